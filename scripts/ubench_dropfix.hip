// Micro-benchmark for SURVEY.md §7 hard part 1, the dropped-feature identity on the fp32 line:
//   (H ⊙ keep) W^T · sf = sf · (H W^T − (H ⊙ drop) W^T)
// H W^T once per instance row (a plain GEMM, priced separately), then per (t, n) row-sample the
// correction sum over its ~10% dropped features, on VALU with W from LDS. This times that
// correction -- the part the identity adds -- for one config-3 bag's worth of row-samples (N = 2048,
// T = 100, L = 512, 512 gate columns), with random drop masks at p = 0.1 and a stand-in epilogue
// (sum of the corrected pre-activations) so nothing is dead code. Diagnostic only.
//
// Layout: lane = row-sample (its own dropped list), 32 columns per pass in registers, the W^T
// column chunk [512 l][32] fp32 (64 KiB) in LDS with its 16-byte pieces rotated by row (random
// rows per lane otherwise fall on 2 bank groups), the drop masks in LDS.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_dropfix.hip -o /tmp/ubench_dropfix
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int L = 512, NCOL = 512, CW = 32, NCHUNK = NCOL / CW, N = 2048, T = 100;
constexpr long long RS = (long long)N * T;

__global__ void make_masks(uint32_t* masks, long long rs, uint32_t thr, uint32_t seed) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rs * 16) return;
    uint32_t w = 0;
    for (int b = 0; b < 32; ++b) {
        uint32_t x = (uint32_t)(i * 32 + b) * 0x9E3779B1u ^ seed;
        x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
        w |= (x < thr ? 1u : 0u) << b;
    }
    masks[i] = w;
}

template <int THREADS, int ROT, int PIPE>
__global__ __launch_bounds__(THREADS) void dropfix(const float* __restrict__ H, const float* __restrict__ Wt,
                                                   const float* __restrict__ P, const uint32_t* __restrict__ masks,
                                                   float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float wl[L * CW];        // 64 KiB
    __shared__ uint32_t ml[16 * THREADS];                            // [word][thread]
    constexpr int HR = THREADS / T + 2;                              // H rows a workgroup touches
    __shared__ __attribute__((aligned(16))) float hl[HR * L];
    const int tid = threadIdx.x;
    const long long rs0 = (long long)blockIdx.x * THREADS;
    const long long rs = rs0 + tid;
    const bool live = rs < RS;
    const long long rr = live ? rs : 0;
    const int n0 = (int)(rs0 / T);
    const int n = (int)(rr / T);
    for (int i = tid; i < HR * L; i += THREADS) {
        const int r = n0 + i / L;
        hl[i] = r < N ? H[(size_t)r * L + (i % L)] : 0.f;
    }
    const float* hrow = hl + (live ? n - n0 : 0) * L;
    for (int w = 0; w < 16; ++w) ml[w * THREADS + tid] = live ? masks[rr * 16 + w] : 0u;
    float tot = 0.f;
    for (int c = 0; c < NCHUNK; ++c) {
        __syncthreads();
        for (int i = tid; i < L * CW / 4; i += THREADS) {          // 16-byte pieces, row l = i / 8
            const int l = i >> 3, q = i & 7;
            const int qs = ROT ? ((q + l) & 7) : q;
            *reinterpret_cast<float4*>(wl + l * CW + qs * 4) =
                *reinterpret_cast<const float4*>(Wt + ((size_t)c * L + l) * CW + q * 4);
        }
        __syncthreads();
        float acc[CW];
#pragma unroll
        for (int j = 0; j < CW; ++j) acc[j] = 0.f;
        int wi = 0;
        uint32_t m = ml[tid];
        auto next = [&]() -> int {      // next dropped feature of this lane, -1 when done
            while (m == 0u && wi < 15) m = ml[++wi * THREADS + tid];
            if (m == 0u) return -1;
            const int l = 32 * wi + __builtin_ctz(m);
            m &= m - 1u;
            return l;
        };
        auto fetch = [&](int l, float& h, float4 (&v)[8]) {
            const int ll = l < 0 ? 0 : l;
            h = l < 0 ? 0.f : hrow[ll];
            const float* wr = wl + ll * CW;
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const float4*>(wr + (ROT ? ((q + ll) & 7) : q) * 4);
        };
        auto accum = [&](float h, const float4 (&v)[8]) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                acc[4 * q + 0] = fmaf(h, v[q].x, acc[4 * q + 0]);
                acc[4 * q + 1] = fmaf(h, v[q].y, acc[4 * q + 1]);
                acc[4 * q + 2] = fmaf(h, v[q].z, acc[4 * q + 2]);
                acc[4 * q + 3] = fmaf(h, v[q].w, acc[4 * q + 3]);
            }
        };
        if constexpr (PIPE) {
            // software-pipelined: the next feature's h and W row are read while the current FMAs run
            int l = next();
            float h; float4 v[8];
            fetch(l, h, v);
            while (__builtin_amdgcn_ballot_w64(l >= 0) != 0) {
                const int ln = l >= 0 ? next() : -1;
                float hn; float4 vn[8];
                fetch(ln, hn, vn);
                accum(h, v);                    // h = 0 for finished lanes
                l = ln; h = hn;
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = vn[q];
            }
        } else {
            while (true) {
                const int l = next();
                if (l < 0) break;
                float h; float4 v[8];
                fetch(l, h, v);
                accum(h, v);
            }
        }
        const float* prow = P + (size_t)n * NCOL + c * CW;
#pragma unroll
        for (int j = 0; j < CW; ++j) tot += prow[j] - acc[j];
    }
    if (live) out[rs] = tot;
}

template <int THREADS, int ROT, int PIPE>
float run(const float* H, const float* Wt, const float* P, const uint32_t* masks, float* out) {
    const int grid = (int)((RS + THREADS - 1) / THREADS);
    hipLaunchKernelGGL((dropfix<THREADS, ROT, PIPE>), dim3(grid), dim3(THREADS), 0, 0, H, Wt, P, masks, out);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int reps = 20;
    hipEventRecord(e0);
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((dropfix<THREADS, ROT, PIPE>), dim3(grid), dim3(THREADS), 0, 0, H, Wt, P, masks, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    float *H, *Wt, *P, *out;
    uint32_t* masks;
    hipMalloc(&H, (size_t)N * L * 4);
    hipMalloc(&Wt, (size_t)NCOL * L * 4);
    hipMalloc(&P, (size_t)N * NCOL * 4);
    hipMalloc(&out, RS * 4);
    hipMalloc(&masks, RS * 16 * 4);
    hipMemset(H, 0, (size_t)N * L * 4);
    hipMemset(Wt, 0, (size_t)NCOL * L * 4);
    hipMemset(P, 0, (size_t)N * NCOL * 4);
    const long long words = RS * 16;
    hipLaunchKernelGGL(make_masks, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, 0, masks, RS,
                       (uint32_t)(0.1 * 4294967296.0), 1234u);
    hipDeviceSynchronize();
    // average dropped count (the identity's FMA count per row-sample = dropped x 512 columns)
    uint32_t* hm = (uint32_t*)malloc(RS * 16 * 4);
    hipMemcpy(hm, masks, RS * 16 * 4, hipMemcpyDeviceToHost);
    double cnt = 0;
    for (long long i = 0; i < RS * 16; ++i) cnt += __builtin_popcount(hm[i]);
    free(hm);
    const double fma = cnt * NCOL;
    struct { const char* name; float ms; } r[5] = {
        {"256 threads, rotated rows, H in LDS", run<256, 1, 0>(H, Wt, P, masks, out)},
        {"256 threads, rotated rows, H in LDS, pipelined", run<256, 1, 1>(H, Wt, P, masks, out)},
        {"512 threads, rotated rows, H in LDS, pipelined", run<512, 1, 1>(H, Wt, P, masks, out)},
        {"256 threads, plain rows, H in LDS, pipelined", run<256, 0, 1>(H, Wt, P, masks, out)},
        {"128 threads, rotated rows, H in LDS, pipelined", run<128, 1, 1>(H, Wt, P, masks, out)}};
    printf("{\"dropped_per_row_sample\": %.2f, \"fma_per_bag\": %.4g}\n", cnt / RS, fma);
    for (auto& x : r)
        printf("{\"variant\": \"%s\", \"ms_per_bag\": %.4f, \"tfma_per_s\": %.2f}\n", x.name, x.ms,
               fma / (x.ms * 1e-3) / 1e12);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e)); return 1; }
    return 0;
}
