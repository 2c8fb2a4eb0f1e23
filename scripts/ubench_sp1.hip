// Micro-benchmark: one wave per SIMD (4-wave workgroup, 512 registers per lane), a persistent
// gate-tile loop whose epilogue is software-pipelined into the MFMA stream -- priced before
// writing the kernel. Per 128-row tile a wave owns 4 gate pairs (8 column tiles) in two halves
// of 2 pairs (accA / accB, 128 accumulators each) and the whole masked H tile sits in LDS
// (128 KB):
//   phase A  16 steps: MFMAs of half A (8 row tiles x 4 column tiles + 1 classifier tile) from
//            the resident tile; meanwhile 4 gated products per lane of half B of the previous
//            tile. No barrier.
//   phase B  16 steps: MFMAs of half B; 4 gated products of half A; the next tile's K slice
//            s-1 (free once every wave has passed step s-1) staged with its dropout masks; one
//            barrier per step.
// Staging modes: 0 = two Philox4x32-10 calls per thread per step (current mask rule),
//                1 = alias-table masks (half a Philox call + two LDS table reads per chunk),
//                2 = no staging (upper bound).
// Against it: the current kernel's shape (8 waves, 33 MFMAs + Philox + staging + barrier per
// step, then the whole epilogue). Work per tile is equal: 4224 MFMAs per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -I montecarlo-gated-mil_amd/csrc scripts/ubench_sp1.hip -o scripts/ubench_sp1.bin
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "mcgmil_device.h"

using namespace mcgmil;

constexpr int kTiles = 32;
constexpr int KS = 16;

__device__ __forceinline__ float gp(float x, float y, float c, float part) {
    const float ax = fmaf(x, -2.88f, 0.1f), by = fmaf(y, -1.44f, 0.2f);
    const float a = __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(ax, -43.f, 43.f));
    const float b = __builtin_amdgcn_exp2f(by);
    const float ia = 1.f + a;
    const float r = __builtin_amdgcn_rcpf(fmaf(ia, b, ia));
    return fmaf(fmaf(-a, c, c), r, part);
}

template <int MODE, int VPM>
__global__ __launch_bounds__(256, 1) void sp1_kern(float* out, const __bf16* W, const __bf16* H,
                                                    uint32_t seed, const uint32_t* tbl) {
    __shared__ __attribute__((aligned(16))) __bf16 Xs[KS][8 * 64 * 8];   // 128 KB: the whole tile
    __shared__ uint32_t atbl[256];
    __shared__ uint4 xtbl[256];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < KS * 8 * 64 * 8; i += 256) (&Xs[0][0])[i] = (__bf16)(0.003f * (i & 255));
    atbl[tid] = tbl[tid];
    xtbl[tid] = keep_expand16((uint32_t)tid);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(W, 1024 * 1024);
    const uint32_t lane_b = (uint32_t)lane * 16u;
    const uint32_t wbase = (uint32_t)__builtin_amdgcn_readfirstlane(wave) * 8u * 16384u;
    const __bf16* hsrc = H + ((size_t)blockIdx.x * 256 + tid) * 8;
    f32x4 accA[8][4], accB[8][4], z = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) accA[r][j] = accB[r][j] = f32x4{0.001f * lane, 0, 0, 0};
    bf16x8 w0[5], w1[5];
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) w0[j][e] = w1[j][e] = (__bf16)(0.001f * (lane + j + e));
    float part[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) part[r] = 0.f;
    uint4 h[2] = {make_uint4(lane, 3, 5, 7), make_uint4(lane, 9, 5, 7)}, hn[2] = {h[0], h[1]};
    uint4 ph = make_uint4(lane, seed, 1, 2);
    int tt = 0;
    int zoff = 0;   // laundered per tile: keeps the unrolled steps' addresses out of the tile loop
    auto step = [&](int s, f32x4 (&acc)[8][4], f32x4 (&fin)[8][4], bool phaseB, bf16x8 (&w)[5],
                    bf16x8 (&wn)[5]) {
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t half = phaseB ? 4u * 16384u : 0u;
#pragma unroll
        for (int j = 0; j < 5; ++j)
            wn[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rs, lane_b, wbase + half + (uint32_t)((s + 1) & 15) * 1024u + j * 16384u, 0));
        if (MODE != 2 && phaseB) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
                hn[i] = *reinterpret_cast<const uint4*>(hsrc + zoff + (size_t)((s + 2) & 63) * 256 * 256 * 8 + i * 2048);
        }
        const __bf16* cur = Xs[s] + zoff;
#pragma unroll
        for (int rt = 0; rt < 8; ++rt) {
            const bf16x8 x = *reinterpret_cast<const bf16x8*>(cur + (rt * 64 + lane) * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], x, s == 0 ? f32x4{0, 0, 0, 0} : acc[rt][j], 0, 0, 0);
        }
        {
            const bf16x8 xz = *reinterpret_cast<const bf16x8*>(cur + ((2 * wave + (phaseB ? 1 : 0)) * 64 + lane) * 8);
            z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[4], xz, z, 0, 0, 0);
        }
        // 4 gated products of the finished half: row tile s/2, pair s&1, values 0..3
        {
            const int rt = s >> 1, jp = s & 1;
#pragma unroll
            for (int v = 0; v < 4; ++v) part[rt] = gp(fin[rt][2 * jp][v], fin[rt][2 * jp + 1][v], 0.3f, part[rt]);
        }
        if (MODE != 2 && phaseB) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                uint4 v = h[i];
                if (MODE == 0) {
                    const uint4 o = philox4x32_10<true>((uint32_t)s * 4 + ((lane + zoff) >> 4) + i, lane + zoff,
                                                        (uint32_t)tt, seed, seed, ~seed);
                    v.x = __builtin_amdgcn_bitop3_b32(v.x, drop_mask16x2_flipped(o.x, 0x19991999u), 0, 0x10);
                    v.y = __builtin_amdgcn_bitop3_b32(v.y, drop_mask16x2(o.y, 0x19991999u), 0, 0x10);
                    v.z = __builtin_amdgcn_bitop3_b32(v.z, drop_mask16x2_flipped(o.z, 0x19991999u), 0, 0x10);
                    v.w = __builtin_amdgcn_bitop3_b32(v.w, drop_mask16x2(o.w, 0x19991999u), 0, 0x10);
                } else {
                    if (i == 0 && (s & 1) == 0)
                        ph = philox4x32_10<false>((uint32_t)s + ((lane + zoff) >> 4), lane + zoff, (uint32_t)tt, seed,
                                                  seed, ~seed);
                    const uint32_t wd = (s & 1) ? (i ? ph.w : ph.z) : (i ? ph.y : ph.x);
                    const uint4 m = xtbl[keep_byte_alias(wd, atbl)];
                    v.x = __builtin_amdgcn_bitop3_b32(v.x, m.x, 0u, 0x40);
                    v.y = __builtin_amdgcn_bitop3_b32(v.y, m.y, 0u, 0x40);
                    v.z = __builtin_amdgcn_bitop3_b32(v.z, m.z, 0u, 0x40);
                    v.w = __builtin_amdgcn_bitop3_b32(v.w, m.w, 0u, 0x40);
                }
                if (s > 0) *reinterpret_cast<uint4*>(&Xs[s - 1][0] + zoff + (tid + 256 * i) * 8) = v;
                h[i] = hn[i];
            }
        }
#pragma unroll
        for (int i = 0; i < 33; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
        }
        if (MODE != 2 && phaseB) __syncthreads();
    };
    for (int t = 0; t < kTiles; ++t) {
        asm volatile("" : "+s"(zoff));
        tt = t;
#pragma unroll
        for (int s = 0; s < KS; s += 2) {      // phase A: half A, finish half B
            step(s, accA, accB, false, w0, w1);
            step(s + 1, accA, accB, false, w1, w0);
        }
#pragma unroll
        for (int s = 0; s < KS; s += 2) {      // phase B: half B, finish half A, stage next tile
            step(s, accB, accA, true, w0, w1);
            step(s + 1, accB, accA, true, w1, w0);
        }
    }
    float t = z[0] + (float)(h[0].x ^ h[1].w);
#pragma unroll
    for (int r = 0; r < 8; ++r) t += part[r] + accA[r][0][0] + accB[r][1][3];
    out[blockIdx.x * 256 + tid] = t + (float)Xs[3][tid];
}

// the current kernel's shape: 8 waves, 33 MFMAs + Philox + staging + barrier per step, then the
// epilogue
__global__ __launch_bounds__(512, 1) void cur_kern(float* out, const __bf16* W, const __bf16* H,
                                                   uint32_t seed, const uint32_t*) {
    __shared__ __attribute__((aligned(16))) __bf16 Xs[2][8 * 64 * 8];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 2 * 8 * 64 * 8; i += 512) (&Xs[0][0])[i] = (__bf16)(0.003f * (i & 255));
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(W, 1024 * 1024);
    const uint32_t lane_b = (uint32_t)lane * 16u;
    const __bf16* hsrc = H + ((size_t)blockIdx.x * 512 + tid) * 8;
    f32x4 acc[8][4], z = {0, 0, 0, 0};
    bf16x8 w0[5], w1[5];
    for (int j = 0; j < 5; ++j)
        for (int e = 0; e < 8; ++e) w0[j][e] = w1[j][e] = (__bf16)(0.001f * (lane + j + e));
    float part[8];
    for (int r = 0; r < 8; ++r) part[r] = 0.f;
    uint4 h = make_uint4(lane, 3, 5, 7), hn = h;
    auto step = [&](int s, bf16x8 (&w)[5], bf16x8 (&wn)[5]) {
#pragma unroll
        for (int j = 0; j < 5; ++j)
            wn[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rs, lane_b, (uint32_t)((s + 1) & 15) * 5120u + j * 1024u, 0));
        hn = *reinterpret_cast<const uint4*>(hsrc + (size_t)((s + 2) & 63) * 512 * 256 * 8);
        const __bf16* cur = Xs[s & 1];
#pragma unroll
        for (int rt = 0; rt < 8; ++rt) {
            const bf16x8 x = *reinterpret_cast<const bf16x8*>(cur + (rt * 64 + lane) * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], x, acc[rt][j], 0, 0, 0);
        }
        const bf16x8 xz = *reinterpret_cast<const bf16x8*>(cur + tid * 8);
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[4], xz, z, 0, 0, 0);
        const uint4 o = philox4x32_10<true>((uint32_t)s * 4 + (lane >> 4), lane, s, seed, seed, ~seed);
        uint4 v = h;
        v.x = __builtin_amdgcn_bitop3_b32(v.x, drop_mask16x2_flipped(o.x, 0x19991999u), 0, 0x10);
        v.y = __builtin_amdgcn_bitop3_b32(v.y, drop_mask16x2(o.y, 0x19991999u), 0, 0x10);
        v.z = __builtin_amdgcn_bitop3_b32(v.z, drop_mask16x2_flipped(o.z, 0x19991999u), 0, 0x10);
        v.w = __builtin_amdgcn_bitop3_b32(v.w, drop_mask16x2(o.w, 0x19991999u), 0, 0x10);
        *reinterpret_cast<uint4*>(&Xs[(s + 1) & 1][0] + tid * 8) = v;
        h = hn;
#pragma unroll
        for (int i = 0; i < 33; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        __syncthreads();
    };
    for (int t = 0; t < kTiles; ++t) {
        for (int r = 0; r < 8; ++r)
            for (int j = 0; j < 4; ++j) acc[r][j] = f32x4{0.001f * lane, 0, 0, 0};
        for (int s = 0; s < KS; s += 2) {
            step(s, w0, w1);
            step(s + 1, w1, w0);
        }
#pragma unroll
        for (int rt = 0; rt < 8; ++rt)
#pragma unroll
            for (int jp = 0; jp < 2; ++jp)
#pragma unroll
                for (int v = 0; v < 4; ++v) part[rt] = gp(acc[rt][2 * jp][v], acc[rt][2 * jp + 1][v], 0.3f, part[rt]);
        __syncthreads();
    }
    float t = z[0] + (float)(h.x ^ h.w);
    for (int r = 0; r < 8; ++r) t += part[r] + acc[r][0][0];
    out[blockIdx.x * 512 + tid] = t + (float)Xs[1][tid];
}

__global__ void fill_kernel(__bf16* p, size_t n, uint32_t seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t x = (uint32_t)i * 0x9E3779B9u ^ seed;
        p[i] = (__bf16)(((x >> 8) & 0xFFFF) * (1.0f / 65536.0f) - 0.25f);
    }
}

template <typename K>
void run(const char* name, K kern, int threads, float* out, const __bf16* W, const __bf16* H,
         const uint32_t* tbl, int cus) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), 0, 0, out, W, H, 7u, tbl);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), 0, 0, out, W, H, 7u, tbl);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)cus * kTiles * 4224.0 * (16.0 * 16 * 32 * 2) * reps;
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"tflops\": %.1f}\n", name, ms / reps, flops / (ms * 1e-3) / 1e12);
    fflush(stdout);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    __bf16 *W, *H;
    uint32_t* tbl;
    const size_t hn = (size_t)cus * 512 * 8 + (size_t)64 * 512 * 256 * 8;
    hipMalloc(&out, (size_t)cus * 512 * sizeof(float));
    hipMalloc(&W, 1024 * 1024);
    hipMalloc(&H, hn * 2);
    hipMalloc(&tbl, 1024);
    hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, W, (size_t)512 * 1024, 1u);
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, H, hn, 2u);
    uint32_t h_tbl[256];
    for (int i = 0; i < 256; ++i) h_tbl[i] = ((uint32_t)(i * 40503u) & 0xFFFFFFu) << 8 | (uint32_t)(255 - (i & 7));
    hipMemcpy(tbl, h_tbl, 1024, hipMemcpyHostToDevice);
    run("current shape (8 waves)", cur_kern, 512, out, W, H, tbl, cus);
    run("sp1 Philox x2 staging, VPM 2", sp1_kern<0, 2>, 256, out, W, H, tbl, cus);
    run("sp1 alias staging, VPM 2", sp1_kern<1, 2>, 256, out, W, H, tbl, cus);
    run("sp1 no staging, VPM 2", sp1_kern<2, 2>, 256, out, W, H, tbl, cus);
    run("sp1 Philox x2 staging, VPM 3", sp1_kern<0, 3>, 256, out, W, H, tbl, cus);
    run("sp1 alias staging, VPM 3", sp1_kern<1, 3>, 256, out, W, H, tbl, cus);
    run("sp1 alias staging, VPM 1", sp1_kern<1, 1>, 256, out, W, H, tbl, cus);
    run("current shape (again)", cur_kern, 512, out, W, H, tbl, cus);
    hipFree(out);
    hipFree(W);
    hipFree(H);
    hipFree(tbl);
    return 0;
}
