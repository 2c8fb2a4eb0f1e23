// Micro-benchmark: the gate kernel's K step built up piece by piece, to see which ingredient
// costs MFMA throughput. 8 waves (2 per SIMD), one workgroup per CU, 33 x
// v_mfma_f32_16x16x32_bf16 per wave per step (128 rows x 64 columns + the 16-row z tile).
//   F_PHILOX  one Philox4x32-10 call + packed keep mask per thread per step (x2 with F_PHILOX2)
//   F_LDS     B fragments from LDS (9 ds_read_b128 per wave per step) + 1 ds_write_b128 staging
//   F_BAR     one workgroup barrier per step (two LDS slots)
//   F_VMEM    5 buffer_load_dwordx4 (weights, one step ahead) + 1 global_load_dwordx4 (H) per step
// Reports TFLOP/s of the MFMA work (wall clock, HIP events). Diagnostic only.
// Build: hipcc --offload-arch=gfx950 -O3 -I montecarlo-gated-mil_amd/csrc scripts/ubench_kstep.hip -o scripts/ubench_kstep.bin
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "mcgmil_device.h"

using namespace mcgmil;

constexpr int kSteps = 1024;
enum { F_PHILOX = 1, F_LDS = 2, F_BAR = 4, F_VMEM = 8, F_PHILOX2 = 16, F_EPI = 32 };

template <int F, int RT, int NJ, int WPC>
__global__ __launch_bounds__(512, WPC) void kern(float* out, const __bf16* W, const __bf16* H, uint32_t wbytes,
                                            uint32_t seed) {
    __shared__ __attribute__((aligned(16))) __bf16 Xs[2][8 * 64 * 8];
    __shared__ float red[8][4][128];
    const int tid = threadIdx.x, lane = tid & 63;
    bf16x8 wA[NJ + 1], wB[NJ + 1], xr[RT];
    for (int j = 0; j <= NJ; ++j)
        for (int e = 0; e < 8; ++e) wA[j][e] = wB[j][e] = (__bf16)(0.001f * (lane + j + e));
    for (int r = 0; r < RT; ++r)
        for (int e = 0; e < 8; ++e) xr[r][e] = (__bf16)(0.002f * (lane - r + e));
    for (int i = tid; i < 2 * 8 * 64 * 8; i += 512) (&Xs[0][0])[i] = (__bf16)(0.003f * (i & 255));
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(W, wbytes);
    const uint32_t lane_b = (uint32_t)lane * 16u;
    const __bf16* hsrc = H + ((size_t)blockIdx.x * 512 + tid) * 8;
    uint4 hA = make_uint4(lane, lane * 3, lane * 5, lane * 7), hB = hA;
    f32x4 acc[RT][NJ];
    for (int r = 0; r < RT; ++r)
        for (int j = 0; j < NJ; ++j) acc[r][j] = f32x4{0, 0, 0, 0};
    f32x4 z = {0, 0, 0, 0};
    const int rbase = (RT == 8) ? 0 : (threadIdx.x >> 6 & 1) * 4;
    auto step = [&](int s, bf16x8 (&w)[NJ + 1], bf16x8 (&wn)[NJ + 1], const uint4& h, uint4& hn) {
        const __bf16* cur = Xs[s & 1];
        __bf16* nxt = Xs[(s + 1) & 1];
        if constexpr (F & F_VMEM) {
            hn = *reinterpret_cast<const uint4*>(hsrc + (size_t)((s + 2) & 63) * 512 * 256 * 8);
#pragma unroll
            for (int j = 0; j <= NJ; ++j)
                wn[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                       rs, lane_b, (uint32_t)(((s + 1) & 15) * 9 + j) * 1024u, 0));
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            bf16x8 x = xr[rt];
            if constexpr (F & F_LDS) x = *reinterpret_cast<const bf16x8*>(cur + ((rbase + rt) * 64 + lane) * 8);
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], x, acc[rt][j], 0, 0, 0);
        }
        {
            bf16x8 xz = xr[0];
            if constexpr (F & F_LDS) xz = *reinterpret_cast<const bf16x8*>(cur + tid * 8);
            z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[NJ], xz, z, 0, 0, 0);
        }
        uint4 v = h;
        if constexpr (F & (F_PHILOX | F_PHILOX2)) {
            const uint4 o = philox4x32_10<true>((uint32_t)s * 4 + (lane >> 4), lane, s, seed, seed, ~seed);
            v.x = __builtin_amdgcn_bitop3_b32(v.x, drop_mask16x2_flipped(o.x, 0x19991999u), 0, 0x10);
            v.y = __builtin_amdgcn_bitop3_b32(v.y, drop_mask16x2(o.y, 0x19991999u), 0, 0x10);
            v.z = __builtin_amdgcn_bitop3_b32(v.z, drop_mask16x2_flipped(o.z, 0x19991999u), 0, 0x10);
            v.w = __builtin_amdgcn_bitop3_b32(v.w, drop_mask16x2(o.w, 0x19991999u), 0, 0x10);
        }
        if constexpr (F & F_LDS) *reinterpret_cast<uint4*>(nxt + tid * 8) = v;
        else hn.x ^= v.x ^ v.y ^ v.z ^ v.w;
#pragma unroll
        for (int i = 0; i < RT * NJ + 1; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        if constexpr (F & F_BAR) __syncthreads();
    };
    float keep = 0.f;
    for (int s = 0; s < kSteps; s += 2) {
        step(s, wA, wB, hB, hA);
        step(s + 1, wB, wA, hA, hB);
        if constexpr (F & F_EPI) {
            if ((s & 15) == 14) {   // end of a 16-step tile: gated products, partials, barrier
                float part[RT];
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    part[rt] = 0.f;
#pragma unroll
                    for (int jp = 0; jp < NJ / 2; ++jp)
#pragma unroll
                        for (int v = 0; v < 4; ++v) {
                            const float ax = fmaf(acc[rt][2 * jp][v], -2.88f, 0.1f);
                            const float by = fmaf(acc[rt][2 * jp + 1][v], -1.44f, 0.2f);
                            const float a = __builtin_amdgcn_exp2f(fminf(fmaxf(ax, -43.f), 43.f));
                            const float b = __builtin_amdgcn_exp2f(by);
                            const float ia = 1.f + a;
                            const float r = __builtin_amdgcn_rcpf(fmaf(ia, b, ia));
                            part[rt] = fmaf(fmaf(-a, 0.3f, 0.3f), r, part[rt]);
                        }
                }
                const int wv = threadIdx.x >> 6;
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) red[wv][lane >> 4][(rt * 16 + (lane & 15)) & 127] = part[rt];
                __syncthreads();
                keep += red[(wv + 1) & 7][lane & 3][threadIdx.x & 127];
                __syncthreads();
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int j = 0; j < NJ; ++j) acc[rt][j] = f32x4{0, 0, 0, 0};
            }
        }
    }
    float t = z[0] + z[3] + (float)(hA.x ^ hB.y) + keep;
    for (int r = 0; r < RT; ++r)
        for (int j = 0; j < NJ; ++j) t += acc[r][j][0] + acc[r][j][3];
    out[blockIdx.x * 512 + tid] = t + (float)Xs[1][tid];
}

template <int F, int RT = 8, int NJ = 4, int WPC = 1>
void run(const char* name, float* out, const __bf16* W, const __bf16* H, int cus) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((kern<F, RT, NJ, WPC>), dim3(cus * WPC), dim3(512), 0, 0, out, W, H, 16u * 9 * 1024, 7u);
    hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((kern<F, RT, NJ, WPC>), dim3(cus * WPC), dim3(512), 0, 0, out, W, H, 16u * 9 * 1024, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)cus * WPC * 8 * kSteps * (RT * 16.0 * NJ * 16 * 32 * 2 + 16.0 * 16 * 32 * 2) * reps;
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"tflops\": %.1f}\n", name, ms / reps, flops / (ms * 1e-3) / 1e12);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    __bf16 *W, *H;
    hipMalloc(&out, (size_t)cus * 2 * 512 * sizeof(float));
    hipMalloc(&W, 16 * 9 * 1024);
    hipMalloc(&H, (size_t)cus * 2 * 512 * 8 * 2 + (size_t)64 * 512 * 256 * 8 * 2);
    hipMemset(W, 0, 16 * 9 * 1024);
    hipMemset(H, 0, (size_t)cus * 2 * 512 * 8 * 2 + (size_t)64 * 512 * 256 * 8 * 2);
    constexpr int K = F_LDS | F_BAR | F_VMEM | F_PHILOX;
    run<K>("8x4 K step", out, W, H, cus);
    run<K | F_EPI>("8x4 K step + epilogue, 1 WG/CU", out, W, H, cus);
    run<K, 4, 4, 2>("4x4 K step, 2 WG/CU", out, W, H, cus);
    run<K | F_EPI, 4, 4, 2>("4x4 K step + epilogue, 2 WG/CU", out, W, H, cus);
    run<K | F_EPI, 4, 8>("4x8 K step + epilogue, 1 WG/CU", out, W, H, cus);
    hipFree(out);
    hipFree(W);
    hipFree(H);
    return 0;
}
