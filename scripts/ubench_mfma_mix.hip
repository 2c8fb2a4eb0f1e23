// Micro-benchmark: one K step of the gate kernel's MFMA work (128 rows x 64 columns per wave)
// issued with or without the staging VALU of that step (one Philox4x32-10 call + the packed keep
// mask), as 33 x v_mfma_f32_16x16x32_bf16 or as 16 x v_mfma_f32_32x32x16_bf16 + 1 x 16x16x32.
// 8 waves per workgroup (2 per SIMD), one workgroup per CU, operands in registers. Reports
// TFLOP/s of the MFMA work (wall clock, HIP events). Diagnostic only.
// Build: hipcc --offload-arch=gfx950 -O3 -I montecarlo-gated-mil_amd/csrc scripts/ubench_mfma_mix.hip -o /tmp/ubench_mix
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "mcgmil_device.h"

using namespace mcgmil;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kSteps = 2048;

template <bool BIG, bool VALU>
__global__ __launch_bounds__(512) void kern(float* out, uint32_t seed) {
    const int lane = threadIdx.x & 63;
    bf16x8 a[4], b[4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) {
            a[i][j] = (__bf16)(0.001f * (lane + i + j));
            b[i][j] = (__bf16)(0.002f * (lane - i + j));
        }
    uint32_t acc_r = seed ^ lane;
    uint4 hv = make_uint4(lane, lane * 3, lane * 5, lane * 7);
    if constexpr (BIG) {
        f32x16 acc[8];
        for (int i = 0; i < 8; ++i) acc[i] = f32x16{};
        f32x4 z = {0, 0, 0, 0};
        for (int s = 0; s < kSteps; ++s) {
#pragma unroll
            for (int rt = 0; rt < 4; ++rt)
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    acc[rt * 2 + ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ct * 2], b[rt], acc[rt * 2 + ct], 0, 0, 0);
                    acc[rt * 2 + ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ct * 2 + 1], b[(rt + 1) & 3], acc[rt * 2 + ct], 0, 0, 0);
                }
            z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], z, 0, 0, 0);
            if constexpr (VALU) {
                const uint4 o = philox4x32_10<true>((uint32_t)s * 4 + (lane >> 4), lane, s, seed, seed, ~seed);
                hv.x = __builtin_amdgcn_bitop3_b32(hv.x, drop_mask16x2_flipped(o.x, 0x19991999u), 0, 0x10);
                hv.y = __builtin_amdgcn_bitop3_b32(hv.y, drop_mask16x2(o.y, 0x19991999u), 0, 0x10);
                hv.z = __builtin_amdgcn_bitop3_b32(hv.z, drop_mask16x2_flipped(o.z, 0x19991999u), 0, 0x10);
                hv.w = __builtin_amdgcn_bitop3_b32(hv.w, drop_mask16x2(o.w, 0x19991999u), 0, 0x10);
#pragma unroll
                for (int i = 0; i < 17; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
                }
            }
        }
        float t = z[0] + z[3];
        for (int i = 0; i < 8; ++i) t += acc[i][0] + acc[i][15];
        out[blockIdx.x * 512 + threadIdx.x] = t + (float)(hv.x ^ hv.y ^ hv.z ^ hv.w ^ acc_r);
    } else {
        f32x4 acc[32];
        for (int i = 0; i < 32; ++i) acc[i] = f32x4{0, 0, 0, 0};
        f32x4 z = {0, 0, 0, 0};
        for (int s = 0; s < kSteps; ++s) {
#pragma unroll
            for (int rt = 0; rt < 8; ++rt)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[rt * 4 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[rt & 3], acc[rt * 4 + j], 0, 0, 0);
            z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], z, 0, 0, 0);
            if constexpr (VALU) {
                const uint4 o = philox4x32_10<true>((uint32_t)s * 4 + (lane >> 4), lane, s, seed, seed, ~seed);
                hv.x = __builtin_amdgcn_bitop3_b32(hv.x, drop_mask16x2_flipped(o.x, 0x19991999u), 0, 0x10);
                hv.y = __builtin_amdgcn_bitop3_b32(hv.y, drop_mask16x2(o.y, 0x19991999u), 0, 0x10);
                hv.z = __builtin_amdgcn_bitop3_b32(hv.z, drop_mask16x2_flipped(o.z, 0x19991999u), 0, 0x10);
                hv.w = __builtin_amdgcn_bitop3_b32(hv.w, drop_mask16x2(o.w, 0x19991999u), 0, 0x10);
#pragma unroll
                for (int i = 0; i < 33; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                }
            }
        }
        float t = z[0] + z[3];
        for (int i = 0; i < 32; ++i) t += acc[i][0] + acc[i][3];
        out[blockIdx.x * 512 + threadIdx.x] = t + (float)(hv.x ^ hv.y ^ hv.z ^ hv.w ^ acc_r);
    }
}

template <bool BIG, bool VALU>
void run(const char* name, float* out, int cus) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((kern<BIG, VALU>), dim3(cus), dim3(512), 0, 0, out, 7u);   // warm-up
    hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((kern<BIG, VALU>), dim3(cus), dim3(512), 0, 0, out, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    // per wave per step: 128 rows x 64 cols x 32 k x 2 + the 16-row z tile (16 x 16 x 32 x 2)
    const double flops = (double)cus * 8 * kSteps * (128.0 * 64 * 32 * 2 + 16.0 * 16 * 32 * 2) * reps;
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"tflops\": %.1f}\n", name, ms / reps, flops / (ms * 1e-3) / 1e12);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, (size_t)cus * 512 * sizeof(float));
    run<false, false>("16x16x32 mfma only", out, cus);
    run<true, false>("32x32x16 mfma only", out, cus);
    run<false, true>("16x16x32 + philox valu", out, cus);
    run<true, true>("32x32x16 + philox valu", out, cus);
    hipFree(out);
    return 0;
}
