// Micro-benchmark: the gate kernel's epilogue in isolation (issue model). Each of the
// 8 waves of a workgroup (two per SIMD, one workgroup per CU, as gate_pipe_kernel) folds 64 gated
// products per lane -- the arithmetic of fold_pairs (mcgmil_kernels.h): two FMAs for the arguments,
// clamp, 2 v_exp_f32, 1 + a, (1 + a)(1 + b) as one FMA, v_rcp_f32, two FMAs into the partial score --
// and reports shader cycles (s_memtime) per tile epilogue and per gated product per SIMD.
// Diagnostic only. Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_epi.hip -o /tmp/ubench_epi
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REPS 32

__global__ __launch_bounds__(512) void epi(const float* seed, float* out, unsigned long long* cyc) {
    const int tid = threadIdx.x;
    float acc[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) acc[i] = seed[(tid + 7 * i) & 1023];
    const float av = seed[1] * -2.885390f, au = seed[2] * -1.442695f;
    const float bv = seed[3], bu = seed[4], w = seed[5];
    float part[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // one chain per row tile
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < REPS; ++r) {
#pragma unroll
        for (int i = 0; i < 64; ++i) asm volatile("" : "+v"(acc[i]));   // no hoisting across reps
#pragma unroll
        for (int i = 0; i < 64; i += 2) {
            const float ax = fmaf(acc[i], av, bv);
            const float by = fmaf(acc[i + 1], au, bu);
            const float a = __builtin_amdgcn_exp2f(fminf(fmaxf(ax, -43.28f), 43.28f));
            const float b = __builtin_amdgcn_exp2f(by);
            const float ia = 1.0f + a;
            const float rr = __builtin_amdgcn_rcpf(fmaf(ia, b, ia));
            part[(i >> 1) & 7] = fmaf(fmaf(-a, w, w), rr, part[(i >> 1) & 7]);
        }
        // one product per (V, U) accumulator pair: 32 per lane per rep; two reps = one tile's 64
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(part[k]));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += part[k];
    out[blockIdx.x * 512 + tid] = sum;
    if ((tid & 63) == 0) cyc[blockIdx.x * 8 + (tid >> 6)] = t1 - t0;
}

int main() {
    const int grid = 256;
    float *seed, *out;
    unsigned long long* cyc;
    hipMalloc(&seed, 1024 * 4);
    hipMalloc(&out, grid * 512 * 4);
    hipMalloc(&cyc, grid * 8 * 8);
    float h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = 0.001f * (float)((i * 37) % 2000 - 1000);
    hipMemcpy(seed, h, sizeof h, hipMemcpyHostToDevice);
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(epi, dim3(grid), dim3(512), 0, 0, seed, out, cyc);
    hipDeviceSynchronize();
    unsigned long long hc[grid * 8];
    hipMemcpy(hc, cyc, sizeof hc, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int i = 0; i < grid * 8; ++i) sum += (double)hc[i];
    const double per_rep = sum / (grid * 8) / REPS;        // cycles per wave per 32 products
    // a tile's epilogue = 64 products per lane per wave, two waves per SIMD sharing its issue
    printf("{\"cycles_per_32_products_per_wave\": %.1f, \"tile_epilogue_cycles\": %.0f, "
           "\"cycles_per_product_per_SIMD\": %.1f}\n", per_rep, 2 * per_rep, per_rep / 64);
    return 0;
}
