// Micro-benchmark: issue cost (cycles per wave-instruction, s_memtime) of the integer ops the
// Philox4x32-10 generator is built from, one and two waves per SIMD. Diagnostic only.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_valu.hip -o /tmp/ubench_valu
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 256

template <int OP>
__global__ void kern(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + 1 + i);
    const uint32_t m = 0xD2511F53u ^ seed;
    __syncthreads();
    unsigned long long t0 = clock64();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) a[i] = a[i] * m + 1u;                              // mul_lo (+add)
            if (OP == 1) a[i] = __umulhi(a[i], m) ^ it;                     // mul_hi
            if (OP == 2) { uint64_t p = (uint64_t)a[i] * m; a[i] = (uint32_t)(p >> 32) ^ (uint32_t)p; }
            if (OP == 3) a[i] = (a[i] ^ m) + it;                            // plain VALU pair
        }
    }
    unsigned long long t1 = clock64();
    uint32_t x = 0;
    for (int i = 0; i < 8; ++i) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int OP>
void run(const char* name, int waves_per_simd) {
    const int blocks = 256, threads = 256 * waves_per_simd;
    uint32_t* out; unsigned long long* cyc;
    hipMalloc(&out, blocks * threads * 4);
    hipMalloc(&cyc, blocks * threads / 64 * 8);
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, out, cyc, 12345u);
    hipDeviceSynchronize();
    const int nw = blocks * threads / 64;
    unsigned long long* h = (unsigned long long*)malloc(nw * 8);
    hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < nw; ++i) s += h[i];
    printf("%-28s waves/SIMD=%d  cycles per wave per op-group: %.2f\n", name, waves_per_simd,
           s / nw / (ITERS * 8.0));
    free(h); hipFree(out); hipFree(cyc);
}

int main() {
    for (int w = 1; w <= 2; ++w) {
        run<0>("mul_lo+add", w);
        run<1>("mul_hi+xor", w);
        run<2>("u64 product (lo^hi)", w);
        run<3>("xor+add", w);
    }
    return 0;
}
