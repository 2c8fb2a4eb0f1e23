// The box's own MFMA ceiling (include/mcgmil_calib.h): a bare MFMA loop at the gate kernels'
// occupancy and operand path, on random data, so bench.py can state each roofline fraction
// against what this chip sustains as well as against the spec peak.
#include "../../include/mcgmil.h"
#include "../../include/mcgmil_calib.h"
#include "mcgmil_device.h"
#include "mcgmil_error.h"

namespace {

using mcgmil::bf16x8;
using mcgmil::f32x4;

constexpr int kThreads = 512;               // 8 waves: two per SIMD
constexpr int kRingBytes = 64 * 1024;       // B fragments cycled through (64 x 1 KiB)
constexpr int kLdsBytes = 96 * 1024;        // > 80 KiB requested: one workgroup per CU
constexpr int kA = 4, kB = 8;               // A fragments in registers, B fragments per step

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du;
    x ^= x >> 15; x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// a full-range uniform value in [-1, 1): 23 random mantissa bits under exponent 0, minus 1, random sign
__device__ __forceinline__ float uniform_pm1(uint32_t h) {
    const float f = __uint_as_float((h >> 9) | 0x3f800000u) - 1.0f;
    return (h & 1u) ? -f : f;
}

__device__ __forceinline__ uint32_t bf16_pair(uint32_t h0, uint32_t h1) {
    return (__float_as_uint(uniform_pm1(h0)) >> 16) | (__float_as_uint(uniform_pm1(h1)) & 0xFFFF0000u);
}

__device__ __forceinline__ void stamp(uint64_t* clock, int i) {
    if (clock && threadIdx.x == 0 && blockIdx.x < (unsigned)MCGMIL_CLOCK_SLOTS) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        const unsigned long long r = __builtin_amdgcn_s_memrealtime();
        clock[(size_t)blockIdx.x * 4 + 2 * i] = t;
        clock[(size_t)blockIdx.x * 4 + 2 * i + 1] = r;
    }
}

template <bool F32>
__global__ __launch_bounds__(kThreads) void mfma_calib_kernel(uint32_t seed, int steps, float* sink,
                                                              uint64_t* clock) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t base = seed * 0x9E3779B9u + blockIdx.x * 0x85EBCA6Bu;
    for (int i = tid; i < kRingBytes / 16; i += kThreads) {
        uint4 v;
        if constexpr (F32) {
            v = make_uint4(__float_as_uint(uniform_pm1(mix32(base + 4 * i))),
                           __float_as_uint(uniform_pm1(mix32(base + 4 * i + 1))),
                           __float_as_uint(uniform_pm1(mix32(base + 4 * i + 2))),
                           __float_as_uint(uniform_pm1(mix32(base + 4 * i + 3))));
        } else {
            v = make_uint4(bf16_pair(mix32(base + 8 * i), mix32(base + 8 * i + 1)),
                           bf16_pair(mix32(base + 8 * i + 2), mix32(base + 8 * i + 3)),
                           bf16_pair(mix32(base + 8 * i + 4), mix32(base + 8 * i + 5)),
                           bf16_pair(mix32(base + 8 * i + 6), mix32(base + 8 * i + 7)));
        }
        reinterpret_cast<uint4*>(lds)[i] = v;
    }
    __syncthreads();
    stamp(clock, 0);
    const uint32_t abase = mix32(base ^ (uint32_t)(tid * 0x27d4eb2du));
    f32x4 acc[kA][kB];
#pragma unroll
    for (int i = 0; i < kA; ++i)
#pragma unroll
        for (int j = 0; j < kB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // each wave walks the 64 KiB ring from its own start, 8 x 1 KiB fragments per step
    uint32_t off = (uint32_t)wave * kB * 1024u + (uint32_t)lane * 16u;
    if constexpr (F32) {
        f32x4 a[kA];
#pragma unroll
        for (int i = 0; i < kA; ++i)
            a[i] = f32x4{uniform_pm1(mix32(abase + 4 * i)), uniform_pm1(mix32(abase + 4 * i + 1)),
                         uniform_pm1(mix32(abase + 4 * i + 2)), uniform_pm1(mix32(abase + 4 * i + 3))};
        for (int s = 0; s < steps; ++s) {
            f32x4 b[kB];
#pragma unroll
            for (int j = 0; j < kB; ++j)
                b[j] = *reinterpret_cast<const f32x4*>(lds + ((off + j * 1024u) & (kRingBytes - 1)));
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int i = 0; i < kA; ++i)
#pragma unroll
                    for (int j = 0; j < kB; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][k], b[j][k], acc[i][j], 0, 0, 0);
            off += kB * 1024u;
        }
    } else {
        bf16x8 a[kA];
#pragma unroll
        for (int i = 0; i < kA; ++i) {
            const uint4 v = make_uint4(bf16_pair(mix32(abase + 8 * i), mix32(abase + 8 * i + 1)),
                                       bf16_pair(mix32(abase + 8 * i + 2), mix32(abase + 8 * i + 3)),
                                       bf16_pair(mix32(abase + 8 * i + 4), mix32(abase + 8 * i + 5)),
                                       bf16_pair(mix32(abase + 8 * i + 6), mix32(abase + 8 * i + 7)));
            a[i] = __builtin_bit_cast(bf16x8, v);
        }
        for (int s = 0; s < steps; ++s) {
            bf16x8 b[kB];
#pragma unroll
            for (int j = 0; j < kB; ++j)
                b[j] = *reinterpret_cast<const bf16x8*>(lds + ((off + j * 1024u) & (kRingBytes - 1)));
#pragma unroll
            for (int i = 0; i < kA; ++i)
#pragma unroll
                for (int j = 0; j < kB; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
            off += kB * 1024u;
        }
    }
    stamp(clock, 1);
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < kA; ++i)
#pragma unroll
        for (int j = 0; j < kB; ++j) sum += acc[i][j].x + acc[i][j].y + acc[i][j].z + acc[i][j].w;
    sink[(size_t)blockIdx.x * kThreads + tid] = sum;
}

}  // namespace

extern "C" {

int64_t mcgmil_mfma_calib_flops_per_step(int dtype) {
    constexpr int64_t waves = kThreads / 64;
    if (dtype == MCGMIL_BF16) return waves * kA * kB * (2ll * 16 * 16 * 32);
    if (dtype == MCGMIL_F32) return waves * kA * kB * 4 * (2ll * 16 * 16 * 4);
    return 0;
}

int mcgmil_mfma_calib(int dtype, int32_t workgroups, int32_t steps, uint32_t seed, float* sink,
                      uint64_t* clock, void* stream) {
    using mcgmil_detail::fail;
    if (dtype != MCGMIL_BF16 && dtype != MCGMIL_F32) return fail(MCGMIL_E_INVALID, "dtype must be MCGMIL_BF16 or MCGMIL_F32");
    if (workgroups < 1 || workgroups > 65536 || steps < 1) return fail(MCGMIL_E_INVALID, "workgroups in 1..65536 and steps >= 1");
    if (!sink) return fail(MCGMIL_E_INVALID, "sink is NULL");
    const void* k = dtype == MCGMIL_BF16 ? reinterpret_cast<const void*>(&mfma_calib_kernel<false>)
                                         : reinterpret_cast<const void*>(&mfma_calib_kernel<true>);
    if (int rc = mcgmil_detail::raise_lds_limit(k, "mfma_calib_kernel LDS limit")) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (dtype == MCGMIL_BF16)
        hipLaunchKernelGGL(mfma_calib_kernel<false>, dim3(workgroups), dim3(kThreads), kLdsBytes, s, seed, steps,
                           sink, clock);
    else
        hipLaunchKernelGGL(mfma_calib_kernel<true>, dim3(workgroups), dim3(kThreads), kLdsBytes, s, seed, steps,
                           sink, clock);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : mcgmil_detail::hip_fail(e, "mfma_calib_kernel launch");
}

}  // extern "C"
