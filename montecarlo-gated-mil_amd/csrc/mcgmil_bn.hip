// Feature-extractor normalisation (include/mcgmil_features.h): BatchNorm2d on the bag's own
// batch statistics (reference infer.py:105-109 deactivate_batchnorm; the backbone of
// model.py:166-177) fused with the ReLU / residual add that follows it in the ResNet blocks.
//
// Channels-last activations are a [rows, C] matrix. Three launches per layer:
//   bn_partial_kernel   per-workgroup fp32 sums of (x - shift_c) and its square, shift_c = x[0, c]
//                       (keeps E[x^2] - E[x]^2 well conditioned), 16-byte loads, LDS reduction
//   bn_finalize_kernel  fp64 combination of the partials in a fixed order (deterministic), then
//                       a_c = gamma_c / sqrt(var_c + eps), b_c = beta_c - mean_c * a_c
//   bn_apply_kernel     y = x * a_c + b_c (+ residual) (relu), 16-byte loads and stores
// HBM-bound elementwise/reduction work: two reads of x, one write of y (+ the residual read).
// Replaces MIOpen's training-mode BN (mean/variance + normalise) and the separate add / clamp
// kernels PyTorch runs for the same layers.
#include <math.h>

#include <numeric>
#include <string>

#include "../../include/mcgmil_features.h"
#include "mcgmil_device.h"
#include "mcgmil_error.h"

namespace {

using mcgmil_detail::fail;
using mcgmil_detail::hip_fail;
using mcgmil::bf16x8;
using mcgmil::f32x4;

constexpr int kThreads = 256;
constexpr int kMaxC = 2048;           // channel groups of 8 <= threads of a workgroup
constexpr int kMaxParts = 1024;       // statistics workgroups
constexpr long long kBytesPerPart = 64 << 10;   // at least this much input per statistics workgroup
constexpr int kFinCh = 8;             // finalize: channels per workgroup
constexpr int kFinLanes = kThreads / kFinCh;    // finalize: lanes per channel
constexpr int kMaxChanParts = 1024;   // (count, mean, M2) blocks the finalize combines directly
constexpr int kChanChunks = 512;      // above that: chunks of consecutive blocks, at most this many

__device__ __forceinline__ void load8(const __bf16* p, float (&v)[8]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xFFFF0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xFFFF0000u);
    v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xFFFF0000u);
    v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xFFFF0000u);
}
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
// streaming forms for the apply / pool passes (each element read or written exactly once):
// nontemporal loads and stores, measured 20-27% faster on a config-5 layer-1 activation
// (scripts/probe_bn.py; MCGMIL_BN_NT=0 builds the plain ones)
#ifndef MCGMIL_BN_NT
#define MCGMIL_BN_NT 1
#endif
#ifndef MCGMIL_BN_UNROLL
#define MCGMIL_BN_UNROLL 2      // 4 (and 8,192 or 2,048 blocks) measured within 2% (profiles/r04/bn_ab/)
#endif
#ifndef MCGMIL_BN_MAXBLOCKS
#define MCGMIL_BN_MAXBLOCKS 4096
#endif
// bn_vpool_col_kernel walks its columns LAST image first: the stem wrote the activation in image
// order, so its most recent part still sits in the 256 MB Infinity Cache when the pass starts
// (same values, same places): 360-364 -> 352-353 us at config 5 (profiles/r06/bnrev/kernel_stats_*.csv). The same
// reversal of bn_apply_kernel's walk measured no change (201-202 us). 0: first image first.
#ifndef MCGMIL_BN_REVERSE
#define MCGMIL_BN_REVERSE 1
#endif
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void load8s(const __bf16* p, float (&v)[8]) {
#if MCGMIL_BN_NT
    const u32x4 u = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xFFFF0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xFFFF0000u);
    v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xFFFF0000u);
    v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xFFFF0000u);
#else
    load8(p, v);
#endif
}
__device__ __forceinline__ void load8s(const float* p, float (&v)[8]) { load8(p, v); }
[[maybe_unused]] __device__ __forceinline__ void store8(__bf16* p, const float (&v)[8]) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (__bf16)v[j];             // round to nearest even
    *reinterpret_cast<bf16x8*>(p) = o;
}
__device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
    *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
__device__ __forceinline__ void store8s(__bf16* p, const float (&v)[8]) {
#if MCGMIL_BN_NT
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (__bf16)v[j];
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), reinterpret_cast<u32x4*>(p));
#else
    store8(p, v);
#endif
}
__device__ __forceinline__ void store8s(float* p, const float (&v)[8]) { store8(p, v); }

// Workgroup b sums rows [b * rpp, (b + 1) * rpp). Thread (rp, cg): channels 8*cg .. 8*cg+7 of
// rows r0 + rp, r0 + rp + RP, ... with RP = 256 / (C / 8) row lanes.
template <typename E>
__global__ __launch_bounds__(kThreads) void bn_partial_kernel(const E* __restrict__ x, long long rows,
                                                              int C, long long rpp,
                                                              float* __restrict__ part) {
    __shared__ float red[2][kThreads * 8];
    const int tid = threadIdx.x, CG = C >> 3, RP = kThreads / CG;
    const int cg = tid % CG, rp = tid / CG;
    const long long r0 = (long long)blockIdx.x * rpp;
    const long long r1 = r0 + rpp < rows ? r0 + rpp : rows;
    float s[8], ss[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = ss[j] = 0.f;
    if (rp < RP) {
        load8(x + cg * 8, sh);                       // shift: row 0
        long long r = r0 + rp;
        // two rows in flight per iteration (independent loads)
        for (; r + RP < r1; r += 2 * RP) {
            float v[8], w[8];
            load8(x + r * C + cg * 8, v);
            load8(x + (r + RP) * C + cg * 8, w);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float d = v[j] - sh[j], e = w[j] - sh[j];
                s[j] += d + e;
                ss[j] = fmaf(d, d, fmaf(e, e, ss[j]));
            }
        }
        if (r < r1) {
            float v[8];
            load8(x + r * C + cg * 8, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float d = v[j] - sh[j];
                s[j] += d;
                ss[j] = fmaf(d, d, ss[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            red[0][rp * C + cg * 8 + j] = s[j];
            red[1][rp * C + cg * 8 + j] = ss[j];
        }
    }
    __syncthreads();
    for (int c = tid; c < C; c += kThreads) {
        float S = 0.f, SS = 0.f;
        for (int k = 0; k < RP; ++k) {
            S += red[0][k * C + c];
            SS += red[1][k * C + c];
        }
        part[((size_t)blockIdx.x * 2) * C + c] = S;
        part[((size_t)blockIdx.x * 2 + 1) * C + c] = SS;
    }
}

// a_c = gamma_c / sqrt(var_c + eps), b_c = beta_c - mean_c a_c (fp64, stored fp32)
__device__ __forceinline__ void write_ab(int c, int C, double mean, double var, const float* gamma,
                                         const float* beta, double eps, float* ab, float* bmean,
                                         float* binvstd) {
    const double inv = 1.0 / sqrt(var + eps);
    const double g = gamma ? (double)gamma[c] : 1.0, bt = beta ? (double)beta[c] : 0.0;
    ab[c] = (float)(g * inv);
    ab[C + c] = (float)(bt - mean * g * inv);
    if (bmean) bmean[c] = (float)mean;
    if (binvstd) binvstd[c] = (float)inv;
}

// One workgroup per 8 channels, 32 lanes per channel each summing every 32nd partial in fp64;
// the 32 lane sums are combined in lane order (deterministic for a given partial count).
template <typename E>
__global__ __launch_bounds__(kThreads) void bn_finalize_kernel(const float* __restrict__ part, int parts,
                                                               long long rows, int C, const E* __restrict__ x,
                                                               const float* gamma, const float* beta,
                                                               const float* rmean, const float* rvar,
                                                               double eps, float* __restrict__ ab,
                                                               float* bmean, float* binvstd) {
    __shared__ double red[2][kThreads];
    const int tid = threadIdx.x, lane = tid / kFinCh, cl = tid % kFinCh;
    const int c = blockIdx.x * kFinCh + cl;
    double S = 0.0, SS = 0.0;
    if (!rmean && c < C) {
        // unrolled so the partial loads are all in flight (same summation order: one chain each)
#pragma unroll 8
        for (int b = lane; b < parts; b += kFinLanes) {
            S += (double)part[((size_t)b * 2) * C + c];
            SS += (double)part[((size_t)b * 2 + 1) * C + c];
        }
    }
    red[0][tid] = S;
    red[1][tid] = SS;
    __syncthreads();
    if (lane != 0 || c >= C) return;
    double mean, var;
    if (rmean) {
        mean = rmean[c];
        var = rvar[c];
    } else {
        S = SS = 0.0;
        for (int k = 0; k < kFinLanes; ++k) {
            S += red[0][k * kFinCh + cl];
            SS += red[1][k * kFinCh + cl];
        }
        float sh[8];
        load8(x + (c & ~7), sh);
        const double m = S / (double)rows;
        var = SS / (double)rows - m * m;
        if (var < 0.0) var = 0.0;
        mean = (double)sh[c & 7] + m;
    }
    write_ab(c, C, mean, var, gamma, beta, eps, ab, bmean, binvstd);
}

// Statistics from (count, mean, M2) blocks [parts][3][C] (mcgmil_conv2d's epilogue). In fp64,
// around the channel's first block mean m0: N = sum n_b, S = sum n_b (m_b - m0),
// Q = sum M2_b + n_b (m_b - m0)^2, so mean = m0 + S / N and var = (Q - S^2 / N) / N -- exact
// Chan combination without a division per block. Each of 32 lanes sums every 32nd block, then
// the lanes in order (deterministic).
__global__ __launch_bounds__(kThreads) void bn_finalize_chan_kernel(const float* __restrict__ part, int parts,
                                                                  int C, const float* gamma, const float* beta,
                                                                  double eps, float* __restrict__ ab,
                                                                  float* bmean, float* binvstd) {
    __shared__ double red[3][kThreads];
    const int tid = threadIdx.x, lane = tid / kFinCh, cl = tid % kFinCh;
    const int c = blockIdx.x * kFinCh + cl;
    double n = 0.0, S = 0.0, Q = 0.0, m0 = 0.0;
    if (c < C) {
        m0 = (double)part[C + c];
#pragma unroll 8
        for (int b = lane; b < parts; b += kFinLanes) {
            const double nb = (double)part[((size_t)b * 3) * C + c];
            const double d = (double)part[((size_t)b * 3 + 1) * C + c] - m0;
            n += nb;
            S = fma(nb, d, S);
            Q += fma(nb * d, d, (double)part[((size_t)b * 3 + 2) * C + c]);
        }
    }
    red[0][tid] = n;
    red[1][tid] = S;
    red[2][tid] = Q;
    __syncthreads();
    if (lane != 0 || c >= C) return;
    for (int k = 1; k < kFinLanes; ++k) {
        n += red[0][k * kFinCh + cl];
        S += red[1][k * kFinCh + cl];
        Q += red[2][k * kFinCh + cl];
    }
    const double mean = n > 0.0 ? m0 + S / n : 0.0;
    double var = n > 0.0 ? (Q - S * S / n) / n : 0.0;
    if (var < 0.0) var = 0.0;
    write_ab(c, C, mean, var, gamma, beta, eps, ab, bmean, binvstd);
}

// More than kMaxChanParts blocks (an fp32 convolution's one block per pixel tile): chunk j of
// `chunk` consecutive blocks -> one block out[j], thread per channel (coalesced across channels),
// the finalize's fp64 combination around the chunk's first mean, stored back as (n, mean, M2).
__global__ __launch_bounds__(kThreads) void bn_chan_reduce_kernel(const float* __restrict__ part, int parts,
                                                                int C, int chunk, float* __restrict__ out) {
    const int c = blockIdx.y * kThreads + threadIdx.x;
    if (c >= C) return;
    const int b0 = blockIdx.x * chunk, b1 = b0 + chunk < parts ? b0 + chunk : parts;
    const double m0 = (double)part[((size_t)b0 * 3 + 1) * C + c];
    double n = 0.0, S = 0.0, Q = 0.0;
#pragma unroll 4
    for (int b = b0; b < b1; ++b) {
        const double nb = (double)part[((size_t)b * 3) * C + c];
        const double d = (double)part[((size_t)b * 3 + 1) * C + c] - m0;
        n += nb;
        S = fma(nb, d, S);
        Q += fma(nb * d, d, (double)part[((size_t)b * 3 + 2) * C + c]);
    }
    const double M2 = n > 0.0 ? Q - S * S / n : 0.0;
    out[((size_t)blockIdx.x * 3) * C + c] = (float)n;
    out[((size_t)blockIdx.x * 3 + 1) * C + c] = (float)(n > 0.0 ? m0 + S / n : 0.0);
    out[((size_t)blockIdx.x * 3 + 2) * C + c] = (float)(M2 > 0.0 ? M2 : 0.0);
}

// Grid-stride over 8-channel vectors; the total thread count is a multiple of C/8, so every
// thread keeps one channel group. Two vectors in flight per iteration.
// RESBN: the residual gets its own BatchNorm first, rounded to E as a separate pass would store it
template <typename E, bool RELU, bool RES, bool RESBN = false>
__global__ __launch_bounds__(kThreads) void bn_apply_kernel(const E* x, const E* res, E* y, long long nvec,
                                                            int C, const float* __restrict__ ab,
                                                            const float* __restrict__ rab = nullptr) {
    const int CG = C >> 3;
    const long long stride = (long long)gridDim.x * kThreads;
    const long long i0 = (long long)blockIdx.x * kThreads + threadIdx.x;
    const int cg = (int)(i0 % CG);
    float a[8], b[8], ra[8], rb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = ab[cg * 8 + j];
        b[j] = ab[C + cg * 8 + j];
        if (RESBN) {
            ra[j] = rab[cg * 8 + j];
            rb[j] = rab[C + cg * 8 + j];
        }
    }
    auto one = [&](long long i, const float (&v)[8], const float (&r)[8]) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float t = fmaf(v[j], a[j], b[j]);
            if (RESBN) t += (float)(E)fmaf(r[j], ra[j], rb[j]);
            else if (RES) t += r[j];
            o[j] = RELU ? fmaxf(t, 0.f) : t;
        }
        store8s(y + i * 8, o);
    };
    long long i = i0;
    // U vectors per thread and iteration, all loads issued before any arithmetic
    constexpr int U = MCGMIL_BN_UNROLL;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        float v[U][8], r[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            load8s(x + (i + u * stride) * 8, v[u]);
            if (RES) load8s(res + (i + u * stride) * 8, r[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) one(i + u * stride, v[u], r[u]);
    }
    for (; i < nvec; i += stride) {
        float v[8], r[8];
        load8s(x + i * 8, v);
        if (RES) load8s(res + i * 8, r);
        one(i, v, r);
    }
}

// statistics workgroups: ~64 KB of input each (at least 4 row passes), at most 1024
// Activation + k x k max-pool (stride s, pad p, -inf padding): thread per (output pixel,
// 8-channel group); the window's inputs are re-read from L2 by the neighbouring outputs.
template <typename E, bool RELU>
__global__ __launch_bounds__(kThreads) void bn_pool_kernel(const E* __restrict__ x, E* __restrict__ y, int H,
                                                           int W, int Ho, int Wo, int k, int st, int pd,
                                                           long long nvec, int C, const float* __restrict__ ab) {
    const int CG = C >> 3;
    const long long stride = (long long)gridDim.x * kThreads;
    const long long i0 = (long long)blockIdx.x * kThreads + threadIdx.x;
    const int cg = (int)(i0 % CG);
    float a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = ab[cg * 8 + j];
        b[j] = ab[C + cg * 8 + j];
    }
    for (long long i = i0; i < nvec; i += stride) {
        const long long pix = i / CG;
        const int ow = (int)(pix % Wo);
        const long long t = pix / Wo;
        const int oh = (int)(t % Ho);
        const long long n = t / Ho;
        float m[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
        const int h0 = oh * st - pd, w0 = ow * st - pd;
        for (int kh = 0; kh < k; ++kh) {
            const int ih = h0 + kh;
            if (ih < 0 || ih >= H) continue;
            const E* row = x + ((n * H + ih) * (long long)W) * C + cg * 8;
            for (int kw = 0; kw < k; ++kw) {
                const int iw = w0 + kw;
                if (iw < 0 || iw >= W) continue;
                float v[8];
                load8(row + (long long)iw * C, v);
#pragma unroll
                for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], fmaf(v[j], a[j], b[j]));
            }
        }
        if (RELU) {
#pragma unroll
            for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], 0.f);
        }
        store8s(y + i * 8, m);
    }
}

// The stem's pooling pass after its convolution took the horizontal half (mcgmil_stem.hip, HP):
// x is [N, H, W / 2, C] of row maxima, stored negated where a_c < 0 (sign of a = sign of gamma).
// Thread per (output pixel, 8-channel group): the vertical 3-row window (stride 2, pad 1), the
// sign restored, then the BN + ReLU -- equal to bn_pool_kernel's max over the 3 x 3 window of
// fmaf(v, a, b) because fmaf is monotonic in v (non-increasing where a_c < 0).
template <bool RELU>
__global__ __launch_bounds__(kThreads) void bn_vpool_kernel(const __bf16* __restrict__ x, __bf16* __restrict__ y,
                                                            int H, int Wp, int Ho, long long nvec, int C,
                                                            const float* __restrict__ ab) {
    const int CG = C >> 3;
    const long long stride = (long long)gridDim.x * kThreads;
    const long long i0 = (long long)blockIdx.x * kThreads + threadIdx.x;
    const int cg = (int)(i0 % CG);
    float a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = ab[cg * 8 + j];
        b[j] = ab[C + cg * 8 + j];
    }
    for (long long i = i0; i < nvec; i += stride) {
        const long long pix = i / CG;
        const int pw = (int)(pix % Wp);
        const long long t = pix / Wp;
        const int oh = (int)(t % Ho);
        const long long n = t / Ho;
        float m[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
        for (int kh = 0; kh < 3; ++kh) {
            const int ih = 2 * oh - 1 + kh;
            if (ih < 0 || ih >= H) continue;
            float v[8];
            load8(x + (((n * H + ih) * (long long)Wp + pw) * C + cg * 8), v);
#pragma unroll
            for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], v[j]);
        }
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = signbit(a[j]) ? -m[j] : m[j];
            const float r = fmaf(v, a[j], b[j]);
            o[j] = RELU ? fmaxf(r, 0.f) : r;
        }
        store8s(y + i * 8, o);
    }
}

// The same pass with a thread per (image, pooled column, 8-channel group): it walks the column's
// Ho output rows top to bottom, so each input row is read once -- the row 2 oh + 1 that pooled rows
// oh and oh + 1 share is carried in registers (bn_vpool_kernel reads it twice, from L2 if lucky).
template <bool RELU>
__global__ __launch_bounds__(kThreads) void bn_vpool_col_kernel(const __bf16* __restrict__ x, __bf16* __restrict__ y,
                                                                int H, int Wp, int Ho, long long ncol, int C,
                                                                const float* __restrict__ ab) {
    const int CG = C >> 3;
    const long long rs = (long long)Wp * C;          // elements per (pooled-width) row
    for (long long walk = (long long)blockIdx.x * kThreads + threadIdx.x; walk < ncol;
         walk += (long long)gridDim.x * kThreads) {
        const long long col = MCGMIL_BN_REVERSE ? ncol - 1 - walk : walk;   // last image first
        const int cg = (int)(col % CG);
        const long long t = col / CG;
        const int pw = (int)(t % Wp);
        const long long n = t / Wp;
        float a[8], b[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            a[j] = ab[cg * 8 + j];
            b[j] = ab[C + cg * 8 + j];
        }
        const __bf16* xc = x + (n * H * Wp + pw) * (long long)C + cg * 8;
        __bf16* yc = y + (n * Ho * Wp + pw) * (long long)C + cg * 8;
        float carry[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) carry[j] = -INFINITY;   // row -1: padding
#pragma unroll 2
        for (int oh = 0; oh < Ho; ++oh) {
            const int r0 = 2 * oh, r1 = 2 * oh + 1;
            float v0[8], v1[8];
            if (r0 < H) load8s(xc + r0 * rs, v0);
            else
#pragma unroll
                for (int j = 0; j < 8; ++j) v0[j] = -INFINITY;
            if (r1 < H) load8s(xc + r1 * rs, v1);
            else
#pragma unroll
                for (int j = 0; j < 8; ++j) v1[j] = -INFINITY;
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float m = fmaxf(fmaxf(carry[j], v0[j]), v1[j]);
                carry[j] = v1[j];
                const float v = signbit(a[j]) ? -m : m;
                const float r = fmaf(v, a[j], b[j]);
                o[j] = RELU ? fmaxf(r, 0.f) : r;
            }
            store8s(yc + oh * rs, o);
        }
    }
}

int pooled_dim(int size, const mcgmil_bn_args* a) {
    return (size + 2 * a->pool_pad - a->pool_kernel) / a->pool_stride + 1;
}

int parts_for(const mcgmil_bn_args* a) {
    const long long esz = a->dtype == MCGMIL_BF16 ? 2 : 4;
    const long long row_bytes = (long long)a->channels * esz;
    const long long RP = kThreads / (a->channels / 8);
    long long rpp = kBytesPerPart / row_bytes;
    if (rpp < 4 * RP) rpp = 4 * RP;
    const long long p = (a->rows + rpp - 1) / rpp;
    return (int)(p < kMaxParts ? (p < 1 ? 1 : p) : kMaxParts);
}

// blocks per chunk when the producer's partials are reduced first (0: combined directly)
int chan_chunk(const mcgmil_bn_args* a) {
    if (!a->partials || a->running_mean || a->num_partials <= kMaxChanParts) return 0;
    return (a->num_partials + kChanChunks - 1) / kChanChunks;
}

// [2][C] a, b, then the statistics pass's [parts][2][C] sums or the reduced [chunks][3][C] blocks
size_t ws_bytes(const mcgmil_bn_args* a) {
    const size_t C = (size_t)a->channels;
    size_t tail = 2 * C * (size_t)parts_for(a);
    if (const int ch = chan_chunk(a)) {
        const size_t red = 3 * C * (size_t)((a->num_partials + ch - 1) / ch);
        tail = red > tail ? red : tail;
    }
    return ((2 * C + tail) * sizeof(float) + 255) & ~(size_t)255;
}

int validate(const mcgmil_bn_args* a) {
    if (!a) return fail(MCGMIL_E_INVALID, "mcgmil_bn_args is NULL");
    if (a->rows < 1) return fail(MCGMIL_E_INVALID, "rows must be >= 1");
    if (a->channels < 8 || a->channels % 8 || a->channels > kMaxC)
        return fail(MCGMIL_E_UNSUPPORTED, "channels must be a multiple of 8 in [8, 2048], got " +
                                              std::to_string(a->channels));
    if (a->dtype != MCGMIL_BF16 && a->dtype != MCGMIL_F32)
        return fail(MCGMIL_E_INVALID, "dtype must be MCGMIL_BF16 or MCGMIL_F32");
    if (!a->x || !a->y) return fail(MCGMIL_E_INVALID, "x and y are required");
    if (((uintptr_t)a->x | (uintptr_t)a->y | (uintptr_t)a->residual) & 15)
        return fail(MCGMIL_E_ALIGN, "x, y and residual must be 16-byte aligned");
    if ((a->running_mean == nullptr) != (a->running_var == nullptr))
        return fail(MCGMIL_E_INVALID, "running_mean and running_var go together");
    if (!(a->eps >= 0.0)) return fail(MCGMIL_E_INVALID, "eps must be >= 0");
    if (a->relu != 0 && a->relu != 1) return fail(MCGMIL_E_INVALID, "relu must be 0 or 1");
    if (a->partials && (a->num_partials < 1 || ((uintptr_t)a->partials & 3)))
        return fail(MCGMIL_E_INVALID, "partials need num_partials >= 1 and 4-byte alignment");
    if (a->residual_ab && (!a->residual || ((uintptr_t)a->residual_ab & 3)))
        return fail(MCGMIL_E_INVALID, "residual_ab needs a residual and 4-byte alignment");
    if (a->pool_kernel < 0) return fail(MCGMIL_E_INVALID, "pool_kernel must be >= 0");
    if (a->pool_kernel > 0) {
        if (a->batch < 1 || a->height < 1 || a->width < 1 ||
            (long long)a->batch * a->height * a->width != a->rows)
            return fail(MCGMIL_E_INVALID, "pooling needs batch * height * width == rows");
        if (a->pool_stride < 1 || a->pool_pad < 0 || 2 * a->pool_pad > a->pool_kernel)
            return fail(MCGMIL_E_INVALID, "pooling needs stride >= 1 and 0 <= pad <= kernel / 2");
        if (pooled_dim(a->height, a) < 1 || pooled_dim(a->width, a) < 1)
            return fail(MCGMIL_E_INVALID, "pooling window larger than the padded input");
        if (a->residual) return fail(MCGMIL_E_UNSUPPORTED, "no residual add with pooling");
        if (a->x == a->y) return fail(MCGMIL_E_INVALID, "pooling cannot run in place");
    }
    return MCGMIL_OK;
}

template <typename E, bool RELU, bool RES, bool RESBN = false>
void launch_apply(const mcgmil_bn_args* a, const float* ab, hipStream_t s) {
    const long long nvec = a->rows * (a->channels / 8);
    const int CG = a->channels / 8;
    // blocks: a multiple of CG / gcd(CG, 256) so that every thread keeps its channel group
    const int unit = CG / std::gcd(CG, kThreads);
    long long want = (nvec + 2LL * kThreads - 1) / (2LL * kThreads);
    if (want > MCGMIL_BN_MAXBLOCKS) want = MCGMIL_BN_MAXBLOCKS;
    long long blocks = (want + unit - 1) / unit * unit;
    hipLaunchKernelGGL((bn_apply_kernel<E, RELU, RES, RESBN>), dim3((unsigned)blocks), dim3(kThreads), 0, s,
                       static_cast<const E*>(a->x), static_cast<const E*>(a->residual),
                       static_cast<E*>(a->y), nvec, a->channels, ab, a->residual_ab);
}

// finalize (statistics from `parts` partial sums around the per-channel shift row `shift`, or
// the running statistics) then the normalise / pool pass; ab lives at the workspace start
// the normalise / pool pass with a, b at ab
template <typename E>
int apply_step(const mcgmil_bn_args* a, const float* ab, hipStream_t s, bool hpooled = false) {
    const int C = a->channels;
    if (hpooled) {      // bf16 only (the stem); a describes the unpooled [N, H, W, C] activation
        const int Ho = pooled_dim(a->height, a), Wp = a->width / 2;
        const long long nvec = (long long)a->batch * Ho * Wp * (C / 8);
        const int unit = (C / 8) / std::gcd(C / 8, kThreads);
        long long want = (nvec + kThreads - 1) / kThreads;
        if (want > 8192) want = 8192;
        const long long blocks = (want + unit - 1) / unit * unit;
#ifndef MCGMIL_VPOOL_COL
#define MCGMIL_VPOOL_COL 1      // measured: the stem layer 0.725-0.733 -> 0.682 ms at k = 916
#endif
        if (MCGMIL_VPOOL_COL && a->pool_kernel == 3 && a->pool_stride == 2 && a->pool_pad == 1) {
            const long long ncol = (long long)a->batch * Wp * (C / 8);
            long long cb = (ncol + kThreads - 1) / kThreads;
            if (cb > 8192) cb = 8192;
            auto k = a->relu ? bn_vpool_col_kernel<true> : bn_vpool_col_kernel<false>;
            hipLaunchKernelGGL(k, dim3((unsigned)cb), dim3(kThreads), 0, s, static_cast<const __bf16*>(a->x),
                               static_cast<__bf16*>(a->y), a->height, Wp, Ho, ncol, C, ab);
        } else {
            auto k = a->relu ? bn_vpool_kernel<true> : bn_vpool_kernel<false>;
            hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(kThreads), 0, s, static_cast<const __bf16*>(a->x),
                               static_cast<__bf16*>(a->y), a->height, Wp, Ho, nvec, C, ab);
        }
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "batchnorm vertical pool launch");
    }
    if (a->pool_kernel > 0) {
        const int Ho = pooled_dim(a->height, a), Wo = pooled_dim(a->width, a);
        const long long nvec = (long long)a->batch * Ho * Wo * (C / 8);
        const int unit = (C / 8) / std::gcd(C / 8, kThreads);
        long long want = (nvec + kThreads - 1) / kThreads;
        if (want > 8192) want = 8192;
        const long long blocks = (want + unit - 1) / unit * unit;
        auto k = a->relu ? bn_pool_kernel<E, true> : bn_pool_kernel<E, false>;
        hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(kThreads), 0, s, static_cast<const E*>(a->x),
                           static_cast<E*>(a->y), a->height, a->width, Ho, Wo, a->pool_kernel,
                           a->pool_stride, a->pool_pad, nvec, C, ab);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "batchnorm pool launch");
    }
    const bool res = a->residual != nullptr;
    if (res && a->residual_ab) {
        if (a->relu) launch_apply<E, true, true, true>(a, ab, s);
        else launch_apply<E, false, true, true>(a, ab, s);
    } else if (a->relu) {
        if (res) launch_apply<E, true, true>(a, ab, s);
        else launch_apply<E, true, false>(a, ab, s);
    } else {
        if (res) launch_apply<E, false, true>(a, ab, s);
        else launch_apply<E, false, false>(a, ab, s);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "batchnorm launch");
}

// finalize (statistics from `parts` partial sums around the per-channel shift row `shift`, or
// the running statistics) then the normalise / pool pass; ab lives at the workspace start
// ab_out: write a, b there and stop (mcgmil_batchnorm_coefficients); NULL: a, b at the workspace
// start, then the apply / pool pass
template <typename E>
int finish(const mcgmil_bn_args* a, const float* part, int parts, const E* shift, hipStream_t s,
           float* ab_out = nullptr, bool hpooled = false) {
    const int C = a->channels;
    float* ab = ab_out ? ab_out : static_cast<float*>(a->workspace);   // [2][C]
    hipLaunchKernelGGL(bn_finalize_kernel<E>, dim3((C + kFinCh - 1) / kFinCh), dim3(kThreads), 0, s, part, parts, a->rows,
                       C, shift, a->gamma, a->beta, a->running_mean, a->running_var, a->eps, ab,
                       a->batch_mean, a->batch_invstd);
    if (ab_out) {
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "batchnorm finalize launch");
    }
    return apply_step<E>(a, ab, s, hpooled);
}

template <typename E>
int run(const mcgmil_bn_args* a, hipStream_t s, float* ab_out = nullptr) {
    const int C = a->channels;
    float* part = static_cast<float*>(a->workspace) + 2 * C;   // [parts][2][C]
    const E* x = static_cast<const E*>(a->x);
    if (!a->running_mean && a->partials) {       // statistics from the producer's (n, mean, M2)
        float* ab = ab_out ? ab_out : static_cast<float*>(a->workspace);
        const float* blocks = a->partials;
        int nblocks = a->num_partials;
        if (const int ch = chan_chunk(a)) {
            float* red = static_cast<float*>(a->workspace) + 2 * C;
            const int chunks = (nblocks + ch - 1) / ch;
            hipLaunchKernelGGL(bn_chan_reduce_kernel, dim3((unsigned)chunks, (unsigned)((C + kThreads - 1) / kThreads)),
                               dim3(kThreads), 0, s, blocks, nblocks, C, ch, red);
            blocks = red;
            nblocks = chunks;
        }
        hipLaunchKernelGGL(bn_finalize_chan_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kThreads), 0, s,
                           blocks, nblocks, C, a->gamma, a->beta, a->eps, ab, a->batch_mean,
                           a->batch_invstd);
        if (ab_out) {
            const hipError_t e = hipGetLastError();
            return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "batchnorm finalize launch");
        }
        return apply_step<E>(a, ab, s);
    }
    int parts = 0;
    if (!a->running_mean) {
        parts = parts_for(a);
        const long long rpp = (a->rows + parts - 1) / parts;
        hipLaunchKernelGGL(bn_partial_kernel<E>, dim3(parts), dim3(kThreads), 0, s, x, a->rows, C, rpp, part);
    }
    return finish<E>(a, part, parts, x, s, ab_out);   // shift row: x[0, :]
}

}  // namespace

namespace mcgmil_detail {

// The normalisation half of mcgmil_batchnorm_act for a caller that produced the per-channel
// partial sums itself (the stem convolution's epilogue): `parts` blocks of [2][C] fp32 sums of
// (x - shift_c) and (x - shift_c)^2, shift_row the bf16 [C] shift. a->workspace needs 2 * C floats.
int bn_finish_bf16(const mcgmil_bn_args* a, const float* part, int parts, const void* shift_row,
                   hipStream_t s, bool hpooled) {
    if (int rc = validate(a)) return rc;
    if (a->dtype != MCGMIL_BF16) return fail(MCGMIL_E_INVALID, "bn_finish_bf16 needs bf16");
    if (!a->workspace || a->workspace_bytes < 2 * (size_t)a->channels * sizeof(float))
        return fail(MCGMIL_E_WORKSPACE, "bn_finish_bf16: workspace smaller than 2 * C floats");
    if (!a->running_mean && (parts < 1 || !part || !shift_row))
        return fail(MCGMIL_E_INVALID, "bn_finish_bf16: batch statistics need partials and a shift");
    if (hpooled && (a->pool_kernel != 3 || a->pool_stride != 2 || a->pool_pad != 1 || (a->width & 1)))
        return fail(MCGMIL_E_INVALID, "bn_finish_bf16: the row-pooled input needs a 3 x 3 / 2 / pad 1 pool, even width");
    return finish<__bf16>(a, part, parts, static_cast<const __bf16*>(shift_row), s, nullptr, hpooled);
}

}  // namespace mcgmil_detail

extern "C" {

size_t mcgmil_bn_args_size(void) { return sizeof(mcgmil_bn_args); }

int mcgmil_bn_workspace_size(const mcgmil_bn_args* a, size_t* bytes) {
    if (int rc = validate(a)) return rc;
    if (!bytes) return fail(MCGMIL_E_INVALID, "bytes is NULL");
    *bytes = ws_bytes(a);
    return MCGMIL_OK;
}

int mcgmil_batchnorm_act(const mcgmil_bn_args* a, void* stream) {
    if (int rc = validate(a)) return rc;
    if (!a->workspace || a->workspace_bytes < ws_bytes(a) || ((uintptr_t)a->workspace & 255))
        return fail(MCGMIL_E_WORKSPACE, "workspace missing, misaligned or smaller than "
                                        "mcgmil_bn_workspace_size()");
    hipStream_t s = static_cast<hipStream_t>(stream);
    return a->dtype == MCGMIL_BF16 ? run<__bf16>(a, s) : run<float>(a, s);
}

int mcgmil_batchnorm_coefficients(const mcgmil_bn_args* a, float* ab, void* stream) {
    if (!a) return fail(MCGMIL_E_INVALID, "mcgmil_bn_args is NULL");
    if (!ab || ((uintptr_t)ab & 3)) return fail(MCGMIL_E_INVALID, "ab must be a 4-byte aligned [2][C] buffer");
    // the apply-side fields do not matter here: validate the rest as mcgmil_batchnorm_act would
    mcgmil_bn_args b = *a;
    b.residual = nullptr;
    b.residual_ab = nullptr;
    b.pool_kernel = 0;
    b.relu = 0;
    // x is only read by the statistics pass; y never (a placeholder keeps validate() generic)
    void* const placeholder = reinterpret_cast<void*>(static_cast<uintptr_t>(256));
    b.y = b.x ? const_cast<void*>(b.x) : placeholder;
    if (!b.x) b.x = placeholder;
    if (int rc = validate(&b)) return rc;
    const bool pass = !b.running_mean && !b.partials;     // statistics from a pass over x
    if (pass && !a->x) return fail(MCGMIL_E_INVALID, "batch statistics without partials need x");
    if ((pass || chan_chunk(&b)) &&
        (!b.workspace || b.workspace_bytes < ws_bytes(&b) || ((uintptr_t)b.workspace & 255)))
        return fail(MCGMIL_E_WORKSPACE, "workspace missing, misaligned or smaller than "
                                        "mcgmil_bn_workspace_size()");
    hipStream_t s = static_cast<hipStream_t>(stream);
    return b.dtype == MCGMIL_BF16 ? run<__bf16>(&b, s, ab) : run<float>(&b, s, ab);
}

}  // extern "C"
