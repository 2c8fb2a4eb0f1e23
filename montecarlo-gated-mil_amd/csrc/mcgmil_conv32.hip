// fp32 convolution for the backbone at the reference precision (config 5's fp32 line): an implicit
// GEMM on v_mfma_f32_16x16x4_f32 with fp32 operands and fp32 accumulation, NHWC in and out.
// Reference: torch.nn.Conv2d.forward in fp32 (model.py:166-179, the ResNet feature extractor).
//
// GEMM view: rows = output channels (the A operand, weights), columns = output pixels (the B
// operand, im2col of x), K = (kh, kw, ci) in steps of 16 input channels of one tap. A workgroup of
// 4 waves computes BN_CO x BM_PX = 128 x 128 (or 64 x 256 when Cout = 64), each wave a 64 x 64
// block = 4 x 4 tiles of 16 x 16 (64 accumulator VGPRs). Per 16-deep K step a wave issues 64 MFMAs
// (32 cycles each on its SIMD) against 32 ds_read_b32 of LDS fragments, so the matrix pipe, not
// LDS or memory, sets the pace. Staging: the next K step's A and B pieces are loaded into
// registers while the current one computes, then written to the other of two LDS stages.
//
// LDS fragments: lane l of a 16x16x4 fp32 MFMA holds A[row l&15][k l>>4] and B[k l>>4][col l&15];
// the stages are k-major rows ([16][BN_CO + 16] and [16][BM_PX + 16] floats), so the 16 lanes of
// one k read 16 consecutive words and the 16-word row pad puts the next k on the next 16 banks:
// every ds_read_b32 is conflict-free. The C layout gives a lane 4 consecutive output channels of
// one pixel: one 16-byte store per tile.
//
// INBN: the input BatchNorm of the previous layer (mcgmil_conv_args.in_ab) is applied to the B
// elements as they are written to LDS (after the step's MFMAs, so the loads stay in flight), so
// relu(bn(x)) is never materialised. STATS: the epilogue also reduces its outputs to one
// (count, mean, M2) block per channel of the tile (shifted sums over a wave's pixels, then the
// waves sharing the channels; tile_stats) for the BatchNorm that follows, so the activation is
// not re-read for statistics.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/mcgmil.h"
#include "../../include/mcgmil_features.h"
#include "mcgmil_device.h"
#include "mcgmil_error.h"

namespace {

using mcgmil_detail::fail;
using mcgmil_detail::hip_fail;

typedef __attribute__((ext_vector_type(4))) float f32x4;

struct Conv32Geom {
    int N, H, W, Cin, Cout, KH, KW, stride, pad, OH, OW;
    long long P;          // N * OH * OW output pixels
    int KS;               // K steps of 16: KH * KW * Cin / 16, or ceil(KH * KW * Cin / 16) (gather)
    int Ktot;             // KH * KW * Cin
    const float* in_ab;   // INBN: [2][Cin] a_c then b_c
    float in_lo;          // INBN: floor after the BatchNorm, 0 (ReLU) or -inf
    float* stats;         // STATS: [pixel tiles][3][Cout] (count, mean, M2)
};

// Gather mode (in_channels not a multiple of 16: the 3-channel stem): K is the flattened
// (kh, kw, ci) of the NHWC window, zero-padded to whole steps, and every B element is its own
// 4-byte load through a per-workgroup LDS table of k -> (offset in the window, kh, kw).
constexpr int kMaxGatherK = 1024;
constexpr int kMaxInBnC = 2048;     // INBN: a_c, b_c of up to this many input channels in LDS

constexpr int kK = 16;    // K step (input channels of one tap)
constexpr int kPad = 16;  // LDS row pad (words)

template <int WCO, int WPX>
struct Tile {
    static constexpr int BN_CO = 64 * WCO, BM_PX = 64 * WPX;
    static constexpr int AS = BN_CO + kPad, BS = BM_PX + kPad;              // row strides (floats)
    static constexpr int STAGE = kK * (AS + BS);                             // floats per stage
    static constexpr int A4 = kK * BN_CO / 4 / 256, B4 = kK * BM_PX / 4 / 256;   // float4 per thread
};

// Lane 15 of every row of 16 lanes gets the row's sum (DPP row_shr 1, 2, 4, 8: four VALU adds,
// no LDS traffic); the other lanes hold partial sums.
__device__ __forceinline__ float row_sum16(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xF, 0xF, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xF, 0xF, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xF, 0xF, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xF, 0xF, true));
    return v;
}

// The tile's statistics (STATS): see the header comment. acc[i][j]: channels 16 i + 4 kl + v of
// the wave's 64, pixels 16 j + cl; the wave's first nval pixels are valid. Per channel the 16
// lanes sum x - sh and (x - sh)^2 around sh = the channel's output at the wave's first pixel
// (lane 16 kl, j = 0), row_sum16 adds the lanes, and lane 16 kl + 15 turns the sums into the
// wave's (count, mean, M2); the waves sharing the channels are merged by chan_merge. One channel quad i
// at a time, so few registers are live beside the accumulators, and no division per lane.
template <int WCO, int WPX>
__device__ __forceinline__ void tile_stats(const f32x4 (&acc)[4][4], int nval, int wco, int wpx, int lane,
                                           float* red, float* stats, long long row, int Cout, int co0) {
    using T = Tile<WCO, WPX>;
    const int kl = lane >> 4, cl = lane & 15;
    const float n = (float)nval, rn = nval > 0 ? 1.f / n : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float sh[4], S[4], Q[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            sh[v] = __shfl(acc[i][0][v], kl * 16, 64);
            float sum = 0.f, sq = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float d = 16 * j + cl < nval ? acc[i][j][v] - sh[v] : 0.f;
                sum += d;
                sq = fmaf(d, d, sq);
            }
            S[v] = sum;
            Q[v] = sq;
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            S[v] = row_sum16(S[v]);
            Q[v] = row_sum16(Q[v]);
        }
        if (cl == 15) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int local = wco * 64 + 16 * i + 4 * kl + v;
                red[(wpx * 3 + 0) * T::BN_CO + local] = n;
                red[(wpx * 3 + 1) * T::BN_CO + local] = nval > 0 ? fmaf(S[v], rn, sh[v]) : 0.f;
                red[(wpx * 3 + 2) * T::BN_CO + local] = nval > 0 ? fmaxf(Q[v] - S[v] * S[v] * rn, 0.f) : 0.f;
            }
        }
    }
    __syncthreads();
    for (int local = threadIdx.x; local < T::BN_CO; local += 256) {
        float cn = red[local], cm[1] = {red[T::BN_CO + local]}, cM2[1] = {red[2 * T::BN_CO + local]};
        for (int w = 1; w < WPX; ++w) {
            const float mb[1] = {red[(w * 3 + 1) * T::BN_CO + local]}, M2b[1] = {red[(w * 3 + 2) * T::BN_CO + local]};
            mcgmil::chan_merge<1>(cn, cm, cM2, red[(w * 3) * T::BN_CO + local], mb, M2b);
        }
        stats[((size_t)row * 3 + 0) * Cout + co0 + local] = cn;
        stats[((size_t)row * 3 + 1) * Cout + co0 + local] = cm[0];
        stats[((size_t)row * 3 + 2) * Cout + co0 + local] = cM2[0];
    }
}

// STATS: 4 waves per SIMD (<= 128 registers with the 64 accumulators): the 128 x 128 tile's LDS
// allows 4 workgroups per CU, and without the bound the statistics epilogue's peak (148 registers)
// cost one of them. The other variants fit 128 unbounded (accumulators in AGPRs).
template <int WCO, int WPX, bool GATHER, bool INBN, bool STATS>
__global__ __launch_bounds__(256, STATS ? 4 : 1) void conv32_kernel(const Conv32Geom g, const float* __restrict__ x,
                                                     const float* __restrict__ w, float* __restrict__ y) {
    using T = Tile<WCO, WPX>;
    static_assert(!(GATHER && INBN), "the gather mode has no input BatchNorm");
    extern __shared__ __attribute__((aligned(16))) float smem32[];
    // gather table after the two stages: k -> window offset (floats) and kh | kw << 8
    int* gtab = reinterpret_cast<int*>(smem32 + 2 * T::STAGE);
    // INBN: the input BatchNorm's a_c, b_c after the two stages
    float* sab = smem32 + 2 * T::STAGE;
    if constexpr (INBN) {
        for (int c = threadIdx.x; c < 2 * g.Cin; c += 256) sab[c] = g.in_ab[c];
        __syncthreads();
    }
    if constexpr (GATHER) {
        const int kpad = g.KS * kK;
        for (int k = threadIdx.x; k < kpad; k += 256) {
            int off = -1, hw = 0;
            if (k < g.Ktot) {
                const int tap = k / g.Cin, ci = k - tap * g.Cin;
                const int kh = tap / g.KW, kw = tap - kh * g.KW;
                off = (kh * g.W + kw) * g.Cin + ci;
                hw = kh | (kw << 8);
            }
            gtab[2 * k] = off;
            gtab[2 * k + 1] = hw;
        }
        __syncthreads();
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wco = wave % WCO, wpx = wave / WCO;
    const long long px0 = (long long)blockIdx.x * T::BM_PX;
    const int co0 = blockIdx.y * T::BN_CO;

    // B staging: every thread owns pixel tid % BM_PX of the block and some of its 4 ci quads
    const int bpx = tid % T::BM_PX;
    const int bq0 = tid / T::BM_PX;               // first ci quad; quads bq0 + (256 / BM_PX) r
    constexpr int QSTEP = 256 / T::BM_PX;
    const long long p = px0 + bpx;
    const bool pvalid = p < g.P;
    int n = 0, oh = 0, ow = 0;
    if (pvalid) {
        const long long ohw = (long long)g.OH * g.OW;
        n = (int)(p / ohw);
        const int r = (int)(p - (long long)n * ohw);
        oh = r / g.OW;
        ow = r - oh * g.OW;
    }
    const int ih0 = oh * g.stride - g.pad, iw0 = ow * g.stride - g.pad;
    const float* xn = x + (long long)n * g.H * g.W * g.Cin;
    const int cchunks = g.Cin / kK > 0 ? g.Cin / kK : 1;

    f32x4 ra[T::A4], rb[T::B4];
    bool bin = false;     // INBN: the staged B quads are in-image x (BatchNorm them; padding stays 0)
    int bci0 = 0;         // INBN: their first input channel
    auto load = [&](int ks) {
        // A: packed weights [KS][16][Cout], rows k of this K step, columns co0 .. co0 + BN_CO
        const float* wk = w + (long long)ks * kK * g.Cout + co0;
#pragma unroll
        for (int r = 0; r < T::A4; ++r) {
            const int f = tid + 256 * r;
            const int k = f / (T::BN_CO / 4), c4 = f % (T::BN_CO / 4);
            ra[r] = *reinterpret_cast<const f32x4*>(wk + (long long)k * g.Cout + 4 * c4);
        }
        if constexpr (GATHER) {   // one 4-byte load per element, window offsets from the table
            const float* base = xn + ((long long)ih0 * g.W + iw0) * g.Cin;
#pragma unroll
            for (int r = 0; r < T::B4; ++r) {
                const int q = bq0 + QSTEP * r;
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = ks * kK + 4 * q + e;
                    const int off = gtab[2 * k], hw = gtab[2 * k + 1];
                    const int ih = ih0 + (hw & 255), iw = iw0 + (hw >> 8);
                    const bool in = pvalid && off >= 0 && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
                    v[e] = in ? base[off] : 0.f;
                }
                rb[r] = f32x4{v[0], v[1], v[2], v[3]};
            }
            return;
        }
        // B: x[n, ih, iw, ci0 + 4q .. +3] of this thread's pixel (zero outside the image)
        const int tap = ks / cchunks, ci0 = (ks - tap * cchunks) * kK;
        const int kh = tap / g.KW, kw = tap - kh * g.KW;
        const int ih = ih0 + kh, iw = iw0 + kw;
        const bool in = pvalid && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        if constexpr (INBN) {
            bin = in;
            bci0 = ci0;
        }
        const float* src = xn + ((long long)(in ? ih : 0) * g.W + (in ? iw : 0)) * g.Cin + ci0;
#pragma unroll
        for (int r = 0; r < T::B4; ++r) {
            const int q = bq0 + QSTEP * r;
            rb[r] = in ? *reinterpret_cast<const f32x4*>(src + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto store = [&](float* st) {
        float* As = st;
        float* Bs = st + kK * T::AS;
#pragma unroll
        for (int r = 0; r < T::A4; ++r) {
            const int f = tid + 256 * r;
            const int k = f / (T::BN_CO / 4), c4 = f % (T::BN_CO / 4);
            *reinterpret_cast<f32x4*>(As + k * T::AS + 4 * c4) = ra[r];
        }
#pragma unroll
        for (int r = 0; r < T::B4; ++r) {
            const int q = bq0 + QSTEP * r;
            if constexpr (INBN) {   // bitwise mcgmil_batchnorm_act's max(fmaf(x, a, b), lo)
                if (bin) {
                    const f32x4 a = *reinterpret_cast<const f32x4*>(sab + bci0 + 4 * q);
                    const f32x4 b = *reinterpret_cast<const f32x4*>(sab + g.Cin + bci0 + 4 * q);
                    rb[r].x = fmaxf(fmaf(rb[r].x, a.x, b.x), g.in_lo);
                    rb[r].y = fmaxf(fmaf(rb[r].y, a.y, b.y), g.in_lo);
                    rb[r].z = fmaxf(fmaf(rb[r].z, a.z, b.z), g.in_lo);
                    rb[r].w = fmaxf(fmaf(rb[r].w, a.w, b.w), g.in_lo);
                }
            }
            Bs[(4 * q + 0) * T::BS + bpx] = rb[r].x;
            Bs[(4 * q + 1) * T::BS + bpx] = rb[r].y;
            Bs[(4 * q + 2) * T::BS + bpx] = rb[r].z;
            Bs[(4 * q + 3) * T::BS + bpx] = rb[r].w;
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int kl = lane >> 4, cl = lane & 15;
    load(0);
    store(smem32);
    __syncthreads();
    for (int ks = 0; ks < g.KS; ++ks) {
        const float* st = smem32 + (ks & 1) * T::STAGE;
        const float* As = st + wco * 64 + cl;
        const float* Bs = st + kK * T::AS + wpx * 64 + cl;
        if (ks + 1 < g.KS) load(ks + 1);
#pragma unroll
        for (int s = 0; s < kK / 4; ++s) {
            const int k = 4 * s + kl;
            float a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[k * T::AS + 16 * i];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[k * T::BS + 16 * j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (ks + 1 < g.KS) store(smem32 + ((ks + 1) & 1) * T::STAGE);
        __syncthreads();
    }

    // D tile (i, j): lane holds channels co0 + wco*64 + 16 i + 4 (lane >> 4) + v of pixel
    // px0 + wpx*64 + 16 j + (lane & 15)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const long long pp = px0 + wpx * 64 + 16 * j + cl;
        if (pp >= g.P) continue;
        float* yp = y + pp * g.Cout + co0 + wco * 64 + 4 * kl;
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<f32x4*>(yp + 16 * i) = acc[i][j];
    }
    if constexpr (STATS) {   // the stages are free: the K loop ended with a barrier
        const long long left = g.P - (px0 + wpx * 64);
        tile_stats<WCO, WPX>(acc, left < 0 ? 0 : (left > 64 ? 64 : (int)left), wco, wpx, lane, smem32,
                             g.stats, blockIdx.x, g.Cout, co0);
    }
}

// torch layout [Cout, Cin, KH, KW] fp32 -> [KS][16][Cout]: row r = ks * 16 + k of K = (kh, kw, ci)
// (Cin % 16 == 0: K step ks = (kh*KW + kw)*(Cin/16) + ci/16; gather mode: r = (kh*KW + kw)*Cin + ci
// itself, zero rows past KH*KW*Cin)
__global__ void pack_conv32_kernel(const float* w, int Cout, int Cin, int KH, int KW, int KS, float* out) {
    const long long total = (long long)KS * kK * Cout;
    const bool gather = Cin % kK != 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int co = (int)(i % Cout);
        const long long r = i / Cout;
        int tap, ci;
        if (gather) {
            if (r >= (long long)KH * KW * Cin) { out[i] = 0.f; continue; }
            tap = (int)(r / Cin);
            ci = (int)(r % Cin);
        } else {
            const int k = (int)(r % kK);
            const long long ks = r / kK;
            const int cchunks = Cin / kK;
            tap = (int)(ks / cchunks);
            ci = (int)(ks % cchunks) * kK + k;
        }
        const int kh = tap / KW, kw = tap % KW;
        out[i] = w[(((long long)co * Cin + ci) * KH + kh) * KW + kw];
    }
}

int validate32(const mcgmil_conv_args* a, Conv32Geom* g) {
    if (!a) return fail(MCGMIL_E_INVALID, "args is NULL");
    if (a->batch < 1 || a->height < 1 || a->width < 1)
        return fail(MCGMIL_E_INVALID, "batch, height and width must be >= 1");
    if (a->in_channels < 1 || a->out_channels < 64 || a->out_channels % 64 != 0)
        return fail(MCGMIL_E_UNSUPPORTED, "fp32 convolution: out_channels a multiple of 64");
    if (a->in_channels % kK != 0 &&
        (long long)a->kernel_h * a->kernel_w * a->in_channels > kMaxGatherK)
        return fail(MCGMIL_E_UNSUPPORTED, "fp32 convolution: in_channels not a multiple of 16 needs "
                                          "kernel_h * kernel_w * in_channels <= 1024");
    if (a->kernel_h < 1 || a->kernel_w < 1 || a->kernel_h > 7 || a->kernel_w > 7)
        return fail(MCGMIL_E_UNSUPPORTED, "kernel size must be in 1..7");
    if (a->stride < 1 || a->pad < 0 || a->pad > 64) return fail(MCGMIL_E_INVALID, "stride >= 1 and 0 <= pad <= 64");
    if (a->in_ab && (a->in_channels % kK != 0 || a->in_channels > kMaxInBnC))
        return fail(MCGMIL_E_UNSUPPORTED, "fp32 convolution: in_ab needs in_channels a multiple of 16, <= 2048");
    if (a->in_relu != 0 && a->in_relu != 1) return fail(MCGMIL_E_INVALID, "in_relu must be 0 or 1");
    const long long oh = ((long long)a->height + 2 * a->pad - a->kernel_h) / a->stride + 1;
    const long long ow = ((long long)a->width + 2 * a->pad - a->kernel_w) / a->stride + 1;
    if (oh < 1 || ow < 1) return fail(MCGMIL_E_INVALID, "the kernel does not fit the padded input");
    const long long P = (long long)a->batch * oh * ow;
    if (P >= (1ll << 31) - 256) return fail(MCGMIL_E_UNSUPPORTED, "too many output pixels");
    if (g) {
        g->N = a->batch; g->H = a->height; g->W = a->width; g->Cin = a->in_channels;
        g->Cout = a->out_channels; g->KH = a->kernel_h; g->KW = a->kernel_w;
        g->stride = a->stride; g->pad = a->pad; g->OH = (int)oh; g->OW = (int)ow; g->P = P;
        g->Ktot = a->kernel_h * a->kernel_w * a->in_channels;
        g->KS = (g->Ktot + kK - 1) / kK;
        g->in_ab = a->in_ab;
        g->in_lo = a->in_relu ? 0.f : -INFINITY;
        g->stats = a->stats;
    }
    return MCGMIL_OK;
}

template <int WCO, int WPX>
long long pixel_tiles(const Conv32Geom& g) { return (g.P + Tile<WCO, WPX>::BM_PX - 1) / Tile<WCO, WPX>::BM_PX; }

// 128 x 128 tiles when Cout is a multiple of 128, else 64 x 256
bool wide_co(const Conv32Geom& g) { return g.Cout % 128 == 0; }

template <int WCO, int WPX, bool GATHER, bool INBN, bool STATS>
int launch32(const Conv32Geom& g, const float* x, const float* w, float* y, hipStream_t s) {
    using T = Tile<WCO, WPX>;
    const size_t lds = (size_t)2 * T::STAGE * sizeof(float) + (GATHER ? (size_t)g.KS * kK * 8 : 0) +
                       (INBN ? (size_t)2 * g.Cin * sizeof(float) : 0);
    dim3 grid((unsigned)pixel_tiles<WCO, WPX>(g), (unsigned)(g.Cout / T::BN_CO));
    hipLaunchKernelGGL((conv32_kernel<WCO, WPX, GATHER, INBN, STATS>), grid, dim3(256), lds, s, g, x, w, y);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "conv32_kernel launch");
}

template <int WCO, int WPX>
int dispatch32(const Conv32Geom& g, const float* x, const float* w, float* y, hipStream_t s) {
    const bool st = g.stats != nullptr;
    if (g.Cin % kK != 0)
        return st ? launch32<WCO, WPX, true, false, true>(g, x, w, y, s)
                  : launch32<WCO, WPX, true, false, false>(g, x, w, y, s);
    if (g.in_ab)
        return st ? launch32<WCO, WPX, false, true, true>(g, x, w, y, s)
                  : launch32<WCO, WPX, false, true, false>(g, x, w, y, s);
    return st ? launch32<WCO, WPX, false, false, true>(g, x, w, y, s)
              : launch32<WCO, WPX, false, false, false>(g, x, w, y, s);
}

}  // namespace

extern "C" {

int mcgmil_pack_conv_weights_f32(const mcgmil_conv_args* a, const void* weight, void* packed, void* stream) {
    if (int rc = validate32(a, nullptr)) return rc;
    if (!weight || !packed) return fail(MCGMIL_E_INVALID, "NULL weight or packed pointer");
    Conv32Geom g;
    validate32(a, &g);
    const long long total = (long long)g.KS * kK * a->out_channels;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(pack_conv32_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       static_cast<const float*>(weight), a->out_channels, a->in_channels, a->kernel_h,
                       a->kernel_w, g.KS, static_cast<float*>(packed));
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "pack_conv32_kernel launch");
}

int mcgmil_conv_packed_size_f32(const mcgmil_conv_args* a, size_t* floats) {
    Conv32Geom g;
    if (int rc = validate32(a, &g)) return rc;
    if (!floats) return fail(MCGMIL_E_INVALID, "floats is NULL");
    *floats = (size_t)g.KS * kK * a->out_channels;
    return MCGMIL_OK;
}

int mcgmil_conv_stats_parts_f32(const mcgmil_conv_args* a, int32_t* parts) {
    Conv32Geom g;
    if (int rc = validate32(a, &g)) return rc;
    if (!parts) return fail(MCGMIL_E_INVALID, "parts is NULL");
    const long long t = wide_co(g) ? pixel_tiles<2, 2>(g) : pixel_tiles<1, 4>(g);
    if (t > 0x7fffffffll) return fail(MCGMIL_E_UNSUPPORTED, "too many pixel tiles");
    *parts = (int32_t)t;
    return MCGMIL_OK;
}

int mcgmil_conv2d_f32(const mcgmil_conv_args* a, void* stream) {
    Conv32Geom g;
    if (int rc = validate32(a, &g)) return rc;
    if (!a->x || !a->w || !a->y) return fail(MCGMIL_E_INVALID, "NULL x, w or y");
    if (((uintptr_t)a->x | (uintptr_t)a->w | (uintptr_t)a->y) & 15u)
        return fail(MCGMIL_E_ALIGN, "x, w and y must be 16-byte aligned");
    if (((uintptr_t)a->stats | (uintptr_t)a->in_ab) & 3u)
        return fail(MCGMIL_E_ALIGN, "stats and in_ab must be 4-byte aligned");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const float* x = static_cast<const float*>(a->x);
    const float* w = static_cast<const float*>(a->w);
    float* y = static_cast<float*>(a->y);
    return wide_co(g) ? dispatch32<2, 2>(g, x, w, y, s) : dispatch32<1, 4>(g, x, w, y, s);
}

}  // extern "C"
