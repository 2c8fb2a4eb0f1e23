// The ResNet stem maxpool(relu(bn1(conv1(x)))) (include/mcgmil_features.h, mcgmil_stem_forward):
// the first four layers of the torchvision backbone the reference builds at model.py:166-177 and
// runs on every instance of a bag at infer.py:191, from the NCHW bf16 instances the patcher
// writes (mcgmil_image_to_bag) to the channels-last activation the block convolutions read.
//
// Convolution (7x7, stride 2, 3 -> 64 channels) as an implicit GEMM on the matrix cores:
//   C[co, m] = sum_k W[co, k] * X[k, m],  m = (n, oh, ow),  k = (ci, kh, j),  j = 0..7
// A K step of v_mfma_f32_16x16x32_bf16 is 4 (ci, kh) rows x 8 horizontal taps: lane chunk q of
// pixel ow reads the 8 input columns iw = 2 ow - P + j, i.e. FOUR 32-bit LDS words at an even
// column -- every read naturally aligned. P = pad rounded up to even, so tap j is kernel
// column kw = j - (P - pad) (the taps outside 0..k-1 carry zero weights; for the 7x7 / pad-3
// stem j = 0 is the dead one). 21 (ci, kh) rows pad to 6 K steps.
//
// Persistent workgroups (2 per CU) walk a contiguous range of 4-output-row tiles; one wave per
// output row, 7 pixel fragments x 4 channel fragments per row. The 3 x 13 staged input rows of
// the next tile are loaded by LDS-DMA (buffer_load_dword ... lds, no registers) into the other half
// of a double-buffered LDS image while this tile computes (one barrier per tile); all 6 x 4 weight fragments
// stay in registers for the whole kernel. LDS row pitch = 16 (mod 64) dwords and channel plane
// = k rows (mod 64), so the four K chunks of a read hit disjoint bank groups.
//
// Batch statistics: each lane accumulates the bf16-rounded outputs of its 16 channels around a
// per-channel shift (the convolution at one central pixel of instance 0, computed first by
// stem_prep_kernel), the lanes of a workgroup are reduced in a fixed order, and the per-
// workgroup sums go to the BatchNorm finalize of mcgmil_bn.hip (fp64, fixed order), which then
// runs the fused normalise + ReLU + max-pool pass. The 64-channel activation is written once
// and read once.
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <string>

#include "../../include/mcgmil_features.h"
#include "mcgmil_device.h"
#include "mcgmil_error.h"

namespace mcgmil_detail {
int bn_finish_bf16(const mcgmil_bn_args* a, const float* part, int parts, const void* shift_row,
                   hipStream_t s, bool hpooled);
}

namespace {

using namespace mcgmil;
using mcgmil_detail::fail;
using mcgmil_detail::hip_fail;

constexpr int kTH = 4;                 // output rows per tile = waves per workgroup
constexpr int kThreads = 64 * kTH;
constexpr int kCout = 64;
constexpr int kMaxWd = 128;            // staged dwords per row (OW + 3)
constexpr int kLdsBytes = 64 * 1024;

struct StemGeom {
    const __bf16* x;
    const bf16x8* w;
    __bf16* y;
    const __bf16* shift;
    float* part;
    const float* gamma;     // HP: the BN weight (its signs), or NULL
    int N, Cin, H, W, OH, OW, k, pad, P;
    int RR;          // staged rows per channel: 2 (kTH - 1) + k
    int pitch;       // LDS dwords per staged row
    int plane;       // LDS dwords per channel
    int wd;          // dwords written per staged row: OW + 3
    int tiles, TPI;  // tiles, tiles per instance
    uint32_t x_bytes;
};

struct Geometry {
    StemGeom g;
    int KS = 0;
    int OH = 0, OW = 0, PH = 0, PW = 0;
    size_t lds = 0;
};

int geometry(const mcgmil_stem_args* a, Geometry* out) {
    if (!a) return fail(MCGMIL_E_INVALID, "mcgmil_stem_args is NULL");
    if (a->batch < 1 || a->height < 1 || a->width < 1)
        return fail(MCGMIL_E_INVALID, "batch, height and width must be >= 1");
    if (a->in_channels < 1 || a->in_channels > 4)
        return fail(MCGMIL_E_UNSUPPORTED, "the stem kernel takes 1..4 input channels");
    if (a->out_channels != kCout) return fail(MCGMIL_E_UNSUPPORTED, "the stem kernel has 64 output channels");
    if (a->kernel < 1 || a->stride != 2 || a->pad < 0 || a->kernel + (a->pad & 1) > 8)
        return fail(MCGMIL_E_UNSUPPORTED, "the stem kernel needs stride 2 and kernel + (pad & 1) <= 8");
    if (a->width & 1) return fail(MCGMIL_E_UNSUPPORTED, "the stem kernel needs an even width");
    if (a->relu != 0 && a->relu != 1) return fail(MCGMIL_E_INVALID, "relu must be 0 or 1");
    if ((a->flags != MCGMIL_STEM_AUTO && a->flags != MCGMIL_STEM_POOL_UNSPLIT) || a->reserved != 0)
        return fail(MCGMIL_E_INVALID, "flags must be an mcgmil_stem_flags value and reserved 0");
    const int OH = (a->height + 2 * a->pad - a->kernel) / 2 + 1;
    const int OW = (a->width + 2 * a->pad - a->kernel) / 2 + 1;
    if (a->height + 2 * a->pad < a->kernel || a->width + 2 * a->pad < a->kernel || OH < 1 || OW < 1)
        return fail(MCGMIL_E_INVALID, "the kernel does not fit the padded input");
    if (OW + 3 > kMaxWd) return fail(MCGMIL_E_UNSUPPORTED, "the stem kernel takes OW <= 125");
    const long long x_bytes = 2LL * a->batch * a->in_channels * a->height * a->width;
    if (x_bytes >= (1LL << 31)) return fail(MCGMIL_E_UNSUPPORTED, "input larger than 2 GiB");
    Geometry G;
    StemGeom& g = G.g;
    g.N = a->batch; g.Cin = a->in_channels; g.H = a->height; g.W = a->width;
    g.OH = OH; g.OW = OW; g.k = a->kernel; g.pad = a->pad; g.P = a->pad + (a->pad & 1);
    g.RR = 2 * (kTH - 1) + g.k;
    g.wd = OW + 3;
    g.pitch = (g.wd + 63) / 64 * 64 + 16;   // whole 64-dword DMA pieces, 16 (mod 64)
    g.plane = g.RR * g.pitch;
    while ((g.plane - g.k * g.pitch) % 64 != 0) ++g.plane;
    G.lds = (size_t)2 * g.Cin * g.plane * 4 + (size_t)kTH * 17 * kCout * 2;   // + epilogue scratch, carry
    if (G.lds > (size_t)kLdsBytes) return fail(MCGMIL_E_UNSUPPORTED, "stem tile exceeds 64 KiB of LDS");
    g.TPI = (OH + kTH - 1) / kTH;
    const long long tiles = (long long)g.N * g.TPI;
    if (tiles >= (1LL << 31) || (long long)g.N * OH * OW * kCout >= (1LL << 40))
        return fail(MCGMIL_E_UNSUPPORTED, "too many tiles");
    g.tiles = (int)tiles;
    g.x_bytes = (uint32_t)x_bytes;
    G.KS = (g.Cin * g.k + 3) / 4;
    G.OH = OH; G.OW = OW;
    if (a->pool_kernel < 0) return fail(MCGMIL_E_INVALID, "pool_kernel must be >= 0");
    if (a->pool_kernel > 0) {
        if (a->pool_stride < 1 || a->pool_pad < 0 || 2 * a->pool_pad > a->pool_kernel)
            return fail(MCGMIL_E_INVALID, "pooling needs stride >= 1 and 0 <= pad <= kernel / 2");
        G.PH = (OH + 2 * a->pool_pad - a->pool_kernel) / a->pool_stride + 1;
        G.PW = (OW + 2 * a->pool_pad - a->pool_kernel) / a->pool_stride + 1;
        if (G.PH < 1 || G.PW < 1) return fail(MCGMIL_E_INVALID, "pooling window larger than the padded input");
    } else {
        G.PH = OH; G.PW = OW;
    }
    *out = G;
    return MCGMIL_OK;
}

// packed[(s * 4 + i) * 64 + lane][j] = W[co = 16 i + (lane & 15), ci, kh, kw = j - (P - pad)]
// with (ci, kh) = divmod(4 s + (lane >> 4), k); zero outside the kernel
template <typename T>
__global__ void pack_stem_weights_kernel(const T* __restrict__ w, int Cin, int k, int e, int KS,
                                         __bf16* __restrict__ out) {
    const int total = KS * 4 * 64 * 8;
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
        const int j = idx & 7, lane = (idx >> 3) & 63, si = idx >> 9;
        const int i = si & 3, s = si >> 2;
        const int co = 16 * i + (lane & 15), r = 4 * s + (lane >> 4), kw = j - e;
        float v = 0.f;
        if (r < Cin * k && kw >= 0 && kw < k) {
            const int ci = r / k, kh = r - ci * k;
            v = (float)w[((co * Cin + ci) * k + kh) * k + kw];
        }
        out[idx] = (__bf16)v;
    }
}

// With batch statistics: the BatchNorm shift row, the convolution at pixel (0, OH/2, OW/2), fp32,
// rounded to bf16 (any value near the channel mean keeps the shifted sums well conditioned; all
// partials share it).
__global__ __launch_bounds__(256) void stem_prep_kernel(const StemGeom g, int KS, int stats) {
    __shared__ float red[4][kCout];
    const int tid = threadIdx.x, c = tid & 63, part = tid >> 6;
    if (!stats) return;
    const int oh = g.OH / 2, ow = g.OW / 2, e = g.P - g.pad;
    const __bf16* wp = reinterpret_cast<const __bf16*>(g.w);
    float acc = 0.f;
    for (int r = part; r < g.Cin * g.k; r += 4) {       // (ci, kh) rows split over 4 waves
        const int s = r >> 2, q = r & 3, ci = r / g.k, kh = r - ci * g.k, ih = 2 * oh - g.pad + kh;
        if (ih < 0 || ih >= g.H) continue;
        for (int j = 0; j < 8; ++j) {
            const int iw = 2 * ow - g.pad + (j - e);
            if (j - e < 0 || j - e >= g.k || iw < 0 || iw >= g.W) continue;
            const float xv = (float)g.x[((size_t)ci * g.H + ih) * g.W + iw];
            const float wv = (float)wp[((size_t)(s * 4 + c / 16) * 64 + (c & 15) + 16 * q) * 8 + j];
            acc = fmaf(xv, wv, acc);
        }
    }
    red[part][c] = acc;
    __syncthreads();
    if (tid < kCout)
        const_cast<__bf16*>(g.shift)[c] = (__bf16)(red[0][c] + red[1][c] + red[2][c] + red[3][c]);
    (void)KS;
}

// The epilogue's reads and writes of the wave's LDS scratch are inline asm: the compiler's wait-count pass
// treats an LDS read after the staging's LDS-DMA as a possible alias and puts an s_waitcnt vmcnt(0)
// in front of it (and of an LDS write), which drains the next tile's staging at the first fragment
// and the previous fragment's output stores at every later one (the same hazard as bn_slot in
// mcgmil_conv.hip).
// The scratch is written and read by one wave only, and LDS serves a wave's operations in order.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)p);
}
__device__ __forceinline__ u32x4 lds_read16(const void* p) {
    u32x4 u;
    asm volatile("ds_read_b128 %0, %1" : "=v"(u) : "v"(lds_addr(p)) : "memory");
    return u;
}
__device__ __forceinline__ void lds_write8(void* p, uint32_t lo, uint32_t hi) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    asm volatile("ds_write_b64 %0, %1" ::"v"(lds_addr(p)), "v"(u32x2{lo, hi}) : "memory");
}
__device__ __forceinline__ void lds_write16(void* p, u32x4 v) {
    asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
// 4 bytes per lane from a buffer straight into LDS at the wave-uniform base + 4 * lane (the
// builtin only exists in the device pass)
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, voff, soff, 0, 0);
#else
    (void)r; (void)lds; (void)voff; (void)soff;
#endif
}
__device__ __forceinline__ void lds_wait(u32x4& a, u32x4& b) {     // names the values read: no use moves above
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b)::"memory");
}
__device__ __forceinline__ void lds_wait(u32x4& a, u32x4& b, u32x4& c) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c)::"memory");
}

// HP (the ResNet 3x3 / 2 / pad 1 max-pool, OW even): the epilogue also takes the horizontal
// 3-wide, stride-2 maximum of each row and stores only that, [N, OH, OW / 2, 64] -- half the
// activation bytes written here and read by the pooling pass (bn_vpool_kernel), which takes the
// vertical maximum. Max-pooling commutes with the BN only channel by channel: where a_c < 0 (the
// sign of gamma_c) the pool of BN(x) is BN of the MINIMUM, so those channels are stored negated
// (bf16 negation is exact) and their maximum is the negated minimum.
template <int KS, bool STATS, bool HP>
__global__ __launch_bounds__(kThreads, 2) void stem_conv_kernel(const StemGeom g) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, p = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: the staging math is scalar
    const int buf_dw = g.Cin * g.plane;
    const int t0 = (int)((long long)blockIdx.x * g.tiles / gridDim.x);
    const int t1 = (int)((long long)(blockIdx.x + 1) * g.tiles / gridDim.x);

    // weights for the whole kernel: KS x 4 fragments of 8 bf16
    bf16x8 wf[KS][4];
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) wf[s][i] = g.w[(s * 4 + i) * 64 + lane];
    // LDS dword offset of this lane's (ci, kh) row per K step (padded rows repeat the last row:
    // their weights are zero, the values only need to be finite)
    int rowoff[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        int r = 4 * s + q;
        if (r > g.Cin * g.k - 1) r = g.Cin * g.k - 1;
        const int ci = r / g.k, kh = r - ci * g.k;
        rowoff[s] = ci * g.plane + (2 * wave + kh) * g.pitch;
    }

    float sh[16], S[16], SS[16];
    if (STATS) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            sh[c] = (float)g.shift[16 * (c >> 2) + 4 * q + (c & 3)];
            S[c] = SS[c] = 0.f;
        }
    }

    // staging by LDS-DMA (buffer_load_dword ... lds: no registers): wave w stages rows
    // sr = w + kTH * it of the Cin x RR image, one 64-dword piece per instruction. The lane's column
    // offset of each piece is fixed for the kernel (coff); rows outside the image and columns
    // outside the row read past the buffer's range, i.e. zeros (offsets >= 2^31 > x_bytes, no
    // wrap: the row base is < 2^31 too); lanes past the row's dwords land in its pitch padding.
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(g.x, g.x_bytes);
    constexpr int kPieces = (kMaxWd + 63) / 64;
    uint32_t coff[kPieces];
#pragma unroll
    for (int d = 0; d < kPieces; ++d) {
        const int gd = 64 * d + lane - (g.P >> 1);  // global dword of the row: columns 2 gd, 2 gd + 1
        coff[d] = gd >= 0 && 2 * gd < g.W ? 4u * (uint32_t)gd : 0x80000000u;
    }
    const int nsr = g.Cin * g.RR;
    auto stage = [&](int t, int buf) {
        const int n = t / g.TPI, oh0 = (t - n * g.TPI) * kTH;
        uint32_t* L = lds + buf * buf_dw;
        int ci = 0, rr = wave;                 // row sr = ci * RR + rr, stepped by kTH (RR >= kTH)
        for (int sr = wave; sr < nsr; sr += kTH, rr += kTH) {
            if (rr >= g.RR) {
                rr -= g.RR;
                ++ci;
            }
            const int ih = 2 * oh0 - g.pad + rr;
            const bool rok = ih >= 0 && ih < g.H;
            const uint32_t rowb = rok ? (uint32_t)((n * g.Cin + ci) * g.H + ih) * (uint32_t)(g.W * 2) : 0u;
            uint32_t* dst = L + ci * g.plane + rr * g.pitch;
#pragma unroll
            for (int d = 0; d < kPieces; ++d) {
                if (64 * d >= g.wd) break;
                const uint32_t vo = rok ? coff[d] : 0x80000000u;
                dma4(xr, dst + 64 * d, vo, rowb);
            }
        }
    };

    const int FR = (g.OW + 15) >> 4;
    __bf16* scratch = reinterpret_cast<__bf16*>(lds + 2 * buf_dw) + wave * 16 * kCout;   // 2 KiB per wave
    // HP: lane = (pooled pixel j of the fragment, 8-channel chunk hc); the chunk's sign flips
    __bf16* carry = reinterpret_cast<__bf16*>(lds + 2 * buf_dw) + kTH * 16 * kCout + wave * kCout;
    const int hj = lane >> 3, hc = lane & 7;
    uint32_t hflip[4] = {0u, 0u, 0u, 0u};
    if (HP && g.gamma) {
#pragma unroll
        for (int d = 0; d < 4; ++d)
            hflip[d] = (__float_as_uint(g.gamma[8 * hc + 2 * d]) >> 31 << 15) |
                       (__float_as_uint(g.gamma[8 * hc + 2 * d + 1]) >> 31 << 31);
    }
    const int PW = g.OW >> 1;
    if (t0 < t1) stage(t0, 0);
    __syncthreads();
    for (int t = t0; t < t1; ++t) {
        const int cur = (t - t0) & 1;
        const bool more = t + 1 < t1;
        if (more) stage(t + 1, cur ^ 1);     // (staging after the compute measured no faster)
        const int n = t / g.TPI, oh = (t - n * g.TPI) * kTH + wave;
        if (oh < g.OH) {
            const uint32_t* L = lds + cur * buf_dw;
            __bf16* yrow = g.y + ((size_t)n * g.OH + oh) * g.OW * kCout;
            for (int f = 0; f < FR; ++f) {
                const int ow = 16 * f + p;
                const int owc = ow < g.OW ? ow : g.OW - 1;
                f32x4 acc[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const uint32_t* src = L + rowoff[s] + owc;
                    const uint4 u = make_uint4(src[0], src[1], src[2], src[3]);
                    const bf16x8 b = __builtin_bit_cast(bf16x8, u);
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s][i], b, acc[i], 0, 0, 0);
                }
                // epilogue: round, transpose the 16 pixels x 64 channels through the wave's LDS
                // scratch (pixel rows of 128 B, 16-B chunks XOR-swizzled by pixel) and store
                // each pixel row as 16-B pieces, 1 KiB contiguous per wave-instruction
                // the rounded outputs as bf16 pairs (channels 4 (q) + 2 h, + 1 of fragment row i): stored
                // to the scratch, and read back out of the same registers for the statistics
                typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
                const bool valid = ow < g.OW;
                uint32_t pk[4][2];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        pk[i][h] = __builtin_bit_cast(uint32_t, bf16x2{(__bf16)acc[i][2 * h], (__bf16)acc[i][2 * h + 1]});
                    const int c = 2 * i + (q >> 1);
                    lds_write8(scratch + p * 64 + ((c ^ (p & 7)) << 3) + ((q & 1) << 2), pk[i][0], pk[i][1]);
                }
                if (STATS && valid) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int v = 0; v < 4; ++v) {
                            const uint32_t u = pk[i][v >> 1];
                            const float y = __uint_as_float((v & 1) ? (u & 0xFFFF0000u) : (u << 16));
                            const float d = y - sh[4 * i + v];
                            S[4 * i + v] += d;
                            SS[4 * i + v] = fmaf(d, d, SS[4 * i + v]);
                        }
                }
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
                if (HP) {
                    // pooled pixel 8 f + hj = max over fragment pixels 2 hj - 1 (the carry from the
                    // previous fragment when hj = 0; padding when f = 0), 2 hj, 2 hj + 1
                    auto px = [&](int pp) { return scratch + pp * 64 + ((hc ^ (pp & 7)) << 3); };
                    const u32x4 flip = {hflip[0], hflip[1], hflip[2], hflip[3]};
                    // pixel 2 hj - 1: the scratch, or (hj = 0) the carry, stored sign-adjusted
                    u32x4 u0 = lds_read16(px(2 * hj)), u1 = lds_read16(px(2 * hj + 1));
                    u32x4 um = lds_read16(hj > 0 ? px(2 * hj - 1) : carry + 8 * hc);
                    lds_wait(u0, u1, um);
                    u0 ^= flip;
                    u1 ^= flip;
                    if (hj > 0) um ^= flip;
                    const bool three = hj > 0 || f > 0;
                    const uint32_t w0[4] = {u0.x, u0.y, u0.z, u0.w}, w1[4] = {u1.x, u1.y, u1.z, u1.w},
                                   wm[4] = {um.x, um.y, um.z, um.w};
                    uint32_t o[4];
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        float lo = fmaxf(__uint_as_float(w0[d] << 16), __uint_as_float(w1[d] << 16));
                        float hi = fmaxf(__uint_as_float(w0[d] & 0xFFFF0000u), __uint_as_float(w1[d] & 0xFFFF0000u));
                        if (three) {
                            lo = fmaxf(lo, __uint_as_float(wm[d] << 16));
                            hi = fmaxf(hi, __uint_as_float(wm[d] & 0xFFFF0000u));
                        }
                        o[d] = (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xFFFF0000u);   // exact
                    }
                    asm volatile("" ::: "memory");
                    if (hj == 7) lds_write16(carry + 8 * hc, u1);   // pixel 15, sign-adjusted
                    const int pw = 8 * f + hj;
                    if (pw < PW)
                        *reinterpret_cast<uint4*>(g.y + (((size_t)n * g.OH + oh) * PW + pw) * kCout + 8 * hc) =
                            make_uint4(o[0], o[1], o[2], o[3]);
                } else {
                    const int pp0 = lane >> 3, c = lane & 7;
                    u32x4 v[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        v[h] = lds_read16(scratch + (pp0 + 8 * h) * 64 + ((c ^ (pp0 & 7)) << 3));
                    lds_wait(v[0], v[1]);
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        if (16 * f + pp0 + 8 * h < g.OW)
                            *reinterpret_cast<u32x4*>(yrow + (size_t)(16 * f + pp0 + 8 * h) * kCout + 8 * c) = v[h];
                }
                asm volatile("" ::: "memory");
            }
        }
        __syncthreads();
    }

    if (STATS) {
        // lanes p = 0..15 of a chunk hold the same 16 channels: butterfly over p, then waves in order
#pragma unroll
        for (int c = 0; c < 16; ++c) {
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                S[c] += __shfl_xor(S[c], o, 64);
                SS[c] += __shfl_xor(SS[c], o, 64);
            }
        }
        float* red = reinterpret_cast<float*>(lds);     // [kTH][2][64]
        if (p == 0) {
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                const int ch = 16 * (c >> 2) + 4 * q + (c & 3);
                red[(wave * 2) * kCout + ch] = S[c];
                red[(wave * 2 + 1) * kCout + ch] = SS[c];
            }
        }
        __syncthreads();
        if (tid < 2 * kCout) {
            float v = 0.f;
            for (int w = 0; w < kTH; ++w) v += red[w * 2 * kCout + tid];
            g.part[(size_t)blockIdx.x * 2 * kCout + tid] = v;   // [2][64]: sums then squares
        }
    }
}

template <int KS>
void launch_conv(const StemGeom& g, int grid, size_t lds, bool stats, bool hp, hipStream_t s) {
    auto k = stats ? (hp ? stem_conv_kernel<KS, true, true> : stem_conv_kernel<KS, true, false>)
                   : (hp ? stem_conv_kernel<KS, false, true> : stem_conv_kernel<KS, false, false>);
    hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), lds, s, g);
}

int cu_count() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
    if (dev < 64) {
        const int c = cache[dev].load(std::memory_order_relaxed);
        if (c > 0) return c;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    if (dev < 64) cache[dev].store(cus, std::memory_order_relaxed);
    return cus;
}

struct Carve {
    size_t conv = 0, shift = 0, part = 0, bn = 0, total = 0;
    int grid = 0;
};

size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

Carve carve(const mcgmil_stem_args* a, const Geometry& G) {
    Carve c;
    c.grid = G.g.tiles < 2 * cu_count() ? G.g.tiles : 2 * cu_count();
    size_t off = 0;
    if (a->pool_kernel > 0) {
        c.conv = off;
        off += al256((size_t)G.g.N * G.OH * G.OW * kCout * 2);
    }
    c.shift = off;          // 64 bf16 shift row
    off += 512;
    c.part = off;
    off += al256((size_t)c.grid * 2 * kCout * sizeof(float));
    c.bn = off;
    off += al256(2 * kCout * sizeof(float));
    c.total = off;
    return c;
}

}  // namespace

extern "C" {

size_t mcgmil_stem_args_size(void) { return sizeof(mcgmil_stem_args); }

int mcgmil_stem_packed_size(const mcgmil_stem_args* a, size_t* bytes) {
    Geometry G;
    if (int rc = geometry(a, &G)) return rc;
    if (!bytes) return fail(MCGMIL_E_INVALID, "bytes is NULL");
    *bytes = (size_t)G.KS * 4 * 64 * 16;
    return MCGMIL_OK;
}

int mcgmil_pack_stem_weights(const mcgmil_stem_args* a, const void* weight, int32_t weight_dtype,
                             void* packed, void* stream) {
    Geometry G;
    if (int rc = geometry(a, &G)) return rc;
    if (!weight || !packed) return fail(MCGMIL_E_INVALID, "NULL weight or packed pointer");
    if ((uintptr_t)packed & 15) return fail(MCGMIL_E_ALIGN, "packed must be 16-byte aligned");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int e = G.g.P - G.g.pad;
    const int blocks = (G.KS * 4 * 64 * 8 + 255) / 256;
    if (weight_dtype == MCGMIL_F32)
        hipLaunchKernelGGL(pack_stem_weights_kernel<float>, dim3(blocks), dim3(256), 0, s,
                           static_cast<const float*>(weight), G.g.Cin, G.g.k, e, G.KS, static_cast<__bf16*>(packed));
    else if (weight_dtype == MCGMIL_BF16)
        hipLaunchKernelGGL(pack_stem_weights_kernel<__bf16>, dim3(blocks), dim3(256), 0, s,
                           static_cast<const __bf16*>(weight), G.g.Cin, G.g.k, e, G.KS, static_cast<__bf16*>(packed));
    else
        return fail(MCGMIL_E_INVALID, "weight_dtype must be MCGMIL_F32 or MCGMIL_BF16");
    const hipError_t err = hipGetLastError();
    return err == hipSuccess ? MCGMIL_OK : hip_fail(err, "pack_stem_weights_kernel launch");
}

int mcgmil_stem_workspace_size(const mcgmil_stem_args* a, size_t* bytes) {
    Geometry G;
    if (int rc = geometry(a, &G)) return rc;
    if (!bytes) return fail(MCGMIL_E_INVALID, "bytes is NULL");
    *bytes = carve(a, G).total;
    return MCGMIL_OK;
}

int mcgmil_stem_forward(const mcgmil_stem_args* a, void* stream) {
    Geometry G;
    if (int rc = geometry(a, &G)) return rc;
    if (!a->x || !a->w || !a->y) return fail(MCGMIL_E_INVALID, "NULL x, w or y");
    if ((((uintptr_t)a->x) & 3) | (((uintptr_t)a->w | (uintptr_t)a->y) & 15))
        return fail(MCGMIL_E_ALIGN, "x must be 4-byte and w, y 16-byte aligned");
    if ((a->running_mean == nullptr) != (a->running_var == nullptr))
        return fail(MCGMIL_E_INVALID, "running_mean and running_var go together");
    const Carve c = carve(a, G);
    if (!a->workspace || a->workspace_bytes < c.total || ((uintptr_t)a->workspace & 255))
        return fail(MCGMIL_E_WORKSPACE, "workspace missing, misaligned or smaller than mcgmil_stem_workspace_size()");
    unsigned char* ws = static_cast<unsigned char*>(a->workspace);
    const bool stats = a->running_mean == nullptr;
    StemGeom g = G.g;
    g.x = static_cast<const __bf16*>(a->x);
    g.w = static_cast<const bf16x8*>(a->w);
    g.y = a->pool_kernel > 0 ? reinterpret_cast<__bf16*>(ws + c.conv) : static_cast<__bf16*>(a->y);
    g.shift = reinterpret_cast<const __bf16*>(ws + c.shift);
    g.part = reinterpret_cast<float*>(ws + c.part);
    g.gamma = a->gamma;
    // the ResNet pool (3 x 3, stride 2, pad 1) on an even width: horizontal half in the epilogue
    // args->flags MCGMIL_STEM_POOL_UNSPLIT, or MCGMIL_STEM_HPOOL=0|1 in the environment (overrides;
    // read once per process)
    static const int hp_env = [] {
        const char* e = getenv("MCGMIL_STEM_HPOOL");
        return e ? (strcmp(e, "0") == 0 ? 1 : 0) : -1;
    }();
    const bool unsplit = hp_env >= 0 ? hp_env == 1 : a->flags == MCGMIL_STEM_POOL_UNSPLIT;
    const bool hp = a->pool_kernel == 3 && a->pool_stride == 2 && a->pool_pad == 1 && G.OW % 2 == 0 && !unsplit;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (stats) hipLaunchKernelGGL(stem_prep_kernel, dim3(1), dim3(256), 0, s, g, G.KS, 1);
    switch (G.KS) {
        case 1: launch_conv<1>(g, c.grid, G.lds, stats, hp, s); break;
        case 2: launch_conv<2>(g, c.grid, G.lds, stats, hp, s); break;
        case 3: launch_conv<3>(g, c.grid, G.lds, stats, hp, s); break;
        case 4: launch_conv<4>(g, c.grid, G.lds, stats, hp, s); break;
        case 5: launch_conv<5>(g, c.grid, G.lds, stats, hp, s); break;
        case 6: launch_conv<6>(g, c.grid, G.lds, stats, hp, s); break;
        case 7: launch_conv<7>(g, c.grid, G.lds, stats, hp, s); break;
        default: launch_conv<8>(g, c.grid, G.lds, stats, hp, s); break;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "stem_conv_kernel launch");
    mcgmil_bn_args b{};
    b.rows = (int64_t)G.g.N * G.OH * G.OW;
    b.channels = kCout;
    b.dtype = MCGMIL_BF16;
    b.x = g.y;
    b.y = a->y;
    b.gamma = a->gamma;
    b.beta = a->beta;
    b.running_mean = a->running_mean;
    b.running_var = a->running_var;
    b.eps = a->eps;
    b.relu = a->relu;
    b.batch = G.g.N;
    b.height = G.OH;
    b.width = G.OW;
    b.pool_kernel = a->pool_kernel;
    b.pool_stride = a->pool_stride;
    b.pool_pad = a->pool_pad;
    b.batch_mean = a->batch_mean;
    b.batch_invstd = a->batch_invstd;
    b.workspace = ws + c.bn;
    b.workspace_bytes = c.total - c.bn;
    return mcgmil_detail::bn_finish_bf16(&b, g.part, stats ? c.grid : 0, g.shift, s, hp);
}

}  // extern "C"
