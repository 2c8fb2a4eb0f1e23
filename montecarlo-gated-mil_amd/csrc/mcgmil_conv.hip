// Implicit-GEMM convolution of the channels-last bf16 backbone (include/mcgmil_features.h,
// mcgmil_conv2d): the 3x3 / 1x1 convolutions of the torchvision BasicBlock / Bottleneck the
// reference builds at model.py:166-177, run in infer.py:191 on every instance of a bag.
//
// GEMM view (one output pixel per row, one output channel per column):
//   C[m, co] = sum_k A[m, k] * B[k, co],  m = (n, oh, ow),  k = (kh, kw, ci)
//   A[m, k]  = x[n, oh*s - pad + kh, ow*s - pad + kw, ci]   (0 outside the image)
//   B[k, co] = w[co, kh, kw, ci]                            (weights packed channels-last)
// A K tile is one (kh, kw) tap and 64 consecutive input channels, so every A row of a K tile is
// ONE contiguous 128-byte run of the NHWC input. v_mfma_f32_16x16x32_bf16 with the weights as
// the A operand: a lane ends with 4 consecutive channels of one pixel (one 8-byte store each).
// fp32 accumulation, one rounding to bf16 -- the arithmetic of MIOpen's bf16 convolution under
// torch.autocast, up to the summation order.
//
// Two kernels, both persistent (one 8-wave workgroup per CU) and fed by LDS-DMA
// (buffer_load_dwordx4 ... lds: no staging registers, no ds_write pass; out-of-image taps use an
// out-of-range offset, which the descriptor's range check turns into zeros):
//   conv_dma_kernel    any layer: 256 pixels x BN channels per tile, three LDS stages, the
//                      (tile, K tile) steps of a workgroup streamed with a counted vmcnt and raw
//                      barriers; every workgroup keeps one channel tile (so its lanes' channels
//                      never change) and walks a contiguous range of pixel tiles.
//   conv3x3c64_kernel  3x3 / stride 1 / 64 -> 64 (ResNet layer 1): weights resident in
//                      registers, each tile's input rows DMA'd once into a zero-padded LDS patch
//                      that all 9 taps read (the generic kernel fetches every pixel 9 times and
//                      is L2-bound on these layers).
//   (and conv3x3_halo_kernel, the same patch idea with streamed weights for Cin >= 128, and
//   conv1x1_kernel, a streaming 1x1 / stride-2 kernel without LDS stages for 64 -> 128.)
// Optional BatchNorm statistics (a->stats, conv_dma_kernel only): each lane keeps running sums of its channels' bf16
// outputs around its first value; at the end the lanes and waves of a workgroup are merged
// (Chan's pairwise update, fixed order) into one (count, mean, M2) block per workgroup, which
// mcgmil_batchnorm_act combines in fp64 -- the activation is then never re-read for statistics.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <string>
#include <type_traits>

#include "../../include/mcgmil_features.h"
#include "mcgmil_device.h"
#include "mcgmil_error.h"

namespace {

using namespace mcgmil;
using mcgmil_detail::fail;
using mcgmil_detail::hip_fail;

constexpr int kThreads = 512;       // 8 waves
constexpr int kBM = 256;            // output pixels per tile
constexpr int kBK = 64;             // K elements per stage (one 128-byte row per pixel/channel)
constexpr int kRowBytes = kBK * 2;
constexpr int kStages = 3;

struct ConvGeom {
    const __bf16* x;
    const __bf16* w;
    __bf16* y;
    float* stats;        // [Gm][3][Cout] (count, mean, M2) per workgroup row, or NULL
    const float* in_ab;  // [2][Cin] input BatchNorm (a_c then b_c; halo kernels only), or NULL
    float in_lo;         // input BatchNorm floor: 0 (ReLU) or -inf
    int N, H, W, Cin, OH, OW, Cout, KH, KW, stride, pad;
    int M;               // N * OH * OW (< 2^31, host-checked)
    int KT;              // K tiles: KH * KW * Cin / 64
    int cin_tiles;       // Cin / 64
    int tiles_m;         // pixel tiles
    int tiles_n;         // channel tiles: Cout / BN
    int Gm;              // workgroups per channel tile
    uint32_t x_bytes;    // buffer range of x (< 2^31, host-checked)
    uint32_t w_bytes;
    // K split of the last pixel tiles (conv_dma_kernel without statistics, split_p >= 2): each
    // workgroup row gm runs full_tiles whole tiles [gm F, (gm + 1) F); the R = tiles_m - F Gm tiles
    // left are cut into split_p K ranges, range p of left tile q run by row q split_p + p, which
    // stores its fp32 sums in part[(tn R + q) split_p + p][BM][BN]; conv_split_fixup_kernel adds
    // the ranges in order and rounds once
    float* part;
    int split_p;         // 0: no split
    int full_tiles;      // F
};

// byte offset of 16-byte chunk c of row r in a swizzled [rows][128 B] stage: rows 2j and 2j+1
// share a bank half, so chunk c sits at slot c ^ ((r >> 1) & 7); the 16 lanes of an MFMA
// fragment read (rows r0..r0+15, one chunk) then hit 16 distinct 4-bank groups
__device__ __forceinline__ uint32_t swz(int r, int c) {
    return (uint32_t)r * kRowBytes + (uint32_t)((c ^ ((r >> 1) & 7)) << 4);
}

// XCD-aware order (guide T1, bijective form): consecutive logical ids land on one XCD's L2
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// 16 bytes per lane from a buffer straight into LDS at the wave-uniform base + 16 * lane. The
// builtin only exists in the device pass; the host pass must still see a kernel body to emit the
// launch stub, hence the guard (device-only code, not a second platform path).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
#else
    (void)r; (void)lds; (void)voff; (void)soff;
#endif
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- Input BatchNorm (mcgmil_conv_args.in_ab) on a halo patch, in place. A lane rewrites the
// 16-byte LDS slot it DMA'd itself (so only its own vmcnt has to cover the DMA, no barrier):
// the 8 channels become bf16(max(fmaf(x, a_c, b_c), lo)) -- mcgmil_batchnorm_act's apply
// arithmetic, so the convolution sees bit-identical inputs to the unfused pair of passes. keep is
// 0 for padding pixels, which must stay zero (BN(0) = b_c is not).
// The LDS read and write are inline asm: the compiler's wait-count pass treats a ds_read after
// an LDS-DMA as a possible alias and would put an s_waitcnt vmcnt(0) in front of it, draining
// the weight and patch DMAs just issued for the next step. The slot's own DMA is covered by the
// caller's counted wait; the caller also waits for the writes (wait_lds_writes) before the
// barrier that publishes the patch.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t lds_addr(const unsigned char* p) {
    return (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const unsigned char*)p);
}
__device__ __forceinline__ u32x4 bn_values(u32x4 u, const float (&a)[8], const float (&b)[8], float lo, bool keep) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        o[2 * j] = (__bf16)fmaxf(fmaf(__uint_as_float(u[j] << 16), a[2 * j], b[2 * j]), lo);
        o[2 * j + 1] = (__bf16)fmaxf(fmaf(__uint_as_float(u[j] & 0xFFFF0000u), a[2 * j + 1], b[2 * j + 1]), lo);
    }
    return __builtin_bit_cast(u32x4, o) & (keep ? 0xFFFFFFFFu : 0u);
}
__device__ __forceinline__ void bn_slot(unsigned char* slot, const float (&a)[8], const float (&b)[8], float lo,
                                        bool keep) {
    const uint32_t addr = lds_addr(slot);
    u32x4 u;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(u) : "v"(addr) : "memory");
    const u32x4 r = bn_values(u, a, b, lo, keep);
    asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(r) : "memory");
}
// Four slots at once (one LDS round trip instead of four); slots past `count` are read (at a
// valid address) but not written. The wait names the read values, so no use moves above it.
__device__ __forceinline__ void bn_slots4(const uint32_t (&addr)[4], int count, uint32_t keep_bits,
                                          const float (&a)[8], const float (&b)[8], float lo) {
    u32x4 u0, u1, u2, u3;
    asm volatile("ds_read_b128 %0, %1" : "=v"(u0) : "v"(addr[0]) : "memory");
    asm volatile("ds_read_b128 %0, %1" : "=v"(u1) : "v"(addr[1]) : "memory");
    asm volatile("ds_read_b128 %0, %1" : "=v"(u2) : "v"(addr[2]) : "memory");
    asm volatile("ds_read_b128 %0, %1" : "=v"(u3) : "v"(addr[3]) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3)::"memory");
    const u32x4 r0 = bn_values(u0, a, b, lo, keep_bits & 1);
    asm volatile("ds_write_b128 %0, %1" ::"v"(addr[0]), "v"(r0) : "memory");
    if (count > 1) {
        const u32x4 r1 = bn_values(u1, a, b, lo, (keep_bits >> 1) & 1);
        asm volatile("ds_write_b128 %0, %1" ::"v"(addr[1]), "v"(r1) : "memory");
    }
    if (count > 2) {
        const u32x4 r2 = bn_values(u2, a, b, lo, (keep_bits >> 2) & 1);
        asm volatile("ds_write_b128 %0, %1" ::"v"(addr[2]), "v"(r2) : "memory");
    }
    if (count > 3) {
        const u32x4 r3 = bn_values(u3, a, b, lo, (keep_bits >> 3) & 1);
        asm volatile("ds_write_b128 %0, %1" ::"v"(addr[3]), "v"(r3) : "memory");
    }
}

__device__ __forceinline__ void wait_lds_writes() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
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

#ifndef MCGMIL_DMA_DIAG
// conv_dma_kernel timing diagnostics (wrong results; after the first NS steps): 1 no DMA wait,
// 2 no barrier, 4 no MFMAs (fragments still read), 8 no fragment reads (MFMAs on register junk),
// 16 no DMA issued
#define MCGMIL_DMA_DIAG 0
#endif
#ifndef MCGMIL_HALO_DIAG
// conv3x3_halo_kernel timing diagnostics (wrong results; after the first 2 steps): 1 no DMA wait,
// 2 no barrier, 4 no MFMAs (fragments still read), 8 no fragment reads, 16 no input-BatchNorm
// rewrite (XF), 32 no DMA issued
#define MCGMIL_HALO_DIAG 0
#endif

// ---- BatchNorm statistics of the output (see the header comment)
// Running sums of NCH channels of one lane: around x0 (the lane's first value per channel).
// PACK keeps the shifts as bf16 pairs (they are bf16 outputs, so exactly): half the registers.
template <int NCH, bool PACK = false>
struct LaneStats {
    float x0f[PACK ? 1 : NCH];
    uint32_t x0p[PACK ? NCH / 2 : 1];
    float S[NCH], SS[NCH];
    float n;
    __device__ __forceinline__ float x0(int c) const {
        if constexpr (PACK) return __uint_as_float((c & 1) ? (x0p[c >> 1] & 0xFFFF0000u) : (x0p[c >> 1] << 16));
        else return x0f[c];
    }
    __device__ __forceinline__ void set_x0(int c, float x) {
        if constexpr (PACK) {
            const uint32_t b = __float_as_uint(x) >> 16;       // x is a bf16 value: exact
            x0p[c >> 1] = (c & 1) ? ((x0p[c >> 1] & 0xFFFFu) | (b << 16)) : ((x0p[c >> 1] & 0xFFFF0000u) | b);
        } else {
            x0f[c] = x;
        }
    }
    __device__ __forceinline__ void init() {
        n = 0.f;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            S[c] = SS[c] = 0.f;
            set_x0(c, 0.f);
        }
    }
};

// End of kernel: lanes -> (n, mean, M2); merged over the 16 pixel lanes of each channel group
// (butterfly, the lane-0 result kept), then over the WGM waves that share channels (LDS, wave
// order). Lane channel of index c = 4 i + v: chan0 + 16 i + 4 (lane >> 4) + v (local to the
// workgroup's channel tile of width BN). Writes stats[(row * 3 + k) * Cout + col0 + local].
template <int NCH, int WGM, int BN, bool PACK>
__device__ void write_stats(const LaneStats<NCH, PACK>& st, int chan0, int wm, float* lds, float* stats,
                            int row, int Cout, int col0) {
    const int lane = threadIdx.x & 63;
    float n = st.n, m[NCH], M2[NCH];
    const float rn = n > 0.f ? 1.f / n : 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        m[c] = st.x0(c) + st.S[c] * rn;
        M2[c] = fmaxf(st.SS[c] - st.S[c] * st.S[c] * rn, 0.f);
        if (!(n > 0.f)) m[c] = M2[c] = 0.f;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
        float mb[NCH], M2b[NCH];
        const float nb = __shfl_xor(n, o, 64);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            mb[c] = __shfl_xor(m[c], o, 64);
            M2b[c] = __shfl_xor(M2[c], o, 64);
        }
        chan_merge<NCH>(n, m, M2, nb, mb, M2b);
    }
    __syncthreads();                                   // LDS stages no longer read
    float* red = lds;                                  // [WGM][3][BN]
    if ((lane & 15) == 0) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int local = chan0 + 16 * (c >> 2) + 4 * (lane >> 4) + (c & 3);
            red[(wm * 3 + 0) * BN + local] = n;
            red[(wm * 3 + 1) * BN + local] = m[c];
            red[(wm * 3 + 2) * BN + local] = M2[c];
        }
    }
    __syncthreads();
    for (int local = threadIdx.x; local < BN; local += blockDim.x) {
        float cn = red[local], cm[1] = {red[BN + local]}, cM2[1] = {red[2 * BN + local]};
        for (int w = 1; w < WGM; ++w) {
            const float mb[1] = {red[(w * 3 + 1) * BN + local]}, M2b[1] = {red[(w * 3 + 2) * BN + local]};
            chan_merge<1>(cn, cm, cM2, red[(w * 3) * BN + local], mb, M2b);
        }
        stats[((size_t)row * 3 + 0) * Cout + col0 + local] = cn;
        stats[((size_t)row * 3 + 1) * Cout + col0 + local] = cm[0];
        stats[((size_t)row * 3 + 2) * Cout + col0 + local] = cM2[0];
    }
}

// The epilogue of one pixel fragment: round to bf16, store 4 x 8 bytes, accumulate statistics.
// PRED: pixels past M are neither stored nor counted (only the last tile can have them).
template <int FI, bool STATS, bool PRED, bool PACK>
__device__ __forceinline__ void store_fragment(const f32x4 (&acc)[FI], __bf16* dst, bool valid,
                                               bool first, LaneStats<4 * FI, PACK>& st) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
        bf16x4 o;
#pragma unroll
        for (int v = 0; v < 4; ++v) o[v] = (__bf16)acc[i][v];
        if (!PRED || valid) *reinterpret_cast<bf16x4*>(dst + i * 16) = o;
        if (STATS) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const float x = (float)o[v];
                if (first) st.set_x0(4 * i + v, x);
                float d = x - st.x0(4 * i + v);
                if (PRED) d = valid ? d : 0.f;
                st.S[4 * i + v] += d;
                st.SS[4 * i + v] = fmaf(d, d, st.SS[4 * i + v]);
            }
        }
    }
    if (STATS) st.n += (!PRED || valid) ? 1.f : 0.f;
}

// ---- conv_dma_kernel: 256 x BN tiles, 8 waves as 4 (pixels) x 2 (channels) for BN = 128 or
// 4 x 2 of 64 x 32 for BN = 64. Workgroup (logical id L): channel tile tn = L % tiles_n and the
// contiguous pixel tiles of row gm = L / tiles_n; ids of one row sit on one XCD (same input rows
// in L2). Its (pixel tile, K tile) steps form one stream through three LDS stages: step s + 2 is
// issued right after the barrier that opens step s (two compute phases to land; the next tile's
// first stages load under this tile's last steps and epilogue); the wait is a counted vmcnt
// before a raw s_barrier (a __syncthreads would drain the stage still in flight).
template <int BM, int BN, int WGM, int NS, bool STATS>
__global__ __launch_bounds__(kThreads, 1) void conv_dma_kernel(const ConvGeom g) {
    constexpr int WGN = 8 / WGM;
    constexpr bool PACK = BM * BN > kBM * 128;        // 128 x 64 wave tiles: bf16-pair shifts
    constexpr int STAGE = (BM + BN) * kRowBytes;
    constexpr int PA = BM / 64, PB = BN / 64;         // 1-KiB pieces per wave per stage (A, B)
    constexpr int WM = BM / WGM, WN = BN / WGN;
    constexpr int FI = WN / 16, FJ = WM / 16;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: LDS-DMA bases (M0) by SALU
    const int L = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    const int tn = L % g.tiles_n, gm = L / g.tiles_n;
    int tm0 = (int)((long long)gm * g.tiles_m / g.Gm);
    int tm1 = (int)((long long)(gm + 1) * g.tiles_m / g.Gm);
    // K split (STATS off, host-checked): whole tiles, then at most one K range of a left tile
    bool piece = false;
    int ptm = 0, k0 = 0, k1 = 0, pslot = 0;
    if (!STATS && g.split_p > 0) {
        tm0 = gm * g.full_tiles;
        tm1 = tm0 + g.full_tiles;
        const int R = g.tiles_m - g.full_tiles * g.Gm, q = gm / g.split_p, pp = gm - q * g.split_p;
        if (q < R) {
            piece = true;
            ptm = g.full_tiles * g.Gm + q;
            k0 = pp * g.KT / g.split_p;
            k1 = (pp + 1) * g.KT / g.split_p;
            pslot = (tn * R + q) * g.split_p + pp;
        }
    }
    const int steps = (tm1 - tm0) * g.KT + (piece ? k1 - k0 : 0);
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(g.x, g.x_bytes);
    const __amdgpu_buffer_rsrc_t wr = make_rsrc(g.w, g.w_bytes);
    const uint32_t K = (uint32_t)(g.KH * g.KW * g.Cin);

    // B (weights) pieces: fixed channel tile
    uint32_t wrow[PB];
#pragma unroll
    for (int j = 0; j < PB; ++j) {
        const int r = 8 * (wave + 8 * j) + (lane >> 3);
        wrow[j] = ((uint32_t)(tn * BN + r) * K + (uint32_t)(((lane & 7) ^ ((r >> 1) & 7)) * 8)) * 2u;
    }
    // A pieces: the pixel rows of the tile being fetched (the issue side runs two steps ahead)
    int itm = -1;
    // per piece, fixed for a tile: the byte offset of the window origin's source chunk (the pixel
    // index may be negative: a valid tap adds a non-negative total) and a bit per (kh, kw) tap that
    // lies inside the image (KH * KW <= 49, host-checked), so a K step's piece costs an add and a
    // bit test -- no multiply and no bounds arithmetic per step. The source chunk of the lane's LDS
    // slot is the same for every piece ((r >> 1) & 7 does not depend on j).
    uint32_t orgb[PA], mlo[PA], mhi[PA];
    const int cha = ((lane & 7) ^ ((4 * wave + (lane >> 4)) & 7)) * 8;
    auto setup = [&](int tm) {
        itm = tm;
#pragma unroll
        for (int j = 0; j < PA; ++j) {
            const int r = 8 * (wave + 8 * j) + (lane >> 3);
            const int m = tm * BM + r;
            const int mm = m < g.M ? m : 0;
            const int n = mm / (g.OH * g.OW);
            const int rem = mm - n * g.OH * g.OW;
            const int oh = rem / g.OW, ow = rem - oh * g.OW;
            const int ih0 = oh * g.stride - g.pad, iw0 = ow * g.stride - g.pad;
            orgb[j] = (uint32_t)(((n * g.H + ih0) * g.W + iw0) * g.Cin + cha) * 2u;
            uint32_t cols = 0;
            for (int kw = 0; kw < g.KW; ++kw) cols |= ((unsigned)(iw0 + kw) < (unsigned)g.W ? 1u : 0u) << kw;
            uint64_t taps = 0;
            if (m < g.M)                                                  // rows past M load zeros
                for (int kh = 0; kh < g.KH; ++kh)
                    if ((unsigned)(ih0 + kh) < (unsigned)g.H) taps |= (uint64_t)cols << (kh * g.KW);
            mlo[j] = (uint32_t)taps;
            mhi[j] = (uint32_t)(taps >> 32);
        }
    };
    // issue() is called for consecutive steps: its (tile, K tile) cursor advances by one per call --
    // kt = (kh * KW + kw) * cin_tiles + cc -- without a runtime division per step
    int i_tm = tm0, i_kt = 0, i_cc = 0, i_kw = 0, i_kh = 0;
    auto to_piece = [&]() {            // the issue cursor jumps to (ptm, k0)
        i_tm = ptm;
        i_kt = k0;
        i_cc = k0 % g.cin_tiles;
        const int t = k0 / g.cin_tiles;
        i_kw = t % g.KW;
        i_kh = t / g.KW;
    };
    if (piece && tm0 == tm1) to_piece();
    auto issue = [&](int buf) {
        if (i_tm != itm) setup(i_tm);
        const int kt = i_kt, cc = i_cc, kh = i_kh, kw = i_kw;
        if (++i_cc == g.cin_tiles) {
            i_cc = 0;
            if (++i_kw == g.KW) {
                i_kw = 0;
                ++i_kh;
            }
        }
        if (++i_kt == g.KT) {
            i_kt = i_cc = i_kw = i_kh = 0;
            ++i_tm;
            if (piece && i_tm == tm1) to_piece();     // the last whole tile's K steps all issued
        }
        const uint32_t koffb = (uint32_t)(((kh * g.W + kw) * g.Cin + cc * 64) * 2);   // wave-uniform
        const int tap = kh * g.KW + kw;
        unsigned char* A = smem + buf * STAGE;
        unsigned char* B = A + BM * kRowBytes;
#pragma unroll
        for (int j = 0; j < PA; ++j) {
            const bool ok = (((tap < 32 ? mlo[j] : mhi[j]) >> (tap & 31)) & 1u) != 0u;
            dma16(xr, A + (wave + 8 * j) * 1024, ok ? orgb[j] + koffb : 0x80000000u, 0);
        }
#pragma unroll
        for (int j = 0; j < PB; ++j)
            dma16(wr, B + (wave + 8 * j) * 1024, wrow[j], (uint32_t)kt * (kBK * 2u));
    };

    const int wm = wave / WGN, wn = wave % WGN;
    f32x4 acc[FJ][FI];
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int i = 0; i < FI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    LaneStats<4 * FI, PACK> st;
    if (STATS) st.init();

    auto compute = [&](int buf) {
        const unsigned char* A = smem + buf * STAGE;
        const unsigned char* B = A + BM * kRowBytes;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int kq = ks * 4 + (lane >> 4);
            bf16x8 wf[FI];
#pragma unroll
            for (int i = 0; i < FI; ++i) {
#if MCGMIL_DMA_DIAG & 8
                asm volatile("" : "=v"(wf[i]));
#else
                wf[i] = *reinterpret_cast<const bf16x8*>(B + swz(wn * WN + i * 16 + (lane & 15), kq));
#endif
            }
            // pixel fragments in groups of 4 (fewer live operand registers with 8 of them)
#pragma unroll
            for (int j0 = 0; j0 < FJ; j0 += 4) {
                bf16x8 xf[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
#if MCGMIL_DMA_DIAG & 8
                    asm volatile("" : "=v"(xf[j]));
#else
                    xf[j] = *reinterpret_cast<const bf16x8*>(A + swz(wm * WM + (j0 + j) * 16 + (lane & 15), kq));
#endif
                }
#if MCGMIL_DMA_DIAG & 4
#pragma unroll
                for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(xf[j]));
#pragma unroll
                for (int i = 0; i < FI; ++i) asm volatile("" ::"v"(wf[i]));
#else
#pragma unroll
                for (int i = 0; i < FI; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[j0 + j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[j0 + j][i], 0, 0, 0);
#endif
            }
        }
    };
    // a K range of a left tile: fp32 sums to part[pslot] ([BM][BN], 4 channels per 16-B store)
    auto store_part = [&]() {
        float* dst = g.part + (size_t)pslot * BM * BN + wn * WN + 4 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            const int ml = wm * WM + j * 16 + (lane & 15);
#pragma unroll
            for (int i = 0; i < FI; ++i) {
                *reinterpret_cast<f32x4*>(dst + (size_t)ml * BN + i * 16) = acc[j][i];
                acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };
    auto epilogue = [&](int tm, bool first) {
        const bool full = (tm + 1) * BM <= g.M;
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            const int m = tm * BM + wm * WM + j * 16 + (lane & 15);
            __bf16* dst = g.y + (size_t)(m < g.M ? m : 0) * g.Cout + tn * BN + wn * WN + 4 * (lane >> 4);
            if (full) store_fragment<FI, STATS, false>(acc[j], dst, true, first && j == 0, st);
            else store_fragment<FI, STATS, true>(acc[j], dst, m < g.M, first && j == 0, st);
#pragma unroll
            for (int i = 0; i < FI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };

    // NS LDS stages: step s + NS - 1 is issued into the stage step s - 1 used
    if (steps > 0) {
        issue(0);
        if (NS == 3 && steps > 1) issue(1);
    }
    int buf = 0, kt = 0, tm = tm0, kend = g.KT;
    bool in_piece = false;
    if (piece && tm0 == tm1) {
        in_piece = true;
        tm = ptm;
        kt = k0;
        kend = k1;
    }
    for (int s = 0; s < steps; ++s) {
        // step s landed (counted: the next step's DMAs may stay in flight; vmcnt retires in order)
#if MCGMIL_DMA_DIAG & 1   // timing only: no wait for the stage's DMA after the first steps (wrong results)
        if (s < NS)
#endif
        {
            if (NS == 3 && s + 1 < steps) wait_vmcnt<PA + PB>();
            else wait_vmcnt<0>();
        }
#if MCGMIL_DMA_DIAG & 2
        if (s < NS)
#endif
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#if MCGMIL_DMA_DIAG & 16
        if (s + NS - 1 < steps && s < NS) issue(buf == 0 ? NS - 1 : buf - 1);
#else
        if (s + NS - 1 < steps) issue(buf == 0 ? NS - 1 : buf - 1);
#endif
        compute(buf);
        buf = buf == NS - 1 ? 0 : buf + 1;
        if (++kt == kend) {
            if (in_piece) {
                store_part();
            } else {
                epilogue(tm, tm == tm0);
                kt = 0;
                ++tm;
                if (piece && tm == tm1) {
                    in_piece = true;
                    tm = ptm;
                    kt = k0;
                    kend = k1;
                }
            }
        }
    }
    if (STATS) write_stats<4 * FI, WGM, BN>(st, wn * WN, wm, reinterpret_cast<float*>(smem), g.stats, gm,
                                             g.Cout, tn * BN);
}

// The K split's second pass (ConvGeom::split_p): one thread per (left tile pixel, 8 channels) adds
// the tile's split_p fp32 K-range sums in range order and rounds once to bf16 -- the split tile's
// outputs differ from the unsplit kernel's only in where the fp32 sum is rounded.
template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_split_fixup_kernel(const ConvGeom g) {
    const int R = g.tiles_m - g.full_tiles * g.Gm, P = g.split_p;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)R * g.tiles_n * BM * (BN / 8)) return;
    const int cg = (int)(idx % (BN / 8));
    const long long r = idx / (BN / 8);
    const int ml = (int)(r % BM), t = (int)(r / BM);            // t = tn R + q
    const int tn = t / R, q = t - tn * R;
    const int m = (g.full_tiles * g.Gm + q) * BM + ml;
    if (m >= g.M) return;
    const float* src = g.part + (size_t)t * P * BM * BN + (size_t)ml * BN + cg * 8;
    f32x4 a = *reinterpret_cast<const f32x4*>(src), b = *reinterpret_cast<const f32x4*>(src + 4);
    for (int p = 1; p < P; ++p) {
        a += *reinterpret_cast<const f32x4*>(src + (size_t)p * BM * BN);
        b += *reinterpret_cast<const f32x4*>(src + (size_t)p * BM * BN + 4);
    }
    bf16x8 o;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        o[v] = (__bf16)a[v];
        o[4 + v] = (__bf16)b[v];
    }
    *reinterpret_cast<bf16x8*>(g.y + (size_t)m * g.Cout + tn * BN + cg * 8) = o;
}

// ---- 3x3 / stride 1 / pad 1, 64 -> 64 channels (ResNet layer 1): halo-tile kernel.
// The whole 64 x 576 weight matrix lives in registers (each wave its 32 channels: 36 fragments).
// Per 256-pixel tile the input rows are DMA'd ONCE into LDS as a zero-padded patch: padded rows
// P = n (H + 2) + ih + 1 of W + 2 pixels x 128 B (XOR-swizzled by patch pixel). All 9 taps read
// their A fragments from the patch at a tap offset -- no barrier inside a tile, 5x less L2
// traffic per FLOP. The next tile's patch loads into the other buffer during this tile.
__device__ __forceinline__ uint32_t swz_lin(int p, int c) {     // swz() for a patch pixel index
    return (uint32_t)p * kRowBytes + (uint32_t)((c ^ ((p >> 1) & 7)) << 4);
}

// Fragment column c (lane & 15) of a halo kernel holds tile pixel frag_px(c) of its 16: the
// ds_read_b128 lane groups pair columns {0-3, 12-15} at chunk kq with columns 4-11 at kq ^ 1, so the
// former take the even pixels and the latter the odd ones. With the swizzle above every tap's read
// of 16 contiguous patch pixels is then conflict-free; a fragment that wraps an output row reads
// 2-way (with contiguous columns layers 1 / 2 averaged 1.71 / 1.81 LDS cycles per group, now
// 1.14 / 1.43). Outputs are the same per pixel; only the BatchNorm statistics' per-lane summation
// order follows the columns.
__device__ __forceinline__ int frag_px(int c) { return c < 4 ? 2 * c : c < 12 ? 2 * c - 7 : 2 * c - 16; }

// The halo kernels' swz_lin(pp + toff, kq) for the 9 taps of a fragment, without re-deriving
// the swizzle from the pixel index each time: with pa = pp * 128 and pb = pp << 3 kept per tile and
// the tap's scalar toff, the address is pa + 128 toff + (((pb + 8 toff) & 0x70) ^ 16 kq) -- three
// VALU (add, bitop3, add3); the second K half (kq + 4, slot ^ 4) is the same offset with bit 6
// flipped. (conv3x3c64_kernel<STATS, XF> keeps swz_lin: it spills with the extra live registers.)
struct PatchPx {
    uint32_t pa, pb;
};
__device__ __forceinline__ PatchPx patch_px(int pp) { return {(uint32_t)pp * kRowBytes, (uint32_t)pp << 3}; }
__device__ __forceinline__ uint32_t tap_addr(PatchPx q, int toff, uint32_t kq16) {
    return q.pa + (uint32_t)toff * kRowBytes + (((q.pb + ((uint32_t)toff << 3)) & 0x70u) ^ kq16);
}

struct HaloGeom {
    ConvGeom g;
    int WP;         // W + 2 (padded row width)
    int NR;         // padded rows per patch (max over tiles)
    int patch_px;   // NR * WP rounded up to whole 8-pixel DMA pieces
    int tiles;
    int q256, r256;   // ring kernel: kBM = q256 * OW + r256 (one tile's advance in output rows / columns)
    int q255, r255;   // kBM - 1 (a tile's first pixel to its last)
};

// With XF (input BatchNorm) the [2][64] a, b table sits after the two patches; each lane rewrites
// its own slots of a tile's patch between its vmcnt wait and the barrier that opens the tile. A
// lane's slots all hold one 8-channel chunk: pieces of a wave are wave + 8 k, so the swizzle
// (p >> 1) & 7 of its pixels p = 8 piece + lane / 8 only depends on the wave's parity.
template <bool STATS, bool XF>
__global__ __launch_bounds__(kThreads, 1) void conv3x3c64_kernel(const HaloGeom hg) {
    const ConvGeom& g = hg.g;
    constexpr int FI = 2, FJ = 4, KSTEPS = 18;          // wave: 64 pixels x 32 channels
    // tap_addr (fewer VALU per fragment read) unless STATS and XF both hold registers: that
    // instantiation spills with it
    constexpr bool kTapAddr = !(STATS && XF);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int t0 = (int)((long long)blockIdx.x * hg.tiles / gridDim.x);
    const int t1 = (int)((long long)(blockIdx.x + 1) * hg.tiles / gridDim.x);
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(g.x, g.x_bytes);
    const int HP = g.H + 2, WP = hg.WP;
    const size_t patch_bytes = (size_t)hg.patch_px * kRowBytes;

    // weights -> registers: K step s = (tap, half) covers k = 32 s .. 32 s + 31
    bf16x8 wf[KSTEPS][FI];
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
        for (int i = 0; i < FI; ++i) {
            const int co = wn * 32 + i * 16 + (lane & 15);
            wf[s][i] = *reinterpret_cast<const bf16x8*>(g.w + (size_t)co * 576 + s * 32 + (lane >> 4) * 8);
        }
    LaneStats<4 * FI, true> st;   // bf16-pair shifts: this kernel is at the register limit
    if (STATS) st.init();

    // No per-tile integer division on the vector side: a tile's first pixel (n0, oh0, ow0) is
    // scalar math, every lane-dependent offset below is split into (rows, cols) once per kernel
    // and carried forward per tile / per DMA piece.
    const int OHW = g.OH * g.OW;
    int dqr[FJ];      // this lane's output pixel offset in the tile per fragment: rows << 16 | cols
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
        const int d = wm * 64 + j * 16 + frag_px(lane & 15), q = d / g.OW;
        dqr[j] = (q << 16) | (d - q * g.OW);
    }
    const int p0 = wave * 8 + (lane >> 3);       // first patch pixel this lane DMAs
    const int rr0 = p0 / WP, col0 = p0 - rr0 * WP;
    const int qstep = 64 / WP, rstep = 64 - qstep * WP;  // pieces advance by 64 patch pixels
    uint32_t okm = 0;     // XF: bit k = piece k of this wave's in-flight patch is inside the image
    float* ab_tbl = reinterpret_cast<float*>(smem + 2 * patch_bytes);
    if (XF) {
        if (threadIdx.x < 128) ab_tbl[threadIdx.x] = g.in_ab[threadIdx.x < 64 ? threadIdx.x : g.Cin + threadIdx.x - 64];
        __syncthreads();
    }

    int need_px = hg.patch_px;   // pixels of the in-flight patch that the tile reads
    auto issue = [&](int tile, int buf) {
        const int m0 = tile * kBM;
        {   // the tile's last output pixel, tap (2, 2), bounds the patch pixels it reads: most tiles
            // need ~3/4 of the worst-case patch (no image boundary inside the tile)
            const int n0 = m0 / OHW, oh0 = (m0 - n0 * OHW) / g.OW;
            const int ml = m0 + kBM - 1 < g.M ? m0 + kBM - 1 : g.M - 1;
            const int nl = ml / OHW, rl = ml - nl * OHW, ohl = rl / g.OW, owl = rl - ohl * g.OW;
            const int need = (((nl - n0) * HP + ohl - oh0 + 2) * WP + owl + 3 + 7) & ~7;
            need_px = need < hg.patch_px ? need : hg.patch_px;
        }
        int n = m0 / OHW;
        int prel = (m0 - n * OHW) / g.OW + rr0;         // padded row (relative to image n) of p
        int col = col0;
        while (prel >= HP) {
            prel -= HP;
            ++n;
        }
        unsigned char* Lp = smem + buf * patch_bytes;
        okm = 0;
        for (int piece = wave, k = 0; piece * 8 < need_px; piece += 8, ++k) {
            const int p = piece * 8 + (lane >> 3);
            const int c = (lane & 7) ^ ((p >> 1) & 7);     // source chunk of this lane's slot
            const int ih = prel - 1, iw = col - 1;
            const bool ok = n < g.N && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
            if (XF) okm |= (uint32_t)ok << k;
            const uint32_t off = ((uint32_t)((n * g.H + ih) * g.W + iw) * 64u + (uint32_t)c * 8u) * 2u;
            dma16(xr, Lp + piece * 1024, ok ? off : 0x80000000u, 0);
            col += rstep;
            prel += qstep;
            if (col >= WP) {
                col -= WP;
                ++prel;
            }
            while (prel >= HP) {
                prel -= HP;
                ++n;
            }
        }
    };

    if (t0 < t1) issue(t0, 0);
    int buf = 0;
    for (int t = t0; t < t1; ++t) {
        // patch t landed; only the previous tile's epilogue stores (FI * FJ per lane) may still fly
        if (t == t0) wait_vmcnt<0>();
        else wait_vmcnt<FI * FJ>();
        if (XF) {
            const int c = (lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7);
            float a[8], b[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                a[j] = ab_tbl[8 * c + j];
                b[j] = ab_tbl[64 + 8 * c + j];
            }
            // this wave's pieces wave + 8 k, four per LDS round trip
            const uint32_t base = lds_addr(smem + buf * patch_bytes) + lane * 16 + wave * 1024;
            const int np = (need_px / 8 - wave + 7) / 8;
            for (int k0 = 0; k0 < np; k0 += 4) {
                uint32_t ad[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) ad[j] = base + (uint32_t)(k0 + j < np ? k0 + j : k0) * 8192u;
                bn_slots4(ad, np - k0, okm >> k0, a, b, g.in_lo);
            }
            wait_lds_writes();
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (t + 1 < t1) issue(t + 1, buf ^ 1);
        const unsigned char* Lp = smem + buf * patch_bytes;
        const int m0 = t * kBM;
        const int n0 = m0 / OHW, r0m = m0 - n0 * OHW, oh0 = r0m / g.OW, ow0 = r0m - oh0 * g.OW;
        int pp[FJ];                                   // patch pixel of tap (0, 0) per fragment
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            int ow = ow0 + (dqr[j] & 0xFFFF), oh = oh0 + (dqr[j] >> 16), dn = 0;
            if (ow >= g.OW) {
                ow -= g.OW;
                ++oh;
            }
            while (oh >= g.OH) {
                oh -= g.OH;
                ++dn;
            }
            // rows past M read a finite patch row and are not stored
            pp[j] = (dn * HP + oh - oh0) * WP + ow;
            if (pp[j] + 2 * WP + 2 >= hg.patch_px) pp[j] = 0;
        }
        PatchPx pq[FJ];
#pragma unroll
        for (int j = 0; j < FJ; ++j) pq[j] = patch_px(pp[j]);
        f32x4 acc[FJ][FI];
#pragma unroll
        for (int j = 0; j < FJ; ++j)
#pragma unroll
            for (int i = 0; i < FI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int toff = (tap / 3) * WP + (tap % 3);
            uint32_t ad[FJ];        // kTapAddr: the tap's K-half-0 addresses (half 1: bit 6 flipped)
            if constexpr (kTapAddr)
#pragma unroll
                for (int j = 0; j < FJ; ++j) ad[j] = tap_addr(pq[j], toff, (uint32_t)(lane >> 4) << 4);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 xf[FJ];
#pragma unroll
                for (int j = 0; j < FJ; ++j) {
                    const uint32_t a = kTapAddr ? (ks ? ad[j] ^ 64u : ad[j])
                                                : swz_lin(pp[j] + toff, ks * 4 + (lane >> 4));
                    xf[j] = *reinterpret_cast<const bf16x8*>(Lp + a);
                }
#pragma unroll
                for (int i = 0; i < FI; ++i)
#pragma unroll
                    for (int j = 0; j < FJ; ++j)
                        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[tap * 2 + ks][i], xf[j], acc[j][i], 0, 0, 0);
            }
        }
        const bool full = m0 + kBM <= g.M, first = t == t0;
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            const int m = m0 + wm * 64 + j * 16 + frag_px(lane & 15);
            __bf16* dst = g.y + (size_t)(m < g.M ? m : 0) * 64 + wn * 32 + 4 * (lane >> 4);
            if (full) store_fragment<FI, STATS, false>(acc[j], dst, true, first && j == 0, st);
            else store_fragment<FI, STATS, true>(acc[j], dst, m < g.M, first && j == 0, st);
        }
        buf ^= 1;
    }
    if (STATS) write_stats<4 * FI, 4, 64>(st, wn * 32, wm, reinterpret_cast<float*>(smem), g.stats,
                                          (int)blockIdx.x, 64, 0);
}

// ---- conv3x3c64_ring_kernel: the same layer-1 convolution on a ring of input rows.
// conv3x3c64_kernel is vector-issue bound (5 VALU per MFMA): each tile re-DMAs its whole patch
// (~1.7 loads per input row) with ~20 VALU of address stepping per 1-KiB piece, and each tap
// read re-derives its XOR-swizzled address. Here:
//  - LDS holds a ring of 16 padded input rows (R = n (H + 2) + ih + 1; rows 0 and H + 1 of an
//    image are zeros) at ring row R % 16, CHUNK-MAJOR: chunk c (8 channels) of padded column q at
//    (R % 16) * 8 KiB + c * 1 KiB + q * 16 (W + 2 <= 64 columns). A tile DMAs only the rows the
//    previous tile did not need: each input row is loaded once per workgroup.
//  - One piece = one (row, chunk): wave w loads chunk w of every row, lane = padded column, so a
//    piece costs one VALU add (row base scalar, column offset per lane fixed) and, with XF, the
//    wave's a / b coefficients are 16 scalars for the whole kernel.
//  - A fragment's 16 pixels read one chunk at consecutive columns: 16 consecutive 16-B slots, no
//    swizzle needed. Columns 0-3 / 12-15 of a fragment take its pixels 0-7 and columns 4-11 pixels
//    8-15 (ring_px), so every ds_read_b128 lane group (chunk kq for one half, kq + 1 for the other;
//    the chunk planes are 1 KiB apart) covers 16 distinct slots mod 256 B.
//  - Tap (kh, kw) and K half ks of a fragment are its per-tile row base for kh plus the immediate
//    kw * 16 + ks * 4 KiB: no address VALU in the tap loop.
// The ring holds the rows of two consecutive tiles (the host checks the span <= 16): tile t + 1's
// new rows load into ring rows tile t does not read, right after the barrier that opens tile t.
#ifndef MCGMIL_RING_DIAG
#define MCGMIL_RING_DIAG 0         // timing diagnostics only (wrong results): 1 no epilogue, 2 no row DMA
#endif                             // after the first tile, 4 no barrier, 8 no wait for the row DMA,
                                   // 16 contiguous DMA sources
#ifndef MCGMIL_RING_WAVES
#define MCGMIL_RING_WAVES 8        // 4: one wave per SIMD (128 x 32 wave tiles)
#endif
#ifndef MCGMIL_RING_PACK
#define MCGMIL_RING_PACK true
#endif
#ifndef MCGMIL_C64_RING
#define MCGMIL_C64_RING 1          // 0: conv3x3c64_kernel for layer 1 (A/B builds)
#endif
constexpr int kRingRows = 16;
constexpr int kRingCols = 64;
constexpr int kRingRowBytes = 8 * kRingCols * 16;
constexpr size_t kRingBytes = (size_t)kRingRows * kRingRowBytes;   // 128 KiB
__device__ __forceinline__ int ring_px(int c) { return c < 4 ? c : c < 12 ? c + 4 : c - 8; }

template <bool STATS, bool XF, int NW>
__global__ __launch_bounds__(NW * 64, 1) void conv3x3c64_ring_kernel(const HaloGeom hg) {
    const ConvGeom& g = hg.g;
    // NW = 8: two waves per SIMD, a wave 64 pixels x 32 channels; NW = 4: one wave per SIMD with the
    // whole register file, a wave 128 pixels x 32 channels (FJ = 8)
    constexpr int FI = 2, FJ = 32 / NW, KSTEPS = 18, PXG = 16 * FJ, CPW = 8 / NW;   // CPW: chunks per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int t0 = (int)((long long)blockIdx.x * hg.tiles / gridDim.x);
    const int t1 = (int)((long long)(blockIdx.x + 1) * hg.tiles / gridDim.x);
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(g.x, g.x_bytes);
    const int HP = g.H + 2, OHW = g.OH * g.OW;

    bf16x8 wf[KSTEPS][FI];
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
        for (int i = 0; i < FI; ++i) {
            const int co = wn * 32 + i * 16 + (lane & 15);
            wf[s][i] = *reinterpret_cast<const bf16x8*>(g.w + (size_t)co * 576 + s * 32 + (lane >> 4) * 8);
        }
    LaneStats<4 * FI, MCGMIL_RING_PACK> st;
    if (STATS) st.init();

    // DMA: lane = padded column, source column lane - 1 (columns 0 and W + 1.. stay zero)
    const bool lane_ok = lane >= 1 && lane <= g.W;
    const uint32_t lane_off = lane_ok ? (uint32_t)(lane - 1) * kRowBytes : 0x80000000u;
    const uint32_t slot_lane = (uint32_t)lane * 16u;
    // the next row to load, R = cn * HP + cr
    int cn = 0, cr = 0;
    auto issue_rows = [&](int Ra, int Rb) {
        for (int R = Ra; R <= Rb; ++R) {
            const bool ok = cr >= 1 && cr <= g.H && cn < g.N;
            const uint32_t row = (uint32_t)((cn * g.H + cr - 1) * g.W) * kRowBytes;
#pragma unroll
            for (int q = 0; q < CPW; ++q) {     // chunk c = wave + NW q of the row
                const int c = wave + NW * q;
#if MCGMIL_RING_DIAG & 16   // timing only: each piece reads 1 KiB of contiguous source (wrong data)
                dma16(xr, smem + (R & (kRingRows - 1)) * kRingRowBytes + c * 1024,
                      ok ? row + (uint32_t)c * 1024u + (uint32_t)lane * 16u : 0x80000000u, 0);
#else
                dma16(xr, smem + (R & (kRingRows - 1)) * kRingRowBytes + c * 1024,
                      ok ? row + (uint32_t)c * 16u + lane_off : 0x80000000u, 0);
#endif
            }
            if (++cr == HP) {
                cr = 0;
                ++cn;
            }
        }
    };
    // XF: the rows just landed, R = xn * HP + xr_ (a second cursor one batch behind)
    int xn = 0, xrr = 0;
    auto rewrite_rows = [&](int Ra, int Rb) {
        // this wave's chunk (channels 8 wave .. 8 wave + 7): scalar loads through the constant
        // address space, so the 16 coefficients take no VGPRs between batches
        typedef __attribute__((address_space(4))) const float* ConstF;
        ConstF ab = (ConstF)g.in_ab;
        int sn = xn, sr = xrr;
#pragma unroll
        for (int q = 0; q < CPW; ++q) {
        const int c = wave + NW * q;
        xn = sn;
        xrr = sr;
        float xa[8], xb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            xa[j] = ab[8 * c + j];
            xb[j] = ab[g.Cin + 8 * c + j];
        }
        const uint32_t base = lds_addr(smem) + slot_lane + (uint32_t)c * 1024u;
        for (int R = Ra; R <= Rb; R += 4) {
            uint32_t ad[4];
            uint32_t keep = 0;
            const int cnt = Rb - R + 1 < 4 ? Rb - R + 1 : 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int Rj = j < cnt ? R + j : R;
                ad[j] = base + (uint32_t)(Rj & (kRingRows - 1)) * kRingRowBytes;
                if (j < cnt) {
                    keep |= (uint32_t)(xrr >= 1 && xrr <= g.H && xn < g.N) << j;
                    if (++xrr == HP) {
                        xrr = 0;
                        ++xn;
                    }
                }
            }
            bn_slots4(ad, cnt, lane_ok ? keep : 0u, xa, xb, g.in_lo);
        }
        }
    };
    // A tile's first pixel (n, oh, ow) advances by kBM = q256 rows + r256 columns: no division in
    // the tile loop (the scalar unit's would be a long serial chain before the tile's barrier).
    struct Px {
        int n, oh, ow;
    };
    auto advance = [&](Px p, int q, int r) {
        p.ow += r;
        p.oh += q;
        if (p.ow >= g.OW) {
            p.ow -= g.OW;
            ++p.oh;
        }
        while (p.oh >= g.OH) {
            p.oh -= g.OH;
            ++p.n;
        }
        return p;
    };
    // rows [lo, hi] that the tile starting at pixel f (index m0) reads
    auto tile_rows = [&](Px f, int m0, int& lo, int& hi) {
        const Px l = m0 + kBM - 1 < g.M ? advance(f, hg.q255, hg.r255) : Px{g.N - 1, g.OH - 1, g.OW - 1};
        lo = f.n * HP + f.oh;
        hi = l.n * HP + l.oh + 2;
    };

    // this lane's output pixel offset in the tile per fragment: rows << 16 | cols
    int dqr[FJ];
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
        const int d = wm * PXG + j * 16 + ring_px(lane & 15), q = d / g.OW;
        dqr[j] = (q << 16) | (d - q * g.OW);
    }
    const uint32_t kq_off = (uint32_t)(lane >> 4) * 1024u;

    int lo = 0, hi = -1, xa_lo = 0, xa_hi = -1;
    Px f{0, 0, 0};                       // first pixel of tile t
    if (t0 < t1) {
        const int m0 = t0 * kBM;
        f.n = m0 / OHW;
        f.oh = (m0 - f.n * OHW) / g.OW;
        f.ow = m0 - f.n * OHW - f.oh * g.OW;
        tile_rows(f, m0, lo, hi);
        cn = lo / HP;
        cr = lo - cn * HP;
        xn = cn;
        xrr = cr;
        issue_rows(lo, hi);
        xa_lo = lo;
        xa_hi = hi;
    }
    for (int t = t0; t < t1; ++t) {
        // tile t's rows landed; only the previous tile's epilogue stores (FI * FJ per lane) may still fly
        if (t == t0) wait_vmcnt<0>();
#if !(MCGMIL_RING_DIAG & 8)
        else wait_vmcnt<FI * FJ>();
#endif
        if (XF) {
            rewrite_rows(xa_lo, xa_hi);
            wait_lds_writes();
        }
#if !(MCGMIL_RING_DIAG & 4)
        __builtin_amdgcn_s_barrier();
#endif
        asm volatile("" ::: "memory");
        const int lo_t = lo, hi_t = hi;
        const Px ft = f;
        const int m0 = t * kBM;
        if (t + 1 < t1) {
            f = advance(f, hg.q256, hg.r256);
            int lo2, hi2;
            tile_rows(f, m0 + kBM, lo2, hi2);
#if !(MCGMIL_RING_DIAG & 2)
            issue_rows(hi_t + 1, hi2);
#endif
            xa_lo = hi_t + 1;
            xa_hi = hi2;
            lo = lo2;
            hi = hi2;
        }
        uint32_t base[FJ][3];              // per fragment and kernel row kh
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            // pixels past M (last tile) read rows inside the ring and are not stored
            int ow = ft.ow + (dqr[j] & 0xFFFF), oh = ft.oh + (dqr[j] >> 16), dn = 0;
            if (ow >= g.OW) {
                ow -= g.OW;
                ++oh;
            }
            while (oh >= g.OH) {
                oh -= g.OH;
                ++dn;
            }
            const int R = lo_t + 2 * dn + oh + dn * g.OH - ft.oh;   // n HP + oh, relative to the tile's row
            const uint32_t col = (uint32_t)ow * 16u + kq_off;
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) base[j][kh] = (uint32_t)((R + kh) & (kRingRows - 1)) * kRingRowBytes + col;
        }
        (void)hi_t;
        f32x4 acc[FJ][FI];
#pragma unroll
        for (int j = 0; j < FJ; ++j)
#pragma unroll
            for (int i = 0; i < FI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int kh = tap / 3, kw = tap % 3;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 xf[FJ];
#pragma unroll
                for (int j = 0; j < FJ; ++j)
                    xf[j] = *reinterpret_cast<const bf16x8*>(smem + base[j][kh] + kw * 16 + ks * 4096);
#pragma unroll
                for (int i = 0; i < FI; ++i)
#pragma unroll
                    for (int j = 0; j < FJ; ++j)
                        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[tap * 2 + ks][i], xf[j], acc[j][i], 0, 0, 0);
            }
        }
        const bool full = m0 + kBM <= g.M, first = t == t0;
#if MCGMIL_RING_DIAG & 1
        // diagnostic (timing only): no epilogue
        for (int j = 0; j < FJ; ++j) asm volatile("" ::"v"(acc[j][0]), "v"(acc[j][1]));
        if (full) continue;
#endif
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            const int m = m0 + wm * PXG + j * 16 + ring_px(lane & 15);
            __bf16* dst = g.y + (size_t)(m < g.M ? m : 0) * 64 + wn * 32 + 4 * (lane >> 4);
            if (full) store_fragment<FI, STATS, false>(acc[j], dst, true, first && j == 0, st);
            else store_fragment<FI, STATS, true>(acc[j], dst, m < g.M, first && j == 0, st);
        }
    }
    if (STATS) write_stats<4 * FI, NW / 2, 64>(st, wn * 32, wm, reinterpret_cast<float*>(smem), g.stats,
                                          (int)blockIdx.x, 64, 0);
}

// ---- 3x3 / stride 1 / pad 1 with Cin = 64 k >= 128 and Cout % 128 == 0 (ResNet layers 2-4):
// halo tiles with streamed weights. conv_dma_kernel re-fetches each pixel once per tap (48 KB of
// L2 traffic per 256 x 128 x 64 step); here a (pixel tile, 64-channel chunk cc) patch is DMA'd
// once into LDS and read by all 9 taps, and only the 16-KB weight tile of each (tap, cc) step is
// streamed (~23 KB per step). Steps run tile-major, then cc, then tap; one barrier per step:
//  - weights of step s + 1 go into the other of two 16-KB stages right after the barrier of s;
//  - the patch of the NEXT (tile, cc) is loaded one 1-KiB piece per wave per tap (taps 0..7),
//    issued after that step's weights, into the other of two 60-KB patch buffers (fixed 480
//    pixels; pieces past the patch read out of range, i.e. zeros, without memory traffic; the
//    four pieces past the buffer are not issued);
//  - so the wait at the top of step s is vmcnt(1) after a patch piece, vmcnt(FI * FJ) after a
//    tile's epilogue stores, else vmcnt(0) (vmcnt retires in order).
// Workgroups are mapped like conv_dma_kernel (one channel tile each, contiguous pixel tiles), so
// the BatchNorm statistics epilogue is the same.
constexpr int kPatchPx = 480;          // 2 patches + 2 weight stages + an 8-KB a, b table = 160 KB

// With XF (input BatchNorm) a lane rewrites its own slot of patch piece k two steps after issuing
// it (tap k + 2, when the counted wait has covered it), piece 7 and the kernel's first patch
// between the wait and the barrier that opens the patch's first step. A lane's slots of one patch
// all hold one 8-channel chunk (see conv3x3c64_kernel), so its 8 a / 8 b values are loaded once
// per patch.
template <bool STATS, bool XF>
__global__ __launch_bounds__(kThreads, 1) void conv3x3_halo_kernel(const HaloGeom hg) {
    const ConvGeom& g = hg.g;
    constexpr int BN = 128, WGM = 4, WGN = 2, WM = 64, WN = 64, FI = 4, FJ = 4;
    constexpr size_t PATCH = (size_t)kPatchPx * kRowBytes, WSTAGE = (size_t)BN * kRowBytes;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: LDS-DMA bases (M0) by SALU
    const int wm = wave / WGN, wn = wave % WGN;
    const int L = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    const int tn = L % g.tiles_n, gm = L / g.tiles_n;
    const int tm0 = (int)((long long)gm * g.tiles_m / g.Gm);
    const int tm1 = (int)((long long)(gm + 1) * g.tiles_m / g.Gm);
    const int CC = g.cin_tiles, SPT = 9 * CC;            // steps per tile
    const int steps = (tm1 - tm0) * SPT;
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(g.x, g.x_bytes);
    const __amdgpu_buffer_rsrc_t wr = make_rsrc(g.w, g.w_bytes);
    const int HP = g.H + 2, WP = hg.WP, OHW = g.OH * g.OW;
    unsigned char* patch0 = smem;                        // [2][kPatchPx][128 B]
    unsigned char* wst0 = smem + 2 * PATCH;              // [2][BN][128 B]
    float* ab_tbl = reinterpret_cast<float*>(wst0 + 2 * WSTAGE);   // XF: [2][Cin] a, b
    if (XF) {
        for (int i = threadIdx.x; i < 2 * g.Cin; i += kThreads) ab_tbl[i] = g.in_ab[i];
        __syncthreads();
    }

    // weights: 2 pieces per wave per step (rows 8 (wave + 8 j) + lane / 8 of the channel tile)
    const uint32_t K = (uint32_t)(9 * g.Cin);
    uint32_t wrow[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int r = 8 * (wave + 8 * j) + (lane >> 3);
        wrow[j] = ((uint32_t)(tn * BN + r) * K + (uint32_t)(((lane & 7) ^ ((r >> 1) & 7)) * 8)) * 2u;
    }
    auto issue_w = [&](int r, int buf) {        // step r of a tile -> (tap, cc): K tile kt = tap * CC + cc
        const int cc = r / 9, tap = r - cc * 9;
        const uint32_t soff = (uint32_t)(tap * CC + cc) * (kBK * 2u);
#pragma unroll
        for (int j = 0; j < 2; ++j) dma16(wr, wst0 + buf * WSTAGE + (wave + 8 * j) * 1024, wrow[j], soff);
    };
    // patch pieces: wave's piece k (k = 0..7) covers patch pixels 8 (wave + 8 k) .. + 7; the lane's
    // pixel advances by 64 per piece, carried as (image, padded row, column) -- no divisions
    const int p0 = wave * 8 + (lane >> 3);
    const int rr0 = p0 / WP, col0 = p0 - rr0 * WP;
    const int qstep = 64 / WP, rstep = 64 - qstep * WP;
    int pn = 0, prel = 0, pcol = 0, pcc = 0;
    unsigned char* pdst = patch0;
    uint32_t okm = 0;                   // XF: bit k = piece k of the patch being loaded is in the image
    float xa[8], xb[8];                 // XF: a, b of this lane's chunk of that patch
    const int xchunk = (lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7);
    // a tile's first pixel advances by kBM = q256 rows + r256 columns: no division per tile or patch
    struct Px {
        int n, oh, ow;
    };
    auto advance = [&](Px f) {
        f.ow += hg.r256;
        f.oh += hg.q256;
        if (f.ow >= g.OW) {
            f.ow -= g.OW;
            ++f.oh;
        }
        while (f.oh >= g.OH) {
            f.oh -= g.OH;
            ++f.n;
        }
        return f;
    };
    auto patch_begin = [&](Px f, int cc, int buf) {
        pn = f.n;
        prel = f.oh + rr0;
        pcol = col0;
        while (prel >= HP) {
            prel -= HP;
            ++pn;
        }
        pcc = cc;
        pdst = patch0 + buf * PATCH;
        if (XF) {
            okm = 0;
            const float* ab = ab_tbl + cc * 64 + xchunk * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                xa[j] = ab[j];
                xb[j] = ab[g.Cin + j];
            }
        }
    };
    auto xform = [&](int k) {
        if (8 * (wave + 8 * k) >= kPatchPx) return;
        bn_slot(pdst + (wave + 8 * k) * 1024 + lane * 16, xa, xb, g.in_lo, (okm >> k) & 1);
    };
    auto patch_piece = [&](int k) -> bool {
        if (8 * (wave + 8 * k) >= kPatchPx) return false;    // wave-uniform: past the buffer
        const int p = 8 * (wave + 8 * k) + (lane >> 3);
        const int c = (lane & 7) ^ ((p >> 1) & 7);
        const int ih = prel - 1, iw = pcol - 1;
        const bool ok = p < hg.patch_px && pn < g.N && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        if (XF) okm |= (uint32_t)ok << k;
        const uint32_t off = ((uint32_t)((pn * g.H + ih) * g.W + iw) * (uint32_t)g.Cin +
                              (uint32_t)(pcc * 64 + c * 8)) * 2u;
        dma16(xr, pdst + (wave + 8 * k) * 1024, ok ? off : 0x80000000u, 0);
        pcol += rstep;
        prel += qstep;
        if (pcol >= WP) {
            pcol -= WP;
            ++prel;
        }
        while (prel >= HP) {
            prel -= HP;
            ++pn;
        }
        return true;
    };

    f32x4 acc[FJ][FI];
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int i = 0; i < FI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    LaneStats<4 * FI> st;
    if (STATS) st.init();
    int dqr[FJ];      // this lane's output pixel offset in the tile per fragment: rows << 16 | cols
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
        const int d = wm * WM + j * 16 + frag_px(lane & 15), q = d / g.OW;
        dqr[j] = (q << 16) | (d - q * g.OW);
    }
    PatchPx pq[FJ];
    auto tile_setup = [&](Px f) {
        const int oh0 = f.oh, ow0 = f.ow;
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            int ow = ow0 + (dqr[j] & 0xFFFF), oh = oh0 + (dqr[j] >> 16), dn = 0;
            if (ow >= g.OW) {
                ow -= g.OW;
                ++oh;
            }
            while (oh >= g.OH) {
                oh -= g.OH;
                ++dn;
            }
            int pp = (dn * HP + oh - oh0) * WP + ow;         // rows past M: a finite patch row
            if (pp + 2 * WP + 2 >= hg.patch_px) pp = 0;
            pq[j] = patch_px(pp);
        }
    };

    if (steps <= 0) return;
    // prologue: the first (tile, cc) patch whole, the first weights
    Px fc;                              // first pixel of tile tm
    {
        const int m0 = tm0 * kBM;
        fc.n = m0 / OHW;
        fc.oh = (m0 - fc.n * OHW) / g.OW;
        fc.ow = m0 - fc.n * OHW - fc.oh * g.OW;
    }
    patch_begin(fc, 0, 0);
#pragma unroll
    for (int k = 0; k < 8; ++k) patch_piece(k);
    issue_w(0, 0);
    tile_setup(fc);
    int tm = tm0, r = 0, pbuf = 0;     // r = step within the tile
    int wait_kind = 0;                 // 0: vmcnt(0), 1: a patch piece after the weights, 2: stores
    for (int s = 0; s < steps; ++s) {
        constexpr int D = MCGMIL_HALO_DIAG;
        const bool live = s < 2;            // the diagnostics keep the first steps intact
        if (!(D & 1) || live) {
            if (wait_kind == 1) wait_vmcnt<1>();
            else if (wait_kind == 2) wait_vmcnt<FI * FJ>();
            else wait_vmcnt<0>();
        }
        const int cc = r / 9, tap = r - cc * 9;
        if (XF && tap == 0 && (!(D & 16) || live)) {       // this step opens a patch: the rest of this lane's slots
            if (s == 0) {
#pragma unroll
                for (int k = 0; k < 8; ++k) xform(k);
            } else {
                xform(7);
            }
            wait_lds_writes();
        }
        if (!(D & 2) || live) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        wait_kind = 0;
        if (s + 1 < steps && (!(D & 32) || live)) issue_w(r + 1 == SPT ? 0 : r + 1, (s + 1) & 1);
        // the next (tile, cc) patch: begun at tap 0, one piece per tap 0..7
        const bool more_patch = (r + 9 < SPT) || (tm + 1 < tm1);
        if (more_patch && tap < 8) {
            if (tap == 0) {
                if (cc + 1 < CC) patch_begin(fc, cc + 1, pbuf ^ 1);
                else patch_begin(advance(fc), 0, pbuf ^ 1);
            }
            // vmcnt(1) at the next step leaves only this piece in flight; without a piece the
            // weights just issued must land: vmcnt(0)
            if ((!(D & 32) || live) && patch_piece(tap)) wait_kind = 1;
        }
        // compute step s: A from the patch at the tap offset, B from the weight stage
        {
            const unsigned char* A = patch0 + pbuf * PATCH;
            const unsigned char* B = wst0 + (s & 1) * WSTAGE;
            const int toff = (tap / 3) * WP + (tap % 3);
            uint32_t ad[FJ];
#pragma unroll
            for (int j = 0; j < FJ; ++j) ad[j] = tap_addr(pq[j], toff, (uint32_t)(lane >> 4) << 4);
            // K half 1's fragments are read before half 0's MFMAs (the scheduler barriers keep
            // that order)
            bf16x8 wf[2][FI], xf[2][FJ];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int kq = ks * 4 + (lane >> 4);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < FI; ++i) {
                    if constexpr ((D & 8) != 0) asm volatile("" : "=v"(wf[ks][i]));
                    else wf[ks][i] = *reinterpret_cast<const bf16x8*>(B + swz(wn * WN + i * 16 + (lane & 15), kq));
                }
#pragma unroll
                for (int j = 0; j < FJ; ++j) {
                    if constexpr ((D & 8) != 0) asm volatile("" : "=v"(xf[ks][j]));
                    else xf[ks][j] = *reinterpret_cast<const bf16x8*>(A + (ks ? ad[j] ^ 64u : ad[j]));
                }
                if (ks == 0) continue;
                if constexpr ((D & 4) != 0) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
#pragma unroll
                        for (int i = 0; i < FI; ++i) asm volatile("" ::"v"(wf[h][i]));
#pragma unroll
                        for (int j = 0; j < FJ; ++j) asm volatile("" ::"v"(xf[h][j]));
                    }
                    continue;
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (h == 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int i = 0; i < FI; ++i)
#pragma unroll
                        for (int j = 0; j < FJ; ++j)
                            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[h][i], xf[h][j], acc[j][i], 0, 0, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // XF: piece tap - 2 of the patch being loaded has landed (the wait above retired it)
        if (XF && more_patch && tap >= 2 && (!(D & 16) || live)) xform(tap - 2);
        if (tap == 8) pbuf ^= 1;                        // next cc (or tile) uses the other patch
        if (++r == SPT) {
            const bool full = (tm + 1) * kBM <= g.M, first = tm == tm0;
#pragma unroll
            for (int j = 0; j < FJ; ++j) {
                const int m = tm * kBM + wm * WM + j * 16 + frag_px(lane & 15);
                __bf16* dst = g.y + (size_t)(m < g.M ? m : 0) * g.Cout + tn * BN + wn * WN + 4 * (lane >> 4);
                if (full) store_fragment<FI, STATS, false>(acc[j], dst, true, first && j == 0, st);
                else store_fragment<FI, STATS, true>(acc[j], dst, m < g.M, first && j == 0, st);
#pragma unroll
                for (int i = 0; i < FI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            wait_kind = 2;
            r = 0;
            ++tm;
            if (tm < tm1) {
                fc = advance(fc);
                tile_setup(fc);
            }
        }
    }
    if (STATS) write_stats<4 * FI, WGM, BN>(st, wn * WN, wm, reinterpret_cast<float*>(smem), g.stats, gm,
                                             g.Cout, tn * BN);
}

// ---- conv1x1_kernel: 1x1 / stride s / no padding, Cin = 32 KS (the plan uses it for 64 -> 128), a
// streaming kernel without LDS stages (conv_dma_kernel moved these at 2.3-3.6 TB/s: one K step per
// tile leaves its stage ring and 8-byte epilogue stores exposed). A wave owns 32 output channels --
// its weights stay in registers -- and walks 16-pixel fragments of one pixel stream: a fragment's
// Cin input channels are loaded by buffer loads straight into MFMA B fragments (16 B per lane; the
// next fragment's are in flight during this one's MFMAs), and the outputs leave as one 16-byte
// store per lane. For that the weight rows are permuted: row r of fragment i is channel
// 32 cb + 8 (r >> 2) + 4 i + (r & 3), so a lane's two accumulators hold 8 consecutive channels.
// The CB = Cout / 32 waves of a pixel stream are neighbours in the grid and share its input in L2.
// Statistics (STATS): one (n, mean, M2) row per pixel stream for each wave's 32 channels.
constexpr int k1x1Threads = 256;
template <int KS, bool STATS>
__global__ __launch_bounds__(k1x1Threads) void conv1x1_kernel(const ConvGeom g) {
    constexpr int FI = 2;
    const int lane = threadIdx.x & 63, q = lane >> 4, c16 = lane & 15;
    const int wid = (int)blockIdx.x * (k1x1Threads / 64) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int CB = g.Cout / 32, PS = (int)gridDim.x * (k1x1Threads / 64) / CB;
    const int cb = wid % CB, ps = wid / CB;
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(g.x, g.x_bytes);

    bf16x8 wf[KS][FI];
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int i = 0; i < FI; ++i) {
            const int ch = 32 * cb + 8 * (c16 >> 2) + 4 * i + (c16 & 3);
            wf[s][i] = *reinterpret_cast<const bf16x8*>(g.w + (size_t)ch * (KS * 32) + s * 32 + 8 * q);
        }
    LaneStats<4 * FI> st;
    if (STATS) st.init();

    const int OHW = g.OH * g.OW, nfrag = (g.M + 15) >> 4;
    auto load = [&](int f, bf16x8 (&xf)[KS]) {
        // the fragment's first pixel in scalar math (f is wave-uniform), then the lane's column
        const int m0 = 16 * f, n0 = m0 / OHW, r0 = m0 - n0 * OHW, oh0 = r0 / g.OW;
        int n = n0, oh = oh0, ow = r0 - oh0 * g.OW + c16;
        if (m0 + c16 >= g.M) {          // past the last pixel: load the last one (not stored)
            n = g.N - 1;
            oh = g.OH - 1;
            ow = g.OW - 1;
        }
        while (ow >= g.OW) {
            ow -= g.OW;
            ++oh;
        }
        while (oh >= g.OH) {
            oh -= g.OH;
            ++n;
        }
        const uint32_t off = ((uint32_t)((n * g.H + oh * g.stride) * g.W + ow * g.stride) * (uint32_t)(KS * 32) +
                              8u * (uint32_t)q) * 2u;
#pragma unroll
        for (int s = 0; s < KS; ++s)
            xf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off + 64u * s, 0, 0));
    };
    bf16x8 xa[KS], xb[KS];
    int f = ps;
    if (f < nfrag) load(f, xa);
    bool first = true;
    while (f < nfrag) {
        const int fn = f + PS;
        if (fn < nfrag) load(fn, xb);
        f32x4 acc[FI];
#pragma unroll
        for (int i = 0; i < FI; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int i = 0; i < FI; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s][i], xa[s], acc[i], 0, 0, 0);
        const int m = 16 * f + c16;
        const bool valid = m < g.M;
        typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
        uint32_t pk[4];
#pragma unroll
        for (int h = 0; h < 4; ++h)
            pk[h] = __builtin_bit_cast(uint32_t, bf16x2{(__bf16)acc[h >> 1][2 * (h & 1)], (__bf16)acc[h >> 1][2 * (h & 1) + 1]});
        if (valid)
            __builtin_nontemporal_store(u32x4{pk[0], pk[1], pk[2], pk[3]},
                                        reinterpret_cast<u32x4*>(g.y + (size_t)m * g.Cout + 32 * cb + 8 * q));
        if (STATS) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t u = pk[c >> 1];
                const float x = __uint_as_float((c & 1) ? (u & 0xFFFF0000u) : (u << 16));
                if (first) st.set_x0(c, x);
                float d = x - st.x0(c);
                d = valid ? d : 0.f;
                st.S[c] += d;
                st.SS[c] = fmaf(d, d, st.SS[c]);
            }
            st.n += valid ? 1.f : 0.f;
        }
        first = false;
#pragma unroll
        for (int s = 0; s < KS; ++s) xa[s] = xb[s];
        f = fn;
    }
    if (STATS) {
        // the lane's channel c (0..7) is 32 cb + 8 q + c: merge the 16 pixel lanes, lanes c16 = 0 write
        float n = st.n, mean[8], M2[8];
        const float rn = n > 0.f ? 1.f / n : 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            mean[c] = st.x0(c) + st.S[c] * rn;
            M2[c] = fmaxf(st.SS[c] - st.S[c] * st.S[c] * rn, 0.f);
            if (!(n > 0.f)) mean[c] = M2[c] = 0.f;
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            float mb[8], M2b[8];
            const float nb = __shfl_xor(n, o, 64);
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                mb[c] = __shfl_xor(mean[c], o, 64);
                M2b[c] = __shfl_xor(M2[c], o, 64);
            }
            chan_merge<8>(n, mean, M2, nb, mb, M2b);
        }
        if (c16 == 0) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const int ch = 32 * cb + 8 * q + c;
                g.stats[((size_t)ps * 3 + 0) * g.Cout + ch] = n;
                g.stats[((size_t)ps * 3 + 1) * g.Cout + ch] = mean[c];
                g.stats[((size_t)ps * 3 + 2) * g.Cout + ch] = M2[c];
            }
        }
    }
}

// ---- launch plan: which kernel, its grid and the statistics rows (Gm x 3 x Cout floats)
struct Plan {
    int kind = 0;          // 1: halo 64 -> 64, 2: dma 256 x 128, 3: dma 256 x 64, 4: halo, streamed
                           // weights, 5: dma 512 x 128, 6: dma 256 x 256, 7: 1x1 streaming,
                           // 8: row-ring 64 -> 64
    int grid = 0;
    int parts = 0;         // statistics rows
    size_t lds = 0;
    HaloGeom hg;
    size_t part_bytes = 0; // K split (kind 6): the fp32 range sums (mcgmil_conv_args.workspace)
};

ConvGeom geom_of(const mcgmil_conv_args* a) {
    ConvGeom g{};
    g.x = static_cast<const __bf16*>(a->x);
    g.w = static_cast<const __bf16*>(a->w);
    g.y = static_cast<__bf16*>(a->y);
    g.stats = a->stats;
    g.in_ab = a->in_ab;
    g.in_lo = a->in_relu ? 0.f : -INFINITY;
    g.N = a->batch; g.H = a->height; g.W = a->width; g.Cin = a->in_channels;
    g.Cout = a->out_channels; g.KH = a->kernel_h; g.KW = a->kernel_w;
    g.stride = a->stride; g.pad = a->pad;
    g.OH = (g.H + 2 * g.pad - g.KH) / g.stride + 1;
    g.OW = (g.W + 2 * g.pad - g.KW) / g.stride + 1;
    g.M = g.N * g.OH * g.OW;
    g.cin_tiles = g.Cin / 64;
    g.KT = g.KH * g.KW * g.cin_tiles;
    g.tiles_m = (g.M + kBM - 1) / kBM;
    g.x_bytes = (uint32_t)((long long)g.N * g.H * g.W * g.Cin * 2);
    g.w_bytes = (uint32_t)((long long)g.Cout * g.KH * g.KW * g.Cin * 2);
    return g;
}

// The tile policy: args->flags (mcgmil_conv_flags), or MCGMIL_CONV_TILE=nohalo|small|big512 in the
// environment, which overrides the flags (A/B timing of an unmodified caller; read once per process)
int tile_policy(int flags) {
    static const int env = [] {
        const char* e = getenv("MCGMIL_CONV_TILE");
        if (e && !strcmp(e, "nohalo")) return (int)MCGMIL_CONV_TILE_NOHALO;
        if (e && !strcmp(e, "small")) return (int)MCGMIL_CONV_TILE_SMALL;
        if (e && !strcmp(e, "big512")) return (int)MCGMIL_CONV_TILE_BIG512;
        return -1;
    }();
    return env >= 0 ? env : flags;
}

Plan make_plan(ConvGeom& g, int flags, bool split_ok = false) {
    Plan p;
    const int cus = cu_count();
    const int policy = tile_policy(flags);
    const bool halo_ok = policy != MCGMIL_CONV_TILE_NOHALO;
    if (halo_ok && g.Cin == 64 && g.Cout == 64 && g.KH == 3 && g.KW == 3 && g.stride == 1 && g.pad == 1 &&
        MCGMIL_C64_RING && g.W + 2 <= kRingCols) {
        // the row ring holds the padded rows of two consecutive tiles: output rows 2 kBM pixels can
        // span, + 2 halo rows, + 2 pad rows per image boundary crossed
        const int rows = (2 * kBM - 1 + g.OW - 1) / g.OW + 1;
        const int imgs = (2 * kBM - 1 + g.OH * g.OW - 1) / (g.OH * g.OW) + 1;
        if (rows + 2 + 2 * (imgs - 1) <= kRingRows) {
            HaloGeom hg{};
            hg.WP = g.W + 2;
            hg.tiles = g.tiles_m;
            hg.q256 = kBM / g.OW;
            hg.r256 = kBM % g.OW;
            hg.q255 = (kBM - 1) / g.OW;
            hg.r255 = (kBM - 1) % g.OW;
            g.tiles_n = 1;
            g.Gm = hg.tiles < cus ? hg.tiles : cus;
            hg.g = g;
            p.kind = 8;
            p.grid = g.Gm;
            p.parts = g.Gm;
            p.lds = kRingBytes;
            p.hg = hg;
            return p;
        }
    }
    if (halo_ok && g.Cin == 64 && g.Cout == 64 && g.KH == 3 && g.KW == 3 && g.stride == 1 && g.pad == 1) {
        HaloGeom hg;
        hg.WP = g.W + 2;
        // output rows a tile can span, + 2 halo rows, + 2 pad rows per image boundary crossed
        const int rows = (kBM - 1 + g.OW - 1) / g.OW + 1;
        const int imgs = (kBM - 1 + g.OH * g.OW - 1) / (g.OH * g.OW) + 1;
        hg.NR = rows + 2 + 2 * (imgs - 1);
        hg.patch_px = (hg.NR * hg.WP + 7) / 8 * 8;
        const size_t lds = (size_t)2 * hg.patch_px * kRowBytes + (g.in_ab ? 512 : 0);
        if (lds <= 160 * 1024) {
            hg.tiles = g.tiles_m;
            g.tiles_n = 1;
            g.Gm = hg.tiles < cus ? hg.tiles : cus;
            hg.g = g;
            p.kind = 1;
            p.grid = g.Gm;
            p.parts = g.Gm;
            p.lds = lds;
            p.hg = hg;
            return p;
        }
    }
    // 1x1 / stride 2 from 64 channels (layer 2's downsample): the streaming kernel, unless the policy
    // pins the dma tiles. Measured at config 5 (scripts/probe_conv.py, k = 916): 64 -> 128 82.6 ->
    // 59.3 us; but 128 -> 256 40.2 -> 54.5 and 256 -> 512 33.1 -> 56.7 (8 / 16 waves per pixel stream
    // re-read its input from L2, and a stream holds only 5-11 fragments), so those stay on the dma tiles
    if (policy == MCGMIL_CONV_TILE_AUTO && g.KH == 1 && g.KW == 1 && g.pad == 0 && g.stride == 2 && g.Cin == 64 &&
        !g.in_ab) {
        const int CB = g.Cout / 32, waves = 32 * cus;    // 8 waves per SIMD
        int ps = waves / CB;
        const int nfrag = (g.M + 15) / 16;
        if (ps > nfrag) ps = nfrag;
        if (ps < 1) ps = 1;
        // 4 waves per workgroup, the CB waves of a pixel stream adjacent: CB * ps waves in all
        while ((CB * ps) % 4) ++ps;
        p.kind = 7;
        p.grid = CB * ps / 4;
        p.parts = ps;
        g.Gm = ps;
        return p;
    }
    const int BN = g.Cout % 128 == 0 ? 128 : 64;
    g.tiles_n = g.Cout / BN;
    int gm = cus / g.tiles_n;
    if (gm < 1) gm = 1;
    if (gm > g.tiles_m) gm = g.tiles_m;
    // measured (scripts/probe_conv.py, one process): +8% at 28 x 28 (layer 2), neutral at 14 x 14,
    // -2% at 7 x 7, where a tile spans many images and the patch is mostly halo
    if (halo_ok && g.Cin >= 128 && BN == 128 && g.KH == 3 && g.KW == 3 && g.stride == 1 && g.pad == 1 &&
        g.OW >= 20) {
        HaloGeom hg;
        hg.WP = g.W + 2;
        const int rows = (kBM - 1 + g.OW - 1) / g.OW + 1;
        const int imgs = (kBM - 1 + g.OH * g.OW - 1) / (g.OH * g.OW) + 1;
        hg.NR = rows + 2 + 2 * (imgs - 1);
        hg.patch_px = hg.NR * hg.WP;
        if (hg.patch_px <= kPatchPx && (!g.in_ab || g.Cin <= 1024)) {
            hg.tiles = g.tiles_m;
            hg.q256 = kBM / g.OW;
            hg.r256 = kBM % g.OW;
            hg.q255 = (kBM - 1) / g.OW;
            hg.r255 = (kBM - 1) % g.OW;
            g.Gm = gm;
            hg.g = g;
            p.kind = 4;
            p.grid = g.tiles_n * gm;
            p.parts = gm;
            p.lds = (size_t)2 * kPatchPx * kRowBytes + (size_t)2 * 128 * kRowBytes +
                    (g.in_ab ? (size_t)8 * g.Cin : 0);
            p.hg = hg;
            return p;
        }
    }
    if (gm < 1) gm = 1;
    if (gm > g.tiles_m) gm = g.tiles_m;
    // 128 x 64 wave tiles (25% less LDS fragment traffic per MFMA than 64 x 64), two LDS stages:
    // 256 x 256 when Cout % 256 == 0 (layer 3: +30-34%, layer 4: +7%, measured in one process);
    // 512 x 128 measured slower on the 128-channel layer (kept for MCGMIL_CONV_TILE=big512);
    // MCGMIL_CONV_TILE_SMALL keeps 256 x 128
    const bool small = policy == MCGMIL_CONV_TILE_SMALL;
    const bool big512 = policy == MCGMIL_CONV_TILE_BIG512;
    if (!small && BN == 128 && (g.Cout % 256 == 0 || big512)) {
        const int bm = g.Cout % 256 == 0 ? 256 : 512, bn = g.Cout % 256 == 0 ? 256 : 128;
        g.tiles_m = (g.M + bm - 1) / bm;
        g.tiles_n = g.Cout / bn;
        int gb = cus / g.tiles_n;
        if (gb < 1) gb = 1;
        if (gb > g.tiles_m) gb = g.tiles_m;
        g.Gm = gb;
        p.kind = bn == 256 ? 6 : 5;
        p.grid = g.tiles_n * gb;
        // tiles_m = F gb + R, 0 < R: the last round of tiles runs on R of gb workgroup rows. With
        // a workspace those R tiles are cut into P = gb / R K ranges (at most 4, each >= 4 K steps),
        // so every row runs F tiles + at most 1 / P of one: layer 4 of config 5 (289 tiles per 128
        // rows, 3 tile times -> 2.33)
        if (split_ok && p.kind == 6) {
            const int F = g.tiles_m / gb, R = g.tiles_m - F * gb;
            int P = R > 0 ? gb / R : 0;
            if (P > 4) P = 4;
            if (F >= 1 && P >= 2 && g.KT >= 4 * P) {
                g.split_p = P;
                g.full_tiles = F;
                p.part_bytes = (size_t)R * g.tiles_n * P * bm * bn * sizeof(float);
            }
        }
        // no statistics from these shapes: with them the kernel spills (256 VGPRs), and the separate
        // statistics pass of a layer-3/4 activation (10-20 us) costs less than that
        p.parts = 0;
        p.lds = (size_t)2 * (bm + bn) * kRowBytes;
        return p;
    }
    g.Gm = gm;
    p.kind = BN == 128 ? 2 : 3;
    p.grid = g.tiles_n * gm;
    p.parts = gm;
    p.lds = (size_t)kStages * (kBM + BN) * kRowBytes;
    return p;
}

// Launch k after raising its dynamic-LDS limit (once per kernel and device; errors returned).
template <typename K, typename A>
int launch_lds(K k, dim3 grid, dim3 block, size_t lds, hipStream_t s, const A& arg) {
    if (int rc = mcgmil_detail::raise_lds_limit(reinterpret_cast<const void*>(k), "convolution kernel LDS limit"))
        return rc;
    hipLaunchKernelGGL(k, grid, block, lds, s, arg);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "convolution kernel launch");
}

int launch(const ConvGeom& g, const Plan& p, hipStream_t s) {
    const bool stats = g.stats != nullptr, xf = g.in_ab != nullptr;
    const dim3 grid((unsigned)p.grid), block(kThreads);
    if (p.kind == 1 || p.kind == 4) {
        HaloGeom hg = p.hg;
        hg.g = g;
        auto k = p.kind == 1 ? (stats ? (xf ? conv3x3c64_kernel<true, true> : conv3x3c64_kernel<true, false>)
                                      : (xf ? conv3x3c64_kernel<false, true> : conv3x3c64_kernel<false, false>))
                             : (stats ? (xf ? conv3x3_halo_kernel<true, true> : conv3x3_halo_kernel<true, false>)
                                      : (xf ? conv3x3_halo_kernel<false, true> : conv3x3_halo_kernel<false, false>));
        return launch_lds(k, grid, block, p.lds, s, hg);
    }
    if (p.kind == 8) {
        HaloGeom hg = p.hg;
        hg.g = g;
        constexpr int NW = MCGMIL_RING_WAVES;
        auto k = stats ? (xf ? conv3x3c64_ring_kernel<true, true, NW> : conv3x3c64_ring_kernel<true, false, NW>)
                       : (xf ? conv3x3c64_ring_kernel<false, true, NW> : conv3x3c64_ring_kernel<false, false, NW>);
        return launch_lds(k, grid, dim3(NW * 64), p.lds, s, hg);
    }
    if (p.kind == 7) {
        const dim3 b1(k1x1Threads);
        auto k = stats ? conv1x1_kernel<2, true> : conv1x1_kernel<2, false>;     // Cin = 64
        hipLaunchKernelGGL(k, grid, b1, 0, s, g);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "conv1x1_kernel launch");
    }
    if (p.kind == 2)
        return stats ? launch_lds(conv_dma_kernel<256, 128, 4, 3, true>, grid, block, p.lds, s, g)
                     : launch_lds(conv_dma_kernel<256, 128, 4, 3, false>, grid, block, p.lds, s, g);
    if (p.kind == 5) return launch_lds(conv_dma_kernel<512, 128, 4, 2, false>, grid, block, p.lds, s, g);
    if (p.kind == 6) {
        if (int rc = launch_lds(conv_dma_kernel<256, 256, 2, 2, false>, grid, block, p.lds, s, g)) return rc;
        if (g.split_p == 0) return MCGMIL_OK;
        const long long n = (long long)(g.tiles_m - g.full_tiles * g.Gm) * g.tiles_n * 256 * (256 / 8);
        hipLaunchKernelGGL((conv_split_fixup_kernel<256, 256>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "conv_split_fixup_kernel launch");
    }
    return stats ? launch_lds(conv_dma_kernel<256, 64, 4, 3, true>, grid, block, p.lds, s, g)
                 : launch_lds(conv_dma_kernel<256, 64, 4, 3, false>, grid, block, p.lds, s, g);
}

// weights [Cout, Cin, KH, KW] (fp32 or bf16) -> [Cout, KH, KW, Cin] bf16
template <typename T>
__global__ void pack_conv_weights_kernel(const T* w, int Cout, int Cin, int KH, int KW, __bf16* out) {
    const long long total = (long long)Cout * Cin * KH * KW;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int ci = (int)(i % Cin);
        long long r = i / Cin;
        const int kw = (int)(r % KW);
        r /= KW;
        const int kh = (int)(r % KH);
        const int co = (int)(r / KH);
        out[i] = (__bf16)(float)w[(((long long)co * Cin + ci) * KH + kh) * KW + kw];
    }
}

int validate(const mcgmil_conv_args* a) {
    if (!a) return fail(MCGMIL_E_INVALID, "args is NULL");
    if (a->batch < 1 || a->height < 1 || a->width < 1)
        return fail(MCGMIL_E_INVALID, "batch, height and width must be >= 1");
    if (a->in_channels < 64 || a->in_channels % 64 != 0 || a->out_channels < 64 || a->out_channels % 64 != 0)
        return fail(MCGMIL_E_UNSUPPORTED, "in_channels and out_channels must be positive multiples of 64");
    if (a->kernel_h < 1 || a->kernel_w < 1 || a->kernel_h > 7 || a->kernel_w > 7)
        return fail(MCGMIL_E_UNSUPPORTED, "kernel size must be in 1..7");
    if (a->stride < 1 || a->pad < 0) return fail(MCGMIL_E_INVALID, "stride must be >= 1 and pad >= 0");
    if (a->in_relu != 0 && a->in_relu != 1) return fail(MCGMIL_E_INVALID, "in_relu must be 0 or 1");
    if (a->flags < MCGMIL_CONV_TILE_AUTO || a->flags > MCGMIL_CONV_TILE_BIG512 || a->reserved != 0)
        return fail(MCGMIL_E_INVALID, "flags must be an mcgmil_conv_flags value and reserved 0");
    if (a->height > 16383 || a->width > 16383 || a->pad > 64)
        return fail(MCGMIL_E_UNSUPPORTED, "height and width must be <= 16383 and pad <= 64");
    const long long oh = ((long long)a->height + 2 * a->pad - a->kernel_h) / a->stride + 1;
    const long long ow = ((long long)a->width + 2 * a->pad - a->kernel_w) / a->stride + 1;
    if (oh < 1 || ow < 1) return fail(MCGMIL_E_INVALID, "the kernel does not fit the padded input");
    const long long x_bytes = (long long)a->batch * a->height * a->width * a->in_channels * 2;
    if (x_bytes >= (1ll << 31) || (long long)a->batch * oh * ow >= (1ll << 31) - kBM)
        return fail(MCGMIL_E_UNSUPPORTED, "input larger than 2 GiB or too many output pixels");
    if ((long long)a->out_channels * a->kernel_h * a->kernel_w * a->in_channels * 2 >= (1ll << 31))
        return fail(MCGMIL_E_UNSUPPORTED, "weights larger than 2 GiB");
    return MCGMIL_OK;
}

}  // namespace

extern "C" {

size_t mcgmil_conv_args_size(void) { return sizeof(mcgmil_conv_args); }

int mcgmil_pack_conv_weights(const mcgmil_conv_args* a, const void* weight, int32_t weight_dtype,
                             void* packed, void* stream) {
    int rc = validate(a);
    if (rc) return rc;
    if (!weight || !packed) return fail(MCGMIL_E_INVALID, "NULL weight or packed pointer");
    const long long total = (long long)a->out_channels * a->in_channels * a->kernel_h * a->kernel_w;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (weight_dtype == MCGMIL_F32)
        hipLaunchKernelGGL(pack_conv_weights_kernel<float>, dim3(blocks), dim3(256), 0, s,
                           static_cast<const float*>(weight), a->out_channels, a->in_channels,
                           a->kernel_h, a->kernel_w, static_cast<__bf16*>(packed));
    else if (weight_dtype == MCGMIL_BF16)
        hipLaunchKernelGGL(pack_conv_weights_kernel<__bf16>, dim3(blocks), dim3(256), 0, s,
                           static_cast<const __bf16*>(weight), a->out_channels, a->in_channels,
                           a->kernel_h, a->kernel_w, static_cast<__bf16*>(packed));
    else
        return fail(MCGMIL_E_INVALID, "weight_dtype must be MCGMIL_F32 or MCGMIL_BF16");
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "pack_conv_weights_kernel launch");
}

int mcgmil_conv_input_bn(const mcgmil_conv_args* a, int32_t* supported) {
    int rc = validate(a);
    if (rc) return rc;
    if (!supported) return fail(MCGMIL_E_INVALID, "supported is NULL");
    mcgmil_conv_args b = *a;
    b.in_ab = reinterpret_cast<const float*>(16);   // a plan with the input BatchNorm
    ConvGeom g = geom_of(&b);
    const int kind = make_plan(g, a->flags).kind;
    *supported = kind == 1 || kind == 4 || kind == 8;
    return MCGMIL_OK;
}

int mcgmil_conv_stats_parts(const mcgmil_conv_args* a, int32_t* parts) {
    int rc = validate(a);
    if (rc) return rc;
    if (!parts) return fail(MCGMIL_E_INVALID, "parts is NULL");
    ConvGeom g = geom_of(a);
    *parts = make_plan(g, a->flags).parts;
    return MCGMIL_OK;
}

int mcgmil_conv_workspace_size(const mcgmil_conv_args* a, size_t* bytes) {
    int rc = validate(a);
    if (rc) return rc;
    if (!bytes) return fail(MCGMIL_E_INVALID, "bytes is NULL");
    ConvGeom g = geom_of(a);
    *bytes = make_plan(g, a->flags, true).part_bytes;
    return MCGMIL_OK;
}

int mcgmil_conv2d(const mcgmil_conv_args* a, void* stream) {
    int rc = validate(a);
    if (rc) return rc;
    if (!a->x || !a->w || !a->y) return fail(MCGMIL_E_INVALID, "NULL x, w or y");
    if (((uintptr_t)a->x | (uintptr_t)a->w | (uintptr_t)a->y) & 15u)
        return fail(MCGMIL_E_ALIGN, "x, w and y must be 16-byte aligned");
    if ((uintptr_t)a->stats & 3u) return fail(MCGMIL_E_ALIGN, "stats must be 4-byte aligned");
    if ((uintptr_t)a->in_ab & 3u) return fail(MCGMIL_E_ALIGN, "in_ab must be 4-byte aligned");
    if ((uintptr_t)a->workspace & 255u) return fail(MCGMIL_E_ALIGN, "workspace must be 256-byte aligned");
    ConvGeom g = geom_of(a);
    Plan p = make_plan(g, a->flags, a->workspace != nullptr);
    if (p.part_bytes > 0 && a->workspace_bytes < p.part_bytes) {
        g = geom_of(a);                          // too small for the K split: the whole-tile plan
        p = make_plan(g, a->flags);
    }
    g.part = static_cast<float*>(a->workspace);
    if (a->in_ab && p.kind != 1 && p.kind != 4 && p.kind != 8)
        return fail(MCGMIL_E_UNSUPPORTED, "in_ab: this layer's kernel has no input BatchNorm "
                                          "(see mcgmil_conv_input_bn)");
    return launch(g, p, reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
