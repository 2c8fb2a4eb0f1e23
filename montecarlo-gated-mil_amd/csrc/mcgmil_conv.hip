// Implicit-GEMM convolution of the channels-last bf16 backbone (include/mcgmil_features.h,
// mcgmil_conv2d): the 3x3 / 1x1 convolutions of the torchvision BasicBlock / Bottleneck the
// reference builds at model.py:166-177, run in infer.py:191 on every instance of a bag.
//
// GEMM view (one output pixel per row, one output channel per column):
//   C[m, co] = sum_k A[m, k] * B[k, co],  m = (n, oh, ow),  k = (kh, kw, ci)
//   A[m, k]  = x[n, oh*s - pad + kh, ow*s - pad + kw, ci]   (0 outside the image)
//   B[k, co] = w[co, kh, kw, ci]                            (weights packed channels-last)
// One 256-thread workgroup computes a 128-pixel x BN-channel tile (BN = 128, or 64 when the
// layer has 64 output channels) over K tiles of 64: each K tile is one (kh, kw) position and 64
// consecutive input channels, so every A row of a K tile is ONE contiguous 128-byte run of the
// NHWC input (a 16-byte buffer load per lane, zero-filled by the descriptor's range check where
// the window leaves the image). Tiles are staged through LDS (double buffered, XOR-swizzled
// 128-byte rows, register staging, one barrier per K tile); 4 waves in a 2 x 2 grid each own a
// 64-pixel x BN/2-channel block of v_mfma_f32_16x16x32_bf16 accumulators (weights as the A
// operand, so a lane ends with 4 consecutive channels of one pixel: one 8-byte store each).
// fp32 accumulation, one rounding to bf16 -- the same arithmetic as MIOpen's bf16 convolution
// under torch.autocast, up to the summation order.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/mcgmil_features.h"
#include "mcgmil_device.h"
#include "mcgmil_error.h"

namespace {

using namespace mcgmil;
using mcgmil_detail::fail;
using mcgmil_detail::hip_fail;

constexpr int kConvThreads = 256;
constexpr int kBM = 128;            // output pixels per tile
constexpr int kBK = 64;             // K elements per stage (one 128-byte row per pixel/channel)
constexpr int kRowBytes = kBK * 2;

struct ConvGeom {
    const __bf16* x;
    const __bf16* w;
    __bf16* y;
    int N, H, W, Cin, OH, OW, Cout, KH, KW, stride, pad;
    int M;               // N * OH * OW (< 2^31, host-checked)
    int KT;              // K tiles: KH * KW * Cin / 64
    int cin_tiles;       // Cin / 64
    int tiles_n;         // Cout / BN
    int tiles;           // tiles_m * tiles_n
    uint32_t x_bytes;    // buffer range of x (< 2^31, host-checked)
    uint32_t w_bytes;
};

// byte offset of 16-byte chunk c of row r in a swizzled [rows][128 B] stage: rows 2j and 2j+1
// share a bank half, so chunk c sits at slot c ^ ((r >> 1) & 7); the 16 lanes of an MFMA
// fragment read (rows r0..r0+15, one chunk) then hit 16 distinct 4-bank groups
__device__ __forceinline__ uint32_t swz(int r, int c) {
    return (uint32_t)r * kRowBytes + (uint32_t)((c ^ ((r >> 1) & 7)) << 4);
}

// XCD-aware tile order (guide T1, bijective form): consecutive logical tiles -- the BN-column
// tiles of one pixel tile, which read the same input rows -- land on the same XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

template <int BN>
__global__ __launch_bounds__(kConvThreads, 2) void conv_kernel(const ConvGeom g) {
    constexpr int STAGE = (kBM + BN) * kRowBytes;     // A rows then B rows
    constexpr int NB = BN / 32;                       // B chunks per thread per stage
    constexpr int WN = BN / 2;                        // channels per wave
    constexpr int FI = WN / 16;                       // channel fragments per wave
    constexpr int FJ = 4;                             // pixel fragments per wave (64 pixels)
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int t = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    if (t >= g.tiles) return;
    const int tm = t / g.tiles_n, tn = t - tm * g.tiles_n;
    const int m0 = tm * kBM, n0 = tn * BN;

    // ---- staging assignment: chunk c of rows (tid >> 3) + 32 i
    const int c = tid & 7, r0 = tid >> 3;
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(g.x, g.x_bytes);
    const __amdgpu_buffer_rsrc_t wr = make_rsrc(g.w, g.w_bytes);
    int pix_base[4], ih0[4], iw0[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + r0 + 32 * i;
        const int mm = m < g.M ? m : 0;
        const int n = mm / (g.OH * g.OW);
        const int rem = mm - n * g.OH * g.OW;
        const int oh = rem / g.OW, ow = rem - (rem / g.OW) * g.OW;
        pix_base[i] = n * g.H * g.W;
        // rows past M get a window that never fits, so they load zeros
        ih0[i] = m < g.M ? oh * g.stride - g.pad : -(1 << 28);
        iw0[i] = ow * g.stride - g.pad;
    }
    const uint32_t K = (uint32_t)(g.KH * g.KW * g.Cin);
    uint32_t wrow[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) wrow[i] = ((uint32_t)(n0 + r0 + 32 * i) * K + (uint32_t)c * 8u) * 2u;

    uint4 ra[4], rb[NB];
    auto load = [&](int kt) {
        const int khw = kt / g.cin_tiles, cc = kt - khw * g.cin_tiles;
        const int kh = khw / g.KW, kw = khw - kh * g.KW;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ih = ih0[i] + kh, iw = iw0[i] + kw;
            const bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
            const uint32_t off = ((uint32_t)(pix_base[i] + ih * g.W + iw) * (uint32_t)g.Cin +
                                  (uint32_t)(cc * 64 + c * 8)) * 2u;
            ra[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  xr, ok ? off : 0x80000000u, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < NB; ++i)
            rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  wr, wrow[i], (uint32_t)kt * (kBK * 2u), 0));
    };
    auto store = [&](int buf) {
        unsigned char* A = smem + buf * STAGE;
        unsigned char* B = A + kBM * kRowBytes;
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4*>(A + swz(r0 + 32 * i, c)) = ra[i];
#pragma unroll
        for (int i = 0; i < NB; ++i) *reinterpret_cast<uint4*>(B + swz(r0 + 32 * i, c)) = rb[i];
    };

    // ---- compute assignment: wave (wm, wn) owns pixels wm*64.. and channels wn*WN..
    const int wm = wave >> 1, wn = wave & 1;
    f32x4 acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int buf) {
        const unsigned char* A = smem + buf * STAGE;
        const unsigned char* B = A + kBM * kRowBytes;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int kq = ks * 4 + (lane >> 4);
            bf16x8 wf[FI], xf[FJ];
#pragma unroll
            for (int i = 0; i < FI; ++i)
                wf[i] = *reinterpret_cast<const bf16x8*>(B + swz(wn * WN + i * 16 + (lane & 15), kq));
#pragma unroll
            for (int j = 0; j < FJ; ++j)
                xf[j] = *reinterpret_cast<const bf16x8*>(A + swz(wm * 64 + j * 16 + (lane & 15), kq));
#pragma unroll
            for (int i = 0; i < FI; ++i)
#pragma unroll
                for (int j = 0; j < FJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
        }
    };

    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < g.KT; ++kt) {
        const bool more = kt + 1 < g.KT;
        if (more) load(kt + 1);
        compute(kt & 1);
        if (more) store((kt + 1) & 1);
        __syncthreads();
    }

    // ---- epilogue: lane holds channels 4*(lane>>4)+v of pixel (lane & 15) per fragment
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
        const int m = m0 + wm * 64 + j * 16 + (lane & 15);
        if (m >= g.M) continue;
        __bf16* dst = g.y + (size_t)m * g.Cout + n0 + wn * WN + 4 * (lane >> 4);
#pragma unroll
        for (int i = 0; i < FI; ++i) {
            typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
            bf16x4 o;
#pragma unroll
            for (int v = 0; v < 4; ++v) o[v] = (__bf16)acc[i][j][v];
            *reinterpret_cast<bf16x4*>(dst + i * 16) = o;
        }
    }
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
    const long long oh = ((long long)a->height + 2 * a->pad - a->kernel_h) / a->stride + 1;
    const long long ow = ((long long)a->width + 2 * a->pad - a->kernel_w) / a->stride + 1;
    if (oh < 1 || ow < 1) return fail(MCGMIL_E_INVALID, "the kernel does not fit the padded input");
    const long long x_bytes = (long long)a->batch * a->height * a->width * a->in_channels * 2;
    const long long y_elems = (long long)a->batch * oh * ow * a->out_channels;
    if (x_bytes >= (1ll << 31) || (long long)a->batch * oh * ow >= (1ll << 31) - kBM)
        return fail(MCGMIL_E_UNSUPPORTED, "input larger than 2 GiB or too many output pixels");
    if ((long long)a->out_channels * a->kernel_h * a->kernel_w * a->in_channels * 2 >= (1ll << 31))
        return fail(MCGMIL_E_UNSUPPORTED, "weights larger than 2 GiB");
    (void)y_elems;
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

int mcgmil_conv2d(const mcgmil_conv_args* a, void* stream) {
    int rc = validate(a);
    if (rc) return rc;
    if (!a->x || !a->w || !a->y) return fail(MCGMIL_E_INVALID, "NULL x, w or y");
    if (((uintptr_t)a->x | (uintptr_t)a->w | (uintptr_t)a->y) & 15u)
        return fail(MCGMIL_E_ALIGN, "x, w and y must be 16-byte aligned");
    ConvGeom g;
    g.x = static_cast<const __bf16*>(a->x);
    g.w = static_cast<const __bf16*>(a->w);
    g.y = static_cast<__bf16*>(a->y);
    g.N = a->batch; g.H = a->height; g.W = a->width; g.Cin = a->in_channels;
    g.Cout = a->out_channels; g.KH = a->kernel_h; g.KW = a->kernel_w;
    g.stride = a->stride; g.pad = a->pad;
    g.OH = (g.H + 2 * g.pad - g.KH) / g.stride + 1;
    g.OW = (g.W + 2 * g.pad - g.KW) / g.stride + 1;
    g.M = g.N * g.OH * g.OW;
    g.cin_tiles = g.Cin / 64;
    g.KT = g.KH * g.KW * g.cin_tiles;
    g.x_bytes = (uint32_t)((long long)g.N * g.H * g.W * g.Cin * 2);
    g.w_bytes = (uint32_t)((long long)g.Cout * g.KH * g.KW * g.Cin * 2);
    const int BN = g.Cout % 128 == 0 ? 128 : 64;
    g.tiles_n = g.Cout / BN;
    const long long tiles = (long long)((g.M + kBM - 1) / kBM) * g.tiles_n;
    if (tiles >= (1ll << 31)) return fail(MCGMIL_E_UNSUPPORTED, "too many tiles");
    g.tiles = (int)tiles;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (BN == 128)
        hipLaunchKernelGGL(conv_kernel<128>, dim3((unsigned)tiles), dim3(kConvThreads), 0, s, g);
    else
        hipLaunchKernelGGL(conv_kernel<64>, dim3((unsigned)tiles), dim3(kConvThreads), 0, s, g);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "conv_kernel launch");
}

}  // extern "C"
