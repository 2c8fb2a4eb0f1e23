#pragma once
// gate_pp_kernel -- the bf16 fast path with TWO independent workgroups per CU.
//
// Same maths and the same K-pipelined staging as gate_pipe_kernel (mcgmil_kernels.h): masked
// features staged 32-deep per step with one Philox4x32-10 call per 8-element chunk, weights as
// the MFMA A operand streamed from L2 through buffer loads, the classifier folded in as one
// more 16-column tile, and the same epilogue. What changes is the shape of the work:
//
//   * 4 waves (256 threads), <= 256 VGPRs: one wave per SIMD, two workgroups per CU. The two
//     workgroups on a CU never synchronise with each other, so one's barriers, epilogue
//     (transcendental VALU) and prologue overlap the other's MFMA stream -- the 8-wave
//     gate_pipe_kernel runs one workgroup per CU and idles its MFMA pipes in all of those.
//   * BM = 16 * RT rows per workgroup; every wave holds all RT row tiles for its PPW gate tile
//     pairs (acc[RT][2 PPW], 128 registers). Separate heads (P = 16): RT = 4, PPW = 4; shared
//     (P = 8): RT = 8, PPW = 2.
//   * MFMAs run column-tile-outer, so each weight fragment is reloaded for the next step as
//     soon as its RT MFMAs are issued: one register set of weights instead of two.
#include "mcgmil_kernels.h"

namespace mcgmil {

constexpr int kPPThreads = 256;
constexpr int kPPWaves = kPPThreads / kWave;

#ifndef MCGMIL_PP_WDB
#define MCGMIL_PP_WDB 0   // 1: weights double-buffered in two named register sets
#endif
#ifndef MCGMIL_PP_PIN
#define MCGMIL_PP_PIN 1   // 1 MFMA : VPM VALU sched_group_barrier pin in the K step
#endif
#ifndef MCGMIL_PP_SB
#define MCGMIL_PP_SB 0    // 1: sched_barrier fences around the per-step workgroup barrier
#endif
#ifndef MCGMIL_PP_STAGE_ROT
#define MCGMIL_PP_STAGE_ROT 0  // diagnostic: wave w stages row tile (w + ROT) % 4
#endif
#ifndef MCGMIL_PP_XRELOAD
#define MCGMIL_PP_XRELOAD 0    // diagnostic: re-read each x fragment before every MFMA
#endif
#ifndef MCGMIL_PP_EXITPAD
#define MCGMIL_PP_EXITPAD 0  // 1: explicit wait states after the K loop (hazard experiment)
#endif

template <typename E, int RT, int MAXC>
__host__ __device__ constexpr size_t pp_lds_bytes() {
    return (size_t)2 * RT * 64 * 8 * sizeof(E)                  // two K-step slots
           + (size_t)kPPWaves * MAXC * 4 * 16 * RT * 4          // partial scores
           + (size_t)MAXC * 16 * RT * 4                         // classifier projections
           + (size_t)kRowInfo * 16 * RT * 4;                    // row table
}

// One BM-row tile of the flattened (bag, t, n) space, rows R0 .. R0 + BM - 1, whose row table is
// in `rinfo` (visible: the caller's barrier). Scores go to lg_out / z_out at row R0 + r - obase.
// The body of gate_pp_kernel.
template <typename E, int RT, int PPW, int MAXC, bool REPLAY, bool ONE_CLASS>
__device__ __forceinline__ void pp_tile(const GateParams& p, long long R0, unsigned char* smem, const int* rinfo,
                                        float* lg_out, float* z_out, long long obase) {
    static_assert(RT % kPPWaves == 0, "row tiles must split over the waves");
    constexpr int BM = 16 * RT;
    constexpr int NJ = 2 * PPW;
    constexpr int CH = RT / kPPWaves;       // staging chunks per thread per step
    constexpr int SLOT = RT * 64 * 8;       // elements of one 32-deep K step
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int KS = p.L >> 5;

    E* Xs = reinterpret_cast<E*>(smem);
    float* red = reinterpret_cast<float*>(smem + (size_t)2 * SLOT * sizeof(E));
    float* zred = red + kPPWaves * MAXC * 4 * BM;

    // staging chunk i of this thread: element (tid + 256 i) * 8 of a step = row tile
    // wave + 4 i, lane slot `lane` (row (wave + 4 i) * 16 + (lane & 15), k-chunk lane >> 4)
    const int kq = lane >> 4;
    const int swave = (wave + MCGMIL_PP_STAGE_ROT) % kPPWaves;   // staging row tile base
    const E* hsrc[CH];
    uint32_t cn[CH], ct[CH], cb[CH], inval[CH];
    const uint8_t* kfe[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        const int row = (swave + kPPWaves * i) * 16 + (lane & 15);
        const int* ri = rinfo + kRowInfo * row;
        const bool valid = ri[0] >= 0;
        hsrc[i] = reinterpret_cast<const E*>(p.H) + (size_t)(valid ? ri[0] : 0) * p.ldh + kq * 8;
        cn[i] = (uint32_t)ri[2];
        ct[i] = (uint32_t)(p.t_base + ri[1]);
        cb[i] = (uint32_t)ri[5];
        inval[i] = valid ? 0u : 0xFFFFFFFFu;
        kfe[i] = REPLAY ? p.keep_feat + (size_t)(valid ? R0 + row : 0) * (p.L >> 3) + kq : nullptr;
    }
    auto stage = [&](int s, const Raw<E> (&h)[CH], E* slot) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            E* dst = slot + (size_t)(swave * 64 + lane + kPPThreads * i) * 8;
            if constexpr (REPLAY) {
                const uint32_t kb = kfe[i][(size_t)(s < KS ? s : KS - 1) * 4];
                store_masked(h[i], kb & ~inval[i], dst);
            } else {
                const uint4 o = philox4x32_10<true>((uint32_t)(s * 4 + kq), cn[i], ct[i], cb[i], p.k0, p.k1);
                store_dropped(h[i], o, p.thrx_f, inval[i], dst);
            }
        }
    };

    // weights: one buffer descriptor, lane byte offset as voffset, wave-uniform soffset
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(p.Wp, p.wp_bytes);
    const uint32_t tile_bytes = (uint32_t)KS * 512u * (uint32_t)sizeof(E);
    constexpr uint32_t kStepBytes = 512u * (uint32_t)sizeof(E);
    const int q0 = __builtin_amdgcn_readfirstlane(wave) * PPW;
    uint32_t wsoff[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        int q = q0 + (j >> 1);
        q = q < p.P ? q : p.P - 1;
        wsoff[j] = (uint32_t)(2 * q + (j & 1)) * tile_bytes;
    }
    const uint32_t zsoff = (uint32_t)(2 * p.P) * tile_bytes;
    const uint32_t lane_b = (uint32_t)lane * 8u * (uint32_t)sizeof(E);

    f32x4 acc[RT][NJ];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 zacc[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) zacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

    // One K step: MFMAs on step s from slot `cur` with weights (w, zc); the weights of step s+1
    // go to (wn, zn) -- the SAME registers when single-buffered (each fragment reloaded right
    // after its RT MFMAs), the other named set when double-buffered. The H chunks of step s+2
    // are prefetched into hn and step s+1 (from h, loaded a step earlier) is staged into `nxt`.
    auto kstep = [&](int s, const E* cur, E* nxt, Frag<E> (&w)[NJ], Frag<E> (&wn)[NJ], Frag<E>& zc,
                     Frag<E>& zn, const Raw<E> (&h)[CH], Raw<E> (&hn)[CH]) {
#if MCGMIL_DIAG & 64   // ablation (timing only): every step reloads the weights of step 0 (L1 hits)
        const int s1 = 0;
#else
        const int s1 = s + 1 < KS ? s + 1 : KS - 1;
#endif
        const int s2 = s + 2 < KS ? s + 2 : KS - 1;
#pragma unroll
        for (int i = 0; i < CH; ++i) hn[i] = load_raw(hsrc[i] + (size_t)s2 * 32);
        Frag<E> x[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) x[rt] = load_frag(cur + (size_t)(rt * 64 + lane) * 8);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                if (MCGMIL_PP_XRELOAD) x[rt] = load_frag(cur + (size_t)(rt * 64 + lane) * 8);
                acc[rt][j] = mma(w[j], x[rt], acc[rt][j]);
            }
#if !(MCGMIL_DIAG & 2)   // ablation (timing only): no weight reloads
            wn[j] = load_frag_buf<E>(wrs, lane_b, wsoff[j] + (uint32_t)s1 * kStepBytes);
#endif
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) {   // classifier tile of row tile wave + 4 i
            const Frag<E> xz = load_frag(cur + (size_t)((wave + kPPWaves * i) * 64 + lane) * 8);
            zacc[i] = mma(zc, xz, zacc[i]);
        }
#if !(MCGMIL_DIAG & 2)
        zn = load_frag_buf<E>(wrs, lane_b, zsoff + (uint32_t)s1 * kStepBytes);
#endif
        stage(s + 1, h, nxt);   // step KS lands in the idle slot and is never read
        if constexpr (sizeof(E) == 2 && MCGMIL_PP_PIN) {
#pragma unroll
            for (int i = 0; i < RT * NJ + CH; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0); // VALU
            }
        }
        if (MCGMIL_PP_SB) __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
        if (MCGMIL_PP_SB) __builtin_amdgcn_sched_barrier(0);
    };

    Frag<E> wA[NJ], zA;
#if MCGMIL_PP_WDB
    Frag<E> wB[NJ], zB;
#else
    Frag<E> (&wB)[NJ] = wA;
    Frag<E>& zB = zA;
#endif
    Raw<E> hA[CH], hB[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) hA[i] = load_raw(hsrc[i]);
    stage(0, hA, Xs);
#pragma unroll
    for (int i = 0; i < CH; ++i) hB[i] = load_raw(hsrc[i] + 32);
#pragma unroll
    for (int j = 0; j < NJ; ++j) wA[j] = load_frag_buf<E>(wrs, lane_b, wsoff[j]);
    zA = load_frag_buf<E>(wrs, lane_b, zsoff);
    __syncthreads();
    MCGMIL_STAMP(p, 2);

    // KS is even and >= 2 (host guarantees L % 64 == 0); the first two steps are peeled so their
    // MFMAs take the zero accumulators as an inline constant (no copies into the loop).
    kstep(0, Xs, Xs + SLOT, wA, wB, zA, zB, hB, hA);
    kstep(1, Xs + SLOT, Xs, wB, wA, zB, zA, hA, hB);
#if MCGMIL_DIAG & 16   // ablation (timing only): 2 of the KS K steps
    if (KS > 1000)
#endif
    for (int s = 2; s < KS; s += 2) {
        kstep(s, Xs, Xs + SLOT, wA, wB, zA, zB, hB, hA);
        kstep(s + 1, Xs + SLOT, Xs, wB, wA, zB, zA, hA, hB);
    }
#if MCGMIL_PP_EXITPAD
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#endif
    MCGMIL_STAMP(p, 3);

    // epilogue: gated products folded into per-lane partial scores (mcgmil_kernels.h)
    float part[MAXC][RT];
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) part[c][rt] = 0.f;
    fold_pairs<RT, PPW, MAXC, ONE_CLASS>(p, acc, q0, lane, part);
    MCGMIL_STAMP(p, 4);

    // partials: red[wave][class][lane group][row] (row fastest: conflict-free both ways)
    const int one_class = ONE_CLASS ? (q0 < p.P ? q0 / (p.D >> 4) : MAXC) : -1;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if (ONE_CLASS && c > 0) break;
        const int cls = ONE_CLASS ? one_class : c;
        if (cls >= MAXC) break;                          // idle wave (no pairs)
        float* dst = red + ((size_t)(wave * MAXC + cls) * 4 + (lane >> 4)) * BM + (lane & 15);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) dst[16 * rt] = part[c][rt];
    }
    if (lane < 16) {
#pragma unroll
        for (int i = 0; i < CH; ++i)
#pragma unroll
            for (int c = 0; c < MAXC; ++c) zred[c * BM + (wave + kPPWaves * i) * 16 + lane] = zacc[i][c];
    }
    MCGMIL_STAMP(p, 5);
    __syncthreads();
    MCGMIL_STAMP(p, 6);

    // one (row, class) item per thread: reduce the partials, bias, logit dropout, stores
    const int waves_per_class = ONE_CLASS ? (p.D >> 4) / PPW : 0;
    for (int item = tid; item < BM * p.C; item += kPPThreads) {
        const int r = item % BM, c = item / BM;
        const int* ri = rinfo + kRowInfo * r;
        if (ri[0] < 0) continue;
        float s = 0.f;
        const int nw = ONE_CLASS ? waves_per_class : kPPWaves;
        for (int k = 0; k < nw; ++k) {
            const int wv = ONE_CLASS ? c * waves_per_class + k : k;
            const float* src = red + (size_t)(wv * MAXC + c) * 4 * BM + r;
            s += src[0] + src[BM] + src[2 * BM] + src[3 * BM];
        }
        s += p.ba[c];
        const int t = ri[1], n = ri[2], bag = ri[3], Nb = ri[4];
        bool keep;
        if (REPLAY) {
            const size_t abase = (size_t)p.T * p.C * (size_t)p.bag_off[bag];
            keep = p.keep_att[abase + ((size_t)t * p.C + c) * Nb + n] != 0;
        } else {
            keep = attention_keep(p.k0, p.k1, (uint32_t)ri[5], (uint32_t)(p.t_base + t), (uint32_t)c,
                                  (uint32_t)n, p.thr_a);
        }
        const size_t o = (size_t)(R0 + r - obase) * p.C + c;
        lg_out[o] = s * (keep ? p.sa : 0.f);
        z_out[o] = zred[c * BM + r] * p.sf;
    }
    MCGMIL_STAMP(p, 7);
}

template <typename E, int RT, int PPW, int MAXC, bool REPLAY, bool ONE_CLASS, bool PROBE = false>
__global__ __launch_bounds__(kPPThreads, 2) void gate_pp_kernel(const GateParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BM = 16 * RT;
    int* rinfo = reinterpret_cast<int*>(smem + (size_t)2 * RT * 64 * 8 * sizeof(E) +
                                        ((size_t)kPPWaves * MAXC * 4 * BM + (size_t)MAXC * BM) * 4);
    const long long R0 = xcd_tile(blockIdx.x, gridDim.x, p.B) * BM;   // XCD-aware order (mcgmil_kernels.h)
    if constexpr (PROBE) clock_probe(p, 0);
    MCGMIL_STAMP(p, 0);
    fill_row_table<BM>(p, R0, rinfo);
    __syncthreads();
    MCGMIL_STAMP(p, 1);
    pp_tile<E, RT, PPW, MAXC, REPLAY, ONE_CLASS>(p, R0, smem, rinfo, p.logits, p.zz, 0);
    if constexpr (PROBE) clock_probe(p, 1);
}

}  // namespace mcgmil
