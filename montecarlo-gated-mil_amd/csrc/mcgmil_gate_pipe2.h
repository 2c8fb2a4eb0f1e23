#pragma once
// gate_pipe2_kernel -- gate_pipe_kernel (mcgmil_kernels.h) with the serial latency chains of a
// tile taken out. Same tile shape (128 rows of the flattened (bag, t, n) space, 8 waves, all
// 2 G D + C output columns), same K-pipelined staging, same arithmetic (outputs bitwise equal to
// gate_pipe_kernel). What changes is where each tile waits:
//
//   * No row-table barrier before the K loop. Every thread derives the (bag, t, n) of the row it
//     stages from the row index itself (the same arithmetic fill_row_table does), so its first H
//     loads issue at kernel entry, beside the step-0 weight loads. The k-chunk-0 thread of each
//     row writes the row table the scoring phase reads; the K loop's barriers publish it.
//   * The head vectors (bv, bu, wa, ba: 3 KB for the reference heads) are copied into LDS at
//     entry, under the same loads. The epilogue used to fetch them from L2 right after its
//     vmcnt(0), once per gate pair: two exposed L2 round trips per wave per tile.
//   * The attention-logit keep decision (one Philox4x32-10 call) of the (row, class) a thread
//     scores is drawn right after its gated products, before the partial-score barrier, so it
//     fills the wait for the slower waves instead of following the barrier.
//   * Waves 4-7 (the younger half, which loses VALU arbitration to its partner on every
//     segment) run at s_setprio 1 (cdna_hip_programming.md T5, static form).
// Reference: model.py:280-303 (masked features, gate linears, gated product, logits, dropout).
#include "mcgmil_kernels.h"

namespace mcgmil {

#ifndef MCGMIL_P2_PRIO
#define MCGMIL_P2_PRIO 1
#endif

// Row info of flattened row R (hrow = -1 past the end): the per-thread form of fill_row_table.
struct RowInfo {
    int hrow, t, n, bag, Nb;
    uint32_t ctr;
};

__device__ __forceinline__ RowInfo row_info(const GateParams& p, long long R, int BM) {
    RowInfo r{-1, 0, 0, 0, 0, 0u};
    if (R >= p.total_samples) return r;
    const bool narrow = p.total_samples <= 0xFFFFFFFFll;
    if (p.uniform_rows > 0) {
        const long long per_bag = (long long)p.T * p.uniform_rows;
        r.Nb = p.uniform_rows;
        if (narrow) {
            const uint32_t x = (uint32_t)R, pb = (uint32_t)per_bag;
            r.bag = (int)(x / pb);
            const uint32_t local = x - (uint32_t)r.bag * pb;
            r.t = (int)(local / (uint32_t)r.Nb);
            r.n = (int)(local - (uint32_t)r.t * (uint32_t)r.Nb);
        } else {
            r.bag = (int)(R / per_bag);
            const long long local = R - (long long)r.bag * per_bag;
            r.t = (int)(local / r.Nb);
            r.n = (int)(local - (long long)r.t * r.Nb);
        }
        r.hrow = r.bag * r.Nb + r.n;
    } else {
        int bag;
        if (p.tile_bag) {
            bag = p.tile_bag[R / BM];
            while ((long long)p.T * p.bag_off[bag + 1] <= R) ++bag;
        } else {
            bag = find_bag(p.bag_off, p.B, p.T, R);
        }
        const int ob = p.bag_off[bag];
        r.bag = bag;
        r.Nb = p.bag_off[bag + 1] - ob;
        const long long local = R - (long long)p.T * ob;
        if (narrow) {
            r.t = (int)((uint32_t)local / (uint32_t)r.Nb);
            r.n = (int)((uint32_t)local - (uint32_t)r.t * (uint32_t)r.Nb);
        } else {
            r.t = (int)(local / r.Nb);
            r.n = (int)(local - (long long)r.t * r.Nb);
        }
        r.hrow = ob + r.n;
    }
    r.ctr = p.bag_ids ? (uint32_t)p.bag_ids[r.bag] : p.bag_base + (uint32_t)r.bag;
    return r;
}

// LDS floats of the head vectors: bv[G*D], bu[G*D], wa[C*D], ba[C] (padded to 4)
__host__ __device__ inline int head_lds_floats(int G, int D, int C) {
    return 2 * G * D + C * D + ((C + 3) & ~3);
}

template <typename E, int MAXC>
__host__ __device__ inline size_t pipe2_lds_bytes(int G, int D, int C) {
    return pipe_lds_bytes<E, MAXC>() + (size_t)head_lds_floats(G, D, C) * 4;
}

// fold_pairs with the head vectors read from LDS (hv = bv | bu | wa | ba).
template <int RT, int PPW, int MAXC, bool ONE_CLASS>
__device__ __forceinline__ void fold_pairs_lds(const GateParams& p, const f32x4 (&acc)[RT][2 * PPW],
                                               int q0, int lane, const float* hv,
                                               float (&part)[MAXC][RT]) {
    const int DB = p.D >> 4;
    const int GD = p.G * p.D;
    const float av_s = p.sf * kM2Log2e, au_s = p.sf * kMLog2e;
#pragma unroll
    for (int jp = 0; jp < PPW; ++jp) {
        const int q = q0 + jp;
        if (q >= p.P) break;
        const int g = q / DB, db = q - g * DB;
        const int d0 = db * 16 + 4 * (lane >> 4);
        f32x4 bvv = *reinterpret_cast<const f32x4*>(hv + g * p.D + d0);
        f32x4 buv = *reinterpret_cast<const f32x4*>(hv + GD + g * p.D + d0);
        bvv *= kM2Log2e;
        buv *= kMLog2e;
        f32x4 coef[MAXC];
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const int cc = ONE_CLASS ? g : c;
            const bool use = ONE_CLASS ? (c == 0) : ((c < p.C) && (p.G == 1 || c == g));
            const f32x4 w = *reinterpret_cast<const f32x4*>(hv + 2 * GD + (use ? cc : 0) * p.D + d0);
            coef[c] = use ? w : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const float ax = fmaf(acc[rt][2 * jp][v], av_s, bvv[v]);
                const float by = fmaf(acc[rt][2 * jp + 1][v], au_s, buv[v]);
                if constexpr (ONE_CLASS) {
                    const float a = __builtin_amdgcn_exp2f(fminf(fmaxf(ax, -43.280851226668903f),
                                                                 43.280851226668903f));
                    const float b = __builtin_amdgcn_exp2f(by);
                    const float ia = 1.0f + a;
                    const float r = __builtin_amdgcn_rcpf(fmaf(ia, b, ia));
                    part[0][rt] = fmaf(fmaf(-a, coef[0][v], coef[0][v]), r, part[0][rt]);
                } else {
                    const float pr = gated_product_scaled(ax, by);
#pragma unroll
                    for (int c = 0; c < MAXC; ++c) part[c][rt] = fmaf(pr, coef[c][v], part[c][rt]);
                }
            }
        }
    }
}

template <typename E, int PPW, int MAXC, bool REPLAY, bool ONE_CLASS>
__global__ __launch_bounds__(kGateThreads) void gate_pipe2_kernel(const GateParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BM = kPipeBM;
    constexpr int RT = BM / 16;                     // 8 row tiles = 8 waves
    constexpr int NJ = 2 * PPW;
    constexpr int SLOT = RT * 64 * 8;               // elements of one 32-deep K step
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int KS = p.L >> 5;

    E* Xs = reinterpret_cast<E*>(smem);                                   // [2][SLOT]
    float* red = reinterpret_cast<float*>(smem + (size_t)2 * SLOT * sizeof(E));
    float* zred = red + red_floats<BM, MAXC>();
    int* rinfo = reinterpret_cast<int*>(zred + MAXC * BM);
    float* hv = reinterpret_cast<float*>(rinfo + kRowInfo * BM);          // head vectors
    const long long R0 = (long long)blockIdx.x * BM;

#if MCGMIL_P2_PRIO
    if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
#endif
    MCGMIL_STAMP(p, 0);

    // weight tiles of this wave: independent of the rows, so they go out first
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
    auto wfrag = [&](uint32_t soff) { return load_frag_buf<E>(wrs, lane_b, soff); };
    Frag<E> wA[NJ], wB[NJ], zA, zB;
#pragma unroll
    for (int j = 0; j < NJ; ++j) wA[j] = wfrag(wsoff[j]);
    zA = wfrag(zsoff);

    // the row this thread stages (row wave*16 + (lane & 15), 8-chunk kq of every K step)
    const int srow = wave * 16 + (lane & 15);
    const int kq = lane >> 4;
    const RowInfo ri = row_info(p, R0 + srow, BM);
    const bool valid = ri.hrow >= 0;
    const E* hsrc = reinterpret_cast<const E*>(p.H) + (size_t)(valid ? ri.hrow : 0) * p.ldh + kq * 8;
    Raw<E> hA = load_raw(hsrc), hB = load_raw(hsrc + 32);
    if (kq == 0) {
        int* w = rinfo + kRowInfo * srow;
        w[0] = ri.hrow; w[1] = ri.t; w[2] = ri.n; w[3] = ri.bag; w[4] = ri.Nb; w[5] = (int)ri.ctr;
    }
    {   // head vectors -> LDS (16-B chunks; G*D, C*D multiples of 16 floats)
        const int GD4 = (p.G * p.D) >> 2, CD4 = (p.C * p.D) >> 2;
        for (int i = tid; i < 2 * GD4 + CD4 + 1; i += kGateThreads) {
            f32x4 v;
            if (i < GD4) v = reinterpret_cast<const f32x4*>(p.bv)[i];
            else if (i < 2 * GD4) v = reinterpret_cast<const f32x4*>(p.bu)[i - GD4];
            else if (i < 2 * GD4 + CD4) v = reinterpret_cast<const f32x4*>(p.wa)[i - 2 * GD4];
            else {
                v = f32x4{0.f, 0.f, 0.f, 0.f};
                for (int c = 0; c < p.C; ++c) v[c] = p.ba[c];
            }
            reinterpret_cast<f32x4*>(hv)[i] = v;
        }
    }

    const uint32_t cn = (uint32_t)ri.n, ct = (uint32_t)(p.t_base + ri.t), cb = ri.ctr;
    const uint8_t* kfe = REPLAY ? p.keep_feat + (size_t)(valid ? R0 + srow : 0) * (p.L >> 3) + kq
                                : nullptr;
    const uint32_t inval = valid ? 0u : 0xFFFFFFFFu;   // padding rows stage zeros
    auto stage = [&](int s, const Raw<E>& h, E* slot) {
        if constexpr (REPLAY) {
            const uint32_t kb = kfe[(size_t)(s < KS ? s : KS - 1) * 4];
            store_masked(h, kb & ~inval, slot + tid * 8);
        } else {
            const uint4 o = philox4x32_10<true>((uint32_t)(s * 4 + kq), cn, ct, cb, p.k0, p.k1);
            store_dropped(h, o, p.thrx_f, inval, slot + tid * 8);
        }
    };

    f32x4 acc[RT][NJ];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 zacc = {0.f, 0.f, 0.f, 0.f};

    // One K step, as gate_pipe_kernel's (see there).
    auto kstep = [&](int s, const E* cur, E* nxt, const Frag<E> (&w)[NJ], const Frag<E>& z,
                     Frag<E> (&wn)[NJ], Frag<E>& zn, const Raw<E>& h, Raw<E>& hn) {
        const int s1 = s + 1 < KS ? s + 1 : KS - 1;
        const int sh = s + HD < KS ? s + HD : KS - 1;
#pragma unroll
        for (int j = 0; j < NJ; ++j) wn[j] = wfrag(wsoff[j] + (uint32_t)s1 * kStepBytes);
        zn = wfrag(zsoff + (uint32_t)s1 * kStepBytes);
        hn = load_raw(hsrc + (size_t)sh * 32);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const Frag<E> x = load_frag(cur + (size_t)(rt * 64 + lane) * 8);
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[rt][j] = mma(w[j], x, acc[rt][j]);
        }
        const Frag<E> xz = load_frag(cur + (size_t)tid * 8);  // row tile `wave`
        zacc = mma(z, xz, zacc);
        stage(s + 1, h, nxt);           // step KS is staged into the idle slot and never read
        if constexpr (sizeof(E) == 2 && PPW == 2) {
#pragma unroll
            for (int i = 0; i < RT * NJ + 1; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0); // VALU
            }
        }
        __syncthreads();
    };

    stage(0, hA, Xs);
    __syncthreads();
    MCGMIL_STAMP(p, 2);

    // KS is even and >= 2 (host guarantees L % 64 == 0); steps 0 and 1 peeled (zero accumulators
    // as inline constants).
    kstep(0, Xs, Xs + SLOT, wA, zA, wB, zB, hB, hA);
    kstep(1, Xs + SLOT, Xs, wB, zB, wA, zA, hA, hB);
    for (int s = 2; s < KS; s += 2) {
        kstep(s, Xs, Xs + SLOT, wA, zA, wB, zB, hB, hA);
        kstep(s + 1, Xs + SLOT, Xs, wB, zB, wA, zA, hA, hB);
    }
    MCGMIL_STAMP(p, 3);

    float part[MAXC][RT];
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) part[c][rt] = 0.f;
    fold_pairs_lds<RT, PPW, MAXC, ONE_CLASS>(p, acc, q0, lane, hv, part);
    MCGMIL_STAMP(p, 4);

    // attention-logit keep of the (row, class) this thread scores (row srow, class lane >> 4)
    bool keep = true;
    if constexpr (!REPLAY) {
        if (valid && kq < p.C)
            keep = attention_keep(p.k0, p.k1, cb, ct, (uint32_t)kq, cn, p.thr_a);
    }
    const int one_class = ONE_CLASS ? (q0 < p.P ? q0 / (p.D >> 4) : MAXC) : -1;
    finish_scores<BM, MAXC>(p, R0, part, zacc, true, red, zred, rinfo, one_class,
                            ONE_CLASS ? (p.D >> 4) / PPW : 0, !REPLAY, keep,
                            hv + 2 * p.G * p.D + p.C * p.D);
    MCGMIL_STAMP(p, 7);
}

}  // namespace mcgmil
