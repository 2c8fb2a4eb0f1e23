#pragma once
// gate_hp_kernel -- the separate-heads gate kernel with the two heads in ping-pong.
//
// gate_pipe_kernel runs one 128-row tile per workgroup as 16 K steps (MFMA) followed by the
// epilogue (transcendental VALU) and the scoring, while the MFMA pipes idle: ~29% of the kernel
// (profiles/r02/gate_ab.log). Two tiles cannot be in flight per SIMD (their accumulators would
// need 2 x 270 KB of a CU's 512 KB register file), and 64-row tiles double the weight bytes per
// MFMA, which costs more than the overlap gains (gate_pp_kernel). With separate heads (reference
// model.py:186-193, shared_attention=False) the two heads need the same masked features and
// nothing else in common, so the 8 waves split by head:
//
//   * team t (waves 4t .. 4t+3, one wave per SIMD) computes head t for all 128 rows of a tile:
//     the V/U columns of class t (model.py:297-298), the gated product and logit of class t
//     (299-301); team 0 also the classifier projection of both classes (313-315). 128
//     accumulators per wave, as in gate_pipe_kernel, and every weight byte still read once per
//     128 rows;
//   * a tile is 21 ticks (one workgroup barrier each). Team 0 runs its 16 K steps in ticks
//     0-15 and its epilogue in 16-20 (4 fold ticks of two row tiles, 1 scoring tick); team 1
//     runs the epilogue of the PREVIOUS tile in ticks 0-4 and its K steps in 5-20. So on every
//     SIMD one head's epilogue and scoring run beside the other head's MFMAs;
//   * the masked features of each K step are staged once (one Philox4x32-10 call per thread,
//     as in gate_pipe_kernel) into a ring of 8 LDS slots that both teams read, team 1 five
//     ticks after team 0 (slot = step mod 8: with 16 steps a tile, compile-time);
//   * persistent: one workgroup per CU walks the row tiles blockIdx.x + k * gridDim.x, the next
//     tile's rows, first features and step-0 weights loading under the current tile's epilogue.
// Every tick is unrolled at compile time, so step parities, ring slots and fold ranges are
// constants and the loop-carried registers are named (no runtime-indexed arrays).
// Arithmetic and summation orders are gate_pipe_kernel's: the outputs are bitwise identical.
#include <type_traits>
#include <utility>

#include "mcgmil_kernels.h"

namespace mcgmil {

#ifndef MCGMIL_HP_DSPIN
#define MCGMIL_HP_DSPIN 0
#endif

constexpr int kHpBM = 128;
constexpr int kHpKS = 16;                // K steps of 32: L = 512 (the reference's ResNet-18)
constexpr int kHpEP = 6;                 // epilogue ticks per tile and team (4 fold, publish, scoring)
constexpr int kHpTicks = kHpKS + kHpEP;
constexpr int kHpSlots = 8;              // feature ring; team 1 reads a slot 5 ticks after team 0
constexpr int kHpD = 128;

template <typename F, int... I>
__device__ __forceinline__ void hp_unroll_impl(F& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void hp_unroll(F&& f) {
    hp_unroll_impl(f, std::make_integer_sequence<int, N>{});
}

struct HpRow {
    int hrow, t, n, bag, Nb;
    uint32_t ctr;
};

// (bag, t, n) of flattened row R: fill_row_table's arithmetic for one row
__device__ __forceinline__ HpRow hp_row(const GateParams& p, long long R0, long long R) {
    HpRow r{-1, 0, 0, 0, 0, 0u};
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
            bag = p.tile_bag[R0 / kHpBM];
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

// LDS: feature ring [8][128 x 32] bf16 | partials [2 teams][4 waves][4 lane groups][128] |
// z [2][128] | row tables [2][128][6] | head vectors bv, bu, wa [2 D] each, ba [4]
__host__ __device__ constexpr size_t hp_lds_bytes() {
    return (size_t)kHpSlots * kHpBM * 32 * 2 + (size_t)2 * 4 * 4 * kHpBM * 4 + (size_t)2 * kHpBM * 4 +
           (size_t)2 * kRowInfo * kHpBM * 4 + (size_t)(6 * kHpD + 4) * 4;
}

__global__ __launch_bounds__(kGateThreads) void gate_hp_kernel(const GateParams p) {
    using E = __bf16;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BM = kHpBM, RT = BM / 16, NJ = 4, KS = kHpKS, EP = kHpEP, D = kHpD;
    constexpr int SLOT = RT * 64 * 8;       // elements of one 32-deep K step of features
    constexpr uint32_t kStepBytes = 1024u;
    int tid = threadIdx.x, lane = tid & 63;
    const int wave = tid >> 6;
    const int team = __builtin_amdgcn_readfirstlane(wave) >> 2;   // = head = class
    const int wt = __builtin_amdgcn_readfirstlane(wave) & 3;      // wave within the team

    E* Xs = reinterpret_cast<E*>(smem);                                          // [8][SLOT]
    float* red = reinterpret_cast<float*>(smem + (size_t)kHpSlots * SLOT * 2);   // [2][4][4][BM]
    float* zred = red + 2 * 4 * 4 * BM;                                          // [2][BM]
    int* rinfo = reinterpret_cast<int*>(zred + 2 * BM);                          // [2][BM][6]
    float* hv = reinterpret_cast<float*>(rinfo + 2 * kRowInfo * BM);             // head vectors

    const long long ntiles = (p.total_samples + BM - 1) / BM;
    const long long G = gridDim.x, b = blockIdx.x;
    const int my_tiles = b < ntiles ? (int)((ntiles - 1 - b) / G + 1) : 0;
    if (my_tiles == 0) return;                                    // workgroup-uniform

    {   // head vectors -> LDS: bv [2D], bu [2D], wa [2D], ba (C = 2)
        constexpr int n4 = (6 * D) >> 2;
        for (int i = tid; i <= n4; i += kGateThreads) {
            f32x4 v;
            if (i < n4) {
                const int f = i * 4, which = f / (2 * D), off = f - which * 2 * D;
                const float* src = which == 0 ? p.bv : which == 1 ? p.bu : p.wa;
                v = *reinterpret_cast<const f32x4*>(src + off);
            } else {
                v = f32x4{p.ba[0], p.ba[1], 0.f, 0.f};
            }
            reinterpret_cast<f32x4*>(hv)[i] = v;
        }
    }

    // ---- staging: thread tid stages row srow = wave*16 + (lane & 15), 8-chunk kq of every step
    const int srow = wave * 16 + (lane & 15);
    int kq = lane >> 4;
    const E* hsrc = reinterpret_cast<const E*>(p.H);
    uint32_t cn = 0, ct = 0, cb = 0, inval = 0xFFFFFFFFu;
    auto set_tile_rows = [&](int k) {       // staging rows (and row table) of the k-th tile
        const long long R0 = (b + (long long)k * G) * BM;
        const HpRow r = hp_row(p, R0, R0 + srow);
        const bool valid = r.hrow >= 0;
        hsrc = reinterpret_cast<const E*>(p.H) + (size_t)(valid ? r.hrow : 0) * p.ldh + kq * 8;
        cn = (uint32_t)r.n;
        ct = (uint32_t)(p.t_base + r.t);
        cb = r.ctr;
        inval = valid ? 0u : 0xFFFFFFFFu;
        if (kq == 0) {
            int* w = rinfo + ((k & 1) * BM + srow) * kRowInfo;
            w[0] = r.hrow; w[1] = r.t; w[2] = r.n; w[3] = r.bag; w[4] = r.Nb; w[5] = (int)r.ctr;
        }
    };
    Raw<E> H0, H1;                          // H chunk of an even / odd step
    auto stage = [&](int s, const Raw<E>& h) {
        const uint4 o = philox4x32_10<true>((uint32_t)(s * 4 + kq), cn, ct, cb, p.k0, p.k1);
        store_dropped(h, o, p.thrx_f, inval, Xs + (size_t)(s % kHpSlots) * SLOT + tid * 8);
    };

    // ---- weights: wave (team, wt) streams gate tiles 2 q0 .. 2 q0 + 3 (q0 = 8 team + 2 wt);
    // team 0 also the classifier tile
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(p.Wp, p.wp_bytes);
    const uint32_t tile_bytes = (uint32_t)KS * kStepBytes;
    const int q0 = team * (D >> 4) + 2 * wt;
    uint32_t wsoff[NJ];   // (not const: relaxed every tick, see `relax`)
#pragma unroll
    for (int j = 0; j < NJ; ++j) wsoff[j] = (uint32_t)(2 * (q0 + (j >> 1)) + (j & 1)) * tile_bytes;
    uint32_t zsoff = (uint32_t)(2 * p.P) * tile_bytes;
    uint32_t lane_b = (uint32_t)lane * 16u;
    // Every tick re-derives its lane / step addresses from these: without the empty asm the
    // compiler hoists all 16 steps' addresses and first Philox products out of the tile loop
    // (~250 registers of invariants) and spills.
    auto relax = [&]() __attribute__((always_inline)) {
        asm volatile("" : "+v"(tid), "+v"(lane), "+v"(kq), "+v"(lane_b));
        asm volatile("" : "+s"(wsoff[0]), "+s"(wsoff[1]), "+s"(wsoff[2]), "+s"(wsoff[3]), "+s"(zsoff));
    };
    auto wfrag = [&](uint32_t soff) { return load_frag_buf<E>(wrs, lane_b, soff); };
    Frag<E> W0[NJ], W1[NJ], Z0, Z1;         // weights of an even / odd step
    auto load_w0 = [&](bool zt) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) W0[j] = wfrag(wsoff[j]);
        if (zt) Z0 = wfrag(zsoff);
    };

    f32x4 acc[RT][NJ];
    f32x4 zacc[2];
    float part[RT];
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

    // one K step of this wave's team on step s (ring slot s % 8); step 0 starts the sums
    auto kstep = [&](auto S, bool zt, const Frag<E> (&w)[NJ], const Frag<E>& z, Frag<E> (&wn)[NJ],
                     Frag<E>& zn) __attribute__((always_inline)) {
        constexpr int s = decltype(S)::value;
        if constexpr (s + 1 < KS) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) wn[j] = wfrag(wsoff[j] + (uint32_t)(s + 1) * kStepBytes);
            if (zt) zn = wfrag(zsoff + (uint32_t)(s + 1) * kStepBytes);
        }
        const E* cur = Xs + (size_t)(s % kHpSlots) * SLOT;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const Frag<E> x = load_frag(cur + (size_t)(rt * 64 + lane) * 8);
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[rt][j] = mma(w[j], x, s == 0 ? zero4 : acc[rt][j]);
        }
        if (zt) {                           // classifier tiles of row tiles 2 wt, 2 wt + 1
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const Frag<E> xz = load_frag(cur + (size_t)((2 * wt + i) * 64 + lane) * 8);
                zacc[i] = mma(z, xz, s == 0 ? zero4 : zacc[i]);
            }
        }
    };
    // Keep a step's MFMAs in its tick: they have no memory side effects, so without this the
    // compiler sinks all 16 steps past the barriers to the fold, with every step's operands
    // live (thousands of bytes of spills). Placed after the staging: an asm statement ends the
    // scheduling region, and the staging VALU must interleave with the MFMAs.
    auto fence_acc = [&](bool zt) __attribute__((always_inline)) {
        if (zt) asm volatile("" : "+v"(zacc[0]), "+v"(zacc[1]));
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
            asm volatile("" : "+v"(acc[rt][0]), "+v"(acc[rt][1]), "+v"(acc[rt][2]), "+v"(acc[rt][3]));
    };
    auto kstep_p = [&](auto S, bool zt) __attribute__((always_inline)) {
        if constexpr ((decltype(S)::value & 1) == 0) kstep(S, zt, W0, Z0, W1, Z1);
        else kstep(S, zt, W1, Z1, W0, Z0);
    };
    auto pin = [&](bool zt) __attribute__((always_inline)) {
        // Spread the staging VALU over the MFMA stream (1 MFMA : VPM VALU), as gate_pipe_kernel,
        // and read each row tile's features two row tiles ahead: with one K-stepping wave per
        // SIMD in the epilogue ticks, an LDS read waited for right before its MFMAs is exposed.
#if MCGMIL_HP_DSPIN
        if (zt) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);    // DS reads: x0, x1, 2 xz
        else __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);       // x0, x1
#endif
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0); // VALU
            }
#if MCGMIL_HP_DSPIN
            if (rt + 2 < RT) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#endif
        }
        if (zt) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
            }
        }
    };

    // fold row tiles 2e, 2e+1 of both pairs into part (fold_pairs' order per row tile)
    const float av_s = p.sf * kM2Log2e, au_s = p.sf * kMLog2e;
    auto fold = [&](auto EE) __attribute__((always_inline)) {
        constexpr int e = decltype(EE)::value;
#pragma unroll
        for (int rt = 2 * e; rt < 2 * e + 2; ++rt) {
            float pr = 0.f;
#pragma unroll
            for (int jp = 0; jp < 2; ++jp) {
                const int db = 2 * wt + jp;
                const int d0 = db * 16 + 4 * (lane >> 4);
                const f32x4 bvv = *reinterpret_cast<const f32x4*>(hv + team * D + d0) * kM2Log2e;
                const f32x4 buv = *reinterpret_cast<const f32x4*>(hv + 2 * D + team * D + d0) * kMLog2e;
                const f32x4 w = *reinterpret_cast<const f32x4*>(hv + 4 * D + team * D + d0);
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const float ax = fmaf(acc[rt][2 * jp][v], av_s, bvv[v]);
                    const float by = fmaf(acc[rt][2 * jp + 1][v], au_s, buv[v]);
                    const float a = __builtin_amdgcn_exp2f(fminf(fmaxf(ax, -43.280851226668903f),
                                                                 43.280851226668903f));
                    const float bb = __builtin_amdgcn_exp2f(by);
                    const float ia = 1.0f + a;
                    const float r = __builtin_amdgcn_rcpf(fmaf(ia, bb, ia));
                    pr = fmaf(fmaf(-a, w[v], w[v]), r, pr);
                }
            }
            part[rt] = pr;
            asm volatile("" : "+v"(part[rt]));     // the fold stays in its tick
        }
    };
    // partial scores (and team 0's z) of tile k to LDS
    auto publish = [&]() __attribute__((always_inline)) {
        float* dst = red + ((size_t)(team * 4 + wt) * 4 + (lane >> 4)) * BM + (lane & 15);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) dst[16 * rt] = part[rt];
        if (team == 0 && lane < 16) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                zred[(2 * wt + i) * 16 + lane] = zacc[i][0];
                zred[BM + (2 * wt + i) * 16 + lane] = zacc[i][1];
            }
        }
    };
    // logits and z of class `team` for tile k (finish_scores' order: waves, then lane groups)
    auto score = [&](int k) __attribute__((always_inline)) {
        const int tt = tid - team * 256;
        if (tt >= BM) return;
        const int* ri = rinfo + ((k & 1) * BM + tt) * kRowInfo;
        if (ri[0] < 0) return;
        float sc = 0.f;
        for (int w4 = 0; w4 < 4; ++w4) {
            const float* src = red + (size_t)(team * 4 + w4) * 4 * BM + tt;
#pragma unroll
            for (int g = 0; g < 4; ++g) sc += src[g * BM];
        }
        sc += hv[6 * D + team];
        const bool keep = attention_keep(p.k0, p.k1, (uint32_t)ri[5], (uint32_t)(p.t_base + ri[1]),
                                         (uint32_t)team, (uint32_t)ri[2], p.thr_a);
        const long long R0 = (b + (long long)k * G) * BM;
        const size_t o = (size_t)(R0 + tt) * 2 + team;
        p.logits[o] = sc * (keep ? p.sa : 0.f);
        p.zz[o] = zred[team * BM + tt] * p.sf;
    };
    // epilogue tick e of this wave's team for tile k (e = 3: weights of the next tile's step 0)
    auto epilogue = [&](auto EE, int k, bool have) __attribute__((always_inline)) {
        constexpr int e = decltype(EE)::value;
        if constexpr (e < RT / 2) {
            if (have) fold(EE);
        } else if constexpr (e == EP - 2) {
            if (have) publish();
            load_w0(team == 0);
        } else {
            if (have) score(k);
        }
    };

    // staging of tick i (steps 1..15 of tile k in ticks 0..14, step 0 of tile k+1 in tick 20)
    auto stage_tick = [&](auto I, bool next) __attribute__((always_inline)) {
        constexpr int i = decltype(I)::value;
        if constexpr (i < KS - 1) stage(i + 1, ((i + 1) & 1) ? H1 : H0);
        else if constexpr (i == kHpTicks - 1) {
            if (next) stage(0, H0);
        }
    };
    // H loads of tick i: step i+2 in ticks 0..13; the next tile's rows in tick 16, its steps 0
    // and 1 in ticks 19 and 20
    auto load_tick = [&](auto I, int k, bool next) __attribute__((always_inline)) {
        constexpr int i = decltype(I)::value;
        if constexpr (i < KS - 2) {
            if constexpr (i & 1) H1 = load_raw(hsrc + (size_t)(i + 2) * 32);
            else H0 = load_raw(hsrc + (size_t)(i + 2) * 32);
        } else if constexpr (i == KS) {
            if (next) set_tile_rows(k + 1);
        } else if constexpr (i == kHpTicks - 2) {
            if (next) H0 = load_raw(hsrc);
        } else if constexpr (i == kHpTicks - 1) {
            if (next) H1 = load_raw(hsrc + 32);
        }
    };

    // prologue: rows of tile 0, step 0 staged, H of step 1 in flight, team 0's step-0 weights
    set_tile_rows(0);
    H0 = load_raw(hsrc);
    if (team == 0) load_w0(true);
    H1 = load_raw(hsrc + 32);
    stage(0, H0);
    __syncthreads();

    // Each team runs its own program (wave-uniform branch, taken once): 22 barriers per tile
    // in both, so the workgroup barriers pair up tick by tick. One program per team keeps one
    // accumulator stream per code path; interleaving both teams' K steps in one tick loop made
    // the register allocator keep two accumulator sets and spill.
    auto run = [&](auto TEAM) __attribute__((always_inline)) {
        constexpr int tm = decltype(TEAM)::value;
        for (int k = 0; k < my_tiles; ++k) {
            const bool next = k + 1 < my_tiles;
            hp_unroll<kHpTicks>([&](auto I) __attribute__((always_inline)) {
                constexpr int i = decltype(I)::value;
                relax();
                if constexpr (tm == 0) {
                    if constexpr (i < KS) {
                        kstep_p(std::integral_constant<int, i>{}, true);
                        stage_tick(I, next);
                        pin(true);
                        fence_acc(true);
                    } else {
                        epilogue(std::integral_constant<int, i - KS>{}, k, true);
                        stage_tick(I, next);
                    }
                } else {
                    if constexpr (i < EP) {
                        epilogue(std::integral_constant<int, i>{}, k - 1, k > 0);
                        stage_tick(I, next);
                    } else {
                        kstep_p(std::integral_constant<int, i - EP>{}, false);
                        stage_tick(I, next);
                        pin(false);
                        fence_acc(false);
                    }
                }
                load_tick(I, k, next);
                __syncthreads();
            });
        }
        // drain: team 1's epilogue of the last tile
        hp_unroll<EP>([&](auto I) __attribute__((always_inline)) {
            if constexpr (tm == 1) epilogue(I, my_tiles - 1, true);
            __syncthreads();
        });
    };
    if (team == 0) run(std::integral_constant<int, 0>{});
    else run(std::integral_constant<int, 1>{});
}

}  // namespace mcgmil
