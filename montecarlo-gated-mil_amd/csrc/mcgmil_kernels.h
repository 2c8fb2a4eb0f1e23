#pragma once
// MI355X (gfx950) kernels of the Monte-Carlo-dropout gated-attention MIL hot path.
//
// Reference: MultiHeadGatedAttentionMIL.mc_inference, xkuubix/MonteCarlo-Gated-MIL
// model.py:279-316 (everything after feature extraction). One launch of gate_scores_kernel
// runs ALL T dropout samples of ALL bags of a batch:
//
//   rows  = flattened (bag, t, n), T * sum(N_b) of them, BM per workgroup
//   X     = H[n] (.) keepF[bag,t,n]                          (model.py:280-281, masks in-register)
//   S     = X . [Wv_g ; Wu_g ; wk]^T   one MFMA GEMM per row tile (model.py:285-286 / 297-298, 313)
//   s_c   = sum_d tanh(S_v*sf + bv) sigmoid(S_u*sf + bu) wa_c + ba_c   (model.py:287-290 / 299)
//   s'_c  = s_c * keepA * sa                                  (model.py:291 / 301)
//   z_c   = sf * S_k                                          (classifier folded into the GEMM)
// softmax_pool_kernel then does A = softmax_n(s') and Y_c = sum_n A z_c (model.py:305-316,
// using Y_c = (sum_n A_n H_drop[n]) . k_c = sum_n A_n (H_drop[n] . k_c)), and bag_stats_kernel
// the callers' uncertainty reductions (infer.py:195,212-219; net_utils.py:207-208).
#include "mcgmil_device.h"

namespace mcgmil {

struct GateParams {
    const void* H;
    long long ldh;
    const int32_t* bag_off;
    int B, T, L, D, C, G, P;       // P = G * D / 16 gate tile pairs
    long long total_samples;       // T * total_rows
    const void* Wp;                // packed weights (see pack_weights_kernel)
    uint32_t wp_bytes;             // their size (buffer-descriptor range)
    const float* bv;
    const float* bu;
    const float* wa;
    const float* ba;
    float sf, sa;                  // dropout scales 1/(1-p) (0 for p = 1)
    uint32_t thr_f, thr_a;         // 16-bit drop thresholds
    uint32_t thrx_f;               // packed_threshold(thr_f)
    uint32_t k0, k1;               // Philox key = seed
    uint32_t bag_base;
    int t_base;
    const uint32_t* bag_ids;       // per-bag Philox counters or nullptr (bag_base + b)
    const int32_t* tile_bag;       // bag of each tile's first row (plan_tiles_kernel) or nullptr
    int uniform_rows;              // N if every bag has N rows (arithmetic row map), else 0
    const uint8_t* keep_feat;      // replay masks (parity mode) or nullptr
    const uint8_t* keep_att;
    float* logits;                 // [T*total_rows, C]
    float* zz;                     // [T*total_rows, C]
    // fused kernel (gate_fused_kernel) only: its outputs and its region table
    float* Y;                      // [B, T, C]
    float* A;                      // per bag [T, C, N_b], or nullptr
    const int32_t* region_off;     // [B+1] prefix of per-bag region counts (ragged bags) or nullptr
    int region_t;                  // t-groups per region when every bag has uniform_rows rows
    unsigned long long* stamps;    // diagnostic build only: [tiles][8] s_memtime stamps
    unsigned long long* clock;     // MCGMIL_CLOCK_PROBE: [kClockSlots][4] clock record, or nullptr
    long long tile_row0;           // short-tile launches (gate_pipe_kernel RTV < 8): first row
};

// The clock probe (MCGMIL_CLOCK_PROBE): thread 0 of workgroups 0..kClockSlots-1 writes
// (s_memtime, s_memrealtime) at its start (i = 0) and end (i = 1). Nothing is kept live in
// between: the marks go to memory at once (vector stores). The tile kernels compile it into a
// separate PROBE instantiation, launched only for a probed call: even an untaken branch at the
// kernel's ends re-schedules gate_fused_kernel's tile loop (-11% measured, profiles/r05).
constexpr int kClockSlots = 1024;
__device__ __forceinline__ void clock_probe(const GateParams& p, int i) {
    if (p.clock && threadIdx.x == 0 && blockIdx.x < (unsigned)kClockSlots) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        const unsigned long long r = __builtin_amdgcn_s_memrealtime();
        p.clock[(size_t)blockIdx.x * 4 + 2 * i] = t;
        p.clock[(size_t)blockIdx.x * 4 + 2 * i + 1] = r;
    }
}

// In-kernel phase stamps (diagnostic build, -DMCGMIL_STAMPS; compiled out otherwise): lane 0
// of wave 0 records s_memtime into stamps[tile * 8 + i].
#ifdef MCGMIL_STAMPS
#define MCGMIL_STAMP(p, i)                                                                 \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        if (threadIdx.x == 0 && (p).stamps)                                                 \
            (p).stamps[(size_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime();        \
        __builtin_amdgcn_sched_barrier(0);                                                  \
    } while (0)
#else
#define MCGMIL_STAMP(p, i) do {} while (0)
#endif


constexpr int kGateThreads = 512;  // 8 waves
constexpr int kGateWaves = kGateThreads / kWave;
constexpr int kRowInfo = 6;        // ints per row: hrow, t, n, bag, Nb, bag counter

// ---------------------------------------------------------------------------------------
// Pieces shared by the two gate-score kernels.
// ---------------------------------------------------------------------------------------

// Row table of one BM-row tile of the flattened (bag, t, n) space (threads < BM). With a tile
// plan (bag of the tile's first row) a row walks forward over at most the few bags that start
// inside the tile instead of binary-searching the CSR offsets (dependent L2 loads). Rows from RV
// on are padding (a short tile: its first RV rows only).
template <int BM, int RV = BM>
__device__ __forceinline__ void fill_row_table(const GateParams& p, long long R0, int* rinfo) {
    const int tid = threadIdx.x;
    if (tid >= BM) return;
    const long long R = tid < RV ? R0 + tid : p.total_samples;
    int hrow = -1, t = 0, n = 0, bag = 0, Nb = 0;
    // 32-bit unsigned division when the launch's sample rows fit (wave-uniform branch); the
    // 64-bit one is a ~50-instruction software routine
    const bool narrow = p.total_samples <= 0xFFFFFFFFll;
    if (R < p.total_samples && p.uniform_rows > 0) {
        const long long per_bag = (long long)p.T * p.uniform_rows;
        Nb = p.uniform_rows;
        if (narrow) {
            const uint32_t r = (uint32_t)R, pb = (uint32_t)per_bag;
            bag = (int)(r / pb);
            const uint32_t local = r - (uint32_t)bag * pb;
            t = (int)(local / (uint32_t)Nb);
            n = (int)(local - (uint32_t)t * (uint32_t)Nb);
        } else {
            bag = (int)(R / per_bag);
            const long long local = R - (long long)bag * per_bag;
            t = (int)(local / Nb);
            n = (int)(local - (long long)t * Nb);
        }
        hrow = bag * Nb + n;
    } else if (R < p.total_samples) {
        if (p.tile_bag) {
            bag = p.tile_bag[R0 / BM];
            while ((long long)p.T * p.bag_off[bag + 1] <= R) ++bag;
        } else {
            bag = find_bag(p.bag_off, p.B, p.T, R);
        }
        const int ob = p.bag_off[bag];
        Nb = p.bag_off[bag + 1] - ob;
        const long long local = R - (long long)p.T * ob;
        if (narrow) {
            t = (int)((uint32_t)local / (uint32_t)Nb);
            n = (int)((uint32_t)local - (uint32_t)t * (uint32_t)Nb);
        } else {
            t = (int)(local / Nb);
            n = (int)(local - (long long)t * Nb);
        }
        hrow = ob + n;
    }
    int* ri = rinfo + kRowInfo * tid;
    ri[0] = hrow; ri[1] = t; ri[2] = n; ri[3] = bag; ri[4] = Nb;
    ri[5] = (int)(p.bag_ids ? p.bag_ids[bag] : p.bag_base + (uint32_t)bag);
}

// Tile plan: bag of the first row of every BM-row tile (one thread per tile).
#ifndef MCGMIL_KERNELS_TEMPLATES_ONLY
__global__ void plan_tiles_kernel(const int32_t* bag_off, int B, int T, long long total_samples,
                                  int BM, long long tiles, int32_t* tile_bag) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= tiles) return;
    const long long R = i * BM;
    tile_bag[i] = R < total_samples ? find_bag(bag_off, B, T, R) : 0;
}
#endif

// tanh(x) * sigmoid(y) (reference model.py:183-184 / 287) evaluated as (1-a) / ((1+a)(1+b)),
// a = e^{-2x} = 2^{ax}, b = e^{-y} = 2^{by}, from the pre-scaled arguments
// ax = -2 log2(e) x, by = -log2(e) y (the scaling is folded into the GEMM epilogue FMA):
// two v_exp_f32 + one v_rcp_f32. ax is clamped to +-15 * 2 log2(e), where tanh is already +-1 in
// fp32, so no inf/inf; b = inf (y < -88) gives the correct 0.
__device__ __forceinline__ float gated_product_scaled(float ax, float by) {
    ax = fminf(fmaxf(ax, -43.280851226668903f), 43.280851226668903f);
    const float a = __builtin_amdgcn_exp2f(ax);
    const float b = __builtin_amdgcn_exp2f(by);
    const float ia = 1.0f + a;
    return (1.0f - a) * __builtin_amdgcn_rcpf(fmaf(ia, b, ia));
}

#ifndef MCGMIL_DIAG
#define MCGMIL_DIAG 0               // ablation bits for timing studies (never in the product)
#endif
#ifndef MCGMIL_PHILOX_ROUNDS
#define MCGMIL_PHILOX_ROUNDS 10     // feature-mask rounds in the pipelined K loop (timing studies only)
#endif

constexpr float kM2Log2e = -2.8853900817779268f;   // -2 / ln 2
constexpr float kMLog2e = -1.4426950408889634f;    // -1 / ln 2

// Head vectors of one gate pair as fold_pairs uses them: bv and bu pre-scaled, wa of its class.
struct HeadVec { f32x4 bv, bu, wa; };

template <int PPW>
__device__ __forceinline__ void load_head_vectors(const GateParams& p, int q0, int lane,
                                                  HeadVec (&hv)[PPW]) {
    const int DB = p.D >> 4;
#pragma unroll
    for (int jp = 0; jp < PPW; ++jp) {
        const int q = q0 + jp < p.P ? q0 + jp : p.P - 1;
        const int g = q / DB, db = q - g * DB;
        const int d0 = db * 16 + 4 * (lane >> 4);
        hv[jp].bv = *reinterpret_cast<const f32x4*>(p.bv + (size_t)g * p.D + d0) * kM2Log2e;
        hv[jp].bu = *reinterpret_cast<const f32x4*>(p.bu + (size_t)g * p.D + d0) * kMLog2e;
        hv[jp].wa = *reinterpret_cast<const f32x4*>(p.wa + (size_t)g * p.D + d0);
    }
}

// Fold the gate pairs of one pass into per-lane partial scores. acc[rt][2j] / acc[rt][2j+1]
// hold V / U pre-activations (before the dropout scale) of pair q0 + j for instance
// rt*16 + (lane & 15) and d = 16*db + 4*(lane >> 4) + v (16x16 C layout, weights as A).
// ONE_CLASS: every pair of this wave belongs to gate g and feeds class g only (separate
// heads): one accumulator, part[0]. Otherwise part[c] for every class (shared gate).
template <int RT, int PPW, int MAXC, bool ONE_CLASS, int RTV = RT>
__device__ __forceinline__ void fold_pairs(const GateParams& p, const f32x4 (&acc)[RT][2 * PPW],
                                           int q0, int lane, float (&part)[MAXC][RT],
                                           const HeadVec* pre = nullptr) {
    const int DB = p.D >> 4;
    const float av_s = p.sf * kM2Log2e, au_s = p.sf * kMLog2e;
#pragma unroll
    for (int jp = 0; jp < PPW; ++jp) {
        const int q = q0 + jp;
        if (q >= p.P) break;
        const int g = q / DB, db = q - g * DB;
        const int d0 = db * 16 + 4 * (lane >> 4);
        f32x4 bvv, buv;
        f32x4 coef[MAXC];
        if (ONE_CLASS && pre) {      // loaded before the K loop (load_head_vectors)
            bvv = pre[jp].bv;
            buv = pre[jp].bu;
            coef[0] = pre[jp].wa;
#pragma unroll
            for (int c = 1; c < MAXC; ++c) coef[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
            bvv = *reinterpret_cast<const f32x4*>(p.bv + (size_t)g * p.D + d0);
            buv = *reinterpret_cast<const f32x4*>(p.bu + (size_t)g * p.D + d0);
            bvv *= kM2Log2e;
            buv *= kMLog2e;
#pragma unroll
            for (int c = 0; c < MAXC; ++c) {
                const int cc = ONE_CLASS ? g : c;
                const bool use = ONE_CLASS ? (c == 0) : ((c < p.C) && (p.G == 1 || c == g));
                // address stays inside wa[C, D] for every c; unused classes get 0
                const f32x4 w = *reinterpret_cast<const f32x4*>(p.wa + (size_t)(use ? cc : 0) * p.D + d0);
                coef[c] = use ? w : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int rt = 0; rt < RTV; ++rt) {           // row tiles past RTV: a short tile's padding
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const float ax = fmaf(acc[rt][2 * jp][v], av_s, bvv[v]);
                const float by = fmaf(acc[rt][2 * jp + 1][v], au_s, buv[v]);
                if constexpr (ONE_CLASS) {
#if MCGMIL_DIAG & 8   // ablation (timing only): no transcendentals in the epilogue
                    part[0][rt] = fmaf(fmaf(ax, coef[0][v], by), ax, part[0][rt]);
                    continue;
#endif
                    // wa (1 - a) / ((1 + a)(1 + b)) as two FMAs around the reciprocal
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

// Cross-wave reduction of the partial scores + attention bias, logit dropout and stores
// (model.py:289-291 / 299-301); z = sf * (X . k_c) for the classifier (model.py:313-315).
// Partial scores in LDS: red[wave][class][lane group g][tile row r] -- a lane of a 16x16 (32x32)
// accumulator holds rows r = rt*16 + (lane & 15) (rt*32 + (lane & 31)) for lane group
// g = lane >> 4 (lane >> 5). No cross-lane shuffles; with the row fastest, the stores (one per
// rt) and the scoring thread's reads (it sums the lane groups of every wave holding its class)
// are bank-conflict free.
template <int BM, int MAXC>
__host__ __device__ constexpr int red_floats() { return kGateWaves * MAXC * 4 * BM; }

// one_class >= 0: part[0] holds the wave's scores for class one_class (other classes 0).
// Output item of a thread: row wave*16 + (lane & 15), class lane >> 4 (C <= 4) -- the (row,
// class) whose attention-dropout draw the pipelined kernel may already have made in its K
// loop (have_keep, keep); otherwise it is drawn here.
template <int BM, int MAXC, int ROWS = 16>
__device__ __forceinline__ void finish_scores(const GateParams& p, long long R0,
                                              float (&part)[MAXC][BM / ROWS], f32x4 zacc,
                                              bool zwave, float* red, float* zred,
                                              const int* rinfo, int one_class, int waves_per_gate,
                                              bool have_keep, bool keep, float* lg_out,
                                              float* z_out, long long obase) {
    constexpr int RT = BM / ROWS;
    constexpr int NG = 64 / ROWS;                  // lane groups per accumulator tile
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ncls = one_class < 0 ? MAXC : 1;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if (c >= ncls) break;
        const int cls = one_class < 0 ? c : one_class;
        if (cls >= MAXC) break;                       // idle wave (no pairs)
        float* dst = red + ((size_t)(wave * MAXC + cls) * NG + lane / ROWS) * BM + (lane % ROWS);
#pragma unroll
        for (int q = 0; q < RT; ++q) dst[ROWS * q] = part[c][q];
    }
    if (zwave && lane < 16) {
#pragma unroll
        for (int c = 0; c < MAXC; ++c) zred[c * BM + wave * 16 + lane] = zacc[c];
    }
    MCGMIL_STAMP(p, 5);
    __syncthreads();
    MCGMIL_STAMP(p, 6);
    const int r = wave * 16 + (lane & 15), c = lane >> 4;
    if (r >= BM || c >= p.C) return;
    const int* ri = rinfo + kRowInfo * r;
    if (ri[0] < 0) return;
    // waves holding class c: every wave (waves_per_gate = 0: shared gate) or, one class per
    // wave, the waves w with w / waves_per_gate == c (their other slots are never written)
    float s = 0.f;
    const int nw = waves_per_gate ? waves_per_gate : kGateWaves;
    for (int k = 0; k < nw; ++k) {
        const int w = waves_per_gate ? c * waves_per_gate + k : k;
        const float* src = red + (size_t)(w * MAXC + c) * NG * BM + r;
#pragma unroll
        for (int g = 0; g < NG; ++g) s += src[g * BM];
    }
    s += p.ba[c];
    const int t = ri[1], n = ri[2], bag = ri[3], Nb = ri[4];
    if (p.keep_att) {
        const size_t abase = (size_t)p.T * p.C * (size_t)p.bag_off[bag];
        keep = p.keep_att[abase + ((size_t)t * p.C + c) * Nb + n] != 0;
    } else if (!have_keep) {
        keep = attention_keep(p.k0, p.k1, (uint32_t)ri[5], (uint32_t)(p.t_base + t), (uint32_t)c,
                              (uint32_t)n, p.thr_a);
    }
    // row R0 + r of the flattened (bag, t, n) space -> lg_out / z_out row R0 + r - obase
    const size_t o = (size_t)(R0 + r - obase) * p.C + c;
    lg_out[o] = s * (keep ? p.sa : 0.f);
    z_out[o] = zred[c * BM + r] * p.sf;
}

// ---------------------------------------------------------------------------------------
// softmax_group: one (bag, t) group's softmax over the bag's instances (model.py:305) and
// Y_c = sum_n A z_c (model.py:308-316), by 256 threads (ltid 0..255, 4 waves). lg / zz: the
// group's logits and classifier projections, row-major [Nb][C] (the global workspace, or LDS
// in the fused kernel); Ao: the group's A [C][Nb] (or nullptr); Yo: its Y[C]; sred: 16 floats of
// LDS for this group's waves. Every caller runs this same code, so A and Y are bitwise the
// same whichever kernel computes them. `active` = false executes only the barriers (the idle half
// of a 512-thread workgroup); both halves of a workgroup must pass the same Nb and C.
// ---------------------------------------------------------------------------------------
constexpr int kSoftmaxRows = 16;    // register path for bags of up to 4096 instances

// A is written once and read by the host: MCGMIL_NT_A streams it past L2 (non-temporal), so the
// ~1.6 MB of A a bag writes does not evict the H rows its other regions are about to re-read
#ifndef MCGMIL_NT_A
#define MCGMIL_NT_A 1
#endif
__device__ __forceinline__ void store_a(float* dst, float v) {
#if MCGMIL_NT_A
    __builtin_nontemporal_store(v, dst);
#else
    *dst = v;
#endif
}

__device__ __forceinline__ void softmax_group(int ltid, bool active, int Nb, int C, const float* lg,
                                              const float* zz, float* Ao, float* Yo, float* sred) {
    const int tid = ltid, lane = ltid & 63, wave = ltid >> 6;
    if (Nb == 0) {
        if (active && tid < C) Yo[tid] = 0.f;
        return;
    }
    const int Nl = active ? Nb : 0;                 // rows this thread may touch
    if (C == 2 && Nb <= 256 * kSoftmaxRows) {
        // The reference's two classes together: one 8-byte load per row of logits and of z, and
        // the two classes' reductions share their barriers. Per class the arithmetic and its
        // order are the register path's below, so A and Y are bitwise the same.
        float (*sred2)[4] = reinterpret_cast<float (*)[4]>(sred);
        float e0[kSoftmaxRows], e1[kSoftmaxRows];
        float2 zr[kSoftmaxRows];          // z loaded with the logits: one memory round trip, not two
        float m0 = -INFINITY, m1 = -INFINITY;
#pragma unroll
        for (int k = 0; k < kSoftmaxRows; ++k) {
            const int n = tid + 256 * k;
            float2 l = make_float2(-INFINITY, -INFINITY);
            zr[k] = make_float2(0.f, 0.f);
            if (n < Nl) {
                l = *reinterpret_cast<const float2*>(lg + (size_t)n * 2);
                zr[k] = *reinterpret_cast<const float2*>(zz + (size_t)n * 2);
            }
            e0[k] = l.x;
            e1[k] = l.y;
            m0 = fmaxf(m0, e0[k]);
            m1 = fmaxf(m1, e1[k]);
        }
        m0 = wave_max(m0);
        m1 = wave_max(m1);
        if (lane == 0) { sred2[0][wave] = m0; sred2[1][wave] = m1; }
        __syncthreads();
        m0 = fmaxf(fmaxf(sred2[0][0], sred2[0][1]), fmaxf(sred2[0][2], sred2[0][3]));
        m1 = fmaxf(fmaxf(sred2[1][0], sred2[1][1]), fmaxf(sred2[1][2], sred2[1][3]));
        __syncthreads();
        float s0 = 0.f, y0 = 0.f, s1 = 0.f, y1 = 0.f;
#pragma unroll
        for (int k = 0; k < kSoftmaxRows; ++k) {
            const int n = tid + 256 * k;
            if (n < Nl) {
                const float2 z = zr[k];
                e0[k] = expf(e0[k] - m0);
                e1[k] = expf(e1[k] - m1);
                s0 += e0[k];
                s1 += e1[k];
                y0 = fmaf(e0[k], z.x, y0);
                y1 = fmaf(e1[k], z.y, y1);
            }
        }
        s0 = wave_sum(s0);
        y0 = wave_sum(y0);
        s1 = wave_sum(s1);
        y1 = wave_sum(y1);
        if (lane == 0) {
            sred2[0][wave] = s0; sred2[1][wave] = y0; sred2[2][wave] = s1; sred2[3][wave] = y1;
        }
        __syncthreads();
        s0 = (sred2[0][0] + sred2[0][1]) + (sred2[0][2] + sred2[0][3]);
        y0 = (sred2[1][0] + sred2[1][1]) + (sred2[1][2] + sred2[1][3]);
        s1 = (sred2[2][0] + sred2[2][1]) + (sred2[2][2] + sred2[2][3]);
        y1 = (sred2[3][0] + sred2[3][1]) + (sred2[3][2] + sred2[3][3]);
        __syncthreads();            // sred is free again for the caller's next group
        const float inv0 = 1.0f / s0, inv1 = 1.0f / s1;
        if (Ao) {
            float* Ao1 = Ao + Nb;
#pragma unroll
            for (int k = 0; k < kSoftmaxRows; ++k) {
                const int n = tid + 256 * k;
                if (n < Nl) {
                    store_a(Ao + n, e0[k] * inv0);
                    store_a(Ao1 + n, e1[k] * inv1);
                }
            }
        }
        if (active && tid == 0) { Yo[0] = y0 * inv0; Yo[1] = y1 * inv1; }
        return;
    }
    float (*sr)[4] = reinterpret_cast<float (*)[4]>(sred);
    for (int c = 0; c < C; ++c) {
        if (Nb <= 256 * kSoftmaxRows) {
            // the bag's logits of class c stay in registers: one read of logits and z, one exp
            // per row (same per-thread order and reduction tree as the streaming path below)
            float e[kSoftmaxRows];
            float m = -INFINITY;
#pragma unroll
            for (int k = 0; k < kSoftmaxRows; ++k) {
                const int n = tid + 256 * k;
                e[k] = n < Nl ? lg[(size_t)n * C + c] : -INFINITY;
                m = fmaxf(m, e[k]);
            }
            m = wave_max(m);
            if (lane == 0) sr[0][wave] = m;
            __syncthreads();
            m = fmaxf(fmaxf(sr[0][0], sr[0][1]), fmaxf(sr[0][2], sr[0][3]));
            __syncthreads();
            float s = 0.f, y = 0.f;
#pragma unroll
            for (int k = 0; k < kSoftmaxRows; ++k) {
                const int n = tid + 256 * k;
                if (n < Nl) {
                    e[k] = expf(e[k] - m);
                    s += e[k];
                    y = fmaf(e[k], zz[(size_t)n * C + c], y);
                }
            }
            s = wave_sum(s);
            y = wave_sum(y);
            if (lane == 0) { sr[0][wave] = s; sr[1][wave] = y; }
            __syncthreads();
            s = (sr[0][0] + sr[0][1]) + (sr[0][2] + sr[0][3]);
            y = (sr[1][0] + sr[1][1]) + (sr[1][2] + sr[1][3]);
            __syncthreads();
            const float inv = 1.0f / s;
            if (Ao) {
                float* Aoc = Ao + (size_t)c * Nb;
#pragma unroll
                for (int k = 0; k < kSoftmaxRows; ++k) {
                    const int n = tid + 256 * k;
                    if (n < Nl) store_a(Aoc + n, e[k] * inv);
                }
            }
            if (active && tid == 0) Yo[c] = y * inv;
            continue;
        }
        float m = -INFINITY;
        for (int n = tid; n < Nl; n += 256) m = fmaxf(m, lg[(size_t)n * C + c]);
        m = wave_max(m);
        if (lane == 0) sr[0][wave] = m;
        __syncthreads();
        m = fmaxf(fmaxf(sr[0][0], sr[0][1]), fmaxf(sr[0][2], sr[0][3]));
        __syncthreads();
        float s = 0.f, y = 0.f;
        for (int n = tid; n < Nl; n += 256) {
            const size_t o = (size_t)n * C + c;
            const float e = expf(lg[o] - m);
            s += e;
            y = fmaf(e, zz[o], y);
        }
        s = wave_sum(s);
        y = wave_sum(y);
        if (lane == 0) { sr[0][wave] = s; sr[1][wave] = y; }
        __syncthreads();
        s = (sr[0][0] + sr[0][1]) + (sr[0][2] + sr[0][3]);
        y = (sr[1][0] + sr[1][1]) + (sr[1][2] + sr[1][3]);
        __syncthreads();
        const float inv = 1.0f / s;
        if (Ao) {
            float* Aoc = Ao + (size_t)c * Nb;
            for (int n = tid; n < Nl; n += 256) store_a(Aoc + n, expf(lg[(size_t)n * C + c] - m) * inv);
        }
        if (active && tid == 0) Yo[c] = y * inv;
    }
}

// softmax_pool_kernel: one 256-thread block per (t, bag) over the gate kernel's workspace.
#ifndef MCGMIL_KERNELS_TEMPLATES_ONLY
__global__ __launch_bounds__(256) void softmax_pool_kernel(const int32_t* bag_off, int T, int C,
                                                           const float* logits, const float* zz,
                                                           float* Y, float* A) {
    __shared__ float sred[16];
    const int t = blockIdx.x, b = blockIdx.y;
    const int ob = bag_off[b];
    const int Nb = bag_off[b + 1] - ob;
    const size_t R0 = (size_t)T * ob + (size_t)t * Nb;
    softmax_group(threadIdx.x, true, Nb, C, logits + R0 * C, zz + R0 * C,
                  A ? A + (size_t)T * C * ob + (size_t)t * C * Nb : nullptr,
                  Y + ((size_t)b * T + t) * C, sred);
}
#endif

// ---------------------------------------------------------------------------------------
// gate_pipe_kernel -- the fast path (gate tile pairs P <= 16, i.e. one pass: the reference's
// C=2/D=128 heads, shared or separate). One workgroup = 128 rows of the flattened (bag, t, n)
// space, 8 waves. The masked features are never materialised whole: the K loop runs over
// 32-deep steps and, while the MFMAs consume step s from one LDS slot, every thread draws
// ONE Philox4x32-10 block (8 keep decisions = its 8-element fragment chunk) for step s+1,
// masks the H chunk it loaded one step earlier and writes it into the other slot (one
// barrier per step). Wave w owns gate tile pairs w*PPW .. w*PPW+PPW-1 for all 128 rows,
// weight fragments streamed from L2 one step ahead, plus the classifier tile for row tile w.
// ---------------------------------------------------------------------------------------
template <typename E> struct Raw;
template <> struct Raw<__bf16> { uint4 v; };
template <> struct Raw<float> { f32x4 lo, hi; };
__device__ __forceinline__ Raw<__bf16> load_raw(const __bf16* p) {
    Raw<__bf16> r; r.v = *reinterpret_cast<const uint4*>(p); return r;
}
__device__ __forceinline__ Raw<float> load_raw(const float* p) {
    Raw<float> r;
    r.lo = *reinterpret_cast<const f32x4*>(p);
    r.hi = *reinterpret_cast<const f32x4*>(p + 4);
    return r;
}
__device__ __forceinline__ void store_masked(const Raw<__bf16>& h, uint32_t kb, __bf16* dst) {
    uint4 v = h.v;
    v.x &= ((kb & 1u) ? 0x0000FFFFu : 0u) | ((kb & 2u) ? 0xFFFF0000u : 0u);
    v.y &= ((kb & 4u) ? 0x0000FFFFu : 0u) | ((kb & 8u) ? 0xFFFF0000u : 0u);
    v.z &= ((kb & 16u) ? 0x0000FFFFu : 0u) | ((kb & 32u) ? 0xFFFF0000u : 0u);
    v.w &= ((kb & 64u) ? 0x0000FFFFu : 0u) | ((kb & 128u) ? 0xFFFF0000u : 0u);
    *reinterpret_cast<uint4*>(dst) = v;
}
__device__ __forceinline__ void store_masked(const Raw<float>& h, uint32_t kb, float* dst) {
    f32x4 a = h.lo, b = h.hi;
    a.x = (kb & 1u) ? a.x : 0.f;   a.y = (kb & 2u) ? a.y : 0.f;
    a.z = (kb & 4u) ? a.z : 0.f;   a.w = (kb & 8u) ? a.w : 0.f;
    b.x = (kb & 16u) ? b.x : 0.f;  b.y = (kb & 32u) ? b.y : 0.f;
    b.z = (kb & 64u) ? b.z : 0.f;  b.w = (kb & 128u) ? b.w : 0.f;
    *reinterpret_cast<f32x4*>(dst) = a;
    *reinterpret_cast<f32x4*>(dst + 4) = b;
}

// Stage 8 features with the keep rule applied straight to the Philox words (2 draws each).
// `o` comes from philox4x32_10<true>: words x and z are already sign-flipped.
__device__ __forceinline__ void store_dropped(const Raw<__bf16>& h, uint4 o, uint32_t thrx,
                                              uint32_t inval, __bf16* dst) {
    // v & ~(drop | inval) as one v_bitop3_b32 (truth table 0x10: a & ~b & ~c)
    uint4 v = h.v;
    v.x = __builtin_amdgcn_bitop3_b32(v.x, drop_mask16x2_flipped(o.x, thrx), inval, 0x10);
    v.y = __builtin_amdgcn_bitop3_b32(v.y, drop_mask16x2(o.y, thrx), inval, 0x10);
    v.z = __builtin_amdgcn_bitop3_b32(v.z, drop_mask16x2_flipped(o.z, thrx), inval, 0x10);
    v.w = __builtin_amdgcn_bitop3_b32(v.w, drop_mask16x2(o.w, thrx), inval, 0x10);
    *reinterpret_cast<uint4*>(dst) = v;
}
__device__ __forceinline__ uint32_t keep_lo(uint32_t m) { return ~(uint32_t)((int32_t)(m << 16) >> 16); }
__device__ __forceinline__ uint32_t keep_hi(uint32_t m) { return ~(uint32_t)((int32_t)m >> 16); }
__device__ __forceinline__ void store_dropped(const Raw<float>& h, uint4 o, uint32_t thrx,
                                              uint32_t inval, float* dst) {
    const uint32_t m0 = drop_mask16x2_flipped(o.x, thrx) | inval, m1 = drop_mask16x2(o.y, thrx) | inval;
    const uint32_t m2 = drop_mask16x2_flipped(o.z, thrx) | inval, m3 = drop_mask16x2(o.w, thrx) | inval;
    f32x4 a = h.lo, b = h.hi;
    a.x = __uint_as_float(__float_as_uint(a.x) & keep_lo(m0));
    a.y = __uint_as_float(__float_as_uint(a.y) & keep_hi(m0));
    a.z = __uint_as_float(__float_as_uint(a.z) & keep_lo(m1));
    a.w = __uint_as_float(__float_as_uint(a.w) & keep_hi(m1));
    b.x = __uint_as_float(__float_as_uint(b.x) & keep_lo(m2));
    b.y = __uint_as_float(__float_as_uint(b.y) & keep_hi(m2));
    b.z = __uint_as_float(__float_as_uint(b.z) & keep_lo(m3));
    b.w = __uint_as_float(__float_as_uint(b.w) & keep_hi(m3));
    *reinterpret_cast<f32x4*>(dst) = a;
    *reinterpret_cast<f32x4*>(dst + 4) = b;
}

constexpr int kPipeBM = 128;
#ifndef MCGMIL_VPM
#define MCGMIL_VPM 2
#endif
constexpr int VPM = MCGMIL_VPM;   // VALU instructions scheduled after each MFMA in a K step
#ifndef MCGMIL_SCHED
#define MCGMIL_SCHED 0
#endif
constexpr int HD = 2;               // H prefetch distance of the pipelined kernel, in K steps (the
                                    // h / hn register rotation of the unrolled loop assumes 2)
// staging slots of the pipelined K loop (a half-step stagger of waves 4-7 needed three; measured
// 20% slower and removed, profiles/r04/gate_ab_r04.log run 2, code in commit 9d17683)
template <typename E>
__host__ __device__ constexpr int pipe_slots() { return 2; }

template <typename E, int MAXC>
__host__ __device__ constexpr size_t pipe_lds_bytes() {
    return (size_t)pipe_slots<E>() * kPipeBM * 32 * sizeof(E) + (size_t)red_floats<kPipeBM, MAXC>() * 4 +
           (size_t)MAXC * kPipeBM * 4 + (size_t)kRowInfo * kPipeBM * 4;
}

// The classifier tile's packed fragments of all KS K steps (tile 2P of the packed weights) into
// LDS [KS][64][8], by the whole workgroup; the caller's next barrier makes them visible.
template <typename E>
__device__ __forceinline__ void load_classifier_lds(__amdgpu_buffer_rsrc_t wrs, uint32_t zsoff, int KS, E* zw) {
    for (int i = threadIdx.x; i < KS * 64; i += kGateThreads)
        *reinterpret_cast<f32x4*>(zw + (size_t)i * 8) = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, (uint32_t)i * 8u * (uint32_t)sizeof(E), zsoff, 0));
}

// One 128-row tile of the flattened (bag, t, n) space, rows R0 .. R0+127, whose row table is
// already in `rinfo` (and visible: the caller's barrier). Scores go to lg_out / z_out at row
// R0 + r - obase. LDS: Xs [2][SLOT] staging slots, red / zred the cross-wave reductions.
// RTV < 8 (a short tile, gate_pipe_kernel's tail launch): row tiles RTV.. are padding -- no
// MFMAs, no staging, no H loads and no epilogue for them; every row computes exactly as in a full
// tile (same K order, same cross-wave sum), so the scores are bitwise the same.
template <typename E, int PPW, int MAXC, bool REPLAY, bool ONE_CLASS, bool EARLY_HV = true,
          bool ZL = false, bool ZLOAD = true, int RTV = kPipeBM / 16>
__device__ __forceinline__ void pipe_tile(const GateParams& p, long long R0, E* Xs, float* red,
                                          float* zred, const int* rinfo, float* lg_out,
                                          float* z_out, long long obase, E* zw = nullptr) {
    constexpr int BM = kPipeBM;
    constexpr int RT = BM / 16;                     // 8 row tiles = 8 waves
    constexpr int NJ = 2 * PPW;
    constexpr int SLOT = RT * 64 * 8;               // elements of one 32-deep K step
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int KS = p.L >> 5;

    // staging item of this thread: row wave*16 + (lane & 15), 8-chunk kq = lane >> 4 of
    // every K step; it lands at lane slot `lane` of row tile `wave` (= element tid*8)
    const int* ri = rinfo + kRowInfo * (wave * 16 + (lane & 15));
    const int hrow = ri[0];
    const bool valid = hrow >= 0;
    const int kq = lane >> 4;
    const E* hsrc = reinterpret_cast<const E*>(p.H) + (size_t)(valid ? hrow : 0) * p.ldh + kq * 8;
    const uint32_t cn = (uint32_t)ri[2], ct = (uint32_t)(p.t_base + ri[1]), cb = (uint32_t)ri[5];
    // replay row (row 0 for padding rows, whose bits are masked off by vmask)
    const uint8_t* kfe = REPLAY ? p.keep_feat + (size_t)(valid ? R0 + wave * 16 + (lane & 15) : 0) *
                                                    (p.L >> 3) + kq
                                : nullptr;

    const uint32_t inval = valid ? 0u : 0xFFFFFFFFu;   // padding rows stage zeros
    auto stage = [&](int s, const Raw<E>& h, E* slot) {
        if constexpr (REPLAY) {
            const uint32_t kb = kfe[(size_t)(s < KS ? s : KS - 1) * 4];  // step KS: dummy, in-row
            store_masked(h, kb & ~inval, slot + tid * 8);
        } else {   // (the staging of step KS lands in the idle slot and is never read)
#if MCGMIL_DIAG & 4   // ablation: no Philox (keep pattern from the counters)
            const uint4 o = make_uint4(cn * 0x9E3779B9u + (uint32_t)s, ct ^ cb, cn + ct, (uint32_t)s * 77u);
#else
            const uint4 o = philox4x32_10<true, MCGMIL_PHILOX_ROUNDS>((uint32_t)(s * 4 + kq), cn, ct, cb, p.k0, p.k1);
#endif
            store_dropped(h, o, p.thrx_f, inval, slot + tid * 8);
        }
    };

    // weight tiles of this wave (idle pair slots read a valid tile; fold_pairs skips them).
    // Buffer loads: one descriptor over the packed weights, the lane's byte offset as voffset
    // and the wave-uniform tile + step offset as soffset, so the per-step address arithmetic
    // is SALU only (no 64-bit VALU pointer increments in the K loop).
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

    f32x4 acc[RT][NJ];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 zacc = {0.f, 0.f, 0.f, 0.f};

    // One K step: MFMAs on step s from slot `cur` with weights (w, z); meanwhile prefetch the
    // weights of step s+1 into (wn, zn) and the H chunk of step s+HD into hn, and stage step
    // s+1 (from h, loaded one step earlier) into slot `nxt`. Loop-carried values alternate
    // between two NAMED register sets (the loop is unrolled by two), so no register copy
    // forces an early wait on the prefetches.
    // (The compiler issues the prefetches late in the step, next to the barrier. Forcing them
    // to the top of the step or after the first 2-12 MFMAs measured 2-4% slower.)
    auto kstep = [&](int s, const E* cur, E* nxt, const Frag<E> (&w)[NJ], const Frag<E>& z,
                     Frag<E> (&wn)[NJ], Frag<E>& zn, const Raw<E>& h, Raw<E>& hn) {
        const int s1 = s + 1 < KS ? s + 1 : KS - 1;          // clamped: no branch in the body
        const int sh = s + HD < KS ? s + HD : KS - 1;
#if MCGMIL_DIAG & 2   // ablation: no weight prefetch
#pragma unroll
        for (int j = 0; j < NJ; ++j) wn[j] = w[j];
        zn = z;
#else
#pragma unroll
        for (int j = 0; j < NJ; ++j) wn[j] = wfrag(wsoff[j] + (uint32_t)s1 * kStepBytes);
        if constexpr (!ZL) zn = wfrag(zsoff + (uint32_t)s1 * kStepBytes);
#endif
#if MCGMIL_DIAG & 1   // ablation (timing only, wrong results): no H prefetch
        hn = h;
#else
        if (RTV == RT || wave < RTV) hn = load_raw(hsrc + (size_t)sh * 32);
#endif
#pragma unroll
        for (int rt = 0; rt < RTV; ++rt) {
            const Frag<E> x = load_frag(cur + (size_t)(rt * 64 + lane) * 8);
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[rt][j] = mma(w[j], x, acc[rt][j]);
        }
        const Frag<E> xz = load_frag(cur + (size_t)tid * 8);  // row tile `wave`
        if constexpr (ZL) zacc = mma(load_frag(zw + (size_t)(s * 64 + lane) * 8), xz, zacc);
        else zacc = mma(z, xz, zacc);
        if (RTV == RT || wave < RTV) stage(s + 1, h, nxt);   // step KS: the idle slot, never read
        if constexpr (sizeof(E) == 2 && PPW == 2) {
            // Spread the Philox/staging VALU over the MFMA stream (1 MFMA : VPM VALU) instead
            // of one block after it: the two waves of a SIMD run the step in lockstep, so a
            // trailing VALU block would not overlap the partner's MFMAs.
#if MCGMIL_SCHED == 1
            // + the global prefetches first and the LDS operand reads two row tiles ahead
            __builtin_amdgcn_sched_group_barrier(0x020, NJ + 2, 0);  // VMEM reads (W, z, H)
            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);       // DS reads x0, x1, xz
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
                }
                if (rt + 2 < RT) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);       // z
            __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
#else
#pragma unroll
            for (int i = 0; i < RTV * NJ + 1; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0); // VALU
            }
#endif
        }
#if MCGMIL_DIAG & 128   // ablation (timing only, wrong results): no barrier between K steps
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
        __syncthreads();
#endif
    };

    // bf16 separate heads: the epilogue's head vectors load under the K loop instead of after it
    // (+0.3-1.4% in same-process A/B, bitwise equal; profiles/r02/gate_ab.log). The fp32 kernel
    // has no registers to spare for them.
    constexpr bool kEarlyHV = EARLY_HV && ONE_CLASS && sizeof(E) == 2;
    HeadVec hvec[PPW];
    {
        // prologue: stage step 0, load the weights of step 0 and H of step 1
        Frag<E> wA[NJ], wB[NJ], zA, zB;
        Raw<E> hA{}, hB{};
        if (RTV == RT || wave < RTV) {
            hA = load_raw(hsrc);
            hB = load_raw(hsrc + 32);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) wA[j] = wfrag(wsoff[j]);
        if constexpr (ZL) {
            // ZL: the classifier tile's fragments of all K steps sit in LDS (ZLOAD: loaded here, by
            // this tile; else by the caller, once), so the K loop reads them with one ds_read per
            // wave instead of 8 waves fetching the same 1 KiB per step. Visible after the barrier.
            if constexpr (ZLOAD) load_classifier_lds<E>(wrs, zsoff, KS, zw);
        } else {
            zA = wfrag(zsoff);
        }
        if (RTV == RT || wave < RTV) stage(0, hA, Xs);
        __syncthreads();
        MCGMIL_STAMP(p, 2);

        if constexpr (kEarlyHV) load_head_vectors<PPW>(p, q0, lane, hvec);
        // KS is even and >= 2 (host guarantees L % 64 == 0). The first two steps are peeled: their
        // MFMAs take the zero accumulators as an inline-constant C operand, so no register copies of
        // the 132 zeroed accumulators are made on the way into the loop.
        kstep(0, Xs, Xs + SLOT, wA, zA, wB, zB, hB, hA);
        kstep(1, Xs + SLOT, Xs, wB, zB, wA, zA, hA, hB);
#if MCGMIL_DIAG & 16   // ablation (timing only): 2 of the KS K steps
        if (KS > 1000)
#endif
        for (int s = 2; s < KS; s += 2) {
            kstep(s, Xs, Xs + SLOT, wA, zA, wB, zB, hB, hA);
            kstep(s + 1, Xs + SLOT, Xs, wB, zB, wA, zA, hA, hB);
        }
    }
    MCGMIL_STAMP(p, 3);

    float part[MAXC][RT];
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) part[c][rt] = 0.f;
    fold_pairs<RT, PPW, MAXC, ONE_CLASS, RTV>(p, acc, q0, lane, part, kEarlyHV ? hvec : nullptr);
    MCGMIL_STAMP(p, 4);
    // ONE_CLASS: the wave's pairs all belong to gate q0 / (D/16) (idle waves: class >= C)
    const int one_class = ONE_CLASS ? (q0 < p.P ? q0 / (p.D >> 4) : MAXC) : -1;
    finish_scores<BM, MAXC>(p, R0, part, zacc, true, red, zred, rinfo, one_class,
                            ONE_CLASS ? (p.D >> 4) / PPW : 0, false, true, lg_out, z_out, obase);
    MCGMIL_STAMP(p, 7);
}

// XCD-aware tile order of the two-kernel gate launches (guide T1, bijective form): workgroup b runs
// logical tile xcd_tile(b, n). Workgroups are dealt to the 8 XCDs round-robin (b % 8), so each XCD
// gets one contiguous chunk of the (bag, t, n)-ordered tiles: all T samples of a bag run on one
// XCD and re-read its H rows from that XCD's L2. With the identity order a ragged bag's tile
// boundaries shift from sample to sample, each XCD saw every bag, and config 4's launch fetched
// 3.7x its algorithmic bytes (profiles/r06/gate_traffic_cfg4.json). Every tile's arithmetic is
// unchanged, so outputs are bitwise the same. Batches of fewer than 8 bags keep the identity
// order: there a chunk would make every XCD read the whole bag, and the one-bag-per-call path
// measured 1-3% slower with it (profiles/r06/xcd_tiles/). MCGMIL_XCD_TILES=0 (A/B builds):
// identity order always.
#ifndef MCGMIL_XCD_TILES
#define MCGMIL_XCD_TILES 1
#endif
__device__ __forceinline__ long long xcd_tile(unsigned b, unsigned n, int bags) {
#if MCGMIL_XCD_TILES
    const unsigned x = b & 7u, q = n >> 3, r = n & 7u;
    const unsigned l = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
    return (long long)(bags >= 8 ? l : b);
#else
    (void)n;
    (void)bags;
    return (long long)b;
#endif
}

// RTV < 8: the tail launch of short tiles (16 RTV rows each from p.tile_row0), so that a last
// round of tiles that would leave most CUs idle is spread over them (launch_gate_pipe)
template <typename E, int PPW, int MAXC, bool REPLAY, bool ONE_CLASS, bool PROBE = false, int RTV = kPipeBM / 16>
__global__ __launch_bounds__(kGateThreads) void gate_pipe_kernel(const GateParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BM = kPipeBM;
    E* Xs = reinterpret_cast<E*>(smem);                                   // [2][SLOT]
    float* red = reinterpret_cast<float*>(smem + (size_t)pipe_slots<E>() * BM * 32 * sizeof(E));
    float* zred = red + red_floats<BM, MAXC>();
    int* rinfo = reinterpret_cast<int*>(zred + MAXC * BM);
    const long long R0 = RTV == BM / 16 ? xcd_tile(blockIdx.x, gridDim.x, p.B) * BM
                                        : p.tile_row0 + (long long)blockIdx.x * (16 * RTV);

    if constexpr (PROBE) clock_probe(p, 0);
    MCGMIL_STAMP(p, 0);
    fill_row_table<BM, 16 * RTV>(p, R0, rinfo);
    __syncthreads();
    MCGMIL_STAMP(p, 1);
    pipe_tile<E, PPW, MAXC, REPLAY, ONE_CLASS, true, false, true, RTV>(p, R0, Xs, red, zred, rinfo, p.logits,
                                                                       p.zz, 0);
    if constexpr (PROBE) clock_probe(p, 1);
}

// ---------------------------------------------------------------------------------------
// gate_fused_kernel -- the whole hot path in ONE launch (model.py:280-316): gate scores,
// softmax over instances and attention pooling. A workgroup owns a REGION: the t-groups
// [t0, t1) of one bag, i.e. the contiguous flattened rows [S, S + (t1-t0)*N_b). It runs the
// region's 128-row tiles one after the other through pipe_tile (the code of gate_pipe_kernel,
// so the logits are bitwise the same), keeping the logits and classifier projections in LDS,
// then runs softmax_group on each t-group, two at a time (threads 0-255 and 256-511): A and
// Y are written once and no logit leaves the CU. Bags of more than fused_cap instances keep
// one t-group per region and go through the global workspace instead (the workgroup re-reads
// its own writes).
// ---------------------------------------------------------------------------------------
#ifndef MCGMIL_FUSED_XCD
#define MCGMIL_FUSED_XCD 1         // 1: regions of bag b on XCD b % 8 (uniform bags, B % 8 == 0)
#endif
#ifndef MCGMIL_FUSED_EARLY_HV
#define MCGMIL_FUSED_EARLY_HV 0   // 1: head vectors before the K loop (as gate_pipe_kernel); in the
                                  // tile loop they left the K loop 16 VGPRs short, and the compiler
                                  // then waited on every B-fragment read (15.6 vs 13.7 ms, gate_ab_r03.log)
#endif
#ifndef MCGMIL_FUSED_NMAJOR
#define MCGMIL_FUSED_NMAJOR 1
#endif
#ifndef MCGMIL_FUSED_CAP
#define MCGMIL_FUSED_CAP 4096      // rows of one region's logits in LDS (C <= 2)
#endif
template <int MAXC>
__host__ __device__ constexpr int fused_cap() { return MAXC <= 2 ? MCGMIL_FUSED_CAP : MCGMIL_FUSED_CAP / 4; }

template <typename E, int MAXC>
__host__ __device__ constexpr size_t fused_lds_bytes() {
    return pipe_lds_bytes<E, MAXC>() + (size_t)kRowInfo * kPipeBM * 4   // second row table
           + (size_t)2 * fused_cap<MAXC>() * MAXC * 4                   // logits + z of a region
           + (size_t)2 * 16 * 4 + 64;                                   // softmax partials, region
}

// bf16: the classifier tile's weight fragments of every K step stay in LDS for the workgroup's
// whole region (L/32 KiB after the rest), loaded once instead of per wave and K step
#ifndef MCGMIL_FUSED_ZL
#define MCGMIL_FUSED_ZL 1
#endif
template <typename E>
__host__ __device__ constexpr bool fused_zl() { return MCGMIL_FUSED_ZL && sizeof(E) == 2; }
template <typename E, int MAXC>
__host__ __device__ constexpr size_t fused_kernel_lds_bytes(int L) {
    return fused_lds_bytes<E, MAXC>() + (fused_zl<E>() ? (size_t)(L / 32) * 512 * sizeof(E) : 0);
}

// t-groups per region for a bag of Nb instances (the host sizes the grid with the same rule)
__host__ __device__ inline int region_t_groups(int Nb, int T, int cap) {
    if (Nb <= 0) return T;
    if (Nb > cap) return 1;
    const int ts = cap / Nb;
    return ts < T ? ts : T;
}

struct Region {
    int bag, t0, t1, Nb, ob;
    int ntiles;                    // 128-row tiles
    long long S, rows;
};

// Tile i of a region's run order. MCGMIL_FUSED_NMAJOR: when the region is G > 1 t-groups of
// whole tiles, instance-block major -- tile i reads the same 128 H rows as tile i-1 for G-1 of
// every G tiles, so each block comes from beyond L2 once per region instead of G times. The order
// changes no result: every tile's logits land at their own rows, and the softmax runs after the
// last tile.
__device__ __forceinline__ int region_tile(const Region& rg, int i) {
#if MCGMIL_FUSED_NMAJOR
    const int G = rg.t1 - rg.t0;
    if (G > 1 && rg.Nb % kPipeBM == 0) return (i % G) * (rg.Nb / kPipeBM) + i / G;
#endif
    return i;
}

// The kernel's parameters (its only argument, at offset 0 of the kernarg segment) read again
// through a pointer the compiler cannot see through, so the loads stay where they are used.
__device__ __forceinline__ GateParams reload_kernarg_params(const GateParams& p) {
#if __HIP_DEVICE_COMPILE__
    typedef __attribute__((address_space(4))) const GateParams* KernargParams;
    KernargParams q = (KernargParams)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(q));
    return *q;
#else
    return p;
#endif
}

__device__ __forceinline__ bool decode_region(const GateParams& p, int g, int cap, Region& rg) {
    int b, j, ts;
    if (p.uniform_rows > 0) {
        ts = p.region_t;
        const int rpb = (p.T + ts - 1) / ts;
        if (MCGMIL_FUSED_XCD && (p.B & 7) == 0) {
            // workgroups g and g + 8 share an XCD (round-robin dispatch): XCD x = g & 7 takes the
            // bags b = x (mod 8), so the ~32 workgroups of an XCD work on one bag's rows at a
            // time and share its H rows in that XCD's L2
            const int k = g >> 3;
            b = 8 * (k / rpb) + (g & 7);
            j = k - (k / rpb) * rpb;
        } else {
            b = g / rpb;
            j = g - b * rpb;
        }
        if (b >= p.B) return false;
    } else {
        if (g >= p.region_off[p.B]) return false;
        b = find_bag(p.region_off, p.B, 1, g);   // region counts are >= 1: strictly increasing
        j = g - p.region_off[b];
        ts = region_t_groups(p.bag_off[b + 1] - p.bag_off[b], p.T, cap);
    }
    rg.bag = b;
    rg.ob = p.bag_off[b];
    rg.Nb = p.bag_off[b + 1] - rg.ob;
    rg.t0 = j * ts;
    rg.t1 = rg.t0 + ts < p.T ? rg.t0 + ts : p.T;
    rg.S = (long long)p.T * rg.ob + (long long)rg.t0 * rg.Nb;
    rg.rows = (long long)(rg.t1 - rg.t0) * rg.Nb;
    rg.ntiles = (int)((rg.rows + kPipeBM - 1) / kPipeBM);
    return true;
}

// Row table of one tile of a region (rows past the region's end are padding).
template <int BM>
__device__ __forceinline__ void fill_row_table_region(const GateParams& p, const Region& rg,
                                                      long long R0, int* rinfo) {
    const int tid = threadIdx.x;
    if (tid >= BM) return;
    const long long rho = R0 + tid - rg.S;
    int hrow = -1, t = 0, n = 0;
    if (rho < rg.rows) {
        const uint32_t r = (uint32_t)rho;          // a region is one t-group or <= fused_cap rows
        const uint32_t tt = r / (uint32_t)rg.Nb;
        n = (int)(r - tt * (uint32_t)rg.Nb);
        t = rg.t0 + (int)tt;
        hrow = rg.ob + n;
    }
    int* ri = rinfo + kRowInfo * tid;
    ri[0] = hrow; ri[1] = t; ri[2] = n; ri[3] = rg.bag; ri[4] = rg.Nb;
    ri[5] = (int)(p.bag_ids ? p.bag_ids[rg.bag] : p.bag_base + (uint32_t)rg.bag);
}


template <typename E, int PPW, int MAXC, bool ONE_CLASS, bool PROBE = false>
__global__ __launch_bounds__(kGateThreads) void gate_fused_kernel(const GateParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BM = kPipeBM;
    constexpr int CAP = fused_cap<MAXC>();
    E* Xs = reinterpret_cast<E*>(smem);                                   // [2][SLOT]
    float* red = reinterpret_cast<float*>(smem + (size_t)pipe_slots<E>() * BM * 32 * sizeof(E));
    float* zred = red + red_floats<BM, MAXC>();
    int* rinfo = reinterpret_cast<int*>(zred + MAXC * BM);               // [2][kRowInfo * BM]
    float* slg = reinterpret_cast<float*>(rinfo + 2 * kRowInfo * BM);    // [CAP][C]
    float* szz = slg + CAP * MAXC;                                        // [CAP][C]
    float* sred = szz + CAP * MAXC;                                       // [2][16]

#if MCGMIL_DIAG & 64   // diagnostic (timing only): gate_pipe_kernel's work in this kernel's frame
    {
        const long long R0 = (long long)blockIdx.x * BM;
        fill_row_table<BM>(p, R0, rinfo);
        __syncthreads();
        pipe_tile<E, PPW, MAXC, false, ONE_CLASS>(p, R0, Xs, red, zred, rinfo, p.logits, p.zz, 0);
        return;
    }
#endif
    Region rg;
    if (!decode_region(p, (int)blockIdx.x, CAP, rg)) return;   // grid rounded up (ragged bags)
    if constexpr (PROBE) clock_probe(p, 0);
    const int ntiles = (int)((rg.rows + BM - 1) / BM);
    // The tile loop keeps almost nothing in registers across tiles: the region sits in LDS and
    // the parameters are re-read from the kernarg segment in every tile, both through pointers
    // the compiler cannot see through. Hoisted out of the loop, the ~40 scalar parameters and
    // the region stay live across it, and the SGPR spills (into VGPR lanes) push the tile over
    // 256 VGPRs.
    Region* srg = reinterpret_cast<Region*>(sred + 32);
    if (threadIdx.x == 0) *srg = rg;
    __syncthreads();                                 // *srg is read by every wave from tile 0 on
    E* zw = reinterpret_cast<E*>(smem + fused_lds_bytes<E, MAXC>());
    if constexpr (fused_zl<E>())
        load_classifier_lds<E>(make_rsrc(p.Wp, p.wp_bytes), (uint32_t)(2 * p.P) * (uint32_t)(p.L >> 5) * 512u *
                                   (uint32_t)sizeof(E), p.L >> 5, zw);   // visible after tile 0's first barrier
    for (int i = 0; i < ntiles; ++i) {
        Region* qr = srg;
        asm volatile("" : "+v"(qr));
        const GateParams pt = reload_kernarg_params(p);
        // two row tables: tile i fills one while tile i-1's scoring may still read the other
        int* ri = rinfo + (i & 1) * kRowInfo * BM;
        MCGMIL_STAMP(pt, 0);
        {
            const Region r = *qr;
            fill_row_table_region<BM>(pt, r, r.S + (long long)region_tile(r, i) * BM, ri);
        }
        __syncthreads();
        MCGMIL_STAMP(pt, 1);
        const Region r = *qr;
        const bool lds = r.Nb <= CAP;
        pipe_tile<E, PPW, MAXC, false, ONE_CLASS, MCGMIL_FUSED_EARLY_HV, fused_zl<E>(), false>(
            pt, r.S + (long long)region_tile(r, i) * BM, Xs, red, zred, ri, lds ? slg : pt.logits,
            lds ? szz : pt.zz, lds ? r.S : 0, zw);
    }
    __syncthreads();
#if MCGMIL_DIAG & 32   // ablation (timing only, no A/Y): no softmax phase
    if (ntiles >= 0) return;
#endif
    rg = *srg;
    const bool in_lds = rg.Nb <= CAP;

    // softmax + pooling per t-group (model.py:305-316), two groups at a time
    const int G = rg.t1 - rg.t0;
    const int half = threadIdx.x >> 8, ltid = threadIdx.x & 255;
    for (int j0 = 0; j0 < G; j0 += 2) {
        const bool act = j0 + half < G;
        const int j = act ? j0 + half : j0;
        const long long row0 = (long long)j * rg.Nb;                    // first row in the region
        const float* lgj = in_lds ? slg + row0 * p.C : p.logits + (rg.S + row0) * p.C;
        const float* zzj = in_lds ? szz + row0 * p.C : p.zz + (rg.S + row0) * p.C;
        float* Ao = p.A ? p.A + (size_t)p.T * p.C * rg.ob + (size_t)(rg.t0 + j) * p.C * rg.Nb : nullptr;
        float* Yo = p.Y + ((size_t)rg.bag * p.T + rg.t0 + j) * p.C;
        softmax_group(ltid, act, rg.Nb, p.C, lgj, zzj, Ao, Yo, sred + half * 16);
    }
    if constexpr (PROBE) clock_probe(p, 1);
}

// ---------------------------------------------------------------------------------------
// gate_scores_kernel -- the generic path (any P): the whole masked BM x L feature tile is
// staged in LDS once, then the gate tile pairs are computed in passes of 8*PPW pairs.
// ---------------------------------------------------------------------------------------
template <int BM>
__host__ __device__ constexpr int gate_row_info_ints() { return kRowInfo * BM; }

template <typename E, int BM, int MAXC>
__host__ __device__ constexpr size_t gate_lds_bytes(int L) {
    // the partial scores alias the masked tile once every pass is done (see the kernel)
    const size_t tile = (size_t)BM * L * sizeof(E), red = (size_t)red_floats<BM, MAXC>() * 4;
    return (tile > red ? tile : red) + (size_t)MAXC * BM * 4 + (size_t)gate_row_info_ints<BM>() * 4;
}

template <typename E, int BM, int PPW, int MAXC>
__global__ __launch_bounds__(kGateThreads) void gate_scores_kernel(const GateParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int RT = BM / 16;
    constexpr int NJ = 2 * PPW;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int L = p.L;
    const int KS = L >> 5;
    const int LC = L >> 3;

    E* Xs = reinterpret_cast<E*>(smem);
    float* red = reinterpret_cast<float*>(smem);     // aliases Xs after the last pass
    const size_t tile_bytes = (size_t)BM * L * sizeof(E), red_bytes = (size_t)red_floats<BM, MAXC>() * 4;
    float* zred = reinterpret_cast<float*>(smem + (tile_bytes > red_bytes ? tile_bytes : red_bytes));
    int* rinfo = reinterpret_cast<int*>(zred + MAXC * BM);
    const long long R0 = (long long)blockIdx.x * BM;

    fill_row_table<BM>(p, R0, rinfo);
    __syncthreads();

    {   // stage the masked feature tile
        const E* H = reinterpret_cast<const E*>(p.H);
        const int items = BM * LC;
        for (int i = tid; i < items; i += kGateThreads) {
            const int blk = i >> 6, slot = i & 63;
            const int rt = blk / KS, ks = blk - rt * KS;
            const int r = rt * 16 + (slot & 15);
            const int kc = ks * 4 + (slot >> 4);
            E* dst = Xs + ((size_t)blk * 64 + slot) * 8;
            const int* ri = rinfo + kRowInfo * r;
            const int hrow = ri[0];
            if (hrow < 0) {
                store_zero8(dst);
                continue;
            }
            uint32_t kb;
            if (p.keep_feat) {
                kb = p.keep_feat[(size_t)(R0 + r) * LC + kc];
            } else {
                const uint4 o = philox4x32_10((uint32_t)kc, (uint32_t)ri[2],
                                              (uint32_t)(p.t_base + ri[1]), (uint32_t)ri[5],
                                              p.k0, p.k1);
                kb = keep_byte(o, p.thr_f);
            }
            load_masked(H + (size_t)hrow * p.ldh + (size_t)kc * 8, kb, dst);
        }
    }
    __syncthreads();

    const E* Wp = reinterpret_cast<const E*>(p.Wp);
    const int pairs_per_pass = kGateWaves * PPW;
    const int npass = (p.P + pairs_per_pass - 1) / pairs_per_pass;
    const size_t tile_elems = (size_t)KS * 512;

    float part[MAXC][RT];
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) part[c][rt] = 0.f;
    f32x4 zacc = {0.f, 0.f, 0.f, 0.f};
    const bool zwave = wave < RT;

    for (int pass = 0; pass < npass; ++pass) {
        const int q0 = pass * pairs_per_pass + wave * PPW;
        const bool active = q0 < p.P;
        const bool doz = (pass == 0) && zwave;
        if (!active && !doz) continue;

        f32x4 acc[RT][NJ];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};

        const E* wbase[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            int q = q0 + (j >> 1);
            q = q < p.P ? q : p.P - 1;
            wbase[j] = Wp + (size_t)(2 * q + (j & 1)) * tile_elems + lane * 8;
        }
        const E* zbase = Wp + (size_t)(2 * p.P) * tile_elems + lane * 8;

        Frag<E> wcur[NJ], wnxt[NJ];
        Frag<E> zcur = zero_frag<E>(), znxt = zero_frag<E>();
#pragma unroll
        for (int j = 0; j < NJ; ++j) wcur[j] = active ? load_frag(wbase[j]) : zero_frag<E>();
        if (doz) zcur = load_frag(zbase);

        for (int ks = 0; ks < KS; ++ks) {
            if (ks + 1 < KS) {
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    if (active) wnxt[j] = load_frag(wbase[j] + (size_t)(ks + 1) * 512);
                if (doz) znxt = load_frag(zbase + (size_t)(ks + 1) * 512);
            }
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const Frag<E> x = load_frag(Xs + ((size_t)(rt * KS + ks) * 64 + lane) * 8);
                if (active) {
#pragma unroll
                    for (int j = 0; j < NJ; ++j) acc[rt][j] = mma(wcur[j], x, acc[rt][j]);
                }
                if (doz && rt == wave) zacc = mma(zcur, x, zacc);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) wcur[j] = wnxt[j];
            zcur = znxt;
        }
        if (!active) continue;
        fold_pairs<RT, PPW, MAXC, false>(p, acc, q0, lane, part);
    }
    __syncthreads();   // every wave is done reading Xs: `red` may overwrite it
    finish_scores<BM, MAXC>(p, R0, part, zacc, zwave, red, zred, rinfo, -1, 0, false, true,
                            p.logits, p.zz, 0);
}

// ---------------------------------------------------------------------------------------
// bag_stats_kernel: mean and unbiased variance of the attention over the T passes
// (infer.py:216-219: torch .mean/.std, var = std^2) per output (bag, c, n), and, in the trailing
// blocks, the mean class probability per (bag, c) (infer.py:195 softmax over classes;
// net_utils.py:207-208 mean over T). A 512-thread block takes 64 consecutive outputs (coalesced
// over n) x 8 interleaved sample groups (t = g, g + 8, ...), so a lone bag of a few thousand
// instances (the per-bag caller, infer.py:187-191) still spreads over dozens of CUs with ~T/8
// loads per thread; the 8 group sums are added in group order (fp64, deterministic).
// ---------------------------------------------------------------------------------------
constexpr int kStatOuts = 64, kStatGroups = 8, kStatThreads = kStatOuts * kStatGroups;
#ifndef MCGMIL_KERNELS_TEMPLATES_ONLY
__global__ __launch_bounds__(kStatThreads) void bag_stats_kernel(const int32_t* bag_off, int B, int T, int C,
                                                                 long long total_rows, int stat_blocks,
                                                                 const float* A, const float* Y,
                                                                 float* A_mean, float* A_var, float* P_mean) {
    if ((int)blockIdx.x < stat_blocks) {
        __shared__ double ssum[kStatGroups][kStatOuts], ssq[kStatGroups][kStatOuts];
        const int o = threadIdx.x % kStatOuts, grp = threadIdx.x / kStatOuts;
        const long long i = (long long)blockIdx.x * kStatOuts + o;
        const bool live = i < total_rows * C;
        double s = 0.0, ss = 0.0;
        if (live) {
            const int bag = find_bag(bag_off, B, C, i);
            const int ob = bag_off[bag];
            const int Nb = bag_off[bag + 1] - ob;
            const long long local = i - (long long)C * ob;
            const int c = (int)(local / Nb);
            const int n = (int)(local - (long long)c * Nb);
            const float* a = A + (size_t)T * C * ob + (size_t)c * Nb + n;
            const size_t step = (size_t)C * Nb;
#pragma unroll 4
            for (int t = grp; t < T; t += kStatGroups) {
                const double v = a[(size_t)t * step];
                s += v;
                ss += v * v;
            }
        }
        ssum[grp][o] = s;
        ssq[grp][o] = ss;
        __syncthreads();
        if (grp != 0 || !live) return;
        s = ssum[0][o];
        ss = ssq[0][o];
#pragma unroll
        for (int g = 1; g < kStatGroups; ++g) {
            s += ssum[g][o];
            ss += ssq[g][o];
        }
        const double mean = s / T;
        if (A_mean) A_mean[i] = (float)mean;
        if (A_var) A_var[i] = T > 1 ? (float)fmax((ss - s * mean) / (T - 1), 0.0) : NAN;
        return;
    }
    // P_mean: one wave per bag, lane l takes the samples t = l, l + 64, ... (the T samples' loads
    // are independent: no serial latency chain over T), fp64 sums reduced over the wave in a
    // fixed butterfly order
    if (!P_mean) return;
    const int b = ((int)blockIdx.x - stat_blocks) * (kStatThreads / kWave) + (int)(threadIdx.x / kWave);
    const int lane = threadIdx.x % kWave;
    if (b >= B) return;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int t = lane; t < T; t += kWave) {
        const float* y = Y + ((size_t)b * T + t) * C;
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = k < C ? y[k] : -INFINITY;
        const float m = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
        float e[4], sum = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            e[k] = k < C ? expf(v[k] - m) : 0.f;
            sum += e[k];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] += (double)(e[k] / sum);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = wave_sum_d(acc[k]);
    if (lane < C) {
        const double a = lane == 0 ? acc[0] : lane == 1 ? acc[1] : lane == 2 ? acc[2] : acc[3];
        P_mean[(size_t)b * C + lane] = (float)(a / T);
    }
}
#endif

// ---------------------------------------------------------------------------------------
// pack_weights_kernel: fp32 nn.Linear weights -> MFMA A-operand tiles of dtype E.
// Tile 2q / 2q+1 = V / U columns d = 16*db .. 16*db+15 of gate g (q = g*D/16 + db);
// tile 2P = classifier rows (c < C), zero-padded to 16. Each tile is KS blocks of
// 64 lanes x 8 elements: lane l, element j = W[col l & 15][k = 32*ks + 8*(l >> 4) + j].
// ---------------------------------------------------------------------------------------
template <typename E>
__global__ void pack_weights_kernel(const float* Wv, const float* Wu, const float* wk, int L, int D,
                                    int C, int P, E* out) {
    const int KS = L >> 5;
    const size_t total = (size_t)(2 * P + 1) * KS * 512;
    const int DB = D >> 4;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int j = (int)(i & 7);
        const int lane = (int)((i >> 3) & 63);
        const size_t blk = i >> 9;
        const int ks = (int)(blk % KS);
        const int tile = (int)(blk / KS);
        const int col = lane & 15;
        const int k = ks * 32 + 8 * (lane >> 4) + j;
        float v;
        if (tile < 2 * P) {
            const int q = tile >> 1;
            const int g = q / DB, db = q - g * DB;
            const float* W = (tile & 1) ? Wu : Wv;
            v = W[((size_t)g * D + db * 16 + col) * L + k];
        } else {
            v = col < C ? wk[(size_t)col * L + k] : 0.f;
        }
        out[i] = static_cast<E>(v);
    }
}

// ---------------------------------------------------------------------------------------
// Mask materialisation (parity tests): the exact decisions gate_scores_kernel draws.
// ---------------------------------------------------------------------------------------
#ifndef MCGMIL_KERNELS_TEMPLATES_ONLY
__global__ void feature_keep_kernel(const int32_t* bag_off, int B, int T, int LC,
                                    long long total_samples, uint32_t k0, uint32_t k1,
                                    uint32_t bag_base, const uint32_t* bag_ids, int t_base,
                                    uint32_t thr, uint8_t* out) {
    const long long total = total_samples * LC;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long R = i / LC;
        const int kc = (int)(i - R * LC);
        const int bag = find_bag(bag_off, B, T, R);
        const int ob = bag_off[bag];
        const int Nb = bag_off[bag + 1] - ob;
        const long long local = R - (long long)T * ob;
        const int t = (int)(local / Nb);
        const int n = (int)(local - (long long)t * Nb);
        const uint32_t bagc = bag_ids ? bag_ids[bag] : bag_base + (uint32_t)bag;
        const uint4 o = philox4x32_10((uint32_t)kc, (uint32_t)n, (uint32_t)(t_base + t), bagc,
                                      k0, k1);
        out[i] = (uint8_t)keep_byte(o, thr);
    }
}
#endif

#ifndef MCGMIL_KERNELS_TEMPLATES_ONLY
__global__ void attention_keep_kernel(const int32_t* bag_off, int B, int T, int C,
                                      long long total, uint32_t k0, uint32_t k1,
                                      uint32_t bag_base, const uint32_t* bag_ids, int t_base,
                                      uint32_t thr, uint8_t* out) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int bag = find_bag(bag_off, B, (long long)T * C, i);
        const int ob = bag_off[bag];
        const int Nb = bag_off[bag + 1] - ob;
        const long long local = i - (long long)T * C * ob;
        const int t = (int)(local / ((long long)C * Nb));
        const long long rem = local - (long long)t * C * Nb;
        const int c = (int)(rem / Nb);
        const int n = (int)(rem - (long long)c * Nb);
        const uint32_t bagc = bag_ids ? bag_ids[bag] : bag_base + (uint32_t)bag;
        out[i] = attention_keep(k0, k1, bagc, (uint32_t)(t_base + t), (uint32_t)c, (uint32_t)n,
                                thr) ? 1 : 0;
    }
}
#endif

}  // namespace mcgmil
