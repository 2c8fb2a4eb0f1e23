#pragma once
// Row-owner gate kernels (round 5): the gate linears, gated product, attention logits, logit
// dropout and classifier projection of model.py:280-316 for bf16 heads whose gate columns form
// at most 16 blocks of 32 (the reference's C = 2 heads at D = 128, shared or separate).
//
// Layout of the work (one 256-thread workgroup per CU, ONE wave per SIMD, 512 registers a lane):
//   - a tile is 128 rows of the flattened (bag, t, n) space; wave w owns rows 32w .. 32w+31 and
//     ALL gate columns, so it makes its own masked features: for K step s (16 features) lane l
//     draws one Philox4x32-10 block for row l & 31, features 16s + 8(l >> 5) .. +7 -- exactly its
//     B fragment of v_mfma_f32_32x32x16_bf16. No feature staging through LDS, no feature barrier,
//     and every keep decision is drawn once (the same counters as gate_pipe_kernel: {l>>3, n, t, bag}).
//   - the weights are the A operands: NCB column blocks of 32 (V and U of each 32-wide d block,
//     gate by gate) stream through a 4-slot LDS ring, one 16-deep K step (NCB KiB) per slot,
//     filled by LDS-DMA three steps ahead (each wave issues NCB/4 of the 1-KiB pieces of a step:
//     no staging registers, no ds_write); each wave reads all NCB fragments of step s+1 while it
//     runs step s's MFMAs, one barrier per K step: each weight byte leaves L2 once per CU per tile.
//   - the classifier projection z = X k_c: v_dot2_f32_bf16 on the lane's own 8 features per K
//     step against k_c from an LDS table (a 32-row MFMA tile for 2 classes would cost 1/16 of the
//     matrix pipe, and 16 accumulator registers more than the AGPR file holds).
//   - accumulators: NCB 32x32 tiles (16 floats a lane each: 256 at NCB = 16) -- the AGPR half of
//     the register file; the lane holds row l & 31 and d = 32 db + (i & 3) + 8 (i >> 2) + 4 (l >> 5).
//   - epilogue: tanh(V) sigmoid(U) wa per (row, d) as in fold_pairs, the two lane halves' partial
//     scores added with one cross-half exchange, attention bias + logit dropout, stores.
// Compared with gate_pipe_kernel (8 waves sharing LDS-staged features, 16x16x32): half the MFMA
// issue slots, no per-K-step barrier over staged features, no cross-wave score reduction.
#include "mcgmil_kernels.h"

namespace mcgmil {

typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kRgWaves = 4;
constexpr int kRgThreads = kRgWaves * kWave;
constexpr int kRgRows = 32 * kRgWaves;      // rows of a tile
constexpr int kRgSlots = 4;                 // weight ring slots (K steps): one being read, two landing, one free

// Column blocks of the row-gate weight stream: V and U of each 32-wide d block of each gate.
__host__ __device__ inline int rg_ncb(int G, int D) { return D % 32 == 0 ? 2 * G * D / 32 : 0; }
// The stream: [L/16 K steps][NCB blocks][64 lanes][8] bf16; lane l, element j of block cb, step s
// = W[g*D + 32*db + (l & 31)][16 s + 8 (l >> 5) + j], cb = g * 2(D/32) + 2 db + (0: Wv, 1: Wu).
__host__ __device__ inline size_t rg_stream_bytes(int L, int G, int D) {
    return (size_t)(L / 16) * rg_ncb(G, D) * 1024;
}
// Followed by the classifier table [4][L] bf16 (rows >= C zero).
__host__ __device__ inline size_t rg_cls_bytes(int L) { return (size_t)4 * L * 2; }
// Only heads the row kernel runs (D = 128, one or two gates, L a multiple of 64, >= 128) get one.
__host__ __device__ inline size_t rg_packed_bytes(int L, int G, int D) {
    const bool fits = D == 128 && (G == 1 || G == 2) && L % 64 == 0 && L >= 128;
    return fits ? rg_stream_bytes(L, G, D) + rg_cls_bytes(L) : 0;
}

template <typename E>
__global__ void pack_rowgate_kernel(const float* Wv, const float* Wu, const float* wk, int L, int D,
                                    int G, int C, __bf16* out) {
    const int NCB = rg_ncb(G, D), DB = D / 32;
    const size_t stream = (size_t)(L / 16) * NCB * 512;     // elements
    const size_t total = stream + (size_t)4 * L;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        float v;
        if (i < stream) {
            const int j = (int)(i & 7), lane = (int)((i >> 3) & 63);
            const size_t blk = i >> 9;
            const int cb = (int)(blk % NCB), s = (int)(blk / NCB);
            const int g = cb / (2 * DB), rem = cb - g * 2 * DB, db = rem >> 1;
            const float* W = (rem & 1) ? Wu : Wv;
            v = W[((size_t)g * D + 32 * db + (lane & 31)) * L + 16 * s + 8 * (lane >> 5) + j];
        } else {
            const size_t e = i - stream;
            const int c = (int)(e / L), k = (int)(e - (size_t)c * L);
            v = c < C ? wk[(size_t)c * L + k] : 0.f;
        }
        out[i] = static_cast<__bf16>(v);
    }
}

// LDS of a row-gate workgroup (bytes): the weight ring, the classifier table [MAXC][L] bf16, the
// head vectors (bv, bu pre-scaled by -2 log2 e / -log2 e; wa).
template <int NCB>
__host__ __device__ constexpr size_t rg_ring_bytes() { return (size_t)kRgSlots * NCB * 1024; }
template <int MAXC>
__host__ __device__ inline size_t rg_ktab_bytes(int L) { return (size_t)MAXC * L * 2; }
__host__ __device__ inline size_t rg_head_bytes(int G, int C, int D) { return (size_t)(2 * G + C) * D * 4; }
template <int NCB, int MAXC>
__host__ __device__ inline size_t rg_lds_bytes(int L, int G, int C, int D) {
    return rg_ring_bytes<NCB>() + rg_ktab_bytes<MAXC>(L) + rg_head_bytes(G, MAXC, D);   // wa zero-padded to MAXC rows
}

// One lane's row of a tile.
struct RgLane {
    const char* h;        // H row + 16 (l >> 5) bytes (a valid row for padding lanes)
    uint32_t n, t, bagc;  // Philox counters (t includes t_base)
    uint32_t inval;       // ~0: padding row (stages zeros, stores nothing)
    long long R;          // flattened (bag, t, n) row (replay masks, outputs)
    int bag;
    const unsigned char* kf;   // replay: the row's keep_feat bytes + (l >> 5) (row 0's for padding)
};

// Row R of the flattened space -> its lane record (the mapping of fill_row_table).
__device__ __forceinline__ RgLane rg_lane_flat(const GateParams& p, long long R, long long tile) {
    RgLane rl;
    int hrow = -1, t = 0, n = 0, bag = 0;
    const bool narrow = p.total_samples <= 0xFFFFFFFFll;
    if (R < p.total_samples && p.uniform_rows > 0) {
        const long long per_bag = (long long)p.T * p.uniform_rows;
        const int Nb = p.uniform_rows;
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
        bag = p.tile_bag ? p.tile_bag[tile] : find_bag(p.bag_off, p.B, p.T, R);
        while ((long long)p.T * p.bag_off[bag + 1] <= R) ++bag;
        const int ob = p.bag_off[bag];
        const int Nb = p.bag_off[bag + 1] - ob;
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
    const int hl = (threadIdx.x >> 5) & 1;
    rl.h = reinterpret_cast<const char*>(p.H) + ((size_t)(hrow >= 0 ? hrow : 0) * p.ldh + 8 * hl) * 2;
    rl.n = (uint32_t)n;
    rl.t = (uint32_t)(p.t_base + t);
    rl.bagc = p.bag_ids ? p.bag_ids[bag] : p.bag_base + (uint32_t)bag;
    rl.inval = hrow >= 0 ? 0u : 0xFFFFFFFFu;
    rl.R = R;
    rl.bag = bag;
    rl.kf = p.keep_feat ? p.keep_feat + (size_t)(hrow >= 0 ? R : 0) * (p.L >> 3) + hl : nullptr;
    return rl;
}

// The X fragment of K step s: the lane's 8 features with the dropped (and padding) ones zeroed.
template <bool REPLAY>
__device__ __forceinline__ bf16x8 rg_stage(const GateParams& p, const RgLane& rl, uint4 h, int s) {
    const int hl = (threadIdx.x >> 5) & 1;
    if constexpr (REPLAY) {
        const uint32_t kb = (uint32_t)rl.kf[2 * s] & ~rl.inval;
        uint4 v = h;
        v.x &= ((kb & 1u) ? 0x0000FFFFu : 0u) | ((kb & 2u) ? 0xFFFF0000u : 0u);
        v.y &= ((kb & 4u) ? 0x0000FFFFu : 0u) | ((kb & 8u) ? 0xFFFF0000u : 0u);
        v.z &= ((kb & 16u) ? 0x0000FFFFu : 0u) | ((kb & 32u) ? 0xFFFF0000u : 0u);
        v.w &= ((kb & 64u) ? 0x0000FFFFu : 0u) | ((kb & 128u) ? 0xFFFF0000u : 0u);
        return __builtin_bit_cast(bf16x8, v);
    } else {
        const uint4 o = philox4x32_10<true>((uint32_t)(2 * s + hl), rl.n, rl.t, rl.bagc, p.k0, p.k1);
        uint4 v;
        v.x = __builtin_amdgcn_bitop3_b32(h.x, drop_mask16x2_flipped(o.x, p.thrx_f), rl.inval, 0x10);
        v.y = __builtin_amdgcn_bitop3_b32(h.y, drop_mask16x2(o.y, p.thrx_f), rl.inval, 0x10);
        v.z = __builtin_amdgcn_bitop3_b32(h.z, drop_mask16x2_flipped(o.z, p.thrx_f), rl.inval, 0x10);
        v.w = __builtin_amdgcn_bitop3_b32(h.w, drop_mask16x2(o.w, p.thrx_f), rl.inval, 0x10);
        return __builtin_bit_cast(bf16x8, v);
    }
}


__device__ __forceinline__ f32x16 mma32(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
// z partial: the lane's 8 features . k_c's 8 (bf16 products exact, fp32 sums)
__device__ __forceinline__ float rg_dot8(bf16x8 x, uint4 k, float acc) {
    const uint4 xv = __builtin_bit_cast(uint4, x);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, xv.x), __builtin_bit_cast(bf16x2, k.x), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, xv.y), __builtin_bit_cast(bf16x2, k.y), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, xv.z), __builtin_bit_cast(bf16x2, k.z), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, xv.w), __builtin_bit_cast(bf16x2, k.w), acc, false);
    return acc;
}

// LDS byte address of a pointer into the dynamic LDS.
__device__ __forceinline__ uint32_t rg_lds(const unsigned char* p) {
    return (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const unsigned char*)p);
}

// 16 bytes per lane from the weight stream into LDS at the wave-uniform `lds` + 16 * lane (LDS-DMA).
// The builtin only exists in the device pass; the host pass must still see a body.
__device__ __forceinline__ void rg_dma(__amdgpu_buffer_rsrc_t r, unsigned char* lds, uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
#else
    (void)r; (void)lds; (void)voff; (void)soff;
#endif
}

// LDS reads of the ring and the classifier table as inline asm: the compiler's wait-count pass
// treats a ds_read after an LDS-DMA as a possible alias and would put an s_waitcnt vmcnt(0) in
// front of it, draining the weight DMAs in flight. The reads are waited for explicitly (the
// end-of-step barrier's lgkmcnt(0), which names their registers).
typedef unsigned int rg_u32x4 __attribute__((ext_vector_type(4)));   // a native vector for asm operands
template <int OFF>
__device__ __forceinline__ rg_u32x4 rg_ds_read(uint32_t addr) {
    rg_u32x4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
    return v;
}
// H rows are ordinary loads: the compiler's wait-count pass then orders every use (and every
// copy) of the loaded registers after the data lands. (An inline-asm load would leave its
// destination registers in flight where the compiler may copy or reuse them.)
__device__ __forceinline__ uint4 rg_hload(const char* p) { return *reinterpret_cast<const uint4*>(p); }
template <int N>
__device__ __forceinline__ void rg_vmwait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Registers a wave carries from one K step to the next (and across tiles): the weight fragments
// and classifier features of the next step (read during this step), X and H of the next steps,
// and (register staging, DMA = false) the weights of steps in flight from L2.
template <int NCB, int MAXC, bool DMA>
struct RgPipe {
    rg_u32x4 af[NCB];  // A fragments of the next step (complete after the step's barrier)
    rg_u32x4 kf[MAXC]; // classifier features of the next step
    bf16x8 x;          // X fragment of the next step
    uint4 h;           // H of the step after it (loaded)
    uint4 ws[DMA ? 1 : 2][NCB / 4];   // register staging: set t & 1 holds step t's pieces
};

// One-time setup of a workgroup: head vectors and classifier table into LDS, the ring's first
// K steps (DMA: steps 0..2 by LDS-DMA into slots 0..2; register staging: steps 0..1 into slots 0..1
// and step 2 into staging set 0). Visible after the caller's barrier.
// LDS: [ring][classifier rows 0..MAXC-1][bv', bu', wa].
template <int NCB, int MAXC, bool DMA>
__device__ __forceinline__ void rg_setup(const GateParams& p, unsigned char* smem, __amdgpu_buffer_rsrc_t& wrs,
                                         RgPipe<NCB, MAXC, DMA>& pp) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned char* kt = smem + rg_ring_bytes<NCB>();
    float* head = reinterpret_cast<float*>(kt + rg_ktab_bytes<MAXC>(p.L));
    const size_t sbytes = rg_stream_bytes(p.L, p.G, p.D);
    wrs = make_rsrc(p.Wr, (uint32_t)(sbytes + rg_cls_bytes(p.L)));
    for (uint32_t i = tid; i < (uint32_t)(MAXC * p.L / 8); i += kRgThreads)
        *reinterpret_cast<uint4*>(kt + (size_t)i * 16) =
            __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, i * 16u, (uint32_t)sbytes, 0));
    const int GD = p.G * p.D;
    for (int i = tid; i < GD; i += kRgThreads) {
        head[i] = p.bv[i] * kM2Log2e;
        head[GD + i] = p.bu[i] * kMLog2e;
    }
    for (int i = tid; i < MAXC * p.D; i += kRgThreads) head[2 * GD + i] = i < p.C * p.D ? p.wa[i] : 0.f;
    const uint32_t lane_b = (uint32_t)lane * 16u;
    if constexpr (DMA) {
#pragma unroll
        for (int st = 0; st < 3; ++st)
#pragma unroll
            for (int i = 0; i < NCB / 4; ++i) {
                const uint32_t cb = (uint32_t)(wave * (NCB / 4) + i);
                rg_dma(wrs, smem + (size_t)(st * NCB + (int)cb) * 1024, lane_b, ((uint32_t)(st * NCB) + cb) * 1024u);
            }
        rg_vmwait<0>();
    } else {
#pragma unroll
        for (int st = 0; st < 3; ++st)
#pragma unroll
            for (int i = 0; i < NCB / 4; ++i) {
                const uint32_t cb = (uint32_t)(wave * (NCB / 4) + i);
                const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                              wrs, lane_b, ((uint32_t)(st * NCB) + cb) * 1024u, 0));
                if (st < 2) *reinterpret_cast<uint4*>(smem + (size_t)(st * NCB + (int)cb) * 1024 + lane_b) = v;
                else pp.ws[0][i] = v;
            }
    }
}

// Timing-only ablations (never in the product; wrong results): 1 no Philox/keep rule, 2 no
// transcendentals in the epilogue, 4 no weight DMA, 8 no H loads, 16 no barrier, 32 no MFMAs,
// 64 no epilogue arithmetic (accumulators kept live).
#ifndef MCGMIL_RG_DIAG
#define MCGMIL_RG_DIAG 0
#endif

// Scheduling of one K step: MFMA i is followed by VPM vector ops.
#ifndef MCGMIL_RG_VPM
#define MCGMIL_RG_VPM 4
#endif

template <int V> using rg_int = std::integral_constant<int, V>;

// Diagnostic build (-DMCGMIL_STAMPS): lane 0 of each wave records s_memtime into
// stamps[(tile * 4 + wave) * 8 + i] (phase boundaries of the row-gate tile).
#ifdef MCGMIL_STAMPS
#define RG_STAMP(p, tile, i)                                                                       \
    do {                                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        if ((threadIdx.x & 63) == 0 && (p).stamps)                                                 \
            (p).stamps[((size_t)(tile) * 4 + (threadIdx.x >> 6)) * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
        __builtin_amdgcn_sched_barrier(0);                                                         \
    } while (0)
#else
#define RG_STAMP(p, tile, i) do {} while (0)
#endif

// Reads of step `s`'s A fragments (ring slot SLOT) and classifier features into pp (asm, waited
// for at the next barrier). The ds_read offset is an immediate: one template instance per block.
// DMA = false: ordinary LDS loads (no LDS-DMA in flight, so the compiler orders them itself).
template <int NCB, int MAXC, bool DMA, int SLOT, int C = 0>
__device__ __forceinline__ void rg_read_frags(RgPipe<NCB, MAXC, DMA>& pp, const unsigned char* smem, uint32_t ring_lane) {
    if constexpr (C < NCB) {
        if constexpr (DMA) pp.af[C] = rg_ds_read<(SLOT * NCB + C) * 1024>(ring_lane);
        else pp.af[C] = *reinterpret_cast<const rg_u32x4*>(smem + (size_t)(SLOT * NCB + C) * 1024 + (threadIdx.x & 63) * 16);
        rg_read_frags<NCB, MAXC, DMA, SLOT, C + 1>(pp, smem, ring_lane);
    }
}
template <int NCB, int MAXC, bool DMA, int SLOT>
__device__ __forceinline__ void rg_prefetch(RgPipe<NCB, MAXC, DMA>& pp, const unsigned char* smem, uint32_t ring_lane,
                                            uint32_t ktab_lane, int L, int s) {
    rg_read_frags<NCB, MAXC, DMA, SLOT>(pp, smem, ring_lane);
    const uint32_t ka = ktab_lane + 32u * (uint32_t)s;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if constexpr (DMA) pp.kf[c] = rg_ds_read<0>(ka + (uint32_t)(c * L * 2));
        else pp.kf[c] = *reinterpret_cast<const rg_u32x4*>(smem + rg_ring_bytes<NCB>() + 16 * ((threadIdx.x & 63) >> 5) +
                                                            32 * s + (size_t)c * L * 2);
    }
}

// The prefetched registers' lgkmcnt(0) wait: one statement naming all of them, so no copy of a
// register whose ds_read is still in flight can be placed before it.
template <int NCB, int MAXC, bool DMA>
__device__ __forceinline__ void rg_wait_frags(RgPipe<NCB, MAXC, DMA>& pp, bool barrier) {
    static_assert((NCB == 16 || NCB == 8) && (MAXC == 2 || MAXC == 4), "row-gate shapes");
#define RG_A8 "+v"(pp.af[0]), "+v"(pp.af[1]), "+v"(pp.af[2]), "+v"(pp.af[3]), "+v"(pp.af[4]), "+v"(pp.af[5]), \
              "+v"(pp.af[6]), "+v"(pp.af[7])
#define RG_A16 RG_A8, "+v"(pp.af[8]), "+v"(pp.af[9]), "+v"(pp.af[10]), "+v"(pp.af[11]), "+v"(pp.af[12]), \
              "+v"(pp.af[13]), "+v"(pp.af[14]), "+v"(pp.af[15])
#define RG_K2 "+v"(pp.kf[0]), "+v"(pp.kf[1])
#define RG_K4 RG_K2, "+v"(pp.kf[2]), "+v"(pp.kf[3])
    if (barrier) {
        if constexpr (NCB == 16 && MAXC == 2) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" : RG_A16, RG_K2::"memory");
        if constexpr (NCB == 16 && MAXC == 4) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" : RG_A16, RG_K4::"memory");
        if constexpr (NCB == 8 && MAXC == 2) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" : RG_A8, RG_K2::"memory");
        if constexpr (NCB == 8 && MAXC == 4) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" : RG_A8, RG_K4::"memory");
    } else {
        if constexpr (NCB == 16 && MAXC == 2) asm volatile("s_waitcnt lgkmcnt(0)" : RG_A16, RG_K2::"memory");
        if constexpr (NCB == 16 && MAXC == 4) asm volatile("s_waitcnt lgkmcnt(0)" : RG_A16, RG_K4::"memory");
        if constexpr (NCB == 8 && MAXC == 2) asm volatile("s_waitcnt lgkmcnt(0)" : RG_A8, RG_K2::"memory");
        if constexpr (NCB == 8 && MAXC == 4) asm volatile("s_waitcnt lgkmcnt(0)" : RG_A8, RG_K4::"memory");
    }
#undef RG_A8
#undef RG_A16
#undef RG_K2
#undef RG_K4
}

// End of a K step: (DMA) my DMA pieces of the step after next have landed (vmcnt: each step issues
// NCB/4 DMA pieces and one H load, so the NCB/4 + 1 youngest vector-memory ops are this step's,
// whatever order the compiler gave them); the prefetched reads and this step's ring writes are
// complete; barrier.
template <int NCB, int MAXC, bool DMA>
__device__ __forceinline__ void rg_step_barrier(RgPipe<NCB, MAXC, DMA>& pp) {
    if constexpr (DMA) rg_vmwait<NCB / 4 + 1>();
    rg_wait_frags<NCB, MAXC, DMA>(pp, !(MCGMIL_RG_DIAG & 16));
}

// One tile's K loop over global steps; `rn` = the next tile's lane record (its X[0] and H[1] are
// made / loaded during this tile's last steps). On entry pp holds this tile's step 0 (A fragments,
// classifier features, X[0]) and H[1]; on return the next tile's. Step s of a tile uses ring slot
// s % 4 (KS = L/16 is a multiple of 4). DMA: step s issues the LDS-DMA of step s + 3 (mod KS: the
// next tile's first steps) into slot (s + 3) % 4. Register staging: step s writes step s + 2's
// pieces (loaded a step earlier) into slot (s + 2) % 4 and loads step s + 3's. Needs KS >= 8.
template <int NCB, int MAXC, bool REPLAY, bool DMA>
__device__ __forceinline__ void rg_kloop(const GateParams& p, unsigned char* smem, __amdgpu_buffer_rsrc_t wrs,
                                         const RgLane& rl, const RgLane& rn, RgPipe<NCB, MAXC, DMA>& pp,
                                         f32x16 (&acc)[NCB], float (&zp)[MAXC]) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int KS = p.L >> 4;
    const uint32_t lane_b = (uint32_t)lane * 16u;
    const uint32_t ring_lane = rg_lds(smem) + lane_b;
    const uint32_t ktab_lane = rg_lds(smem + rg_ring_bytes<NCB>()) + 16u * (uint32_t)(lane >> 5);
#pragma unroll
    for (int c = 0; c < MAXC; ++c) zp[c] = 0.f;
    // MODE 0: inside the tile; 1: the first step (accumulators start at zero); 2: step s+2 is the
    // next tile's step 0; 3: steps s+1 and s+2 are the next tile's steps 0 and 1.
    auto kstep = [&](auto sl_c, auto mode_c, int s) {
        constexpr int SL = decltype(sl_c)::value, MODE = decltype(mode_c)::value;
        constexpr bool N1 = MODE == 3, N2 = MODE >= 2;
        const RgLane& l1 = N1 ? rn : rl;
        const RgLane& l2 = N2 ? rn : rl;
        const int s1 = N1 ? s + 1 - KS : s + 1, s2 = N2 ? s + 2 - KS : s + 2;
        const int s3 = s + 3 < KS ? s + 3 : s + 3 - KS;
        __builtin_amdgcn_sched_barrier(0);
        // this step's operands; the next step's are read into pp below
        rg_u32x4 af[NCB];
#pragma unroll
        for (int c = 0; c < NCB; ++c) af[c] = pp.af[c];
        rg_u32x4 kf[MAXC];
#pragma unroll
        for (int c = 0; c < MAXC; ++c) kf[c] = pp.kf[c];
        const bf16x8 x = pp.x;
        const uint4 h1 = pp.h;                             // H[s+1] (issued a step ago)
        // this step's vector-memory ops: H[s+2] and the DMA of step s+3
#if MCGMIL_RG_DIAG & 8
        const uint4 h2 = h1;
#else
        const uint4 h2 = rg_hload(l2.h + 32 * s2);
#endif
#if !(MCGMIL_RG_DIAG & 4)
        if constexpr (DMA) {
#pragma unroll
            for (int i = 0; i < NCB / 4; ++i) {
                const uint32_t cb = (uint32_t)(wave * (NCB / 4) + i);
                rg_dma(wrs, smem + (size_t)(((SL + 3) & 3) * NCB + (int)cb) * 1024, lane_b,
                       ((uint32_t)s3 * (uint32_t)NCB + cb) * 1024u);
            }
        } else {
#pragma unroll
            for (int i = 0; i < NCB / 4; ++i) {
                const uint32_t cb = (uint32_t)(wave * (NCB / 4) + i);
                *reinterpret_cast<uint4*>(smem + (size_t)(((SL + 2) & 3) * NCB + (int)cb) * 1024 + lane_b) = pp.ws[SL & 1][i];
                pp.ws[(SL + 1) & 1][i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                       wrs, lane_b, ((uint32_t)s3 * (uint32_t)NCB + cb) * 1024u, 0));
            }
        }
#endif
        rg_prefetch<NCB, MAXC, DMA, (SL + 1) & 3>(pp, smem, ring_lane, ktab_lane, p.L, N1 ? 0 : s + 1);
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
#if MCGMIL_RG_DIAG & 32
            acc[c][c & 15] += __uint_as_float(af[c].x ^ 0u);
#else
            acc[c] = mma32(__builtin_bit_cast(bf16x8, af[c]), x, MODE == 1 ? f32x16{} : acc[c]);
#endif
        }
#pragma unroll
        for (int c = 0; c < MAXC; ++c) zp[c] = rg_dot8(x, __builtin_bit_cast(uint4, kf[c]), zp[c]);
        // X[s+1] from H[s+1] (the compiler waits for the load)
#if MCGMIL_RG_DIAG & 1
        pp.x = __builtin_bit_cast(bf16x8, make_uint4(h1.x & ~l1.inval, h1.y, h1.z, h1.w ^ (uint32_t)s1));
#else
        pp.x = rg_stage<REPLAY>(p, l1, h1, s1);
#endif
        pp.h = h2;
#pragma unroll
        for (int i = 0; i < NCB; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);              // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, MCGMIL_RG_VPM, 0);  // VALU
        }
        __builtin_amdgcn_sched_barrier(0);
        rg_step_barrier<NCB, MAXC, DMA>(pp);
    };
    const rg_int<0> S0{}, M0{};
    const rg_int<1> S1{}, M1{};
    const rg_int<2> S2{}, M2{};
    const rg_int<3> S3{}, M3{};
    kstep(S0, M1, 0);
    kstep(S1, M0, 1);
    kstep(S2, M0, 2);
    kstep(S3, M0, 3);
    for (int s = 4; s < KS - 4; s += 4) {
        kstep(S0, M0, s);
        kstep(S1, M0, s + 1);
        kstep(S2, M0, s + 2);
        kstep(S3, M0, s + 3);
    }
    kstep(S0, M0, KS - 4);
    kstep(S1, M0, KS - 3);
    kstep(S2, M2, KS - 2);     // H[s+2] = the next tile's H[0]
    kstep(S3, M3, KS - 1);     // X[s+1] = the next tile's X[0], H[s+2] its H[1]
}

// Prologue of a workgroup's first tile: its step-0 operands and H[1] into pp (after rg_setup's
// DMA and the caller's barrier).
template <int NCB, int MAXC, bool REPLAY, bool DMA>
__device__ __forceinline__ void rg_first(const GateParams& p, unsigned char* smem, const RgLane& rl,
                                         RgPipe<NCB, MAXC, DMA>& pp) {
    const int lane = threadIdx.x & 63;
    const uint32_t ring_lane = rg_lds(smem) + (uint32_t)lane * 16u;
    const uint32_t ktab_lane = rg_lds(smem + rg_ring_bytes<NCB>()) + 16u * (uint32_t)(lane >> 5);
    rg_prefetch<NCB, MAXC, DMA, 0>(pp, smem, ring_lane, ktab_lane, p.L, 0);
    const uint4 h0 = rg_hload(rl.h);
    pp.h = rg_hload(rl.h + 32);
    pp.x = rg_stage<REPLAY>(p, rl, h0, 0);
    rg_wait_frags<NCB, MAXC, DMA>(pp, false);
}

// The epilogue of a tile: scores, logit dropout, z; store(rl, c, logit, z) per (row, class).
// G gates of DB 32-wide d blocks; shared heads (G = 1) feed every class, separate (G = C) class g.
// With one wave per SIMD no other wave hides a product's exp -> add -> fma -> rcp chain, so the
// 16 products of an accumulator pair go through each stage together (scheduling barriers keep the
// stages apart: 16 independent instructions back to back), and each class sums into 4 partials.
template <int G, int DB, int MAXC, bool REPLAY, typename Store>
__device__ __forceinline__ void rg_epilogue(const GateParams& p, const unsigned char* smem, const RgLane& rl,
                                            const f32x16 (&acc)[2 * G * DB], const float (&zp)[MAXC], Store store) {
    constexpr int NCB = 2 * G * DB, D = 32 * DB;
    const int lane = threadIdx.x & 63, hl = lane >> 5;
#if MCGMIL_RG_DIAG & 64
    {   // every accumulator stays live (its MFMAs are kept), no epilogue arithmetic
        float t = zp[0];
#pragma unroll
        for (int c = 0; c < NCB; ++c) t += acc[c][c & 15];
        if (!rl.inval) store(rl, hl, t, 0.f);
        return;
    }
#endif
    const float* head = reinterpret_cast<const float*>(smem + rg_ring_bytes<NCB>() + rg_ktab_bytes<MAXC>(p.L));
    const float av_s = p.sf * kM2Log2e, au_s = p.sf * kMLog2e;
    float part[MAXC][4], z[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int k = 0; k < 4; ++k) part[c][k] = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int db = 0; db < DB; ++db) {
            // keeps the compiler from hoisting every d block's head-vector reads to the top (their
            // registers, live through the whole epilogue, spill the shared-heads kernels)
            asm volatile("" ::: "memory");
            const int cb = g * 2 * DB + 2 * db;
            float ax[16], by[16], w[MAXC][16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int d0 = 32 * db + 8 * q + 4 * hl;
                const f32x4 bv = *reinterpret_cast<const f32x4*>(head + g * D + d0);
                const f32x4 bu = *reinterpret_cast<const f32x4*>(head + G * D + g * D + d0);
#pragma unroll
                for (int c = 0; c < MAXC; ++c) {
                    const bool use = G == 1 || c == g;   // rows c >= C are zero
                    const f32x4 wq = use ? *reinterpret_cast<const f32x4*>(head + 2 * G * D + c * D + d0)
                                         : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int r = 0; r < 4; ++r) w[c][4 * q + r] = wq[r];
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    ax[4 * q + r] = fmaf(acc[cb][4 * q + r], av_s, bv[r]);
                    by[4 * q + r] = fmaf(acc[cb + 1][4 * q + r], au_s, bu[r]);
                }
            }
#if MCGMIL_RG_DIAG & 2
#pragma unroll
            for (int i = 0; i < 16; ++i) part[G == 1 ? 0 : g][i & 3] = fmaf(fmaf(ax[i], w[G == 1 ? 0 : g][i], by[i]), ax[i], part[G == 1 ? 0 : g][i & 3]);
            continue;
#endif
            float a[16], b[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) a[i] = __builtin_amdgcn_exp2f(fminf(ax[i], 43.280851226668903f));
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; ++i) b[i] = __builtin_amdgcn_exp2f(by[i]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float ia = 1.0f + a[i];
                b[i] = fmaf(ia, b[i], ia);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; ++i) b[i] = __builtin_amdgcn_rcpf(b[i]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if constexpr (G == 1) {
                    const float pr = (1.0f - a[i]) * b[i];
#pragma unroll
                    for (int c = 0; c < MAXC; ++c) part[c][i & 3] = fmaf(pr, w[c][i], part[c][i & 3]);
                } else {
                    part[g][i & 3] = fmaf(fmaf(-a[i], w[g][i], w[g][i]), b[i], part[g][i & 3]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // the other lane half holds the row's other d values and other 8 features of each K step;
    // lane half hl scores classes hl, hl + 2 (selected value by value: a select between two
    // elements of one array becomes a dynamically indexed stack array)
    float pcs[MAXC / 2], zcs[MAXC / 2];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        float sc = (part[c][0] + part[c][1]) + (part[c][2] + part[c][3]);
        sc += __shfl_xor(sc, 32);
        z[c] = zp[c] + __shfl_xor(zp[c], 32);
        if ((c & 1) == 0) {
            pcs[c / 2] = sc;
            zcs[c / 2] = z[c];
        } else {
            pcs[c / 2] = hl ? sc : pcs[c / 2];
            zcs[c / 2] = hl ? z[c] : zcs[c / 2];
        }
    }
#pragma unroll
    for (int c0 = 0; c0 < MAXC; c0 += 2) {
        const int c = c0 + hl;
        const float pc = pcs[c0 / 2], zc = zcs[c0 / 2];
        if (c >= p.C || rl.inval) continue;
        bool keep;
        if constexpr (REPLAY) {
            const size_t abase = (size_t)p.T * p.C * (size_t)p.bag_off[rl.bag];
            const int Nb = p.bag_off[rl.bag + 1] - p.bag_off[rl.bag];
            keep = p.keep_att[abase + ((size_t)(rl.t - (uint32_t)p.t_base) * p.C + c) * Nb + rl.n] != 0;
        } else {
            keep = attention_keep(p.k0, p.k1, rl.bagc, rl.t, (uint32_t)c, rl.n, p.thr_a);
        }
        store(rl, c, (pc + p.ba[c]) * (keep ? p.sa : 0.f), zc * p.sf);
    }
}

// Two-kernel path: persistent workgroups over the 128-row tiles; logits and z to the workspace.
// DMA: the LDS-DMA weight stream with asm operand reads -- only for instantiations the compiler
// fits without spills (tests/test_codegen_guard.py); else register staging, all compiler-visible.
template <int G, int DB, int MAXC, bool REPLAY, bool DMA>
__global__ __launch_bounds__(kRgThreads, 1) void rowgate_scores_kernel(const GateParams p, long long tiles) {
    constexpr int NCB = 2 * G * DB;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    clock_probe(p, 0);
    __amdgpu_buffer_rsrc_t wrs;
    RgPipe<NCB, MAXC, DMA> pp;
    rg_setup<NCB, MAXC, DMA>(p, smem, wrs, pp);
    long long tile = blockIdx.x;
    auto row_of = [&](long long tl) { return tl < tiles ? tl * kRgRows + 32 * wave + (lane & 31) : p.total_samples; };
    RgLane rl = rg_lane_flat(p, row_of(tile), tile);
    __syncthreads();
    rg_first<NCB, MAXC, REPLAY, DMA>(p, smem, rl, pp);
    f32x16 acc[NCB];
    float zp[MAXC];
    for (; tile < tiles; tile += gridDim.x) {
        RG_STAMP(p, tile, 0);
        const long long nt = tile + gridDim.x;
        const RgLane rn = rg_lane_flat(p, row_of(nt), nt);
        RG_STAMP(p, tile, 1);
        rg_kloop<NCB, MAXC, REPLAY, DMA>(p, smem, wrs, rl, rn, pp, acc, zp);
        RG_STAMP(p, tile, 2);
        rg_epilogue<G, DB, MAXC, REPLAY>(p, smem, rl, acc, zp, [&](const RgLane& r, int c, float lg, float z) {
            p.logits[(size_t)r.R * p.C + c] = lg;
            p.zz[(size_t)r.R * p.C + c] = z;
        });
        RG_STAMP(p, tile, 3);
        rl = rn;
    }
    clock_probe(p, 1);
}

// ---------------------------------------------------------------------------------------
// rowgate_fused_kernel -- the whole path in ONE launch on the row-owner tile: a workgroup owns a
// region (the t-groups [t0, t1) of one bag, decode_region), runs its 128-row tiles through the
// K loop + epilogue above with the logits and z kept in LDS, then softmax_group per t-group
// (model.py:305-316) with its 256 threads. Bags of more than CAP instances keep one t-group per
// region and go through the global workspace. A and Y are bitwise those of rowgate_scores_kernel
// + softmax_pool_kernel (same tile code, same softmax_group).
// ---------------------------------------------------------------------------------------
template <int MAXC>
__host__ __device__ constexpr int rg_fused_cap() { return fused_cap<MAXC>(); }
template <int NCB, int MAXC>
__host__ __device__ inline size_t rg_fused_lds_bytes(int L, int G, int C, int D) {
    return rg_lds_bytes<NCB, MAXC>(L, G, C, D) + (size_t)2 * rg_fused_cap<MAXC>() * MAXC * 4 + 16 * 4 + 64;
}

// Lane record of row S + rho of a region (rho >= rows: padding).
__device__ __forceinline__ RgLane rg_lane_region(const GateParams& p, const Region& rg, long long rho) {
    RgLane rl;
    int hrow = -1, t = 0, n = 0;
    if (rho < rg.rows) {
        const uint32_t r = (uint32_t)rho;
        const uint32_t tt = r / (uint32_t)rg.Nb;
        n = (int)(r - tt * (uint32_t)rg.Nb);
        t = rg.t0 + (int)tt;
        hrow = rg.ob + n;
    }
    const int hl = (threadIdx.x >> 5) & 1;
    rl.h = reinterpret_cast<const char*>(p.H) + ((size_t)(hrow >= 0 ? hrow : 0) * p.ldh + 8 * hl) * 2;
    rl.n = (uint32_t)n;
    rl.t = (uint32_t)(p.t_base + t);
    rl.bagc = p.bag_ids ? p.bag_ids[rg.bag] : p.bag_base + (uint32_t)rg.bag;
    rl.inval = hrow >= 0 ? 0u : 0xFFFFFFFFu;
    rl.R = rg.S + rho;
    rl.bag = rg.bag;
    rl.kf = nullptr;   // the fused kernel makes its own masks
    return rl;
}

template <int G, int DB, int MAXC, bool DMA>
__global__ __launch_bounds__(kRgThreads, 1) void rowgate_fused_kernel(const GateParams p) {
    constexpr int NCB = 2 * G * DB;
    constexpr int CAP = rg_fused_cap<MAXC>();
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* slg = reinterpret_cast<float*>(smem + rg_lds_bytes<NCB, MAXC>(p.L, p.G, p.C, p.D));   // [CAP][C]
    float* szz = slg + CAP * MAXC;                                                             // [CAP][C]
    float* sred = szz + CAP * MAXC;                                                            // [16]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Region rg;
    if (!decode_region(p, (int)blockIdx.x, CAP, rg)) return;   // grid rounded up (ragged bags)
    clock_probe(p, 0);
    __amdgpu_buffer_rsrc_t wrs;
    RgPipe<NCB, MAXC, DMA> pp;
    rg_setup<NCB, MAXC, DMA>(p, smem, wrs, pp);
    const bool in_lds = rg.Nb <= CAP;
    float* lg_out = in_lds ? slg : p.logits;
    float* z_out = in_lds ? szz : p.zz;
    const long long obase = in_lds ? rg.S : 0;
    auto rho_of = [&](int i) {
        return i < rg.ntiles ? (long long)region_tile(rg, i) * kRgRows + 32 * wave + (lane & 31) : rg.rows;
    };
    RgLane rl = rg_lane_region(p, rg, rho_of(0));
    __syncthreads();
    rg_first<NCB, MAXC, false, DMA>(p, smem, rl, pp);
    f32x16 acc[NCB];
    float zp[MAXC];
    for (int i = 0; i < rg.ntiles; ++i) {
        const RgLane rn = rg_lane_region(p, rg, rho_of(i + 1));
        rg_kloop<NCB, MAXC, false, DMA>(p, smem, wrs, rl, rn, pp, acc, zp);
        rg_epilogue<G, DB, MAXC, false>(p, smem, rl, acc, zp, [&](const RgLane& r, int c, float lg, float z) {
            const size_t o = (size_t)(r.R - obase) * p.C + c;
            lg_out[o] = lg;
            z_out[o] = z;
        });
        rl = rn;
    }
    __syncthreads();
    // softmax + pooling per t-group (model.py:305-316)
    const int ng = rg.t1 - rg.t0;
    for (int j = 0; j < ng; ++j) {
        const long long row0 = (long long)j * rg.Nb;
        const float* lgj = in_lds ? slg + row0 * p.C : p.logits + (rg.S + row0) * p.C;
        const float* zzj = in_lds ? szz + row0 * p.C : p.zz + (rg.S + row0) * p.C;
        float* Ao = p.A ? p.A + (size_t)p.T * p.C * rg.ob + (size_t)(rg.t0 + j) * p.C * rg.Nb : nullptr;
        float* Yo = p.Y + ((size_t)rg.bag * p.T + rg.t0 + j) * p.C;
        softmax_group(threadIdx.x, true, rg.Nb, p.C, lgj, zzj, Ao, Yo, sred);
    }
    clock_probe(p, 1);
}

}  // namespace mcgmil
