#pragma once
// gate_w4_kernel -- timing study (MCGMIL_GATE=w4, two-kernel path only): the pipelined gate tile of
// gate_pipe_kernel with ONE wave per SIMD instead of two. A 4-wave workgroup owns a 128-row tile;
// wave w owns gate tile pairs 4w .. 4w+3 (one class: bf16 separate heads, P = 16) for all 8 row
// tiles, i.e. 64 accumulator tiles (256 registers, AGPR-resident), and the classifier tile of row
// tiles 2w, 2w+1. Per K step a wave issues 66 MFMAs against the same per-SIMD VALU (two Philox
// draws per thread), with no co-resident partner: the question it answers is whether a single,
// register-rich wave per SIMD keeps the matrix pipe busier than two lock-stepped ones
// (DESIGN.md §5, round 4). Reference semantics: model.py:280-303 (as gate_pipe_kernel).
#include "mcgmil_kernels.h"

namespace mcgmil {

constexpr int kW4Threads = 256;
constexpr int kW4Waves = kW4Threads / kWave;

template <int MAXC>
__host__ __device__ constexpr size_t w4_lds_bytes() {
    return (size_t)2 * kPipeBM * 32 * 2                 // two staging slots (bf16)
           + (size_t)kW4Waves * 4 * kPipeBM * 4          // partial scores [wave][lane group][row]
           + (size_t)MAXC * kPipeBM * 4                  // classifier projections
           + (size_t)kRowInfo * kPipeBM * 4;             // row table
}

template <int MAXC>
__global__ __launch_bounds__(kW4Threads, 1) void gate_w4_kernel(const GateParams p) {
    using E = __bf16;
    constexpr int BM = kPipeBM, RT = BM / 16, PPW = 4, NJ = 2 * PPW;
    constexpr int SLOT = RT * 64 * 8;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    E* Xs = reinterpret_cast<E*>(smem);
    float* red = reinterpret_cast<float*>(smem + (size_t)2 * SLOT * sizeof(E));
    float* zred = red + kW4Waves * 4 * BM;
    int* rinfo = reinterpret_cast<int*>(zred + MAXC * BM);
    const long long R0 = (long long)blockIdx.x * BM;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int KS = p.L >> 5;

    fill_row_table<BM>(p, R0, rinfo);
    __syncthreads();

    // staging items tid and tid + 256: rows (wave + 4h) * 16 + (lane & 15), chunk kq = lane >> 4
    const int kq = lane >> 4;
    const E* hsrc[2];
    uint32_t cn[2], ct[2], cb[2], inval[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int* ri = rinfo + kRowInfo * ((wave + 4 * h) * 16 + (lane & 15));
        const int hrow = ri[0];
        hsrc[h] = reinterpret_cast<const E*>(p.H) + (size_t)(hrow >= 0 ? hrow : 0) * p.ldh + kq * 8;
        cn[h] = (uint32_t)ri[2];
        ct[h] = (uint32_t)(p.t_base + ri[1]);
        cb[h] = (uint32_t)ri[5];
        inval[h] = hrow >= 0 ? 0u : 0xFFFFFFFFu;
    }
    struct Raw2 { Raw<E> r[2]; };
    auto load2 = [&](int s) {
        Raw2 x;
        x.r[0] = load_raw(hsrc[0] + (size_t)s * 32);
        x.r[1] = load_raw(hsrc[1] + (size_t)s * 32);
        return x;
    };
    auto stage = [&](int s, const Raw2& h, E* slot) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint4 o = philox4x32_10<true>((uint32_t)(s * 4 + kq), cn[k], ct[k], cb[k], p.k0, p.k1);
            store_dropped(h.r[k], o, p.thrx_f, inval[k], slot + (size_t)(tid + 256 * k) * 8);
        }
    };

    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(p.Wp, p.wp_bytes);
    const uint32_t tile_bytes = (uint32_t)KS * 512u * (uint32_t)sizeof(E);
    constexpr uint32_t kStepBytes = 512u * (uint32_t)sizeof(E);
    const int q0 = __builtin_amdgcn_readfirstlane(wave) * PPW;
    uint32_t wsoff[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) wsoff[j] = (uint32_t)(2 * (q0 + (j >> 1)) + (j & 1)) * tile_bytes;
    const uint32_t zsoff = (uint32_t)(2 * p.P) * tile_bytes;
    const uint32_t lane_b = (uint32_t)lane * 8u * (uint32_t)sizeof(E);
    auto wfrag = [&](uint32_t soff) { return load_frag_buf<E>(wrs, lane_b, soff); };
    const int zr0 = 2 * __builtin_amdgcn_readfirstlane(wave);   // classifier row tiles zr0, zr0 + 1

    f32x4 acc[RT][NJ];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 zacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};

    auto kstep = [&](int s, const E* cur, E* nxt, const Frag<E> (&w)[NJ], const Frag<E>& z,
                     Frag<E> (&wn)[NJ], Frag<E>& zn, const Raw2& h, Raw2& hn) {
        const int s1 = s + 1 < KS ? s + 1 : KS - 1;
        const int sh = s + HD < KS ? s + HD : KS - 1;
#pragma unroll
        for (int j = 0; j < NJ; ++j) wn[j] = wfrag(wsoff[j] + (uint32_t)s1 * kStepBytes);
        zn = wfrag(zsoff + (uint32_t)s1 * kStepBytes);
        hn = load2(sh);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const Frag<E> x = load_frag(cur + (size_t)(rt * 64 + lane) * 8);
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[rt][j] = mma(w[j], x, acc[rt][j]);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k)
            zacc[k] = mma(z, load_frag(cur + (size_t)((zr0 + k) * 64 + lane) * 8), zacc[k]);
        stage(s + 1, h, nxt);
#pragma unroll
        for (int i = 0; i < RT * NJ + 2; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // VALU
        }
        __syncthreads();
    };

    Frag<E> wA[NJ], wB[NJ], zA, zB;
    Raw2 hA = load2(0), hB = load2(1);
#pragma unroll
    for (int j = 0; j < NJ; ++j) wA[j] = wfrag(wsoff[j]);
    zA = wfrag(zsoff);
    stage(0, hA, Xs);
    __syncthreads();
    kstep(0, Xs, Xs + SLOT, wA, zA, wB, zB, hB, hA);
    kstep(1, Xs + SLOT, Xs, wB, zB, wA, zA, hA, hB);
    for (int s = 2; s < KS; s += 2) {
        kstep(s, Xs, Xs + SLOT, wA, zA, wB, zB, hB, hA);
        kstep(s + 1, Xs + SLOT, Xs, wB, zB, wA, zA, hA, hB);
    }

    // epilogue: this wave's 4 pairs belong to class q0 / (D / 16)
    float part[MAXC][RT];
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) part[c][rt] = 0.f;
    fold_pairs<RT, PPW, MAXC, true>(p, acc, q0, lane, part);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) red[((size_t)wave * 4 + (lane >> 4)) * BM + rt * 16 + (lane & 15)] = part[0][rt];
    if (lane < 16) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int c = 0; c < MAXC; ++c) zred[c * BM + (zr0 + k) * 16 + lane] = zacc[k][c];
    }
    __syncthreads();
    // scores: thread -> (row tid & 127, class tid >> 7); class c's partials come from waves
    // c * wpg .. c * wpg + wpg - 1
    const int r = tid & (BM - 1), c = tid >> 7;
    if (c >= p.C) return;
    const int* ri = rinfo + kRowInfo * r;
    if (ri[0] < 0) return;
    const int wpg = (p.D >> 4) / PPW;
    float s = 0.f;
    for (int k = 0; k < wpg; ++k) {
        const float* src = red + (size_t)((c * wpg + k) * 4) * BM + r;
#pragma unroll
        for (int g = 0; g < 4; ++g) s += src[g * BM];
    }
    s += p.ba[c];
    const bool keep = attention_keep(p.k0, p.k1, (uint32_t)ri[5], (uint32_t)(p.t_base + ri[1]), (uint32_t)c,
                                     (uint32_t)ri[2], p.thr_a);
    const size_t o = (size_t)(R0 + r) * p.C + c;
    p.logits[o] = s * (keep ? p.sa : 0.f);
    p.zz[o] = zred[c * BM + r] * p.sf;
}

}  // namespace mcgmil
