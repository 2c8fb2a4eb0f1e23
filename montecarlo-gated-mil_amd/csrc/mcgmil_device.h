// Device-side building blocks shared by the MCDO kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcgmil {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int kWave = 64;

// ---------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. SC'11). Bit-exact with oracle/philox_oracle.c; the key words
// are wave-uniform (the seed), so the key schedule lives in SGPRs.
// ---------------------------------------------------------------------------------------
// FLIP_XZ: output words x and z come out XORed with 0x80008000 (the sign flip of the packed
// keep rule, drop_mask16x2_flipped) -- folded into the last round's key words, i.e. free.
// ROUNDS: 10 is the product stream (Random123's default); other counts exist for timing studies.
template <bool FLIP_XZ = false, int ROUNDS = 10>
__device__ __forceinline__ uint4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        if (FLIP_XZ && r == ROUNDS - 1) {
            k0 ^= 0x80008000u;
            k1 ^= 0x80008000u;
        }
        // one v_mad_u64_u32 per product gives both halves (measured: the cost of one
        // v_mul_hi_u32, half of a separate mul_lo + mul_hi pair)
        const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u;
        const uint64_t p1 = (uint64_t)c2 * 0xCD9E8D57u;
        // hi ^ c ^ key as ONE v_bitop3_b32 (truth table 0x96; gfx950 has no v_xor3_b32)
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

// Packed form of the keep rule for the two 16-bit draws of one Philox word: returns 0xFFFF in
// each half whose draw is DROPPED (u16 < thr) and 0 where it is kept. thrx = the threshold
// (clamped to 65535; p = 1 is handled by the zero dropout scale) with its sign bit flipped, in
// both halves: u >= thr (unsigned) <=> (u ^ 0x8000) >= (thr ^ 0x8000) (signed), and a
// saturating signed difference keeps the sign. v_xor + v_pk_sub_i16 clamp + v_pk_ashrrev_i16.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t drop_mask16x2(uint32_t word, uint32_t thrx) {
    const s16x2 u = __builtin_bit_cast(s16x2, word ^ 0x80008000u);
    const s16x2 d = __builtin_elementwise_sub_sat(u, __builtin_bit_cast(s16x2, thrx));
    return __builtin_bit_cast(uint32_t, d >> (s16x2){15, 15});
}

// drop_mask16x2 of a word that is already XORed with 0x80008000.
__device__ __forceinline__ uint32_t drop_mask16x2_flipped(uint32_t flipped, uint32_t thrx) {
    const s16x2 u = __builtin_bit_cast(s16x2, flipped);
    const s16x2 d = __builtin_elementwise_sub_sat(u, __builtin_bit_cast(s16x2, thrx));
    return __builtin_bit_cast(uint32_t, d >> (s16x2){15, 15});
}

__host__ __device__ inline uint32_t packed_threshold(uint32_t thr) {
    const uint32_t t = (thr > 65535u ? 65535u : thr) ^ 0x8000u;
    return t | (t << 16);
}

// Eight keep decisions (bit m = draw m) from one Philox block: keep iff u16 >= thr.
__device__ __forceinline__ uint32_t keep_byte(uint4 o, uint32_t thr) {
    uint32_t b = 0;
    b |= (uint32_t)((o.x & 0xFFFFu) >= thr) << 0;
    b |= (uint32_t)((o.x >> 16) >= thr) << 1;
    b |= (uint32_t)((o.y & 0xFFFFu) >= thr) << 2;
    b |= (uint32_t)((o.y >> 16) >= thr) << 3;
    b |= (uint32_t)((o.z & 0xFFFFu) >= thr) << 4;
    b |= (uint32_t)((o.z >> 16) >= thr) << 5;
    b |= (uint32_t)((o.w & 0xFFFFu) >= thr) << 6;
    b |= (uint32_t)((o.w >> 16) >= thr) << 7;
    return b;
}

__device__ __forceinline__ uint32_t draw_u16(uint4 o, int m) {
    const uint32_t w = (m >> 1) == 0 ? o.x : (m >> 1) == 1 ? o.y : (m >> 1) == 2 ? o.z : o.w;
    return (w >> (16 * (m & 1))) & 0xFFFFu;
}

// Attention-logit keep decision for (bag counter, sample counter, class, instance).
__device__ __forceinline__ bool attention_keep(uint32_t k0, uint32_t k1, uint32_t bagc, uint32_t tc,
                                               uint32_t c, uint32_t n, uint32_t thr) {
    const uint4 o = philox4x32_10(n >> 3, c, tc | 0x80000000u, bagc, k0, k1);
    return draw_u16(o, (int)(n & 7u)) >= thr;
}

// ---------------------------------------------------------------------------------------
// 8-element MFMA operand fragments. For both dtypes lane l of a 16x16 tile carries
// row/col (l & 15) and the 8 consecutive k values 8*(l >> 4) + j of a 32-deep K step:
//   bf16: one v_mfma_f32_16x16x32_bf16 per K step;
//   f32 : eight v_mfma_f32_16x16x4_f32 (MFMA j sums k = 8*kk + j over kk = l >> 4).
// C/D layout (both): col = l & 15, row = 4*(l >> 4) + v.
// ---------------------------------------------------------------------------------------
template <typename E> struct Frag;
template <> struct Frag<__bf16> { bf16x8 v; };
template <> struct Frag<float> { f32x4 lo, hi; };

__device__ __forceinline__ Frag<__bf16> load_frag(const __bf16* p) {
    Frag<__bf16> f; f.v = *reinterpret_cast<const bf16x8*>(p); return f;
}
__device__ __forceinline__ Frag<float> load_frag(const float* p) {
    Frag<float> f;
    f.lo = *reinterpret_cast<const f32x4*>(p);
    f.hi = *reinterpret_cast<const f32x4*>(p + 4);
    return f;
}
// Fragment loads through a buffer descriptor: voffset = the lane's byte offset, soffset = a
// wave-uniform byte offset (SGPR), so address arithmetic stays scalar. DATA_FORMAT=32 in
// word 3 (0x00020000), stride 0, range = bytes.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <typename E>
__device__ __forceinline__ Frag<E> load_frag_buf(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff);
template <>
__device__ __forceinline__ Frag<__bf16> load_frag_buf<__bf16>(__amdgpu_buffer_rsrc_t r, uint32_t voff,
                                                              uint32_t soff) {
    Frag<__bf16> f;
    f.v = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
    return f;
}
template <>
__device__ __forceinline__ Frag<float> load_frag_buf<float>(__amdgpu_buffer_rsrc_t r, uint32_t voff,
                                                            uint32_t soff) {
    Frag<float> f;
    f.lo = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
    f.hi = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16u, soff, 0));
    return f;
}

template <typename E> __device__ __forceinline__ Frag<E> zero_frag();
template <> __device__ __forceinline__ Frag<__bf16> zero_frag<__bf16>() {
    Frag<__bf16> f; f.v = bf16x8{}; return f;
}
template <> __device__ __forceinline__ Frag<float> zero_frag<float>() {
    Frag<float> f; f.lo = f32x4{0.f, 0.f, 0.f, 0.f}; f.hi = f.lo; return f;
}

__device__ __forceinline__ f32x4 mma(const Frag<__bf16>& a, const Frag<__bf16>& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma(const Frag<float>& a, const Frag<float>& b, f32x4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.x, b.lo.x, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.y, b.lo.y, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.z, b.lo.z, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo.w, b.lo.w, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.x, b.hi.x, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.y, b.hi.y, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.z, b.hi.z, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi.w, b.hi.w, c, 0, 0, 0);
    return c;
}

// Load 8 consecutive features of one instance row and zero the dropped ones (bit m of kb).
// The dropout scale is applied to the fp32 GEMM result instead (exact selection here).
__device__ __forceinline__ void load_masked(const __bf16* src, uint32_t kb, __bf16* dst) {
    uint4 h = *reinterpret_cast<const uint4*>(src);
    const uint32_t m0 = ((kb & 1u) ? 0x0000FFFFu : 0u) | ((kb & 2u) ? 0xFFFF0000u : 0u);
    const uint32_t m1 = ((kb & 4u) ? 0x0000FFFFu : 0u) | ((kb & 8u) ? 0xFFFF0000u : 0u);
    const uint32_t m2 = ((kb & 16u) ? 0x0000FFFFu : 0u) | ((kb & 32u) ? 0xFFFF0000u : 0u);
    const uint32_t m3 = ((kb & 64u) ? 0x0000FFFFu : 0u) | ((kb & 128u) ? 0xFFFF0000u : 0u);
    h.x &= m0; h.y &= m1; h.z &= m2; h.w &= m3;
    *reinterpret_cast<uint4*>(dst) = h;
}
__device__ __forceinline__ void load_masked(const float* src, uint32_t kb, float* dst) {
    f32x4 a = *reinterpret_cast<const f32x4*>(src);
    f32x4 b = *reinterpret_cast<const f32x4*>(src + 4);
    a.x = (kb & 1u) ? a.x : 0.f;   a.y = (kb & 2u) ? a.y : 0.f;
    a.z = (kb & 4u) ? a.z : 0.f;   a.w = (kb & 8u) ? a.w : 0.f;
    b.x = (kb & 16u) ? b.x : 0.f;  b.y = (kb & 32u) ? b.y : 0.f;
    b.z = (kb & 64u) ? b.z : 0.f;  b.w = (kb & 128u) ? b.w : 0.f;
    *reinterpret_cast<f32x4*>(dst) = a;
    *reinterpret_cast<f32x4*>(dst + 4) = b;
}
__device__ __forceinline__ void store_zero8(__bf16* dst) {
    *reinterpret_cast<uint4*>(dst) = make_uint4(0u, 0u, 0u, 0u);
}
__device__ __forceinline__ void store_zero8(float* dst) {
    *reinterpret_cast<f32x4*>(dst) = f32x4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4*>(dst + 4) = f32x4{0.f, 0.f, 0.f, 0.f};
}

// Bag lookup in the flattened (bag, t, n) row space: largest b with T*off[b] <= R.
__device__ __forceinline__ int find_bag(const int32_t* off, int B, long long scale, long long R) {
    int lo = 0, hi = B;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (scale * (long long)off[mid] <= R) lo = mid; else hi = mid;
    }
    return lo;
}

// Block-wide reductions for 256-thread blocks.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// BatchNorm statistics blocks (count, mean, M2): (n, m, M2) <- merge with (nb, mb, M2b) for every
// channel, Chan's pairwise update (the counts are shared by the channels). The convolution
// epilogues (mcgmil_conv.hip, mcgmil_conv32.hip) reduce their outputs' statistics with it.
template <int NCH>
__device__ __forceinline__ void chan_merge(float& n, float (&m)[NCH], float (&M2)[NCH], float nb,
                                           const float (&mb)[NCH], const float (&M2b)[NCH]) {
    const float nn = n + nb;
    const float f = nn > 0.f ? nb / nn : 0.f, h = n * f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const float d = mb[c] - m[c];
        m[c] = fmaf(d, f, m[c]);
        M2[c] = M2[c] + M2b[c] + d * d * h;
    }
    n = nn;
}

}  // namespace mcgmil
