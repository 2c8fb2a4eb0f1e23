/*
 * TEST INFRASTRUCTURE -- CPU oracle for the dropout keep-masks of the MCDO hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker. The product path (montecarlo-gated-mil_amd/) never
 * links or calls it.
 *
 * What it restates
 * ----------------
 * The reference draws its dropout masks from torch's global CPU RNG:
 *   - feature dropout on the expanded features  H_drop = feature_dropout(H.expand(T,1,N,L))
 *     (reference model.py:280-281, module created at model.py:206);
 *   - attention-logit dropout per class          attention_dropouts[c](A[:, :, c, :])
 *     (reference model.py:291 shared / model.py:301 separate; modules model.py:207-209).
 * No GPU can reproduce torch's CPU generator, so the MI355X build replaces it with a
 * counter-based generator whose stream is a pure function of (seed, bag, t, n, l). This file
 * is the bit-exact CPU definition of that stream; the HIP kernel must match it bit for bit.
 * Parity with the reference's arithmetic is established by *mask replay*: the same keep
 * masks are fed into the reference module (tests/golden/make_golden.py) and the oracle.
 *
 * Generator: Philox4x32-10 (Salmon et al., SC'11, "Parallel random numbers: as easy as
 * 1, 2, 3"; Random123's philox4x32 with R=10). Known answers from Random123's kat_vectors
 * are checked in tests/test_philox.py.
 *
 * Keep rule (one 16-bit uniform per draw, eight draws per Philox call):
 *   thr  = min(65536, floor(p * 65536 + 0.5))           (drop probability = thr / 65536)
 *   keep = (u16 >= thr)
 * Counters (key = {seed_lo, seed_hi}; b = 32-bit bag counter = bag_id_base + bag index):
 *   feature   draw (b, t, n, l):  ctr = {l >> 3, n, t,              b}, lane m = l & 7
 *   attention draw (b, t, c, n):  ctr = {n >> 3, c, t | 0x80000000u, b}, lane m = n & 7
 *   u16 = (out[m >> 1] >> (16 * (m & 1))) & 0xFFFF
 * Survivors are scaled by torch's dropout factor 1.0f / (float)(1 - p) (verified against
 * torch.nn.functional.dropout on CPU: the scalar (1-p) is rounded to fp32 first).
 */
#include <stdint.h>
#include <string.h>
#include <math.h>

#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

static inline void mulhilo32(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    *lo = (uint32_t)p;
}

void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo32(PHILOX_M0, c0, &hi0, &lo0);
        mulhilo32(PHILOX_M1, c2, &hi1, &lo1);
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += PHILOX_W0; k1 += PHILOX_W1;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint32_t oracle_drop_threshold(double p) {
    if (!(p > 0.0)) return 0u;
    double x = floor(p * 65536.0 + 0.5);
    if (x >= 65536.0) return 65536u;
    return (uint32_t)x;
}

float oracle_dropout_scale(double p) {
    if (p >= 1.0) return 0.0f;
    return 1.0f / (float)(1.0 - p);
}

static inline uint32_t u16_of(const uint32_t out[4], int m) {
    return (out[m >> 1] >> (16 * (m & 1))) & 0xFFFFu;
}

/* Feature keep bits, packed little-endian: byte (t, n, l>>3), bit (l & 7).
 * out has T*N*(L/8) bytes; L must be a multiple of 8. t runs over [t0, t0+T). */
int oracle_feature_keep(uint64_t seed, uint32_t bag_ctr, int32_t t0, int32_t T, int32_t N,
                        int32_t L, uint32_t thr, uint8_t* out) {
    if (L % 8 != 0 || T < 0 || N < 0) return -1;
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    const int32_t LB = L / 8;
    for (int32_t t = 0; t < T; ++t)
        for (int32_t n = 0; n < N; ++n)
            for (int32_t lb = 0; lb < LB; ++lb) {
                uint32_t ctr[4] = {(uint32_t)lb, (uint32_t)n, (uint32_t)(t0 + t), bag_ctr};
                uint32_t o[4];
                oracle_philox4x32_10(ctr, key, o);
                uint8_t byte = 0;
                for (int m = 0; m < 8; ++m)
                    if (u16_of(o, m) >= thr) byte |= (uint8_t)(1u << m);
                out[((size_t)t * N + n) * LB + lb] = byte;
            }
    return 0;
}

/* Attention keep flags, one byte (0/1) per (t, c, n). t runs over [t0, t0+T). */
int oracle_attention_keep(uint64_t seed, uint32_t bag_ctr, int32_t t0, int32_t T, int32_t C,
                          int32_t N, uint32_t thr, uint8_t* out) {
    if (T < 0 || C < 0 || N < 0) return -1;
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int32_t t = 0; t < T; ++t)
        for (int32_t c = 0; c < C; ++c)
            for (int32_t n0 = 0; n0 < N; n0 += 8) {
                uint32_t ctr[4] = {(uint32_t)(n0 >> 3), (uint32_t)c,
                                   (uint32_t)(t0 + t) | 0x80000000u, bag_ctr};
                uint32_t o[4];
                oracle_philox4x32_10(ctr, key, o);
                for (int m = 0; m < 8 && n0 + m < N; ++m)
                    out[((size_t)t * C + c) * N + n0 + m] = (uint8_t)(u16_of(o, m) >= thr);
            }
    return 0;
}
