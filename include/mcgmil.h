/*
 * mcgmil.h -- C ABI of the MI355X (gfx950) Monte-Carlo-dropout gated-attention MIL hot path.
 *
 * Drop-in boundary for xkuubix/MonteCarlo-Gated-MIL's inference hot path: everything in
 * MultiHeadGatedAttentionMIL.mc_inference after feature extraction (reference model.py:279-328),
 * i.e. feature dropout -> gated attention (tanh/sigmoid gates, per-class attention logits)
 * -> logit dropout -> softmax over instances -> attention pooling -> per-class classifier,
 * for all T Monte-Carlo samples and any number of bags in one call.
 *
 * Reference interfaces replaced (the reference has no FFI; its "operator API" is the
 * nn.Module, so each entry cites the method it serves):
 *   mcgmil_mcdo_forward   <- MultiHeadGatedAttentionMIL.mc_inference   (model.py:256-328)
 *                            MultiHeadGatedAttentionMIL.mc_inference_serial (model.py:330-401,
 *                              called per sample with T=1, t_base=t)
 *                            MultiHeadGatedAttentionMIL.forward in eval mode (model.py:211-253,
 *                              T=1, p_feat=p_att=0)
 *                            + the callers' uncertainty statistics (infer.py:195,212-219;
 *                              net_utils.py:207-208) when A_mean/A_var/P_mean are requested
 *   mcgmil_pack_weights   <- the parameter layout of __init__ (model.py:182-203), re-laid out
 *                            for the kernel once per model
 *   mcgmil_gate_softmax_pool
 *                         <- model.py:280-316 for all T samples: the two stages below, or ONE
 *                            fused launch (args->flags); A and Y are bitwise the same either way
 *   mcgmil_gate_scores / mcgmil_softmax_pool / mcgmil_bag_stats
 *                         <- the stages of mcgmil_mcdo_forward, exposed for profiling
 *   mcgmil_feature_keep / mcgmil_attention_keep
 *                         <- the dropout masks the kernel draws (nn.Dropout at model.py:206-209),
 *                            materialised for parity tests
 *
 * Conventions
 *   - All pointers are DEVICE pointers unless stated; the caller owns every buffer (no
 *     allocation inside). `stream` is a hipStream_t (NULL = default stream). Every call is
 *     asynchronous and stream-ordered; no host synchronisation happens inside.
 *   - Return value 0 on success, a negative MCGMIL_E* code on error; the message is then
 *     available from mcgmil_last_error() (thread-local).
 *   - Re-entrant: the library keeps no mutable global state besides the thread-local error.
 *   - Layouts follow the reference tensors: Y[b] is the reference's Y[T,1,C] (as [T,C]), A of a
 *     bag is the reference's A[T,1,C,N] (as [T,C,N]).
 */
#ifndef MCGMIL_H_
#define MCGMIL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCGMIL_ABI_VERSION 6   /* 2: mcgmil_args.flags (path selection); 3: mcgmil_conv_args.flags,
                                  mcgmil_stem_args.flags (mcgmil_features.h); 4: MCGMIL_CLOCK_PROBE (and a
                                  row-gate flag); 5: the row-gate flag (3 << 2) and its weight stream in the
                                  packed weights removed -- measured slower everywhere, DESIGN.md §5;
                                  6: mcgmil_conv_args.workspace / workspace_bytes and
                                  mcgmil_conv_workspace_size (the convolutions' K split) */

enum mcgmil_status {
    MCGMIL_OK = 0,
    MCGMIL_E_INVALID = -1,   /* bad size / pointer / probability */
    MCGMIL_E_UNSUPPORTED = -2, /* valid for the reference but not built here (e.g. C > 4) */
    MCGMIL_E_ALIGN = -3,     /* H / ldh not 16-byte aligned */
    MCGMIL_E_WORKSPACE = -4, /* workspace missing or too small */
    MCGMIL_E_HIP = -5        /* a HIP runtime call failed (message has the HIP error) */
};

enum mcgmil_dtype { MCGMIL_F32 = 0, MCGMIL_BF16 = 1 };

/* mcgmil_args.flags: which launch path mcgmil_gate_softmax_pool / mcgmil_mcdo_forward take. All
 * paths give bitwise the same A and Y (tests/test_gpu_fused.py); the choice is performance only.
 * The environment variables MCGMIL_FUSED (0 | 1 | auto) and MCGMIL_GATE (pipe | pp), when
 * set, override the flags (A/B timing of an unmodified caller); they are read once per process. */
enum mcgmil_flags {
    MCGMIL_PATH_AUTO = 0,        /* fused launch for bf16 batches of equal-size bags with >= 16,384
                                    regions whose heads run gate_pipe_kernel (separate heads), else
                                    the two kernels */
    MCGMIL_PATH_FUSED = 1,       /* the fused launch (gate_fused_kernel) whenever it applies: bf16 or
                                    fp32, L % 64 == 0, L >= 128, the tile within 160 KiB of LDS
                                    (bf16: L <= 1024), <= 16 gate tile pairs, no replay masks, and
                                    for bf16 heads the two-kernel path would run on gate_pipe_kernel
                                    (> 8 gate tile pairs, or MCGMIL_GATE_PIPE) -- the fused launch
                                    runs that kernel's tile code; heads on gate_pp_kernel (shared
                                    heads) always take the two kernels */
    MCGMIL_PATH_TWO_KERNEL = 2,  /* never fused: gate scores -> workspace -> softmax/pooling */
    MCGMIL_PATH_MASK = 3,
    MCGMIL_GATE_AUTO = 0 << 2,   /* two-kernel path, bf16 heads: gate_pipe_kernel for > 8 gate tile
                                    pairs (separate heads), gate_pp_kernel for <= 8 (shared) */
    MCGMIL_GATE_PIPE = 1 << 2,   /* always gate_pipe_kernel (one 8-wave workgroup per CU) */
    MCGMIL_GATE_PP = 2 << 2,     /* gate_pp_kernel (two 4-wave workgroups per CU) where it applies;
                                    3 << 2 is invalid since ABI 5 */
    MCGMIL_GATE_MASK = 3 << 2,
    MCGMIL_CLOCK_PROBE = 1 << 4  /* measurement: the gate launch's workgroups 0..MCGMIL_CLOCK_SLOTS-1
                                    write their (s_memtime, s_memrealtime) at start and end into
                                    args->debug ([MCGMIL_CLOCK_SLOTS][4] uint64, required): the shader
                                    clock the launch ran at = d(memtime) / d(realtime) x 100 MHz.
                                    Outputs are unchanged; no stamp executes without the flag.
                                    Stamped launches: gate_fused_kernel, gate_pipe_kernel and
                                    gate_pp_kernel with their own Philox masks; the replay-mask,
                                    generic (gate_scores_kernel) and softmax/statistics kernels write
                                    no record, so a record stays all zero when only they ran */
};
#define MCGMIL_CLOCK_SLOTS 1024

typedef struct mcgmil_args {
    /* ---- sizes ---- */
    int32_t L;            /* feature dim (reference L, model.py:140; 512 for r18/r34) */
    int32_t D;            /* gate dim (reference D, model.py:141; 128) */
    int32_t C;            /* classes = attention heads (num_classes, model.py:137; 2), 1..4 */
    int32_t G;            /* distinct gate pairs: 1 if shared_attention else C (model.py:182-193) */
    int32_t T;            /* Monte-Carlo samples (mc_inference's `N` argument, model.py:256) */
    int32_t num_bags;     /* B >= 1 */
    int64_t total_rows;   /* sum of bag sizes = rows of H (host-known) */
    /* ---- instances ---- */
    int32_t h_dtype;      /* mcgmil_dtype of H and of the GEMM operands */
    int32_t uniform_bag_rows; /* optional hint: N if every bag has N rows (bag_offsets[b] = b*N),
                                 0 otherwise; lets the kernels map rows to bags arithmetically */
    const void* H;        /* [total_rows, ldh] row-major; bag b = rows bag_offsets[b]..[b+1] */
    int64_t ldh;          /* row stride of H in elements (>= L) */
    const int32_t* bag_offsets; /* [B+1] CSR row offsets, bag_offsets[0] = 0 */
    /* ---- parameters: fp32, torch nn.Linear layout ---- */
    const float* Wv;      /* [G, D, L]  attention_V[g][0].weight */
    const float* bv;      /* [G, D]     attention_V[g][0].bias   */
    const float* Wu;      /* [G, D, L]  attention_U[g][0].weight */
    const float* bu;      /* [G, D]     attention_U[g][0].bias   */
    const float* wa;      /* [C, D]     attention_weights[c].weight */
    const float* ba;      /* [C]        attention_weights[c].bias   */
    const float* wk;      /* [C, L]     classifiers[c].weight (no bias) */
    const void* packed_w; /* optional: output of mcgmil_pack_weights for these parameters;
                             NULL = pack into the workspace on every call */
    /* ---- dropout ---- */
    float p_feat;         /* feature_dropout.p   (model.py:206), 0 = off */
    float p_att;          /* attention_dropouts[c].p (model.py:207-209), 0 = off */
    uint64_t seed;        /* Philox key */
    uint32_t bag_id_base; /* bag b draws with bag counter bag_id_base + b ... */
    int32_t t_base;       /* sample t draws with sample counter t_base + t */
    const uint32_t* bag_ids; /* ... or, if not NULL, with bag counter bag_ids[b] ([B], device):
                                lets a shard of a larger batch draw its bags' global streams */
    const uint8_t* keep_feat; /* optional replay mask (parity mode): packed bits
                                 [sum_b T*N_b rows (order bag,t,n)][L/8], bit l&7 of byte l>>3 */
    const uint8_t* keep_att;  /* optional replay mask: [sum_b T*C*N_b] bytes (order bag,t,c,n) */
    /* ---- outputs (fp32) ---- */
    float* Y;             /* [B, T, C] class logits (required) */
    float* A;             /* [sum_b T*C*N_b] attention (order bag,t,c,n), or NULL */
    float* A_mean;        /* [sum_b C*N_b] mean over T (order bag,c,n), or NULL */
    float* A_var;         /* [sum_b C*N_b] unbiased variance over T, or NULL */
    float* P_mean;        /* [B, C] mean over T of softmax(Y), or NULL */
    /* ---- scratch ---- */
    void* workspace;      /* >= mcgmil_workspace_size() bytes, 256-byte aligned */
    size_t workspace_bytes;
    void* debug;          /* with MCGMIL_CLOCK_PROBE: the clock record; diagnostic builds
                             (-DMCGMIL_STAMPS): per-tile s_memtime stamps. NULL otherwise */
    /* ---- policy ---- */
    int32_t flags;        /* mcgmil_flags: MCGMIL_PATH_* | MCGMIL_GATE_* (0 = auto) */
    int32_t reserved;     /* must be 0 */
} mcgmil_args;

int mcgmil_abi_version(void);
size_t mcgmil_args_size(void);          /* sizeof(mcgmil_args), for binding checks */
const char* mcgmil_last_error(void);

/* Bytes of scratch mcgmil_mcdo_forward needs for these sizes. */
int mcgmil_workspace_size(const mcgmil_args* a, size_t* bytes);
/* Bytes of the packed-weight buffer for (L, D, C, G, h_dtype). */
int mcgmil_packed_weights_size(const mcgmil_args* a, size_t* bytes);
/* Re-lay the fp32 parameters out as MFMA operand tiles of dtype h_dtype into `packed`. */
int mcgmil_pack_weights(const mcgmil_args* a, void* packed, void* stream);

/* The whole hot path: [pack] -> gate scores + softmax + pooling -> [statistics]. */
int mcgmil_mcdo_forward(const mcgmil_args* a, void* stream);

/* Its stages (same args/workspace; call in this order, after packing if packed_w is NULL):
 * mcgmil_gate_softmax_pool, then mcgmil_bag_stats. mcgmil_gate_softmax_pool is
 * ONE fused launch (gate scores, softmax, pooling) or mcgmil_gate_scores followed by
 * mcgmil_softmax_pool, as args->flags selects (MCGMIL_PATH_*; default auto: fused for bf16
 * batches of equal-size bags with >= 16,384 regions). Both give bitwise the same A and Y. */
int mcgmil_gate_softmax_pool(const mcgmil_args* a, void* stream);
/* The fused launch mcgmil_gate_softmax_pool would make for these args: *regions = its number of
 * workgroups (one per region of t-groups of a bag; an upper bound for ragged bags), or 0 when
 * it would run the two-kernel path. Launches nothing. */
int mcgmil_fused_regions(const mcgmil_args* a, int64_t* regions);
int mcgmil_gate_scores(const mcgmil_args* a, void* stream);
int mcgmil_softmax_pool(const mcgmil_args* a, void* stream);
int mcgmil_bag_stats(const mcgmil_args* a, void* stream);

/* Materialise the masks the kernel draws for a batch (same layouts as keep_feat/keep_att).
 * Uses L, C, T, num_bags, total_rows, bag_offsets, p_feat/p_att, seed, bag_id_base, t_base. */
int mcgmil_feature_keep(const mcgmil_args* a, uint8_t* keep_feat, void* stream);
int mcgmil_attention_keep(const mcgmil_args* a, uint8_t* keep_att, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MCGMIL_H_ */
