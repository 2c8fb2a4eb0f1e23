/* mcgmil_features.h -- C ABI of the feature extractor's normalisation layers (SURVEY.md §8(f)
 * row 1: the ResNet backbone that feeds the MCDO kernel, with BatchNorm on the bag's own batch
 * statistics). libmcgmil.so exports these next to include/mcgmil.h.
 *
 * Reference interface replaced:
 *   mcgmil_batchnorm_act   torch.nn.BatchNorm2d.forward of the backbone's BN layers
 *                          (torchvision BasicBlock/Bottleneck as built at model.py:166-177),
 *                          with the ReLU / residual add / stem max-pool that follows them, after
 *                          deactivate_batchnorm (infer.py:105-109: track_running_stats=False,
 *                          running stats None -> every forward normalises with the statistics
 *                          of the bag itself)
 *
 *   mcgmil_stem_forward    the torchvision stem maxpool(relu(bn1(conv1(x)))) of the same
 *                          backbone (ResNet.forward's first four layers), from the NCHW
 *                          instances the image patcher writes
 *
 *   mcgmil_conv2d          torch.nn.Conv2d.forward (bias=False, groups=1, dilation=1) of the
 *                          backbone's 3x3 / 1x1 convolutions (torchvision BasicBlock /
 *                          Bottleneck, model.py:166-177) under torch.autocast bf16, applied to
 *                          every instance of the bag at infer.py:191 -> model.py:275-277
 *
 * Layout: activations are channels-last (NHWC), i.e. a row-major [rows = N*H*W, C] matrix;
 * C a multiple of 8, rows >= 1, x / residual / y 16-byte aligned.
 *
 * Semantics (torch.nn.functional.batch_norm + relu):
 *   batch statistics (running_mean == running_var == NULL): mean_c = (1/rows) sum x[:, c],
 *     var_c = (1/rows) sum (x[:, c] - mean_c)^2 (biased, as torch normalises in training mode),
 *     accumulated in fp32 per workgroup around a per-channel shift (x[0, c]) and combined in fp64;
 *   running statistics (both given): mean_c, var_c as passed;
 *   y = x * a_c + b_c [+ residual] [then max(., 0)], with a_c = gamma_c / sqrt(var_c + eps) and
 *     b_c = beta_c - mean_c * a_c in fp32 (gamma = 1, beta = 0 when NULL); one rounding to the
 *     output dtype. torch rounds the BN output before the residual add; the fused form rounds
 *     once (<= 1 bf16 ulp apart).
 *   pooling (the torchvision stem, maxpool(relu(bn1(conv1(x))))): y[n, oh, ow, c] = max over the
 *     window of the activated values, computed from x without materialising them (rounding is
 *     monotonic, so this equals pooling the rounded activations); no residual with pooling.
 * y may alias x (in place) without pooling. Stream-ordered, no allocation, no host
 * synchronisation; errors are MCGMIL_E_* codes with mcgmil_last_error().
 */
#ifndef MCGMIL_FEATURES_H_
#define MCGMIL_FEATURES_H_

#include <stddef.h>
#include <stdint.h>

#include "mcgmil.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mcgmil_bn_args {
    int64_t rows;               /* N * H * W */
    int32_t channels;           /* C, multiple of 8, <= 2048 */
    int32_t dtype;              /* MCGMIL_BF16 or MCGMIL_F32 (x, residual and y) */
    const void* x;              /* [rows, C] */
    const void* residual;       /* [rows, C] added before the activation, or NULL */
    void* y;                    /* [rows, C], may alias x */
    const float* gamma;         /* [C] BN weight or NULL (1) */
    const float* beta;          /* [C] BN bias or NULL (0) */
    const float* running_mean;  /* [C]: running-statistics mode when both are given */
    const float* running_var;   /* [C] */
    double eps;                 /* BN eps (torch default 1e-5) */
    int32_t relu;               /* 1: max(., 0) after the (residual) add */
    int32_t batch, height, width;   /* N, H, W with rows == N * H * W (needed with pooling) */
    int32_t pool_kernel;        /* 0: none; k > 0: max-pool k x k after the activation */
    int32_t pool_stride, pool_pad;  /* torch MaxPool2d(k, stride, pad): -inf padding, floor mode;
                                       y is then [N * Ho * Wo, C], Ho = (H + 2 pad - k) / stride + 1 */
    int32_t num_partials;       /* rows of `partials` (0: none) */
    float* batch_mean;          /* optional out [C]: the mean used */
    float* batch_invstd;        /* optional out [C]: 1 / sqrt(var + eps) */
    void* workspace;            /* >= mcgmil_bn_workspace_size() bytes, 256-byte aligned */
    size_t workspace_bytes;
    const float* partials;      /* optional [num_partials][3][C] (count, mean, M2) blocks of x, as
                                   mcgmil_conv2d's / mcgmil_conv2d_f32's stats: batch statistics
                                   from them (Chan's combination in fp64, fixed order) instead of
                                   a pass over x. More than 1024 blocks are first combined in
                                   chunks of consecutive blocks (fp64, stored as fp32 blocks) in
                                   the workspace, so size it after setting partials */
    const float* residual_ab;   /* optional [2][C] (a_c, b_c) of the residual's own BatchNorm (as
                                   mcgmil_batchnorm_coefficients writes them): the added residual
                                   is dtype(fmaf(r, a_c, b_c)) -- bit-identical to normalising the
                                   residual in a pass of its own first (the ResNet downsample
                                   branch). Needs residual. NULL: r as is */
} mcgmil_bn_args;

size_t mcgmil_bn_args_size(void);   /* sizeof(mcgmil_bn_args), for binding checks */

/* Convolution y = conv2d(x, w, stride, pad) of channels-last bf16 activations as an implicit GEMM
 * on the matrix cores (fp32 accumulation, one rounding to bf16 -- torch.autocast's arithmetic up
 * to the summation order). x is [batch, height, width, in_channels], y is [batch, OH, OW,
 * out_channels] with OH = (height + 2 pad - kernel_h) / stride + 1 (likewise OW), both NHWC;
 * w is the packed weight [out_channels, kernel_h, kernel_w, in_channels] bf16 made by
 * mcgmil_pack_conv_weights from the torch layout [out, in, kh, kw] (fp32 or bf16). Zero padding.
 * in/out channels multiples of 64; kernel 1..7; x < 2 GiB; pointers 16-byte aligned. */
typedef struct mcgmil_conv_args {
    int32_t batch, height, width, in_channels;
    int32_t out_channels, kernel_h, kernel_w, stride, pad;
    int32_t in_relu;            /* with in_ab: 1 = ReLU after the input BatchNorm, 0 = none */
    const void* x;              /* bf16 [batch, height, width, in_channels] */
    const void* w;              /* packed bf16 [out_channels, kernel_h, kernel_w, in_channels] */
    void* y;                    /* bf16 [batch, OH, OW, out_channels] */
    float* stats;               /* optional out: BatchNorm statistics of y, [parts][3][out_channels]
                                   = (count, mean, M2) of the bf16 outputs per workgroup row
                                   (per pixel stream for the 1x1 streaming kernel),
                                   parts = mcgmil_conv_stats_parts() (0 when the layer's
                                   kernel emits none: then stats is ignored and the BN computes
                                   its statistics from y); hand them to mcgmil_batchnorm_act as
                                   partials. NULL: not computed */
    const float* in_ab;         /* optional [2][in_channels] fp32 input BatchNorm (a_c, then b_c,
                                   as mcgmil_batchnorm_coefficients writes them): the convolution
                                   reads bf16(max(fmaf(x, a_c, b_c), 0)) (in_relu; without it
                                   bf16(fmaf(x, a_c, b_c))) in place of every in-image x, padding
                                   staying zero -- conv(relu(bn(x))) bit-identical to
                                   mcgmil_batchnorm_act followed by mcgmil_conv2d, without
                                   writing and re-reading bn(x). Only where
                                   mcgmil_conv_input_bn() reports support (the 3x3 / stride 1 halo
                                   kernels), else MCGMIL_E_UNSUPPORTED. NULL: x as is */
    void* workspace;            /* optional device scratch, 256-byte aligned, of
                                   mcgmil_conv_workspace_size() bytes (0 for most layers). With it
                                   a layer whose last round of 256 x 256 pixel tiles would leave
                                   most CUs idle cuts those tiles' K loop into 2-4 ranges (fp32
                                   sums added in range order, then one rounding to bf16 -- within
                                   the fp32 accumulation bound of the whole-tile sums, not bitwise
                                   them). NULL or smaller: whole tiles. mcgmil_conv2d_f32 ignores it */
    size_t workspace_bytes;
    int32_t flags;              /* mcgmil_conv_flags: the kernel shape (0 = auto; performance only;
                                   every shape sums each output's K terms in the same order, so
                                   they agree bitwise where no K split applies; MCGMIL_CONV_TILE in
                                   the environment -- nohalo | small | big512 -- overrides) */
    int32_t reserved;           /* must be 0 */
} mcgmil_conv_args;

/* mcgmil_conv_args.flags */
enum mcgmil_conv_flags {
    MCGMIL_CONV_TILE_AUTO = 0,     /* the measured-fastest kernel per layer shape (1x1 / stride 2
                                      from 64 channels: a streaming kernel) */
    MCGMIL_CONV_TILE_NOHALO = 1,   /* no halo-patch or streaming kernels (generic LDS-DMA kernel
                                      everywhere) */
    MCGMIL_CONV_TILE_SMALL = 2,    /* 256 x 128 tiles where auto would take 256 x 256 */
    MCGMIL_CONV_TILE_BIG512 = 3    /* 512 x 128 tiles on 128-channel layers */
};

size_t mcgmil_conv_args_size(void);
int mcgmil_pack_conv_weights(const mcgmil_conv_args* a, const void* weight, int32_t weight_dtype,
                             void* packed, void* stream);

/* The ResNet stem pool(relu(bn1(conv1(x)))) in one call -- replaces torchvision ResNet.forward's
 * first four layers (conv1 7x7/2 pad 3, bn1, relu, maxpool 3x3/2 pad 1; model.py:166-177 builds
 * the backbone, infer.py:191 runs it on every instance of a bag) under torch.autocast bf16.
 * x is the instance batch straight from mcgmil_image_to_bag: NCHW bf16 [batch, in_channels,
 * height, width]; y is channels-last bf16 [batch, PH, PW, 64] (NHWC), PH/PW the pooled sizes
 * (or OH/OW without pooling). The convolution is an implicit GEMM on the matrix cores (fp32
 * accumulation, one rounding to bf16, as autocast's convolution); with batch statistics its
 * epilogue also accumulates the per-channel sums that BatchNorm needs (around a per-channel
 * shift taken from the convolution at one pixel), so the 64-channel activation is read once,
 * by the pooling pass. BatchNorm / ReLU / pooling semantics are those of mcgmil_batchnorm_act.
 * Supported: in_channels 1..4, out_channels 64, square kernel <= 8 (kernel + (pad & 1) <= 8),
 * stride 2, width even, OW <= 125; otherwise MCGMIL_E_UNSUPPORTED (the caller keeps torch's
 * layers). w is packed by mcgmil_pack_stem_weights from the torch layout [64, in, k, k]. */
typedef struct mcgmil_stem_args {
    int32_t batch, in_channels, height, width;
    int32_t out_channels, kernel, stride, pad;
    int32_t pool_kernel, pool_stride, pool_pad;   /* 0: no pooling */
    int32_t relu;
    double eps;
    const void* x;              /* bf16 NCHW [batch, in_channels, height, width] */
    const void* w;              /* packed bf16 weights (mcgmil_stem_packed_size bytes) */
    const float* gamma;         /* [64] or NULL (1) */
    const float* beta;          /* [64] or NULL (0) */
    const float* running_mean;  /* [64]: running-statistics mode when both are given */
    const float* running_var;
    void* y;                    /* bf16 NHWC [batch, PH, PW, 64] */
    float* batch_mean;          /* optional out [64] */
    float* batch_invstd;        /* optional out [64] */
    void* workspace;            /* >= mcgmil_stem_workspace_size() bytes, 256-byte aligned */
    size_t workspace_bytes;
    int32_t flags;              /* mcgmil_stem_flags (0 = auto; performance only, same results;
                                   MCGMIL_STEM_HPOOL=0 in the environment overrides) */
    int32_t reserved;           /* must be 0 */
} mcgmil_stem_args;

/* mcgmil_stem_args.flags */
enum mcgmil_stem_flags {
    MCGMIL_STEM_AUTO = 0,            /* the 3x3/2 max-pool split: horizontal half in the convolution
                                        epilogue, vertical half in the BatchNorm pass */
    MCGMIL_STEM_POOL_UNSPLIT = 1     /* the convolution writes the whole activation; one pooling pass */
};

size_t mcgmil_stem_args_size(void);
int mcgmil_stem_packed_size(const mcgmil_stem_args* a, size_t* bytes);
int mcgmil_pack_stem_weights(const mcgmil_stem_args* a, const void* weight, int32_t weight_dtype,
                             void* packed, void* stream);
int mcgmil_stem_workspace_size(const mcgmil_stem_args* a, size_t* bytes);
int mcgmil_stem_forward(const mcgmil_stem_args* a, void* stream);
int mcgmil_conv_stats_parts(const mcgmil_conv_args* a, int32_t* parts);
/* Bytes of mcgmil_conv_args.workspace this layer's plan can use (0: none). Replaces nothing in the
 * reference (torch.nn.Conv2d allocates its own scratch through the caching allocator). */
int mcgmil_conv_workspace_size(const mcgmil_conv_args* a, size_t* bytes);
/* *supported = 1 when mcgmil_conv2d accepts in_ab for this geometry (in_ab itself not read) */
int mcgmil_conv_input_bn(const mcgmil_conv_args* a, int32_t* supported);
int mcgmil_conv2d(const mcgmil_conv_args* a, void* stream);
/* The same convolution in fp32 (the reference precision: fp32 operands, fp32 accumulation on
 * v_mfma_f32_16x16x4_f32): x [batch, height, width, in_channels] fp32 NHWC, y fp32 NHWC, w the
 * packed fp32 weight made by mcgmil_pack_conv_weights_f32 from the torch layout [out, in, kh, kw]
 * fp32 (mcgmil_conv_packed_size_f32 floats). out_channels a multiple of 64, kernel 1..7, and
 * in_channels a multiple of 16 or kernel_h * kernel_w * in_channels <= 1024 (the 3-channel stem,
 * one 4-byte gather per element). 16-byte aligned pointers.
 *   stats: as mcgmil_conv2d's, one (count, mean, M2) block per output-pixel tile of the fp32
 *     outputs, parts = mcgmil_conv_stats_parts_f32().
 *   in_ab / in_relu: as mcgmil_conv2d's, in fp32 (max(fmaf(x, a_c, b_c), 0) or fmaf(x, a_c, b_c),
 *     bit-identical to mcgmil_batchnorm_act then mcgmil_conv2d_f32); in_channels a multiple of 16
 *     and <= 2048 (not the gather mode), else MCGMIL_E_UNSUPPORTED. */
int mcgmil_conv_packed_size_f32(const mcgmil_conv_args* a, size_t* floats);
int mcgmil_conv_stats_parts_f32(const mcgmil_conv_args* a, int32_t* parts);
int mcgmil_pack_conv_weights_f32(const mcgmil_conv_args* a, const void* weight, void* packed, void* stream);
int mcgmil_conv2d_f32(const mcgmil_conv_args* a, void* stream);
int mcgmil_bn_workspace_size(const mcgmil_bn_args* a, size_t* bytes);
int mcgmil_batchnorm_act(const mcgmil_bn_args* a, void* stream);
/* The per-channel coefficients mcgmil_batchnorm_act would apply, without the apply pass:
 * ab[c] = a_c = gamma_c / sqrt(var_c + eps), ab[C + c] = b_c = beta_c - mean_c * a_c (fp32,
 * [2][C], 4-byte aligned). Statistics as mcgmil_batchnorm_act: from partials, from the running
 * statistics, or from a pass over x (then, and with more than 1024 partials, workspace as
 * mcgmil_bn_workspace_size). y, residual and
 * the pooling fields are ignored; batch_mean / batch_invstd are written when given. For a consumer
 * that applies the BatchNorm itself (mcgmil_conv_args.in_ab). */
int mcgmil_batchnorm_coefficients(const mcgmil_bn_args* a, float* ab, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MCGMIL_FEATURES_H_ */
