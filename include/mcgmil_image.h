/* mcgmil_image.h -- C ABI of the image side around the MCDO kernel:
 * the tile grid, non-empty tile selection and bag gather that feed the feature extractor, and
 * the attention-map reconstruction (with infer.py's mean/std over passes) that consumes the
 * kernel's A. libmcgmil.so exports these next to include/mcgmil.h.
 *
 * Reference interface replaced (ImagePatcher, image_patcher.py):
 *   mcgmil_tile_grid           get_tiles / _start_points                image_patcher.py:16-41
 *   mcgmil_image_to_bag        convert_img_to_bag + _select_bag         image_patcher.py:43-59,115-131
 *   mcgmil_attention_maps      reconstruct_attention_map                image_patcher.py:83-110
 *                              + mean/std over passes                   infer.py:212-219
 *   mcgmil_reconstruct_image   reconstruct_image_from_patches           image_patcher.py:62-80
 *
 * Geometry. The tiles are the reference's grid: start points 0, s, 2s, ... with
 * s = (int)(ps * (1 - overlap)) evaluated in double, the last one moved to size - ps; tile k =
 * (row i, column j) with k = i * n_cols + j. All tile boundaries together cut the image into
 * disjoint "cells"; every cell lies either inside or outside each tile, which is what lets the
 * device code count and reconstruct per cell instead of per pixel.
 *
 * Semantics kept from the reference:
 *   - px[k] = 100 * (non-zero pixels of channel 0 in tile k) / ps^2, bit-exact fp32
 *     ((float)count / (float)(ps*ps) * 100.0f == torch's mean()*100).
 *   - a tile is kept iff px > (float)(empty_thresh * 100) (torch compares in fp32); the bag is
 *     the kept tiles ordered by px descending, capped at bag_size when bag_size > 0.
 *   - ties: the reference orders equal px with numpy's unstable quicksort and then shuffles
 *     with sklearn (numpy's global RNG). Here equal px are ordered by tile index (stable), and
 *     the shuffle, when requested, is a Philox-keyed permutation of shuffle_seed. The SET of
 *     selected tiles is the reference's; the MIL head is permutation-equivariant.
 *   - attention maps: per (pass, class) sum of the covering instances' attention in instance
 *     order (fp32), divided by the covering count taken modulo 256 (the reference counts in
 *     uint8; 0 -> 1), then divided by the map's maximum. Bit-exact with the reference.
 *   - mean / unbiased std over passes accumulate in fp64 (torch's CPU accumulation type).
 *
 * All entry points are stream-ordered, allocate nothing and never synchronise the host;
 * errors are returned as MCGMIL_E_* codes (include/mcgmil.h) with mcgmil_last_error().
 */
#ifndef MCGMIL_IMAGE_H_
#define MCGMIL_IMAGE_H_

#include <stddef.h>
#include <stdint.h>

#include "mcgmil.h"

#ifdef __cplusplus
extern "C" {
#endif

/* image_dtype values beyond MCGMIL_F32 / MCGMIL_BF16 */
#define MCGMIL_U8 2
#define MCGMIL_U16 3

typedef struct mcgmil_image_args {
    /* ---- ImagePatcher(patch_size, overlap, bag_size, empty_thresh) ---- */
    int32_t height, width;      /* image H, W (pixels) */
    int32_t channels;           /* c */
    int32_t patch_size;         /* ps, 1 <= ps <= min(H, W) */
    double overlap;             /* in [0, 1); stride (int)(ps * (1 - overlap)) must be >= 1 */
    double empty_thresh;        /* fraction; compared as (float)(empty_thresh * 100) */
    int32_t bag_size;           /* -1: every kept tile; > 0: at most bag_size */
    int32_t shuffle;            /* 1: Philox(shuffle_seed) permutation of the bag; 0: rank order */
    uint64_t shuffle_seed;
    /* ---- image (device), [c, H, W] with strides in elements ---- */
    int32_t image_dtype;        /* MCGMIL_F32, MCGMIL_BF16, MCGMIL_U8 or MCGMIL_U16 */
    int32_t out_dtype;          /* instances: MCGMIL_F32 or MCGMIL_BF16 */
    int32_t normalize;          /* 1: instances = (x - norm_mean[ch]) / norm_std[ch] in fp32, the
                                   dataset's T.Normalize (reference utils.py:50-51); c <= 4 */
    float norm_mean[4], norm_std[4];
    const void* image;
    int64_t ld_row;             /* elements between rows (>= W) */
    int64_t ld_channel;         /* elements between channels (>= H * ld_row) */
    /* ---- mcgmil_image_to_bag outputs (device) ---- */
    float* px;                  /* [n_tiles] non-zero percentages, or NULL */
    int32_t* tile_ids;          /* [n_tiles] capacity: the bag's tile indices (instances_idx) */
    int32_t* num_selected;      /* [1] number of instances k */
    void* instances;            /* [instance_capacity, c, ps, ps] (out_dtype) or NULL; only the
                                   first k are written */
    int32_t instance_capacity;  /* >= k; min(n_tiles, bag_size) always suffices */
    /* ---- attention maps: A of one bag (device) ---- */
    int32_t T, C, k;            /* passes, classes, instances */
    const float* attention;     /* [T, C, k] fp32 (the kernel's A for one bag) */
    const int32_t* map_tile_ids;/* [k] tile index of instance n (instances_idx) */
    float* maps;                /* [T, C, H, W] normalised maps, or NULL */
    float* map_mean;            /* [C, H, W] mean over passes, or NULL */
    float* map_std;             /* [C, H, W] unbiased std over passes (NaN at T == 1), or NULL */
    /* ---- image reconstruction ---- */
    const float* patches;       /* [k, c, ps, ps] fp32 */
    float* image_out;           /* [c, H, W] fp32 */
    /* ---- scratch ---- */
    void* workspace;            /* >= mcgmil_image_workspace_size() bytes, 256-byte aligned */
    size_t workspace_bytes;
} mcgmil_image_args;

size_t mcgmil_image_args_size(void);    /* sizeof(mcgmil_image_args), for binding checks */

/* Host-only: the reference tile grid. Writes n_tiles (and n_rows, n_cols when non-NULL); when
 * tiles is non-NULL also fills tiles[n_tiles][6] = (y, x, ps, ps, i, j) as get_tiles does. */
int mcgmil_tile_grid(const mcgmil_image_args* a, int64_t* tiles, int32_t* n_tiles,
                     int32_t* n_rows, int32_t* n_cols);

/* Scratch for any image entry point with these sizes (uses H, W, ps, overlap, T, C). */
int mcgmil_image_workspace_size(const mcgmil_image_args* a, size_t* bytes);

/* px, selection, optional shuffle and the instance gather. */
int mcgmil_image_to_bag(const mcgmil_image_args* a, void* stream);

/* maps and/or map_mean / map_std from (attention, map_tile_ids). */
int mcgmil_attention_maps(const mcgmil_image_args* a, void* stream);

/* image_out from (patches, map_tile_ids): overlap-averaged, uncovered pixels 0. */
int mcgmil_reconstruct_image(const mcgmil_image_args* a, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MCGMIL_IMAGE_H_ */
