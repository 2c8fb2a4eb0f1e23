// Image side of the path (include/mcgmil_image.h): the reference ImagePatcher's tile grid,
// non-empty tile selection and bag gather (image_patcher.py:16-59,115-131), and the attention
// maps with infer.py's mean/std over passes (image_patcher.py:62-110, infer.py:212-219).
//
// Everything is computed per *cell*: the union of all tile boundaries cuts the image into
// disjoint rectangles, each lying wholly inside or outside every tile. One pass over channel 0
// counts non-zero pixels per cell and adds the count to the (few) tiles covering the cell; the
// attention maps are constant on each cell, so a map is T*C*cells values until the final
// (write-bound) expansion to pixels. Byte/integer work, HBM-bound: no MFMA here.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/mcgmil_image.h"
#include "mcgmil_device.h"
#include "mcgmil_error.h"

namespace {

using mcgmil_detail::fail;
using mcgmil_detail::hip_fail;
using mcgmil::f32x4;
using mcgmil::philox4x32_10;
using mcgmil::wave_max;

constexpr int kThreads = 256;
constexpr int kMaxStarts = 4096;     // tile start points per dimension
constexpr int kMaxCover = 4096;      // instances covering one cell (LDS list)
constexpr int kMaxSide = 65535;      // pixels per axis (grid_kernel's LDS byte map)
constexpr uint32_t kShuffleTag = 0x5348464cu;   // "SHFL": Philox counter word of the shuffle

// ---------------------------------------------------------------------------------------
// Geometry, shared verbatim by host and device so both derive the same grid.
// ---------------------------------------------------------------------------------------

// image_patcher.py:16-28. The caller guarantees stride >= 1 and ps <= size.
__host__ __device__ inline int start_points(int size, int ps, int stride, int32_t* out) {
    int n = 0;
    if (out) out[n] = 0;
    ++n;
    for (long long counter = 1;; ++counter) {
        const long long pt = (long long)stride * counter;
        if (pt + ps >= size) {
            if (out) out[n] = size - ps;
            ++n;
            break;
        }
        if (out) out[n] = (int)pt;
        ++n;
    }
    return n;
}

// Sorted union of {s[i]} and {s[i] + ps} (s non-decreasing): the cell boundaries of one axis.
__host__ __device__ inline int merge_bounds(const int32_t* s, int n, int ps, int32_t* out) {
    int i = 0, j = 0, m = 0, last = -1;
    while (i < n || j < n) {
        int v;
        if (j >= n || (i < n && s[i] <= s[j] + ps)) v = s[i++];
        else v = s[j++] + ps;
        if (v != last) {
            if (out) out[m] = v;
            ++m;
            last = v;
        }
    }
    return m;
}

struct Geom {
    int H, W, ps, stride;
    int ny, nx;        // tile start points (rows, columns)
    int nby, nbx;      // cell boundaries per axis (cells = boundaries - 1)
    __host__ __device__ int cy() const { return nby - 1; }
    __host__ __device__ int cx() const { return nbx - 1; }
    __host__ __device__ long long cells() const { return (long long)cy() * cx(); }
    __host__ __device__ long long tiles() const { return (long long)ny * nx; }
};

// Largest number of start points s with s <= p < s + ps over all positions p of one axis.
int max_cover_1d(const std::vector<int32_t>& s, const std::vector<int32_t>& b, int ps) {
    int best = 0;
    for (size_t c = 0; c + 1 < b.size(); ++c) {
        const int p = b[c];
        const int hi = (int)(std::upper_bound(s.begin(), s.end(), p) - s.begin());
        const int lo = (int)(std::upper_bound(s.begin(), s.end(), p - ps) - s.begin());
        best = std::max(best, hi - lo);
    }
    return best;
}

int validate_geometry(const mcgmil_image_args* a, Geom* g, int* max_cover = nullptr) {
    if (!a) return fail(MCGMIL_E_INVALID, "args is NULL");
    if (a->height < 1 || a->width < 1) return fail(MCGMIL_E_INVALID, "image height/width must be >= 1");
    if (a->height > kMaxSide || a->width > kMaxSide)
        return fail(MCGMIL_E_UNSUPPORTED, "image sides above 65535 pixels are not built");
    if (a->patch_size < 1) return fail(MCGMIL_E_INVALID, "patch_size must be >= 1");
    if (a->patch_size > a->height || a->patch_size > a->width)
        return fail(MCGMIL_E_UNSUPPORTED, "patch_size larger than the image");
    if (!(a->overlap >= 0.0 && a->overlap < 1.0)) return fail(MCGMIL_E_INVALID, "overlap must be in [0, 1)");
    const int stride = (int)(a->patch_size * (1.0 - a->overlap));   // int(ps * (1 - overlap))
    if (stride < 1) return fail(MCGMIL_E_INVALID, "stride int(patch_size * (1 - overlap)) is 0");
    g->H = a->height;
    g->W = a->width;
    g->ps = a->patch_size;
    g->stride = stride;
    g->ny = start_points(g->H, g->ps, stride, nullptr);
    g->nx = start_points(g->W, g->ps, stride, nullptr);
    if (g->ny > kMaxStarts || g->nx > kMaxStarts)
        return fail(MCGMIL_E_UNSUPPORTED, "more than 4096 tile start points per axis");
    std::vector<int32_t> ys(g->ny), xs(g->nx);
    start_points(g->H, g->ps, stride, ys.data());
    start_points(g->W, g->ps, stride, xs.data());
    g->nby = merge_bounds(ys.data(), g->ny, g->ps, nullptr);
    g->nbx = merge_bounds(xs.data(), g->nx, g->ps, nullptr);
    if (max_cover) {
        std::vector<int32_t> yb(g->nby), xb(g->nbx);
        merge_bounds(ys.data(), g->ny, g->ps, yb.data());
        merge_bounds(xs.data(), g->nx, g->ps, xb.data());
        *max_cover = max_cover_1d(ys, yb, g->ps) * max_cover_1d(xs, xb, g->ps);
    }
    return MCGMIL_OK;
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct Layout {
    size_t ys, xs, yb, xb, rowcell, colcell, counts, sorted, rank, pos, above, cellval, cellstat, total;
};

Layout layout(const Geom& g, int T, int C) {
    Layout l;
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t at = o; o = align_up(o + bytes, 256); return at; };
    l.ys = take(4 * (size_t)g.ny);
    l.xs = take(4 * (size_t)g.nx);
    l.yb = take(4 * (size_t)g.nby);
    l.xb = take(4 * (size_t)g.nbx);
    l.rowcell = take(4 * (size_t)g.H);
    l.colcell = take(4 * (size_t)g.W);
    l.counts = take(4 * (size_t)g.tiles());
    l.sorted = take(4 * (size_t)g.tiles());
    l.rank = take(4 * (size_t)g.tiles());
    l.pos = take(4 * (size_t)g.tiles());
    l.above = take(4);
    l.cellval = take(4 * (size_t)std::max(T, 0) * std::max(C, 0) * g.cells());
    l.cellstat = take(8 * (size_t)std::max(C, 0) * g.cells());
    l.total = o;
    return l;
}

struct Ws {
    int32_t *ys, *xs, *yb, *xb, *rowcell, *colcell, *counts, *sorted, *rank, *pos, *above;
    float *cellval, *cellstat;
};

Ws carve(void* base, const Layout& l) {
    char* b = (char*)base;
    return Ws{(int32_t*)(b + l.ys), (int32_t*)(b + l.xs), (int32_t*)(b + l.yb), (int32_t*)(b + l.xb),
              (int32_t*)(b + l.rowcell), (int32_t*)(b + l.colcell), (int32_t*)(b + l.counts),
              (int32_t*)(b + l.sorted), (int32_t*)(b + l.rank), (int32_t*)(b + l.pos),
              (int32_t*)(b + l.above), (float*)(b + l.cellval), (float*)(b + l.cellstat)};
}

// ---------------------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------------------

// Grid setup, one 1024-thread block per axis (block 0: rows, block 1: columns). Every start
// s_i and end s_i + ps is flagged in an LDS byte map over positions 0..size; a block-wide
// prefix count over the map then yields the sorted, de-duplicated cell boundaries and the
// cell index of every pixel (last boundary <= p) in one pass. The start points have a closed
// form: s_i = i * stride for i < n - 1 and s_{n-1} = size - ps (image_patcher.py:16-28).
constexpr int kGridThreads = 1024;

__global__ void __launch_bounds__(kGridThreads) grid_kernel(Geom g, Ws w, int zero_counts) {
    __shared__ uint8_t s_flag[kMaxSide + 1];
    __shared__ int s_scan[kGridThreads / 64];
    const bool rows = blockIdx.x == 0;
    const int size = rows ? g.H : g.W;
    const int n = rows ? g.ny : g.nx;
    int32_t* starts = rows ? w.ys : w.xs;
    int32_t* bounds = rows ? w.yb : w.xb;
    int32_t* cell = rows ? w.rowcell : w.colcell;
    const int tid = threadIdx.x;
    for (int q = tid; q <= size; q += kGridThreads) s_flag[q] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += kGridThreads) {
        const int st = i < n - 1 ? i * g.stride : size - g.ps;
        starts[i] = st;
        s_flag[st] = 1;          // racing writes store the same value
        s_flag[st + g.ps] = 1;
    }
    __syncthreads();
    // chunk of positions per thread, its flag count, then a block-wide exclusive scan
    const int chunk = (size + 1 + kGridThreads - 1) / kGridThreads;
    const int q0 = tid * chunk, q1 = min(q0 + chunk, size + 1);
    int cnt = 0;
    for (int q = q0; q < q1; ++q) cnt += s_flag[q];
    const int lane = tid & 63, wv = tid >> 6;
    int incl = cnt;
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) s_scan[wv] = incl;
    __syncthreads();
    int base = 0;
    for (int v = 0; v < wv; ++v) base += s_scan[v];
    int running = base + incl - cnt;           // boundaries before this chunk
    for (int q = q0; q < q1; ++q) {
        if (s_flag[q]) bounds[running++] = q;
        if (q < size) cell[q] = running - 1;
    }
    if (zero_counts) {   // counters of the selection (cell_count, rank and order kernels)
        const long long nt = g.tiles();
        for (long long i = (long long)blockIdx.x * kGridThreads + tid; i < nt; i += 2ll * kGridThreads) {
            w.counts[i] = 0;
            w.rank[i] = 0;
            w.pos[i] = 0;
        }
        if (blockIdx.x == 0 && tid == 0) *w.above = 0;
    }
}

template <typename In> __device__ __forceinline__ float pixel(const In* p);
template <> __device__ __forceinline__ float pixel<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float pixel<__bf16>(const __bf16* p) { return (float)*p; }
template <> __device__ __forceinline__ float pixel<uint8_t>(const uint8_t* p) { return (float)*p; }
template <> __device__ __forceinline__ float pixel<uint16_t>(const uint16_t* p) { return (float)*p; }

// Non-zero pixels of channel 0 per cell (image_patcher.py:53 counts `> 0`), added to every
// tile covering the cell. Integer atomics: the result is order-independent.
template <typename In>
__global__ void __launch_bounds__(kThreads) cell_count_kernel(Geom g, const In* img, long long ld_row,
                                                              Ws w) {
    const int cell = blockIdx.x;
    const int cy = cell / g.cx(), cx = cell % g.cx();
    const int y0 = w.yb[cy], y1 = w.yb[cy + 1], x0 = w.xb[cx], x1 = w.xb[cx + 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int cnt = 0;
    for (int y = y0 + wave; y < y1; y += kThreads / 64) {
        const In* row = img + (long long)y * ld_row;
        for (int x = x0 + lane; x < x1; x += 64) cnt += pixel<In>(row + x) > 0.f;
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    __shared__ int s_cnt[kThreads / 64];
    if (lane == 0) s_cnt[wave] = cnt;
    __syncthreads();
    const int total = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    if (total == 0) return;
    // tile rows covering y0 x tile columns covering x0 (starts are non-decreasing)
    for (int i = threadIdx.x; i < g.ny; i += kThreads) {
        const int ty = w.ys[i];
        if (!(ty <= y0 && y0 < ty + g.ps)) continue;
        for (int j = 0; j < g.nx; ++j) {
            const int tx = w.xs[j];
            if (tx > x0) break;
            if (x0 < tx + g.ps) atomicAdd(w.counts + (long long)i * g.nx + j, total);
        }
    }
}

__device__ __forceinline__ float nonzero_percent(int count, float area) {
    return (float)count / area * 100.0f;   // == torch (mask.float().mean() * 100), fp32
}

// Stable rank of every tile (px descending, tile index ascending), split over a 2-D grid:
// block (bx, by) compares tiles bx*256.. against the j-chunk by*256.. and adds its partial
// counts with integer atomics (order-independent). Blocks of column 0 also count the tiles
// above the threshold, chunk by chunk.
__global__ void __launch_bounds__(kThreads) rank_kernel(Geom g, float thr, Ws w) {
    __shared__ float s_px[kThreads];
    __shared__ int s_above[kThreads / 64];
    const int nt = (int)g.tiles();
    const float area = (float)(g.ps * g.ps);   // numel of a tile
    const int i = blockIdx.x * kThreads + threadIdx.x;
    const int base = blockIdx.y * kThreads;
    const int j = base + threadIdx.x;
    const float pj = j < nt ? nonzero_percent(w.counts[j], area) : -1.f;
    s_px[threadIdx.x] = pj;
    if (blockIdx.x == 0) {
        const unsigned long long m = __ballot(j < nt && pj > thr);
        if ((threadIdx.x & 63) == 0) s_above[threadIdx.x >> 6] = __popcll(m);
    }
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int a = s_above[0] + s_above[1] + s_above[2] + s_above[3];
        if (a) atomicAdd(w.above, a);
    }
    if (i >= nt) return;
    const float pi = nonzero_percent(w.counts[i], area);
    const int m = min(kThreads, nt - base);
    int rank = 0;
    for (int jj = 0; jj < m; ++jj) {
        const float q = s_px[jj];
        rank += (q > pi) || (q == pi && base + jj < i);
    }
    if (rank) atomicAdd(w.rank + i, rank);
}

// px, k = min(#above, cap) and the rank-ordered tile list.
__global__ void __launch_bounds__(kThreads) scatter_kernel(Geom g, int cap, Ws w, float* px_out,
                                                           int32_t* num_selected) {
    const int nt = (int)g.tiles();
    const int i = blockIdx.x * kThreads + threadIdx.x;
    const int k = min(*w.above, cap);
    if (i == 0) *num_selected = k;
    if (i >= nt) return;
    if (px_out) px_out[i] = nonzero_percent(w.counts[i], (float)(g.ps * g.ps));
    const int r = w.rank[i];
    if (r < k) w.sorted[r] = i;
}

// The bag order. shuffle: position of rank r = #{r' < k : key_r' < key_r or (== and r' < r)},
// key_r = Philox4x32-10(counter {r, 0, 0, "SHFL"}, key = seed) word 0 -- a seeded permutation
// standing in for sklearn.utils.shuffle (image_patcher.py:131). A 2-D split like rank_kernel's,
// with kShuffleChunk-key chunks: k is only known on the device (k <= tiles), so most blocks of
// the (tiles/256) x (tiles/kShuffleChunk) grid exit at once and the rest each compare 64 keys
// (integer atomics: order-free).
constexpr int kShuffleChunk = 64;
__global__ void __launch_bounds__(kThreads) shuffle_rank_kernel(uint32_t k0, uint32_t k1,
                                                                const int32_t* num_selected, Ws w) {
    __shared__ uint32_t s_key[kShuffleChunk];
    const int k = *num_selected;
    const int base = blockIdx.y * kShuffleChunk;
    if (base >= k) return;                       // uniform per block
    if (threadIdx.x < kShuffleChunk)
        s_key[threadIdx.x] = philox4x32_10((uint32_t)(base + threadIdx.x), 0u, 0u, kShuffleTag, k0, k1).x;
    __syncthreads();
    const int r = blockIdx.x * kThreads + threadIdx.x;
    if (r >= k) return;
    const uint32_t kr = philox4x32_10((uint32_t)r, 0u, 0u, kShuffleTag, k0, k1).x;
    const int m = min(kShuffleChunk, k - base);
    int pos = 0;
    for (int jj = 0; jj < m; ++jj) {
        const uint32_t q = s_key[jj];
        pos += (q < kr) || (q == kr && base + jj < r);
    }
    if (pos) atomicAdd(w.pos + r, pos);
}

__global__ void __launch_bounds__(kThreads) order_kernel(Ws w, int shuffle, const int32_t* num_selected,
                                                         int32_t* ids) {
    const int k = *num_selected;
    const int r = blockIdx.x * kThreads + threadIdx.x;
    if (r < k) ids[shuffle ? w.pos[r] : r] = w.sorted[r];
}

template <typename Out> __device__ __forceinline__ Out to_out(float v);
template <> __device__ __forceinline__ float to_out<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 to_out<__bf16>(float v) { return (__bf16)v; }

template <typename T, int N> using vec_t = T __attribute__((ext_vector_type(N)));

struct Norm {
    int on;
    float mean[4], std[4];
};

// instances[n, ch, r, :] = image[ch, y + r, x : x + ps] for n < k (image_patcher.py:52, the
// float copy new_img[i] = image[...] then new_img[sorted_idx]), optionally normalised per
// channel as the dataset's T.Normalize does: (x - mean) / std in fp32 (utils.py:50-51).
// 32 threads per tile row, VEC elements each (VEC = 8 when rows and tiles are 8-aligned), 8
// rows per 256-thread block; rows of ps > 32*VEC loop.
template <typename In, typename Out, int VEC>
__global__ void __launch_bounds__(kThreads) gather_kernel(Geom g, int channels, const In* img,
                                                          long long ld_row, long long ld_ch, Ws w,
                                                          const int32_t* ids, const int32_t* num_selected,
                                                          Norm nm, Out* out) {
    const long long row = (long long)blockIdx.x * (kThreads / 32) + (threadIdx.x >> 5);   // (n, ch, r)
    const int ps = g.ps;
    const long long n = row / ((long long)channels * ps);
    if (n >= *num_selected) return;
    const int rem = (int)(row - n * channels * ps);
    const int ch = rem / ps, r = rem % ps;
    const int t = ids[n];
    const int ty = w.ys[t / g.nx], tx = w.xs[t % g.nx];
    const In* src = img + ch * ld_ch + (long long)(ty + r) * ld_row + tx;
    Out* dst = out + row * ps;
    const float m = nm.on ? nm.mean[ch] : 0.f, sd = nm.on ? nm.std[ch] : 1.f;
    for (int x = (threadIdx.x & 31) * VEC; x < ps; x += 32 * VEC) {
        const vec_t<In, VEC> v = *reinterpret_cast<const vec_t<In, VEC>*>(src + x);
        vec_t<Out, VEC> o;
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
            float f = (float)v[e];
            if (nm.on) f = (f - m) / sd;
            o[e] = to_out<Out>(f);
        }
        *reinterpret_cast<vec_t<Out, VEC>*>(dst + x) = o;
    }
}

// The same copy walked in TILE order: block (tile, channel) in ascending tile index, the blocks
// dealt to the 8 XCDs in contiguous chunks (guide T1, bijective form), each block writing its
// tile's rows to the tile's bag position n = pos[rank] (rank when not shuffled). In the bag's own
// (shuffled) order the overlapping tiles that share pixels are far apart, so every instance
// re-read its pixels from HBM (stride ps / 4 at config 5: each pixel sits in up to 16 tiles);
// in tile order neighbours run together on one XCD and share its L2. Same values, same places.
#ifndef MCGMIL_GATHER_TILES
#define MCGMIL_GATHER_TILES 1
#endif
#ifndef MCGMIL_GATHER_NT
#define MCGMIL_GATHER_NT 1
#endif
template <typename In, typename Out, int VEC>
__global__ void __launch_bounds__(kThreads) gather_tiles_kernel(Geom g, int channels, const In* __restrict__ img,
                                                                long long ld_row, long long ld_ch, Ws w,
                                                                int shuffle, long long capacity,
                                                                const int32_t* num_selected, Norm nm,
                                                                Out* __restrict__ out) {
    const unsigned b = blockIdx.x, nb = gridDim.x, x8 = b & 7u, q = nb >> 3, r8 = nb & 7u;
    const long long L = (long long)(x8 < r8 ? x8 * (q + 1) : r8 * (q + 1) + (x8 - r8) * q) + (b >> 3);
    const long long i = L / channels;
    const int ch = (int)(L - i * channels);
    const int rk = w.rank[i];
    if (rk >= *num_selected) return;
    const long long n = shuffle ? w.pos[rk] : rk;
    if (n >= capacity) return;
    const int ps = g.ps;
    const int ty = w.ys[i / g.nx], tx = w.xs[i % g.nx];
    const In* src = img + ch * ld_ch + (long long)ty * ld_row + tx;
    Out* dst = out + (n * channels + ch) * ps * ps;
    const float m = nm.on ? nm.mean[ch] : 0.f, sd = nm.on ? nm.std[ch] : 1.f;
    const int x0 = (threadIdx.x & 31) * VEC;
#pragma unroll 4
    for (int r = threadIdx.x >> 5; r < ps; r += kThreads / 32) {
        for (int x = x0; x < ps; x += 32 * VEC) {
            const vec_t<In, VEC> v = *reinterpret_cast<const vec_t<In, VEC>*>(src + (long long)r * ld_row + x);
            vec_t<Out, VEC> o;
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                float f = (float)v[e];
                if (nm.on) f = (f - m) / sd;
                o[e] = to_out<Out>(f);
            }
#if MCGMIL_GATHER_NT
            if constexpr (sizeof(vec_t<Out, VEC>) == 16)
                __builtin_nontemporal_store(__builtin_bit_cast(vec_t<uint32_t, 4>, o),
                                            reinterpret_cast<vec_t<uint32_t, 4>*>(dst + (long long)r * ps + x));
            else
#endif
                *reinterpret_cast<vec_t<Out, VEC>*>(dst + (long long)r * ps + x) = o;
        }
    }
}

// Ordered list (instance order) of the instances whose tile covers the cell with top-left
// (y0, x0), built in LDS chunk by chunk with ballot compaction. Returns the count.
__device__ int collect_cover(const Geom& g, const Ws& w, const int32_t* ids, int k, int y0, int x0,
                             int32_t* list, int* s_wave) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long nt = g.tiles();
    int count = 0;
    for (int base = 0; base < k; base += kThreads) {
        const int item = base + threadIdx.x;
        bool cov = false;
        if (item < k) {
            const int t = ids[item];
            if (t >= 0 && t < nt) {
                const int ty = w.ys[t / g.nx], tx = w.xs[t % g.nx];
                cov = ty <= y0 && y0 < ty + g.ps && tx <= x0 && x0 < tx + g.ps;
            }
        }
        const unsigned long long mask = __ballot(cov);
        const int before = __popcll(mask & ((1ull << lane) - 1ull));
        __syncthreads();                      // previous chunk's s_wave reads are done
        if (lane == 0) s_wave[wave] = __popcll(mask);
        __syncthreads();
        int off = count;
        for (int v = 0; v < wave; ++v) off += s_wave[v];
        if (cov && off + before < kMaxCover) list[off + before] = item;
        for (int v = 0; v < kThreads / 64; ++v) count += s_wave[v];
    }
    __syncthreads();
    return count;
}

// Per (pass, class, cell): the covering instances' attention summed in instance order in fp32,
// divided by the uint8 covering count (0 -> 1), as image_patcher.py:92-106 does per pixel.
__global__ void __launch_bounds__(kThreads) cell_attention_kernel(Geom g, int TC, int k, const float* A,
                                                                  const int32_t* ids, Ws w) {
    __shared__ int32_t s_list[kMaxCover];
    __shared__ int s_wave[kThreads / 64];
    const long long cells = g.cells();
    const int cell = blockIdx.x;
    const int cy = cell / g.cx(), cx = cell % g.cx();
    const int n = collect_cover(g, w, ids, k, w.yb[cy], w.xb[cx], s_list, s_wave);
    const int c8 = n & 255;
    const float div = (float)(c8 ? c8 : 1);
    const int nl = min(n, kMaxCover);
    for (int p = threadIdx.x; p < TC; p += kThreads) {
        const float* a = A + (long long)p * k;
        float acc = 0.f;
        for (int q = 0; q < nl; ++q) acc += a[s_list[q]];
        w.cellval[p * cells + cell] = acc / div;
    }
}

// Per (pass, class): divide by the map's maximum (image_patcher.py:107-108). Every cell holds
// at least one pixel, so the max over cells is the max over pixels.
__global__ void __launch_bounds__(kThreads) normalize_kernel(Geom g, Ws w) {
    __shared__ float s_max[kThreads / 64];
    const long long cells = g.cells();
    float* v = w.cellval + blockIdx.x * cells;
    float m = -INFINITY;
    for (long long i = threadIdx.x; i < cells; i += kThreads) m = fmaxf(m, v[i]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(s_max[0], s_max[1]), fmaxf(s_max[2], s_max[3]));
    for (long long i = threadIdx.x; i < cells; i += kThreads) v[i] = v[i] / m;
}

// Mean and unbiased std over the T passes per (class, cell), accumulated in fp64
// (infer.py:216-219). A block takes 64 (class, cell) items; its 4 waves split the passes and
// combine their sums of v and v^2 in LDS (values lie in [0, 1]: no cancellation issue in fp64).
__global__ void __launch_bounds__(kThreads) cell_stats_kernel(Geom g, int T, int C, Ws w) {
    __shared__ double s_sum[kThreads / 64][64], s_sq[kThreads / 64][64];
    const long long cells = g.cells();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long i = (long long)blockIdx.x * 64 + lane;    // over (c, cell)
    double s = 0.0, q = 0.0;
    if (i < C * cells) {
        const int c = (int)(i / cells);
        const long long cell = i % cells;
        for (int t = wv; t < T; t += kThreads / 64) {
            const double v = (double)w.cellval[((long long)t * C + c) * cells + cell];
            s += v;
            q += v * v;
        }
    }
    s_sum[wv][lane] = s;
    s_sq[wv][lane] = q;
    __syncthreads();
    if (wv != 0 || i >= C * cells) return;
    for (int k = 1; k < kThreads / 64; ++k) {
        s += s_sum[k][lane];
        q += s_sq[k][lane];
    }
    const double mean = s / T;
    w.cellstat[i] = (float)mean;
    w.cellstat[C * cells + i] = T > 1 ? (float)sqrt(fmax(q - s * mean, 0.0) / (T - 1)) : NAN;
}

// Expand per-cell planes to pixels: planes [0, P0) come from src0 into out0, planes [P0, P)
// from src1 into out1 (each plane H x W). Nontemporal 16-byte stores when W % 4 == 0.
__global__ void __launch_bounds__(kThreads) expand_kernel(Geom g, Ws w, int P0, const float* src0, float* out0,
                                                          const float* src1, float* out1) {
    const int y = blockIdx.x;
    const int plane = blockIdx.y;
    const long long cells = g.cells();
    const bool first = plane < P0;
    const float* src = first ? src0 + (long long)plane * cells : src1 + (long long)(plane - P0) * cells;
    float* out = (first ? out0 + (long long)plane * g.H * g.W : out1 + (long long)(plane - P0) * g.H * g.W) +
                 (long long)y * g.W;
    const float* srow = src + (long long)w.rowcell[y] * g.cx();
    if ((g.W & 3) == 0) {
        const int4* cc = reinterpret_cast<const int4*>(w.colcell);
        f32x4* o4 = reinterpret_cast<f32x4*>(out);
        for (int x = threadIdx.x; x < g.W / 4; x += kThreads) {
            const int4 c = cc[x];
            f32x4 v = {srow[c.x], srow[c.y], srow[c.z], srow[c.w]};
            __builtin_nontemporal_store(v, o4 + x);
        }
    } else {
        for (int x = threadIdx.x; x < g.W; x += kThreads) __builtin_nontemporal_store(srow[w.colcell[x]], out + x);
    }
}

// image_out[ch] = overlap average of the patches (image_patcher.py:62-80): per pixel the
// covering patches summed in instance order in fp32, divided by the float count (0 -> 1).
__global__ void __launch_bounds__(kThreads) reconstruct_kernel(Geom g, int channels, int k, const float* patches,
                                                               const int32_t* ids, Ws w, float* out) {
    __shared__ int32_t s_list[kMaxCover];
    __shared__ int s_wave[kThreads / 64];
    const int cell = blockIdx.x;
    const int ch = blockIdx.y;
    const int cy = cell / g.cx(), cx = cell % g.cx();
    const int y0 = w.yb[cy], y1 = w.yb[cy + 1], x0 = w.xb[cx], x1 = w.xb[cx + 1];
    const int n = collect_cover(g, w, ids, k, y0, x0, s_list, s_wave);
    const float div = (float)(n ? n : 1);
    const int nl = min(n, kMaxCover);
    const int ps = g.ps;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int y = y0 + wave; y < y1; y += kThreads / 64) {
        for (int x = x0 + lane; x < x1; x += 64) {
            float acc = 0.f;
            for (int q = 0; q < nl; ++q) {
                const int item = s_list[q];
                const int t = ids[item];
                const int ty = w.ys[t / g.nx], tx = w.xs[t % g.nx];
                acc += patches[(((long long)item * channels + ch) * ps + (y - ty)) * ps + (x - tx)];
            }
            out[((long long)ch * g.H + y) * g.W + x] = acc / div;
        }
    }
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, what);
}

int launch_grid(const Geom& g, const Ws& w, bool zero_counts, hipStream_t s) {
    hipLaunchKernelGGL(grid_kernel, dim3(2), dim3(kGridThreads), 0, s, g, w, zero_counts ? 1 : 0);
    return check_launch("grid_kernel");
}

int check_workspace(const mcgmil_image_args* a, const Layout& l) {
    if (!a->workspace) return fail(MCGMIL_E_WORKSPACE, "workspace is NULL");
    if (((uintptr_t)a->workspace & 255u) != 0) return fail(MCGMIL_E_ALIGN, "workspace must be 256-byte aligned");
    if (a->workspace_bytes < l.total)
        return fail(MCGMIL_E_WORKSPACE, "workspace too small: need " + std::to_string(l.total) + " bytes");
    return MCGMIL_OK;
}

template <typename In>
int launch_count(const Geom& g, const mcgmil_image_args* a, const Ws& w, hipStream_t s) {
    hipLaunchKernelGGL(cell_count_kernel<In>, dim3((unsigned)g.cells()), dim3(kThreads), 0, s, g,
                       (const In*)a->image, (long long)a->ld_row, w);
    return check_launch("cell_count_kernel");
}

template <typename In, typename Out>
int launch_gather(const Geom& g, const mcgmil_image_args* a, const Ws& w, hipStream_t s) {
    const long long rows = (long long)a->instance_capacity * a->channels * g.ps;
    const long long blocks = (rows + kThreads / 32 - 1) / (kThreads / 32);
    if (blocks == 0) return MCGMIL_OK;
    Norm nm;
    nm.on = a->normalize ? 1 : 0;
    for (int c = 0; c < 4; ++c) {
        nm.mean[c] = a->norm_mean[c];
        nm.std[c] = a->norm_std[c];
    }
    // 8-wide when every tile row starts 8-aligned: base, strides, tile starts and ps
    const bool vec8 = ((uintptr_t)a->image % (8 * sizeof(In))) == 0 && a->ld_row % 8 == 0 &&
                      (a->channels == 1 || a->ld_channel % 8 == 0) && g.ps % 8 == 0 && g.stride % 8 == 0 &&
                      (g.W - g.ps) % 8 == 0 && ((uintptr_t)a->instances % (8 * sizeof(Out))) == 0;
    const dim3 grid((unsigned)blocks), block(kThreads);
    if (MCGMIL_GATHER_TILES && g.tiles() * a->channels < (1ll << 31)) {
        const dim3 tgrid((unsigned)(g.tiles() * a->channels));
        const int sh = a->shuffle ? 1 : 0;
        if (vec8)
            hipLaunchKernelGGL((gather_tiles_kernel<In, Out, 8>), tgrid, block, 0, s, g, a->channels,
                               (const In*)a->image, (long long)a->ld_row, (long long)a->ld_channel, w, sh,
                               (long long)a->instance_capacity, a->num_selected, nm, (Out*)a->instances);
        else
            hipLaunchKernelGGL((gather_tiles_kernel<In, Out, 1>), tgrid, block, 0, s, g, a->channels,
                               (const In*)a->image, (long long)a->ld_row, (long long)a->ld_channel, w, sh,
                               (long long)a->instance_capacity, a->num_selected, nm, (Out*)a->instances);
        return check_launch("gather_tiles_kernel");
    }
    if (vec8)
        hipLaunchKernelGGL((gather_kernel<In, Out, 8>), grid, block, 0, s, g, a->channels, (const In*)a->image,
                           (long long)a->ld_row, (long long)a->ld_channel, w, a->tile_ids, a->num_selected, nm,
                           (Out*)a->instances);
    else
        hipLaunchKernelGGL((gather_kernel<In, Out, 1>), grid, block, 0, s, g, a->channels, (const In*)a->image,
                           (long long)a->ld_row, (long long)a->ld_channel, w, a->tile_ids, a->num_selected, nm,
                           (Out*)a->instances);
    return check_launch("gather_kernel");
}

template <typename In>
int launch_gather_out(const Geom& g, const mcgmil_image_args* a, const Ws& w, hipStream_t s) {
    return a->out_dtype == MCGMIL_BF16 ? launch_gather<In, __bf16>(g, a, w, s) : launch_gather<In, float>(g, a, w, s);
}

}  // namespace

extern "C" {

size_t mcgmil_image_args_size(void) { return sizeof(mcgmil_image_args); }

int mcgmil_tile_grid(const mcgmil_image_args* a, int64_t* tiles, int32_t* n_tiles, int32_t* n_rows,
                     int32_t* n_cols) {
    Geom g;
    int rc = validate_geometry(a, &g);
    if (rc) return rc;
    if (!n_tiles) return fail(MCGMIL_E_INVALID, "n_tiles is NULL");
    *n_tiles = (int32_t)g.tiles();
    if (n_rows) *n_rows = g.ny;
    if (n_cols) *n_cols = g.nx;
    if (tiles) {
        std::vector<int32_t> ys(g.ny), xs(g.nx);
        start_points(g.H, g.ps, g.stride, ys.data());
        start_points(g.W, g.ps, g.stride, xs.data());
        int64_t* t = tiles;
        for (int i = 0; i < g.ny; ++i)
            for (int j = 0; j < g.nx; ++j) {   // image_patcher.py:38 (y, x, ps, ps, i, j)
                t[0] = ys[i]; t[1] = xs[j]; t[2] = g.ps; t[3] = g.ps; t[4] = i; t[5] = j;
                t += 6;
            }
    }
    return MCGMIL_OK;
}

int mcgmil_image_workspace_size(const mcgmil_image_args* a, size_t* bytes) {
    Geom g;
    int rc = validate_geometry(a, &g);
    if (rc) return rc;
    if (!bytes) return fail(MCGMIL_E_INVALID, "bytes is NULL");
    *bytes = layout(g, a->T, a->C).total;
    return MCGMIL_OK;
}

int mcgmil_image_to_bag(const mcgmil_image_args* a, void* stream) {
    Geom g;
    int rc = validate_geometry(a, &g);
    if (rc) return rc;
    if (a->bag_size != -1 && a->bag_size <= 0) return fail(MCGMIL_E_INVALID, "Invalid bag size");
    if (a->channels < 1) return fail(MCGMIL_E_INVALID, "channels must be >= 1");
    if (!a->image || !a->tile_ids || !a->num_selected)
        return fail(MCGMIL_E_INVALID, "image, tile_ids and num_selected are required");
    const int it = a->image_dtype;
    if (it != MCGMIL_F32 && it != MCGMIL_BF16 && it != MCGMIL_U8 && it != MCGMIL_U16)
        return fail(MCGMIL_E_INVALID, "image_dtype must be F32, BF16, U8 or U16");
    if (a->ld_row < a->width || (a->channels > 1 && a->ld_channel < (int64_t)a->height * a->ld_row))
        return fail(MCGMIL_E_INVALID, "image strides too small");
    const long long nt = g.tiles();
    // the O(n^2) ranking runs as a (n/256)^2 grid: cap n at 2^20 tiles (a 16k x 16k image at ps 16)
    if (nt > (1ll << 20)) return fail(MCGMIL_E_UNSUPPORTED, "more than 2^20 tiles");
    const int cap = a->bag_size > 0 ? a->bag_size : 0x7fffffff;
    if (a->instances) {
        if (a->normalize && a->channels > 4) return fail(MCGMIL_E_UNSUPPORTED, "normalize supports c <= 4");
        if (a->out_dtype != MCGMIL_F32 && a->out_dtype != MCGMIL_BF16)
            return fail(MCGMIL_E_INVALID, "out_dtype must be F32 or BF16");
        if ((long long)a->instance_capacity < std::min<long long>(nt, cap))
            return fail(MCGMIL_E_INVALID, "instance_capacity < min(n_tiles, bag_size)");
    }
    const Layout l = layout(g, 0, 0);
    if ((rc = check_workspace(a, l))) return rc;
    const Ws w = carve(a->workspace, l);
    hipStream_t s = (hipStream_t)stream;
    if ((rc = launch_grid(g, w, true, s))) return rc;
    switch (it) {
        case MCGMIL_F32: rc = launch_count<float>(g, a, w, s); break;
        case MCGMIL_BF16: rc = launch_count<__bf16>(g, a, w, s); break;
        case MCGMIL_U8: rc = launch_count<uint8_t>(g, a, w, s); break;
        default: rc = launch_count<uint16_t>(g, a, w, s); break;
    }
    if (rc) return rc;
    const float thr = (float)(a->empty_thresh * 100.0);   // torch: fp32 tensor > python float
    const unsigned tb = (unsigned)((nt + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(rank_kernel, dim3(tb, tb), dim3(kThreads), 0, s, g, thr, w);
    if ((rc = check_launch("rank_kernel"))) return rc;
    hipLaunchKernelGGL(scatter_kernel, dim3(tb), dim3(kThreads), 0, s, g, cap, w, a->px, a->num_selected);
    if ((rc = check_launch("scatter_kernel"))) return rc;
    if (a->shuffle) {
        const unsigned tc = (unsigned)((nt + kShuffleChunk - 1) / kShuffleChunk);
        hipLaunchKernelGGL(shuffle_rank_kernel, dim3(tb, tc), dim3(kThreads), 0, s, (uint32_t)a->shuffle_seed,
                           (uint32_t)(a->shuffle_seed >> 32), a->num_selected, w);
        if ((rc = check_launch("shuffle_rank_kernel"))) return rc;
    }
    hipLaunchKernelGGL(order_kernel, dim3(tb), dim3(kThreads), 0, s, w, a->shuffle ? 1 : 0, a->num_selected,
                       a->tile_ids);
    if ((rc = check_launch("order_kernel"))) return rc;
    if (!a->instances) return MCGMIL_OK;
    switch (it) {
        case MCGMIL_F32: return launch_gather_out<float>(g, a, w, s);
        case MCGMIL_BF16: return launch_gather_out<__bf16>(g, a, w, s);
        case MCGMIL_U8: return launch_gather_out<uint8_t>(g, a, w, s);
        default: return launch_gather_out<uint16_t>(g, a, w, s);
    }
}

int mcgmil_attention_maps(const mcgmil_image_args* a, void* stream) {
    Geom g;
    int max_cover = 0;
    int rc = validate_geometry(a, &g, &max_cover);
    if (rc) return rc;
    if (a->T < 1 || a->C < 1 || a->k < 0) return fail(MCGMIL_E_INVALID, "need T >= 1, C >= 1, k >= 0");
    if (a->k > 0 && (!a->attention || !a->map_tile_ids))
        return fail(MCGMIL_E_INVALID, "attention and map_tile_ids are required");
    if (!a->maps && !a->map_mean && !a->map_std) return fail(MCGMIL_E_INVALID, "no output requested");
    if (max_cover > kMaxCover) return fail(MCGMIL_E_UNSUPPORTED, "more than 4096 tiles overlap one pixel");
    if ((long long)a->T * a->C > 65535) return fail(MCGMIL_E_UNSUPPORTED, "T * C > 65535");
    if (g.cells() > 0x7fffffffll) return fail(MCGMIL_E_UNSUPPORTED, "too many cells");
    const Layout l = layout(g, a->T, a->C);
    if ((rc = check_workspace(a, l))) return rc;
    const Ws w = carve(a->workspace, l);
    hipStream_t s = (hipStream_t)stream;
    if ((rc = launch_grid(g, w, false, s))) return rc;
    const int TC = a->T * a->C;
    hipLaunchKernelGGL(cell_attention_kernel, dim3((unsigned)g.cells()), dim3(kThreads), 0, s, g, TC, a->k,
                       a->attention, a->map_tile_ids, w);
    if ((rc = check_launch("cell_attention_kernel"))) return rc;
    hipLaunchKernelGGL(normalize_kernel, dim3(TC), dim3(kThreads), 0, s, g, w);
    if ((rc = check_launch("normalize_kernel"))) return rc;
    const bool stats = a->map_mean || a->map_std;
    if (stats) {
        const unsigned sb = (unsigned)((a->C * g.cells() + 63) / 64);
        hipLaunchKernelGGL(cell_stats_kernel, dim3(sb), dim3(kThreads), 0, s, g, a->T, a->C, w);
        if ((rc = check_launch("cell_stats_kernel"))) return rc;
    }
    const long long plane = (long long)g.H * g.W;
    // maps: T*C planes from cellval; statistics: C planes each, written where requested
    if (a->maps) {
        hipLaunchKernelGGL(expand_kernel, dim3(g.H, TC), dim3(kThreads), 0, s, g, w, TC, w.cellval, a->maps,
                           w.cellval, a->maps);
        if ((rc = check_launch("expand_kernel"))) return rc;
    }
    if (a->map_mean && a->map_std && a->map_std == a->map_mean + a->C * plane) {
        hipLaunchKernelGGL(expand_kernel, dim3(g.H, 2 * a->C), dim3(kThreads), 0, s, g, w, 2 * a->C, w.cellstat,
                           a->map_mean, w.cellstat, a->map_mean);
        return check_launch("expand_kernel");
    }
    if (a->map_mean) {
        hipLaunchKernelGGL(expand_kernel, dim3(g.H, a->C), dim3(kThreads), 0, s, g, w, a->C, w.cellstat,
                           a->map_mean, w.cellstat, a->map_mean);
        if ((rc = check_launch("expand_kernel"))) return rc;
    }
    if (a->map_std) {
        const float* sd = w.cellstat + a->C * g.cells();
        hipLaunchKernelGGL(expand_kernel, dim3(g.H, a->C), dim3(kThreads), 0, s, g, w, a->C, sd, a->map_std, sd,
                           a->map_std);
        if ((rc = check_launch("expand_kernel"))) return rc;
    }
    return MCGMIL_OK;
}

int mcgmil_reconstruct_image(const mcgmil_image_args* a, void* stream) {
    Geom g;
    int max_cover = 0;
    int rc = validate_geometry(a, &g, &max_cover);
    if (rc) return rc;
    if (a->channels < 1 || a->k < 0) return fail(MCGMIL_E_INVALID, "need channels >= 1, k >= 0");
    if (!a->image_out || (a->k > 0 && (!a->patches || !a->map_tile_ids)))
        return fail(MCGMIL_E_INVALID, "patches, map_tile_ids and image_out are required");
    if (max_cover > kMaxCover) return fail(MCGMIL_E_UNSUPPORTED, "more than 4096 tiles overlap one pixel");
    if (a->channels > 65535) return fail(MCGMIL_E_UNSUPPORTED, "channels > 65535");
    const Layout l = layout(g, 0, 0);
    if ((rc = check_workspace(a, l))) return rc;
    const Ws w = carve(a->workspace, l);
    hipStream_t s = (hipStream_t)stream;
    if ((rc = launch_grid(g, w, false, s))) return rc;
    hipLaunchKernelGGL(reconstruct_kernel, dim3((unsigned)g.cells(), a->channels), dim3(kThreads), 0, s, g,
                       a->channels, a->k, a->patches, a->map_tile_ids, w, a->image_out);
    return check_launch("reconstruct_kernel");
}

}  // extern "C"
