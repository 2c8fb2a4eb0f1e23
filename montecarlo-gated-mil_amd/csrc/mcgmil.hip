// C ABI (include/mcgmil.h) over the gfx950 MCDO kernels: validation, workspace layout,
// kernel selection and stream-ordered launches. No allocation, no host synchronisation.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <set>
#include <string>
#include <utility>

#include "../../include/mcgmil.h"
#include "mcgmil_error.h"
#include "mcgmil_kernels.h"
#include "mcgmil_gate_pp.h"
#include "mcgmil_fused.h"

namespace mcgmil_detail {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(MCGMIL_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

int raise_lds_limit(const void* k, const char* what) {
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, what);
    std::lock_guard<std::mutex> lock(mu);
    if (done.count({k, dev})) return MCGMIL_OK;
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return hip_fail(e, what);
    done.insert({k, dev});
    return MCGMIL_OK;
}

}  // namespace mcgmil_detail

namespace {

using mcgmil_detail::fail;
using mcgmil_detail::hip_fail;

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

uint32_t drop_threshold(float p) {
    // identical to oracle_drop_threshold (oracle/philox_oracle.c), p taken as double
    const double pd = (double)p;
    if (!(pd > 0.0)) return 0u;
    const double x = floor(pd * 65536.0 + 0.5);
    return x >= 65536.0 ? 65536u : (uint32_t)x;
}

float dropout_scale(float p) {
    // torch's nn.Dropout factor: 1.0f / (float)(1 - p) (see oracle/philox_oracle.c)
    const double pd = (double)p;
    return pd >= 1.0 ? 0.0f : 1.0f / (float)(1.0 - pd);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

size_t elem_size(int dtype) { return dtype == MCGMIL_BF16 ? 2 : 4; }

// Largest row tile whose masked feature tile fits the 128 KiB LDS budget.
int pick_bm(int dtype, int L) {
    const size_t es = elem_size(dtype);
    if (dtype == MCGMIL_BF16) return (size_t)128 * L * es <= 131072 ? 128 : 32;
    return (size_t)64 * L * es <= 131072 ? 64 : 16;
}

int validate_sizes(const mcgmil_args* a) {
    if (!a) return fail(MCGMIL_E_INVALID, "args is NULL");
    if (a->L <= 0 || a->L % 32 != 0) return fail(MCGMIL_E_UNSUPPORTED, "L must be a positive multiple of 32");
    if (a->L > 2048) return fail(MCGMIL_E_UNSUPPORTED, "L > 2048 is not built");
    if (a->D <= 0 || a->D % 16 != 0) return fail(MCGMIL_E_UNSUPPORTED, "D must be a positive multiple of 16");
    if (a->C < 1 || a->C > 4) return fail(MCGMIL_E_UNSUPPORTED, "num_classes C must be in 1..4");
    if (!(a->G == 1 || a->G == a->C)) return fail(MCGMIL_E_INVALID, "G must be 1 (shared) or C (separate)");
    if (a->h_dtype != MCGMIL_F32 && a->h_dtype != MCGMIL_BF16) return fail(MCGMIL_E_INVALID, "h_dtype must be MCGMIL_F32 or MCGMIL_BF16");
    return MCGMIL_OK;
}

int validate_batch(const mcgmil_args* a) {
    int rc = validate_sizes(a);
    if (rc) return rc;
    if (a->T < 1) return fail(MCGMIL_E_INVALID, "T (number of MC samples) must be >= 1");
    if (a->num_bags < 1) return fail(MCGMIL_E_INVALID, "num_bags must be >= 1");
    if (a->total_rows < 0) return fail(MCGMIL_E_INVALID, "total_rows must be >= 0");
    if ((long long)a->T * a->total_rows > (1ll << 46)) return fail(MCGMIL_E_UNSUPPORTED, "T * total_rows too large");
    if (a->total_rows > 0x7fffffffll) return fail(MCGMIL_E_UNSUPPORTED, "total_rows must fit int32");
    if (!a->bag_offsets) return fail(MCGMIL_E_INVALID, "bag_offsets is NULL");
    if (a->uniform_bag_rows < 0 ||
        (a->uniform_bag_rows > 0 && (long long)a->uniform_bag_rows * a->num_bags != a->total_rows))
        return fail(MCGMIL_E_INVALID, "uniform_bag_rows must be 0 or total_rows / num_bags");
    if (!(a->p_feat >= 0.f && a->p_feat <= 1.f) || !(a->p_att >= 0.f && a->p_att <= 1.f))
        return fail(MCGMIL_E_INVALID, "dropout probabilities must be in [0, 1]");
    if ((a->flags & ~(MCGMIL_PATH_MASK | MCGMIL_GATE_MASK | MCGMIL_CLOCK_PROBE)) != 0 ||
        (a->flags & MCGMIL_PATH_MASK) == 3 || (a->flags & MCGMIL_GATE_MASK) == (3 << 2) || a->reserved != 0)
        return fail(MCGMIL_E_INVALID, "flags must be MCGMIL_PATH_* | MCGMIL_GATE_* [| MCGMIL_CLOCK_PROBE] and reserved 0");
    if ((a->flags & MCGMIL_CLOCK_PROBE) && !a->debug)
        return fail(MCGMIL_E_INVALID, "MCGMIL_CLOCK_PROBE needs args->debug ([MCGMIL_CLOCK_SLOTS][4] uint64)");
    return MCGMIL_OK;
}

struct Layout {
    size_t packed_bytes;   // 0 when args->packed_w is supplied
    size_t logits_off, zz_off, plan_off, region_off, total;
};

// Smallest row tile any gate kernel uses (sizes the tile plan).
constexpr int kMinBM = 16;

// The 16x16x32 operand tiles of gate_pipe/pp/scores_kernel.
size_t packed_bytes_for(const mcgmil_args* a) {
    const size_t P = (size_t)a->G * (a->D / 16);
    return (2 * P + 1) * (size_t)(a->L / 32) * 512 * elem_size(a->h_dtype);
}

Layout layout_for(const mcgmil_args* a) {
    Layout l;
    l.packed_bytes = a->packed_w ? 0 : align_up(packed_bytes_for(a), 256);
    const size_t scores = align_up((size_t)a->T * a->total_rows * a->C * sizeof(float), 256);
    l.logits_off = l.packed_bytes;
    l.zz_off = l.logits_off + scores;
    l.plan_off = l.zz_off + scores;
    const size_t max_tiles = ((size_t)a->T * a->total_rows + kMinBM - 1) / kMinBM;
    l.region_off = l.plan_off + align_up(max_tiles * sizeof(int32_t), 256);
    l.total = l.region_off + align_up(((size_t)a->num_bags + 1) * sizeof(int32_t), 256);
    return l;
}

int check_workspace(const mcgmil_args* a, const Layout& l) {
    if (l.total > 0 && (!a->workspace || a->workspace_bytes < l.total))
        return fail(MCGMIL_E_WORKSPACE, "workspace missing or smaller than mcgmil_workspace_size()");
    if (((uintptr_t)a->workspace & 255u) != 0) return fail(MCGMIL_E_ALIGN, "workspace must be 256-byte aligned");
    return MCGMIL_OK;
}

const void* packed_ptr(const mcgmil_args* a) {
    return a->packed_w ? a->packed_w : a->workspace;
}

// The tile plan for BM-row tiles (written into the workspace; gp.tile_bag points there).
int launch_plan(const mcgmil::GateParams& gp, int BM, hipStream_t s) {
    const long long tiles = (gp.total_samples + BM - 1) / BM;
    if (tiles == 0) return MCGMIL_OK;
    hipLaunchKernelGGL(mcgmil::plan_tiles_kernel, dim3((unsigned)((tiles + 255) / 256)), dim3(256), 0,
                       s, gp.bag_off, gp.B, gp.T, gp.total_samples, BM, tiles,
                       const_cast<int32_t*>(gp.tile_bag));
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "plan_tiles_kernel launch");
}

template <typename E, int BM, int PPW, int MAXC>
int launch_gate_generic(const mcgmil::GateParams& gp, hipStream_t s) {
    auto* k = &mcgmil::gate_scores_kernel<E, BM, PPW, MAXC>;
    // all scratch is dynamic LDS (> 64 KiB)
    if (int rc = mcgmil_detail::raise_lds_limit(reinterpret_cast<const void*>(k), "gate_scores_kernel LDS limit"))
        return rc;
    const long long tiles = (gp.total_samples + BM - 1) / BM;
    if (tiles == 0) return MCGMIL_OK;
    if (gp.uniform_rows <= 0)
        if (int rc = launch_plan(gp, BM, s)) return rc;
    const size_t lds = mcgmil::gate_lds_bytes<E, BM, MAXC>(gp.L);
    hipLaunchKernelGGL(k, dim3((unsigned)tiles), dim3(mcgmil::kGateThreads), lds, s, gp);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "gate_scores_kernel launch");
}

int device_cus() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
    if (dev < 64) {
        const int c = cache[dev].load(std::memory_order_relaxed);
        if (c > 0) return c;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    if (dev < 64) cache[dev].store(cus, std::memory_order_relaxed);
    return cus;
}

// Short tiles for a sparse last round (bf16, two gate pairs per wave: the reference's separate
// heads). gate_pipe_kernel holds one workgroup per CU, so `tiles` 128-row tiles run in
// ceil(tiles / CUs) rounds; when the last round would fill at most half the CUs (one bag per call:
// N = 2,048, T = 100 is 1,600 tiles = 6.25 rounds; T = 50 3.125) its rows go to a second launch of
// 32- or 64-row tiles (rows' scores bitwise the same), at most one round of them.
// MCGMIL_SHORT_TILES=0 in the environment: whole tiles only (A/B timing; read once per process).
int short_tile_rows(long long tiles) {
    static const bool off = [] {
        const char* e = getenv("MCGMIL_SHORT_TILES");
        return e && strcmp(e, "0") == 0;
    }();
    if (off) return 0;
    const long long cus = device_cus(), full = tiles / cus * cus, rem = tiles - full;
    if (full == 0 || rem == 0) return 0;
    if (4 * rem <= cus) return 32;
    if (2 * rem <= cus) return 64;
    return 0;
}

template <typename E, int PPW, int MAXC, bool REPLAY, bool ONE>
int launch_gate_pipe(const mcgmil::GateParams& gp, hipStream_t s) {
    auto* k = &mcgmil::gate_pipe_kernel<E, PPW, MAXC, REPLAY, ONE>;
    if constexpr (!REPLAY)
        if (gp.clock) k = &mcgmil::gate_pipe_kernel<E, PPW, MAXC, REPLAY, ONE, true>;   // MCGMIL_CLOCK_PROBE
    if (int rc = mcgmil_detail::raise_lds_limit(reinterpret_cast<const void*>(k), "gate_pipe_kernel LDS limit"))
        return rc;
    const long long tiles = (gp.total_samples + mcgmil::kPipeBM - 1) / mcgmil::kPipeBM;
    if (tiles == 0) return MCGMIL_OK;
    if (gp.uniform_rows <= 0)
        if (int rc = launch_plan(gp, mcgmil::kPipeBM, s)) return rc;
    const size_t lds = mcgmil::pipe_lds_bytes<E, MAXC>();
    int srows = 0;
    if constexpr (sizeof(E) == 2 && PPW == 2)
        if (!gp.clock) srows = short_tile_rows(tiles);
    const long long main_tiles = srows ? tiles / device_cus() * device_cus() : tiles;
    hipLaunchKernelGGL(k, dim3((unsigned)main_tiles), dim3(mcgmil::kGateThreads), lds, s, gp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "gate_pipe_kernel launch");
    if constexpr (sizeof(E) == 2 && PPW == 2) {
        if (srows) {
            mcgmil::GateParams gt = gp;
            gt.tile_row0 = main_tiles * mcgmil::kPipeBM;
            const long long n = (gp.total_samples - gt.tile_row0 + srows - 1) / srows;
            auto* ks = srows == 32 ? &mcgmil::gate_pipe_kernel<E, PPW, MAXC, REPLAY, ONE, false, 2>
                                   : &mcgmil::gate_pipe_kernel<E, PPW, MAXC, REPLAY, ONE, false, 4>;
            if (int rc = mcgmil_detail::raise_lds_limit(reinterpret_cast<const void*>(ks), "gate_pipe_kernel LDS limit"))
                return rc;
            hipLaunchKernelGGL(ks, dim3((unsigned)n), dim3(mcgmil::kGateThreads), lds, s, gt);
            e = hipGetLastError();
            if (e != hipSuccess) return hip_fail(e, "gate_pipe_kernel (short tiles) launch");
        }
    }
    return MCGMIL_OK;
}

template <typename E, int RT, int PPW, int MAXC, bool REPLAY, bool ONE>
int launch_gate_pp(const mcgmil::GateParams& gp, hipStream_t s) {
    constexpr int BM = 16 * RT;
    auto* k = &mcgmil::gate_pp_kernel<E, RT, PPW, MAXC, REPLAY, ONE>;
    if constexpr (!REPLAY)
        if (gp.clock) k = &mcgmil::gate_pp_kernel<E, RT, PPW, MAXC, REPLAY, ONE, true>;   // MCGMIL_CLOCK_PROBE
    const long long tiles = (gp.total_samples + BM - 1) / BM;
    if (tiles == 0) return MCGMIL_OK;
    if (gp.uniform_rows <= 0)
        if (int rc = launch_plan(gp, BM, s)) return rc;
    const size_t lds = mcgmil::pp_lds_bytes<E, RT, MAXC>();
    hipLaunchKernelGGL(k, dim3((unsigned)tiles), dim3(mcgmil::kPPThreads), lds, s, gp);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "gate_pp_kernel launch");
}

// Kernel choice for bf16 heads of up to 16 gate tile pairs (measured, config 3, MI355X):
// separate heads (P = 16) run the one-workgroup-per-CU gate_pipe_kernel (914 vs 853 TFLOP/s),
// shared heads (P = 8) the two-workgroups-per-CU gate_pp_kernel (820 vs 781).
// args->flags MCGMIL_GATE_PIPE / _PP force one of them; MCGMIL_GATE=pipe / pp in the environment
// overrides the flags (A/B timing). Variants measured slower and removed are listed with their
// numbers in profiles/r02/gate_ab.log and DESIGN.md §5.
#ifndef MCGMIL_GATE_DEFAULT
#define MCGMIL_GATE_DEFAULT 0       // A/B builds: 1 pipe, 2 pp
#endif
int gate_mode(int flags) {   // 0 auto, 1 pipe, 2 pp
    static const int env = [] {
        const char* e = getenv("MCGMIL_GATE");
        if (e && strcmp(e, "pipe") == 0) return 1;
        if (e && strcmp(e, "pp") == 0) return 2;
        return -1;
    }();
    if (env >= 0) return env;
    const int f = (flags & MCGMIL_GATE_MASK) >> 2;
    return f ? f : MCGMIL_GATE_DEFAULT;
}

template <int RT, int PPW, int MAXC>
int dispatch_gate_pp(const mcgmil::GateParams& gp, hipStream_t s) {
    const bool replay = gp.keep_feat != nullptr;
    const bool one = gp.G > 1 && gp.G == gp.C && (gp.D / 16) % PPW == 0;
    if (replay) return one ? launch_gate_pp<__bf16, RT, PPW, MAXC, true, true>(gp, s)
                           : launch_gate_pp<__bf16, RT, PPW, MAXC, true, false>(gp, s);
    return one ? launch_gate_pp<__bf16, RT, PPW, MAXC, false, true>(gp, s)
               : launch_gate_pp<__bf16, RT, PPW, MAXC, false, false>(gp, s);
}

template <typename E, int PPW, int MAXC>
int dispatch_gate_pipe(const mcgmil::GateParams& gp, hipStream_t s) {
    const bool replay = gp.keep_feat != nullptr;
    // separate heads whose gate tile pairs split evenly over the waves: one class per wave
    const bool one = gp.G > 1 && gp.G == gp.C && (gp.D / 16) % PPW == 0;
    if (replay) return one ? launch_gate_pipe<E, PPW, MAXC, true, true>(gp, s)
                           : launch_gate_pipe<E, PPW, MAXC, true, false>(gp, s);
    return one ? launch_gate_pipe<E, PPW, MAXC, false, true>(gp, s)
               : launch_gate_pipe<E, PPW, MAXC, false, false>(gp, s);
}

template <typename E, int MAXC>
int dispatch_gate_maxc(const mcgmil::GateParams& gp, int L, int dtype, int flags, hipStream_t s) {
    const bool pipe_ok = L % 64 == 0;          // the pipelined K loop is unrolled by two steps
    if constexpr (sizeof(E) == 2) {
        const int mode = gate_mode(flags);
        if (pipe_ok && mode != 1) {
            if (gp.P <= 2 * mcgmil::kPPWaves) return dispatch_gate_pp<8, 2, MAXC>(gp, s);
            if (mode == 2 && gp.P <= 4 * mcgmil::kPPWaves) return dispatch_gate_pp<4, 4, MAXC>(gp, s);
        }
    }
    if (pipe_ok && gp.P <= mcgmil::kGateWaves) return dispatch_gate_pipe<E, 1, MAXC>(gp, s);
    if (pipe_ok && gp.P <= 2 * mcgmil::kGateWaves) return dispatch_gate_pipe<E, 2, MAXC>(gp, s);
    // larger heads: whole masked tile in LDS, several passes of 16 pairs
    return pick_bm(dtype, L) == (dtype == MCGMIL_BF16 ? 128 : 64)
               ? launch_gate_generic<E, (sizeof(E) == 2 ? 128 : 64), 2, MAXC>(gp, s)
               : launch_gate_generic<E, (sizeof(E) == 2 ? 32 : 16), 2, MAXC>(gp, s);
}

template <typename E>
int dispatch_gate(const mcgmil::GateParams& gp, int L, int dtype, int flags, hipStream_t s) {
    return gp.C <= 2 ? dispatch_gate_maxc<E, 2>(gp, L, dtype, flags, s)
                     : dispatch_gate_maxc<E, 4>(gp, L, dtype, flags, s);
}

// Fused single launch (gate_fused_kernel) or the two-kernel path (gate scores into the
// workspace, then softmax_pool_kernel)? The fused kernel runs the pipelined gate kernel's tiles
// (Philox masks, no replay); a workgroup owns a whole region (~32 tiles at config 3), so it
// needs many regions to fill 256 CUs without a tail. By default (MCGMIL_FUSED unset or "auto")
// it takes batches of equal-size bags with >= 16,384 regions (64 per CU): at config 3 it is 0.1-0.8% faster than the
// two-kernel path in the same process (bitwise the same outputs) and moves 40% fewer
// HBM bytes (no logits/z workspace round trip). args->flags MCGMIL_PATH_FUSED takes it whenever it
// applies, MCGMIL_PATH_TWO_KERNEL never; MCGMIL_FUSED=1 / 0 / auto in the environment overrides.
constexpr long long kFusedMinRegions = 16384;

int fused_mode(int flags) {   // -1 auto, 0 off, 1 on
    // MCGMIL_FUSED overrides the flags; read once per process (in-process callers switch paths
    // through args->flags)
    static const int env = [] {
        const char* e = getenv("MCGMIL_FUSED");
        if (e && strcmp(e, "1") == 0) return 1;
        if (e && strcmp(e, "0") == 0) return 0;
        if (e && strcmp(e, "auto") == 0) return -1;
        return -2;
    }();
    if (env != -2) return env;
    const int path = flags & MCGMIL_PATH_MASK;
    return path == MCGMIL_PATH_FUSED ? 1 : path == MCGMIL_PATH_TWO_KERNEL ? 0 : -1;
}

// Returns 1 if the fused kernel was launched (with `regions` set: nothing is launched, *regions
// = its grid), 0 if the caller must run the two-kernel path.
template <typename E, int MAXC>
int try_fused_maxc(const mcgmil::GateParams& gp, long long total_rows, int L, int flags, hipStream_t s,
                   int* rc, long long* regions = nullptr) {
    *rc = MCGMIL_OK;
    // (L >= 128: the fused pipeline peels two K steps at each end of a tile)
    if (gp.keep_feat) return 0;
    // bf16: only heads the two-kernel path runs on gate_pipe_kernel fuse (separate heads of > 8
    // gate tile pairs, or any head under MCGMIL_GATE_PIPE): the fused launch runs that kernel's
    // tile code, so A and Y stay bitwise the two-kernel path's. Heads on gate_pp_kernel (shared
    // heads under auto / MCGMIL_GATE_PP) have no single-launch form and always take two kernels.
    if constexpr (sizeof(E) == 2) {
        const int mode = gate_mode(flags);
        if (!(mode == 1 || (mode == 0 && gp.P > 2 * mcgmil::kPPWaves))) return 0;
    }
    if (L % 64 != 0 || L < 128 || gp.P > 2 * mcgmil::kGateWaves) return 0;
    if (mcgmil::fused_kernel_lds_bytes<E, MAXC>(L) > 160 * 1024) return 0;   // bf16 L > 1024
    const int fm = fused_mode(flags);
    if (fm == 0) return 0;
    constexpr int cap = mcgmil::fused_cap<MAXC>();
    // auto: bf16 uniform batches only -- on ragged ones (config 4) the fused launch measured 2.8%
    // slower (regions of 16-32 tiles straddling t-groups; profiles/r03/bench_cfg4*.log), and in fp32
    // (which spills in the tile loop) 13-18% slower (profiles/r03/probe_fused_f32.log). (bf16 shared
    // heads: the 8-wave tile in one launch measured 5.53 vs 4.04-4.10 ms per 64 bags for
    // gate_pp_kernel + softmax_pool_kernel, profiles/r05/fused_ab_*; a fused form of gate_pp_kernel's
    // own tile 16.68 vs 16.56 ms per 256 bags, profiles/r05/pp_fused_probe.log, removed in round 6.)
    if (fm < 0 && (sizeof(E) != 2 || gp.uniform_rows <= 0 ||
                   mcgmil_detail::fused_regions(gp, total_rows, cap, true) < kFusedMinRegions))
        return 0;
    // same kernel shape as dispatch_gate_pipe: one class per wave for separate heads
    const int ppw = gp.P <= mcgmil::kGateWaves ? 1 : 2;
    const bool one = gp.G > 1 && gp.G == gp.C && (gp.D / 16) % ppw == 0;
    if (regions) {
        *regions = mcgmil_detail::fused_regions(gp, total_rows, cap, false);
        return 1;
    }
    *rc = mcgmil_detail::launch_gate_fused(gp, sizeof(E) == 2, ppw, MAXC, one, total_rows, s);
    return 1;
}

template <typename E>
int try_fused(const mcgmil::GateParams& gp, long long total_rows, int L, int flags, hipStream_t s, int* rc,
              long long* regions = nullptr) {
    return gp.C <= 2 ? try_fused_maxc<E, 2>(gp, total_rows, L, flags, s, rc, regions)
                     : try_fused_maxc<E, 4>(gp, total_rows, L, flags, s, rc, regions);
}

}  // namespace

extern "C" {

int mcgmil_abi_version(void) { return MCGMIL_ABI_VERSION; }

size_t mcgmil_args_size(void) { return sizeof(mcgmil_args); }

const char* mcgmil_last_error(void) { return mcgmil_detail::g_last_error.c_str(); }

int mcgmil_packed_weights_size(const mcgmil_args* a, size_t* bytes) {
    int rc = validate_sizes(a);
    if (rc) return rc;
    if (!bytes) return fail(MCGMIL_E_INVALID, "bytes is NULL");
    *bytes = packed_bytes_for(a);
    return MCGMIL_OK;
}

int mcgmil_workspace_size(const mcgmil_args* a, size_t* bytes) {
    int rc = validate_batch(a);
    if (rc) return rc;
    if (!bytes) return fail(MCGMIL_E_INVALID, "bytes is NULL");
    *bytes = layout_for(a).total;
    return MCGMIL_OK;
}

int mcgmil_pack_weights(const mcgmil_args* a, void* packed, void* stream) {
    int rc = validate_sizes(a);
    if (rc) return rc;
    if (!packed || !a->Wv || !a->Wu || !a->wk) return fail(MCGMIL_E_INVALID, "NULL weight or output pointer");
    const int P = a->G * (a->D / 16);
    const size_t total = (size_t)(2 * P + 1) * (a->L / 32) * 512;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (a->h_dtype == MCGMIL_BF16) {
        hipLaunchKernelGGL(mcgmil::pack_weights_kernel<__bf16>, dim3(blocks), dim3(256), 0, s, a->Wv,
                           a->Wu, a->wk, a->L, a->D, a->C, P, reinterpret_cast<__bf16*>(packed));
    } else
        hipLaunchKernelGGL(mcgmil::pack_weights_kernel<float>, dim3(blocks), dim3(256), 0, s, a->Wv,
                           a->Wu, a->wk, a->L, a->D, a->C, P, reinterpret_cast<float*>(packed));
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "pack_weights_kernel launch");
}

}  // extern "C"

namespace {

// Validation of the gate kernels' inputs and their launch parameters (mcgmil_gate_scores,
// mcgmil_gate_softmax_pool).
int gate_params(const mcgmil_args* a, mcgmil::GateParams& gp) {
    int rc = validate_batch(a);
    if (rc) return rc;
    const Layout l = layout_for(a);
    if ((rc = check_workspace(a, l))) return rc;
    if (!a->H && a->total_rows > 0) return fail(MCGMIL_E_INVALID, "H is NULL");
    if (!a->bv || !a->bu || !a->wa || !a->ba) return fail(MCGMIL_E_INVALID, "NULL bias / attention weight pointer");
    if (a->ldh < a->L) return fail(MCGMIL_E_INVALID, "ldh must be >= L");
    if (!aligned16(a->H) || (a->ldh * (long long)elem_size(a->h_dtype)) % 16 != 0)
        return fail(MCGMIL_E_ALIGN, "H and its row stride must be 16-byte aligned");
    if (!aligned16(a->bv) || !aligned16(a->bu) || !aligned16(a->wa))
        return fail(MCGMIL_E_ALIGN, "bv, bu and wa must be 16-byte aligned");
    if ((a->keep_feat == nullptr) != (a->keep_att == nullptr))
        return fail(MCGMIL_E_INVALID, "replay mode needs both keep_feat and keep_att");
    if (a->packed_w && !aligned16(a->packed_w)) return fail(MCGMIL_E_ALIGN, "packed_w must be 16-byte aligned");

    gp.H = a->H;
    gp.ldh = a->ldh;
    gp.bag_off = a->bag_offsets;
    gp.B = a->num_bags;
    gp.T = a->T;
    gp.L = a->L;
    gp.D = a->D;
    gp.C = a->C;
    gp.G = a->G;
    gp.P = a->G * (a->D / 16);
    gp.total_samples = (long long)a->T * a->total_rows;
    gp.Wp = packed_ptr(a);
    gp.wp_bytes = (uint32_t)packed_bytes_for(a);
    gp.bv = a->bv;
    gp.bu = a->bu;
    gp.wa = a->wa;
    gp.ba = a->ba;
    gp.sf = dropout_scale(a->p_feat);
    gp.sa = dropout_scale(a->p_att);
    gp.thr_f = drop_threshold(a->p_feat);
    gp.thr_a = drop_threshold(a->p_att);
    gp.thrx_f = mcgmil::packed_threshold(gp.thr_f);
    gp.k0 = (uint32_t)a->seed;
    gp.k1 = (uint32_t)(a->seed >> 32);
    gp.bag_base = a->bag_id_base;
    gp.t_base = a->t_base;
    gp.bag_ids = a->bag_ids;
    gp.keep_feat = a->keep_feat;
    gp.keep_att = a->keep_att;
    gp.logits = reinterpret_cast<float*>(static_cast<char*>(a->workspace) + l.logits_off);
    gp.zz = reinterpret_cast<float*>(static_cast<char*>(a->workspace) + l.zz_off);
#ifdef MCGMIL_STAMPS
    gp.stamps = static_cast<unsigned long long*>(a->debug);
    gp.clock = nullptr;
#else
    gp.stamps = nullptr;
    gp.clock = (a->flags & MCGMIL_CLOCK_PROBE) ? static_cast<unsigned long long*>(a->debug) : nullptr;
#endif
    gp.tile_bag = reinterpret_cast<const int32_t*>(static_cast<char*>(a->workspace) + l.plan_off);
    gp.tile_row0 = 0;
    gp.uniform_rows = a->uniform_bag_rows;
    gp.Y = a->Y;
    gp.A = a->A;
    gp.region_off = reinterpret_cast<const int32_t*>(static_cast<char*>(a->workspace) + l.region_off);
    gp.region_t = a->uniform_bag_rows > 0
                      ? mcgmil::region_t_groups(a->uniform_bag_rows, a->T,
                                                a->C <= 2 ? mcgmil::fused_cap<2>() : mcgmil::fused_cap<4>())
                      : 0;
    return MCGMIL_OK;
}

}  // namespace

extern "C" {

int mcgmil_gate_scores(const mcgmil_args* a, void* stream) {
    mcgmil::GateParams gp;
    if (int rc = gate_params(a, gp)) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (a->h_dtype == MCGMIL_BF16) return dispatch_gate<__bf16>(gp, a->L, a->h_dtype, a->flags, s);
    return dispatch_gate<float>(gp, a->L, a->h_dtype, a->flags, s);
}

int mcgmil_fused_regions(const mcgmil_args* a, int64_t* regions) {
    if (!regions) return fail(MCGMIL_E_INVALID, "regions is NULL");
    mcgmil::GateParams gp;
    if (int rc = gate_params(a, gp)) return rc;
    int rc = MCGMIL_OK;
    long long r = 0;
    const int fused = a->h_dtype == MCGMIL_BF16 ? try_fused<__bf16>(gp, a->total_rows, a->L, a->flags, nullptr, &rc, &r)
                                                : try_fused<float>(gp, a->total_rows, a->L, a->flags, nullptr, &rc, &r);
    *regions = fused ? r : 0;
    return MCGMIL_OK;
}

int mcgmil_gate_softmax_pool(const mcgmil_args* a, void* stream) {
    mcgmil::GateParams gp;
    if (int rc = gate_params(a, gp)) return rc;
    if (!a->Y) return fail(MCGMIL_E_INVALID, "Y is NULL");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc = MCGMIL_OK;
    const int fused = a->h_dtype == MCGMIL_BF16 ? try_fused<__bf16>(gp, a->total_rows, a->L, a->flags, s, &rc)
                                                : try_fused<float>(gp, a->total_rows, a->L, a->flags, s, &rc);
    if (fused) return rc;
    if ((rc = mcgmil_gate_scores(a, stream))) return rc;
    return mcgmil_softmax_pool(a, stream);
}

int mcgmil_softmax_pool(const mcgmil_args* a, void* stream) {
    int rc = validate_batch(a);
    if (rc) return rc;
    const Layout l = layout_for(a);
    if ((rc = check_workspace(a, l))) return rc;
    if (!a->Y) return fail(MCGMIL_E_INVALID, "Y is NULL");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const float* logits = reinterpret_cast<const float*>(static_cast<const char*>(a->workspace) + l.logits_off);
    const float* zz = reinterpret_cast<const float*>(static_cast<const char*>(a->workspace) + l.zz_off);
    hipLaunchKernelGGL(mcgmil::softmax_pool_kernel, dim3(a->T, a->num_bags), dim3(256), 0, s,
                       a->bag_offsets, a->T, a->C, logits, zz, a->Y, a->A);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "softmax_pool_kernel launch");
}

int mcgmil_bag_stats(const mcgmil_args* a, void* stream) {
    int rc = validate_batch(a);
    if (rc) return rc;
    if (!a->A_mean && !a->A_var && !a->P_mean) return MCGMIL_OK;
    if ((a->A_mean || a->A_var) && !a->A) return fail(MCGMIL_E_INVALID, "A_mean/A_var need the A output");
    if (!a->Y) return fail(MCGMIL_E_INVALID, "Y is NULL");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const long long outs = (a->A_mean || a->A_var) ? a->total_rows * a->C : 0;
    const long long sb = (outs + mcgmil::kStatOuts - 1) / mcgmil::kStatOuts;
    if (sb > 0x7fffffffll) return fail(MCGMIL_E_UNSUPPORTED, "too many attention outputs for bag_stats_kernel");
    const int stat_blocks = (int)sb;
    constexpr int kBagsPerBlock = mcgmil::kStatThreads / mcgmil::kWave;   // P_mean: one wave per bag
    const int p_blocks = a->P_mean ? (a->num_bags + kBagsPerBlock - 1) / kBagsPerBlock : 0;
    if (stat_blocks + p_blocks == 0) return MCGMIL_OK;
    hipLaunchKernelGGL(mcgmil::bag_stats_kernel, dim3(stat_blocks + p_blocks), dim3(mcgmil::kStatThreads), 0, s,
                       a->bag_offsets, a->num_bags, a->T, a->C, (long long)a->total_rows,
                       stat_blocks, a->A, a->Y, a->A_mean, a->A_var, a->P_mean);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "bag_stats_kernel launch");
}

int mcgmil_mcdo_forward(const mcgmil_args* a, void* stream) {
    int rc = validate_batch(a);
    if (rc) return rc;
    const Layout l = layout_for(a);
    if ((rc = check_workspace(a, l))) return rc;
    if (!a->packed_w) {
        if ((rc = mcgmil_pack_weights(a, a->workspace, stream))) return rc;
    }
    if ((rc = mcgmil_gate_softmax_pool(a, stream))) return rc;
    return mcgmil_bag_stats(a, stream);
}

int mcgmil_feature_keep(const mcgmil_args* a, uint8_t* keep_feat, void* stream) {
    int rc = validate_batch(a);
    if (rc) return rc;
    if (!keep_feat) return fail(MCGMIL_E_INVALID, "keep_feat is NULL");
    const long long total = (long long)a->T * a->total_rows * (a->L / 8);
    if (total == 0) return MCGMIL_OK;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    hipLaunchKernelGGL(mcgmil::feature_keep_kernel, dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), a->bag_offsets, a->num_bags, a->T,
                       a->L / 8, (long long)a->T * a->total_rows, (uint32_t)a->seed,
                       (uint32_t)(a->seed >> 32), a->bag_id_base, a->bag_ids, a->t_base,
                       drop_threshold(a->p_feat), keep_feat);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "feature_keep_kernel launch");
}

int mcgmil_attention_keep(const mcgmil_args* a, uint8_t* keep_att, void* stream) {
    int rc = validate_batch(a);
    if (rc) return rc;
    if (!keep_att) return fail(MCGMIL_E_INVALID, "keep_att is NULL");
    const long long total = (long long)a->T * a->C * a->total_rows;
    if (total == 0) return MCGMIL_OK;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    hipLaunchKernelGGL(mcgmil::attention_keep_kernel, dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), a->bag_offsets, a->num_bags, a->T,
                       a->C, total, (uint32_t)a->seed, (uint32_t)(a->seed >> 32), a->bag_id_base,
                       a->bag_ids, a->t_base, drop_threshold(a->p_att), keep_att);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "attention_keep_kernel launch");
}

}  // extern "C"
