// Launcher of gate_fused_kernel (mcgmil_kernels.h), the single-launch MCDO hot path, in its own
// translation unit: the tile loop fits the register file (no scratch) with LLVM's default
// machine scheduler and spills under the max-ILP strategy the two-kernel path's source uses
// (mcgmil/_build.py SOURCE_FLAGS).
#define MCGMIL_KERNELS_TEMPLATES_ONLY   // the plain kernels live in mcgmil.hip's object
#include "../../include/mcgmil.h"
#include "mcgmil_kernels.h"
#include "mcgmil_error.h"
#include "mcgmil_fused.h"


namespace mcgmil {

// Region counts per bag -> their prefix (one block; ragged batches only).
__global__ __launch_bounds__(1024) void plan_regions_kernel(const int32_t* bag_off, int B, int T,
                                                            int cap, int32_t* region_off) {
    __shared__ int part[1024];
    const int tid = threadIdx.x;
    const int per = (B + 1023) / 1024;
    const int b0 = tid * per, b1 = b0 + per < B ? b0 + per : B;
    int sum = 0;
    for (int b = b0; b < b1; ++b) {
        const int ts = region_t_groups(bag_off[b + 1] - bag_off[b], T, cap);
        sum += (T + ts - 1) / ts;
    }
    part[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {           // inclusive scan (Hillis-Steele)
        const int v = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int run = part[tid] - sum;                      // exclusive prefix of this thread's bags
    for (int b = b0; b < b1; ++b) {
        region_off[b] = run;
        const int ts = region_t_groups(bag_off[b + 1] - bag_off[b], T, cap);
        run += (T + ts - 1) / ts;
    }
    if (tid == 1023) region_off[B] = part[1023];
}

}  // namespace mcgmil

namespace mcgmil_detail {

long long fused_regions(const mcgmil::GateParams& gp, long long total_rows, int cap, bool estimate) {
    if (gp.uniform_rows > 0) {
        const int ts = mcgmil::region_t_groups(gp.uniform_rows, gp.T, cap);
        return (long long)gp.B * ((gp.T + ts - 1) / ts);
    }
    if (estimate) return (long long)gp.T * total_rows / cap;
    // grid bound: regions_b <= 2 T N_b / cap + 1 (region_t_groups); surplus workgroups exit
    return (2ll * gp.T * total_rows + cap - 1) / cap + gp.B + 1;
}

namespace {

template <typename E, int PPW, int MAXC, bool ONE>
int launch(const mcgmil::GateParams& gp, long long total_rows, hipStream_t s) {
    auto* k = gp.clock ? &mcgmil::gate_fused_kernel<E, PPW, MAXC, ONE, true>   // MCGMIL_CLOCK_PROBE
                       : &mcgmil::gate_fused_kernel<E, PPW, MAXC, ONE>;
    if (int rc = raise_lds_limit(reinterpret_cast<const void*>(k), "gate_fused_kernel LDS limit")) return rc;
    constexpr int cap = mcgmil::fused_cap<MAXC>();
    if (gp.uniform_rows <= 0) {
        hipLaunchKernelGGL(mcgmil::plan_regions_kernel, dim3(1), dim3(1024), 0, s, gp.bag_off, gp.B,
                           gp.T, cap, const_cast<int32_t*>(gp.region_off));
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "plan_regions_kernel launch");
    }
    const long long grid = fused_regions(gp, total_rows, cap, false);
    if (grid == 0) return MCGMIL_OK;
    if (grid > 0x7fffffffll) return fail(MCGMIL_E_UNSUPPORTED, "too many regions for one launch");
    const size_t lds = mcgmil::fused_kernel_lds_bytes<E, MAXC>(gp.L);
    if (lds > 160 * 1024) return fail(MCGMIL_E_UNSUPPORTED, "fused kernel: L too large for its LDS");
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(mcgmil::kGateThreads), lds, s, gp);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? MCGMIL_OK : hip_fail(e, "gate_fused_kernel launch");
}

template <typename E, int MAXC>
int launch_maxc(const mcgmil::GateParams& gp, int ppw, bool one, long long total_rows, hipStream_t s) {
    if (ppw == 1) return one ? launch<E, 1, MAXC, true>(gp, total_rows, s) : launch<E, 1, MAXC, false>(gp, total_rows, s);
    return one ? launch<E, 2, MAXC, true>(gp, total_rows, s) : launch<E, 2, MAXC, false>(gp, total_rows, s);
}

}  // namespace

int launch_gate_fused(const mcgmil::GateParams& gp, bool bf16, int ppw, int maxc, bool one,
                      long long total_rows, hipStream_t s) {
    if (bf16) return maxc == 2 ? launch_maxc<__bf16, 2>(gp, ppw, one, total_rows, s)
                               : launch_maxc<__bf16, 4>(gp, ppw, one, total_rows, s);
    return maxc == 2 ? launch_maxc<float, 2>(gp, ppw, one, total_rows, s)
                     : launch_maxc<float, 4>(gp, ppw, one, total_rows, s);
}

}  // namespace mcgmil_detail
