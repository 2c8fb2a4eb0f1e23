// Host entry points of the fused MCDO kernel (mcgmil_fused.hip), used by mcgmil.hip.
#pragma once
#include "mcgmil_kernels.h"

namespace mcgmil_detail {

// Workgroups of a fused launch: exact for uniform bags; for ragged bags the grid bound, or
// with `estimate` T * total_rows / cap (the dispatch policy's size measure).
long long fused_regions(const mcgmil::GateParams& gp, long long total_rows, int cap, bool estimate);

// gate_fused_kernel<bf16 ? __bf16 : float, ppw, maxc, one> (+ the region plan for ragged bags).
int launch_gate_fused(const mcgmil::GateParams& gp, bool bf16, int ppw, int maxc, bool one,
                      long long total_rows, hipStream_t s);

// gate_pp_fused_kernel<bf16, 8, 2, maxc, one> (mcgmil_gate_pp.h; bf16 heads of <= 8 gate tile
// pairs, e.g. shared heads; regions of pp_fused_cap<maxc> rows).
int launch_pp_fused(const mcgmil::GateParams& gp, int maxc, bool one, long long total_rows, hipStream_t s);

// rowgate_fused_kernel<G, D/32, maxc> (mcgmil_rowgate.h; bf16, D = 128, G = 1 or 2).
int launch_rowgate_fused(const mcgmil::GateParams& gp, int maxc, long long total_rows, hipStream_t s);

}  // namespace mcgmil_detail
