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

}  // namespace mcgmil_detail
