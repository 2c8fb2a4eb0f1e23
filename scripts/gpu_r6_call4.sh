# Round-6 call: final-tree HBM traffic of the gate launches (config 3 fused, config 4 two-kernel),
# the GRBM clock cross-check with the steady-state probe, and the single-bag path's kernel trace.
STEPS="pmcfinal pmc4 grbm profsingle" bash scripts/gpu_round6.sh
