# Round-4 end: the BN apply / vertical-pool A/B (scripts/ab_bn.sh), then the evidence steps of
# scripts/gpu_round4.sh on the tree as built (smoke, every GPU test, the headline bench and its rocprof
# summary, config 5 and its trace). Stops at the first step that faults or times out.
set -o pipefail
timeout -k 10 600 bash scripts/ab_bn.sh > gpurun_out/ab_bn.log 2>&1
echo "== ab_bn rc=$?"
STEPS="smoke all bench prof cfg5 profcfg5" bash scripts/gpu_round4.sh
