# Round-6 final-tree evidence in one lease: smoke, every GPU test, the driver's bench command, the
# rocprofv3 summary of that same command, config 4 and config 5 (bf16 and fp32). Each step has its
# own limit; a fault / abort / timeout ends the script (scripts/gpu_round6.sh).
STEPS="${STEPS:-smoke all bench prof cfg4 cfg5 cfg5f32}" bash scripts/gpu_round6.sh
