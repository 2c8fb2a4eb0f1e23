# Round-6 call: conv_dma_kernel layer-3/4 A/B (interleaved DMA issue, timing diagnostics), then the
# final-tree traffic passes (config 3 fused, config 4 two-kernel).
timeout -k 10 600 env AB_LIBS=abvar/base.so,abvar/il.so,abvar/nowait.so,abvar/nobar.so,abvar/nomfma.so,abvar/noread.so,abvar/nodma.so,abvar/il.so,abvar/base.so python -u scripts/ab_conv_libs.py > gpurun_out/ab_dma_diag.log 2>&1 && grep -h "layers_3_4\|bitwise\|verdict" gpurun_out/ab_dma_diag.log && STEPS="pmcfinal pmc4" bash scripts/gpu_round6.sh
