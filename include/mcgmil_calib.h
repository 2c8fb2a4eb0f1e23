/*
 * mcgmil_calib.h -- measurement entry point: the MFMA rate this MI355X actually sustains.
 *
 * Not part of the drop-in boundary (the reference has nothing like it). bench.py prices every
 * MFMA-bound kernel twice: against the spec peak (2.5 PFLOP/s bf16, 157.3 TFLOP/s fp32 at 2.4 GHz)
 * and against this calibration loop run on the same box in the same process, so that a roofline
 * fraction says how far a kernel is from what the chip sustains under a comparable load
 * (MI355X_MICROARCH.md, "DVFS give-back": on random bf16 data the chip holds ~1.9 GHz, not 2.4).
 *
 * The loop (csrc/mcgmil_calib.hip): one 512-thread workgroup per CU (two waves per SIMD, the
 * occupancy of gate_pipe_kernel / gate_fused_kernel), each wave 4 A fragments in registers and 8 B
 * fragments re-read from LDS by ds_read_b128 every step (as pipe_tile reads its instance tiles),
 * 32 independent accumulators, random full-range operands in [-1, 1), no barrier, no global
 * memory in the loop.
 *   bf16: 32 v_mfma_f32_16x16x32_bf16 per wave-step (16,384 FLOP each);
 *   fp32: 128 v_mfma_f32_16x16x4_f32 per wave-step (2,048 FLOP each).
 */
#ifndef MCGMIL_CALIB_H_
#define MCGMIL_CALIB_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* FLOPs one workgroup-step of the loop performs (8 waves), for dtype MCGMIL_BF16 / MCGMIL_F32
 * (mcgmil.h enum mcgmil_dtype); 0 for any other dtype. */
int64_t mcgmil_mfma_calib_flops_per_step(int dtype);

/* Launch the loop: `workgroups` workgroups (one per CU: the CU count) x `steps` steps, operands
 * drawn from `seed`. sink: float [workgroups * 512] (device; every thread's accumulator sum, so
 * nothing is dead code). clock: NULL or uint64 [MCGMIL_CLOCK_SLOTS][4] (device): workgroups
 * 0..MCGMIL_CLOCK_SLOTS-1 write (s_memtime, s_memrealtime) after their LDS fill and after the
 * loop, the layout of MCGMIL_CLOCK_PROBE (mcgmil.h). Asynchronous on `stream`. */
int mcgmil_mfma_calib(int dtype, int32_t workgroups, int32_t steps, uint32_t seed, float* sink,
                      uint64_t* clock, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MCGMIL_CALIB_H_ */
