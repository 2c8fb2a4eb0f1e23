// Micro-benchmark: a software-pipelined gate tile, to price it before writing the kernel.
// 8 waves (2 per SIMD), one workgroup per CU. A tile's K loop is split into two phases over
// half of the wave's gate pairs each (8 row tiles x 2 column tiles = 16 MFMAs per step + the
// classifier tile in phase A):
//   phase A  MFMAs of half A from the LDS-resident H tile; meanwhile the epilogue of half B of
//            the previous tile (2 gated products per lane per step); no barrier
//   phase B  MFMAs of half B; meanwhile the epilogue of half A, one Philox4x32-10 call +
//            masked staging of the next tile's slice (ds_write) and one barrier per step
// Against it: the current kernel's shape (33 MFMAs + Philox + staging + barrier per step, a
// 16-step tile, then the whole epilogue). TFLOP/s of the MFMA work, wall clock (HIP events).
// Build: hipcc --offload-arch=gfx950 -O3 -I montecarlo-gated-mil_amd/csrc scripts/ubench_sp.hip -o scripts/ubench_sp.bin
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "mcgmil_device.h"

using namespace mcgmil;

constexpr int kTiles = 32;
constexpr int KS = 16;

__device__ __forceinline__ float gp(float x, float y, float c, float part) {
    const float ax = fmaf(x, -2.88f, 0.1f), by = fmaf(y, -1.44f, 0.2f);
    const float a = __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(ax, -43.f, 43.f));
    const float b = __builtin_amdgcn_exp2f(by);
    const float ia = 1.f + a;
    const float r = __builtin_amdgcn_rcpf(fmaf(ia, b, ia));
    return fmaf(fmaf(-a, c, c), r, part);
}

// software-pipelined tile loop
template <int VPM>
__global__ __launch_bounds__(512, 1) void sp_kern(float* out, const __bf16* W, const __bf16* H, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) __bf16 Xs[KS][8 * 64 * 8];   // 128 KB: the whole tile
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < KS * 8 * 64 * 8; i += 512) (&Xs[0][0])[i] = (__bf16)(0.003f * (i & 255));
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(W, 64 * 1024);
    const uint32_t lane_b = (uint32_t)lane * 16u;
    const __bf16* hsrc = H + ((size_t)blockIdx.x * 512 + tid) * 8;
    f32x4 accA[8][2], accB[8][2], z = {0, 0, 0, 0};
    for (int r = 0; r < 8; ++r)
        for (int j = 0; j < 2; ++j) accA[r][j] = accB[r][j] = f32x4{0.001f * lane, 0, 0, 0};
    bf16x8 w0[3], w1[3];
    for (int j = 0; j < 3; ++j)
        for (int e = 0; e < 8; ++e) w0[j][e] = w1[j][e] = (__bf16)(0.001f * (lane + j + e));
    float part[8];
    for (int r = 0; r < 8; ++r) part[r] = 0.f;
    uint4 h = make_uint4(lane, 3, 5, 7), hn = h;
    int tt = 0;     // tile counter (Philox counter word)
    int zoff = 0;   // laundered per tile: keeps the unrolled steps' addresses out of the tile loop
    // one step: MFMAs of half `acc` (+ z in phase A); epilogue of 2 products of `fin`
    auto step = [&](int s, f32x4 (&acc)[8][2], f32x4 (&fin)[8][2], bool phaseB,
                    bf16x8 (&w)[3], bf16x8 (&wn)[3]) {
        __builtin_amdgcn_sched_barrier(0);   // no hoisting across steps of the unrolled phases
#pragma unroll
        for (int j = 0; j < 3; ++j)
            wn[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rs, lane_b, (uint32_t)((s + 1) & 15) * 3072u + j * 1024u, 0));
        if (phaseB) hn = *reinterpret_cast<const uint4*>(hsrc + zoff + (size_t)((s + 2) & 63) * 512 * 256 * 8);
        const __bf16* cur = Xs[s] + zoff;
#pragma unroll
        for (int rt = 0; rt < 8; ++rt) {
            const bf16x8 x = *reinterpret_cast<const bf16x8*>(cur + (rt * 64 + lane) * 8);
#pragma unroll
            for (int j = 0; j < 2; ++j)   // a phase starts a fresh half: zero C operand
                acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], x, s == 0 ? f32x4{0, 0, 0, 0} : acc[rt][j], 0, 0, 0);
        }
        {   // (in both phases: with the classifier tile in phase A only, the compiler sinks the
            // z chain into phase B and spills its operands)
            const bf16x8 xz = *reinterpret_cast<const bf16x8*>(cur + tid * 8);
            z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], xz, z, 0, 0, 0);
        }
        // 2 gated products of the finished half: row tile s/2, values 2*(s&1), +1
        {
            const int rt = s >> 1, v0 = 2 * (s & 1);
            part[rt] = gp(fin[rt][0][v0], fin[rt][1][v0], 0.3f, part[rt]);
            part[rt] = gp(fin[rt][0][v0 + 1], fin[rt][1][v0 + 1], 0.3f, part[rt]);
        }
        if (phaseB) {
            const uint4 o = philox4x32_10<true>((uint32_t)s * 4 + ((lane + zoff) >> 4), lane + zoff, (uint32_t)tt, seed, seed, ~seed);
            uint4 v = h;
            v.x = __builtin_amdgcn_bitop3_b32(v.x, drop_mask16x2_flipped(o.x, 0x19991999u), 0, 0x10);
            v.y = __builtin_amdgcn_bitop3_b32(v.y, drop_mask16x2(o.y, 0x19991999u), 0, 0x10);
            v.z = __builtin_amdgcn_bitop3_b32(v.z, drop_mask16x2_flipped(o.z, 0x19991999u), 0, 0x10);
            v.w = __builtin_amdgcn_bitop3_b32(v.w, drop_mask16x2(o.w, 0x19991999u), 0, 0x10);
            if (s > 0) *reinterpret_cast<uint4*>(&Xs[s - 1][0] + zoff + tid * 8) = v;   // slice s-1 is free
            h = hn;
        }
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
        }
        if (phaseB) __syncthreads();
    };
    for (int t = 0; t < kTiles; ++t) {
        asm volatile("" : "+s"(zoff));
        tt = t;
#pragma unroll
        for (int s = 0; s < KS; s += 2) {      // phase A: half A, finish half B
            step(s, accA, accB, false, w0, w1);
            step(s + 1, accA, accB, false, w1, w0);
        }
#pragma unroll
        for (int s = 0; s < KS; s += 2) {      // phase B: half B, finish half A, stage next tile
            step(s, accB, accA, true, w0, w1);
            step(s + 1, accB, accA, true, w1, w0);
        }
    }
    float t = z[0] + (float)(h.x ^ h.w);
    for (int r = 0; r < 8; ++r) t += part[r] + accA[r][0][0] + accB[r][1][3];
    out[blockIdx.x * 512 + tid] = t + (float)Xs[3][tid];
}

// the current kernel's shape: 33 MFMAs + Philox + staging + barrier per step, then the epilogue
__global__ __launch_bounds__(512, 1) void cur_kern(float* out, const __bf16* W, const __bf16* H, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) __bf16 Xs[2][8 * 64 * 8];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 2 * 8 * 64 * 8; i += 512) (&Xs[0][0])[i] = (__bf16)(0.003f * (i & 255));
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(W, 64 * 1024);
    const uint32_t lane_b = (uint32_t)lane * 16u;
    const __bf16* hsrc = H + ((size_t)blockIdx.x * 512 + tid) * 8;
    f32x4 acc[8][4], z = {0, 0, 0, 0};
    bf16x8 w0[5], w1[5];
    for (int j = 0; j < 5; ++j)
        for (int e = 0; e < 8; ++e) w0[j][e] = w1[j][e] = (__bf16)(0.001f * (lane + j + e));
    float part[8];
    for (int r = 0; r < 8; ++r) part[r] = 0.f;
    uint4 h = make_uint4(lane, 3, 5, 7), hn = h;
    auto step = [&](int s, bf16x8 (&w)[5], bf16x8 (&wn)[5]) {
#pragma unroll
        for (int j = 0; j < 5; ++j)
            wn[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rs, lane_b, (uint32_t)((s + 1) & 15) * 5120u + j * 1024u, 0));
        hn = *reinterpret_cast<const uint4*>(hsrc + (size_t)((s + 2) & 63) * 512 * 256 * 8);
        const __bf16* cur = Xs[s & 1];
#pragma unroll
        for (int rt = 0; rt < 8; ++rt) {
            const bf16x8 x = *reinterpret_cast<const bf16x8*>(cur + (rt * 64 + lane) * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], x, acc[rt][j], 0, 0, 0);
        }
        const bf16x8 xz = *reinterpret_cast<const bf16x8*>(cur + tid * 8);
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[4], xz, z, 0, 0, 0);
        const uint4 o = philox4x32_10<true>((uint32_t)s * 4 + (lane >> 4), lane, s, seed, seed, ~seed);
        uint4 v = h;
        v.x = __builtin_amdgcn_bitop3_b32(v.x, drop_mask16x2_flipped(o.x, 0x19991999u), 0, 0x10);
        v.y = __builtin_amdgcn_bitop3_b32(v.y, drop_mask16x2(o.y, 0x19991999u), 0, 0x10);
        v.z = __builtin_amdgcn_bitop3_b32(v.z, drop_mask16x2_flipped(o.z, 0x19991999u), 0, 0x10);
        v.w = __builtin_amdgcn_bitop3_b32(v.w, drop_mask16x2(o.w, 0x19991999u), 0, 0x10);
        *reinterpret_cast<uint4*>(&Xs[(s + 1) & 1][0] + tid * 8) = v;
        h = hn;
#pragma unroll
        for (int i = 0; i < 33; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        __syncthreads();
    };
    for (int t = 0; t < kTiles; ++t) {
        for (int r = 0; r < 8; ++r)
            for (int j = 0; j < 4; ++j) acc[r][j] = f32x4{0.001f * lane, 0, 0, 0};
        for (int s = 0; s < KS; s += 2) {
            step(s, w0, w1);
            step(s + 1, w1, w0);
        }
#pragma unroll
        for (int rt = 0; rt < 8; ++rt)
#pragma unroll
            for (int jp = 0; jp < 2; ++jp)
#pragma unroll
                for (int v = 0; v < 4; ++v) part[rt] = gp(acc[rt][2 * jp][v], acc[rt][2 * jp + 1][v], 0.3f, part[rt]);
        __syncthreads();
    }
    float t = z[0] + (float)(h.x ^ h.w);
    for (int r = 0; r < 8; ++r) t += part[r] + acc[r][0][0];
    out[blockIdx.x * 512 + tid] = t + (float)Xs[1][tid];
}

template <typename K>
void run(const char* name, K kern, int mfma_per_tile, float* out, const __bf16* W, const __bf16* H, int cus) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(cus), dim3(512), 0, 0, out, W, H, 7u);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(cus), dim3(512), 0, 0, out, W, H, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    // MFMAs of 16x16x32 issued per wave per tile (sp: 32 steps x 17, current: 16 x 33)
    const double flops = (double)cus * 8 * kTiles * mfma_per_tile * (16.0 * 16 * 32 * 2) * reps;
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"tflops\": %.1f}\n", name, ms / reps, flops / (ms * 1e-3) / 1e12);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    __bf16 *W, *H;
    const size_t hbytes = (size_t)cus * 512 * 8 * 2 + (size_t)64 * 512 * 256 * 8 * 2;
    hipMalloc(&out, (size_t)cus * 512 * sizeof(float));
    hipMalloc(&W, 64 * 1024);
    hipMalloc(&H, hbytes);
    hipMemset(W, 0, 64 * 1024);
    hipMemset(H, 0, hbytes);
    run("current shape: 33 MFMA/step + Philox + barrier, epilogue after the tile", cur_kern, 528, out, W, H, cus);
    run("software-pipelined halves, VPM 2", sp_kern<2>, 544, out, W, H, cus);
    run("software-pipelined halves, VPM 3", sp_kern<3>, 544, out, W, H, cus);
    run("software-pipelined halves, VPM 4", sp_kern<4>, 544, out, W, H, cus);
    run("current shape (again)", cur_kern, 528, out, W, H, cus);
    hipFree(out);
    hipFree(W);
    hipFree(H);
    return 0;
}
