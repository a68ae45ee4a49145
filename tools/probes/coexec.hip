// MFMA / VALU co-execution probe (diagnostic): does the SIMD run VALU work
// under bf16 MFMAs, and does it matter whether the MFMA accumulators live in
// the architectural VGPRs (what the compiler picks for k_scan_split: the
// kernel's "amdgpu-agpr-alloc" is inferred 0) or in the AGPRs?
//   8 waves per workgroup (2 per SIMD), per wave and iteration 8
//   v_mfma_f32_32x32x16_bf16 on NACC accumulators and NV packed
//   FP32 FMAs on independent chains; AGPR = 1 makes the compiler take the
//   MFMAs' AGPR form (an "a"-constraint inline-asm hint).  DEP = 1: the VALU chain of iteration i
//   forms (v_cvt_pk_bf16_f32) the A operand of iteration i + 1's MFMAs, as the
//   scan's w formation feeds its products.  DEP = 2: producer / consumer --
//   half the waves issue only VALU, the other half only MFMAs.  KIND: the
//   VALU instruction (packed / plain FP32 FMA, integer, bf16 packing).
// Prints one JSON line per variant: ms, MFMA issue rate as a fraction of the
// fastest MFMA-only run, VALU ops per MFMA.
//   hipcc -O3 --offload-arch=gfx950 coexec.hip -o coexec_bin && ./coexec_bin
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 2048;

// KIND of the VALU work: 0 v_pk_fma_f32, 1 v_fma_f32 (non-packed), 2 integer
// v_xad / shifts (the split's bit operations), 3 v_cvt_pk_bf16_f32
template <int KIND>
__device__ __forceinline__ void valu(f32x2& x, f32x2 y, f32x2 z)
{
    if (KIND == 0) x = __builtin_elementwise_fma(x, y, z);
    if (KIND == 1) x.x = __builtin_fmaf(x.x, y.x, z.x);
    if (KIND == 2) x.x = __uint_as_float((__float_as_uint(x.x) ^ __float_as_uint(y.x)) + 0x9e37u);
    if (KIND == 3) x.x = __builtin_bit_cast(float, bf16x2{(__bf16)(x.x * 1.0001f), (__bf16)y.y});
}

template <int AGPR, int NV, int DEP, int NACC = 8, int KIND = 0>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
k_coexec(float* out, float seed)
{
    const int lane = threadIdx.x & 63;
    // AGPR: an inline-asm operand in the AGPR class keeps the attributor from
    // inferring "amdgpu-agpr-alloc"="0", and instruction selection then takes
    // the MFMAs' AGPR form (accumulators in a[...], half the registers each)
    if (AGPR) { float h = 0.f; asm volatile("; agpr hint %0" : "+a"(h)); }
    f32x16 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; i++)
#pragma unroll
        for (int j = 0; j < 16; j++) acc[i][j] = 0.f;
    u32x4 ab;
    for (int k = 0; k < 4; k++) ab[k] = __builtin_bit_cast(unsigned, bf16x2{(__bf16)(seed + lane), (__bf16)(seed * k)});
    bf16x8 a = __builtin_bit_cast(bf16x8, ab), b = a;
    f32x2 x[8], y = {seed, seed * 0.5f}, z = {1e-3f, 2e-3f};
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = f32x2{seed + k, seed - k};
    // DEP == 2: producer / consumer split -- waves 0-3 (one per SIMD) issue
    // only the VALU chains (twice NV per iteration, the same total), waves
    // 4-7 only the MFMAs: time = max of the two if the SIMD overlaps another
    // wave's VALU with its MFMAs, their sum if it does not
    const int wave = threadIdx.x >> 6;
    if (DEP == 2 && wave < 4) {
        for (int it = 0; it < ITERS; it++)
#pragma unroll
            for (int v = 0; v < 2 * NV; v++) valu<KIND>(x[v & 7], y, z);
    } else
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            acc[i % NACC] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i % NACC], 0, 0, 0);
#pragma unroll
            for (int v = 0; v < (DEP == 2 ? 0 : NV / 8); v++) {
                const int k = (i * (NV / 8) + v) & 7;
                valu<KIND>(x[k], y, z);
            }
        }
        if (DEP == 1) {
            u32x4 q;
#pragma unroll
            for (int k = 0; k < 4; k++)
                q[k] = __builtin_bit_cast(unsigned, bf16x2{(__bf16)x[2 * k].x, (__bf16)x[2 * k + 1].y});
            a = __builtin_bit_cast(bf16x8, q);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NACC; i++)
#pragma unroll
        for (int j = 0; j < 16; j++) s += acc[i][j];
#pragma unroll
    for (int k = 0; k < 8; k++) s += x[k].x + x[k].y;
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int AGPR, int NV, int DEP, int NACC = 8, int KIND = 0>
void run(float* out, double& best_mfma_rate)
{
    const int grid = 256 * 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((k_coexec<AGPR, NV, DEP, NACC, KIND>), dim3(grid), dim3(512), 0, 0, out, 1.0f);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_coexec<AGPR, NV, DEP, NACC, KIND>), dim3(grid), dim3(512), 0, 0, out, 1.0f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double mfma = (double)grid * (DEP == 2 ? 4 : 8) * ITERS * 8;   // wave-level MFMA instructions
    const double rate = mfma / (best * 1e-3);
    if (rate > best_mfma_rate) best_mfma_rate = rate;
    printf("{\"agpr\": %d, \"nacc\": %d, \"valu_kind\": %d, \"valu_per_mfma\": %.2f, \"dep\": %d, "
           "\"ms\": %.4f, \"mfma_per_s\": %.4e, \"bf16_TFLOPs\": %.1f, \"rate_vs_best\": %.3f}\n",
           AGPR, NACC, KIND, NV / 8.0, DEP, best, rate, rate * 32768.0 / 1e12, rate / best_mfma_rate);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main()
{
    float* out;
    hipMalloc(&out, sizeof(float) * 256 * 4 * 512);
    double best = 0;
    // warm the clocks, then VGPR- and AGPR-form MFMAs (4 accumulators: the
    // AGPR form's half split of the 256 registers holds them without spills)
    run<0, 0, 0, 4>(out, best);
    run<0, 0, 0, 4>(out, best);
    run<1, 0, 0, 4>(out, best);
    run<0, 8, 0, 4>(out, best);
    run<1, 8, 0, 4>(out, best);
    run<0, 16, 0, 4>(out, best);
    run<1, 16, 0, 4>(out, best);
    run<0, 32, 0, 4>(out, best);
    run<1, 32, 0, 4>(out, best);
    run<0, 64, 0, 4>(out, best);
    run<1, 64, 0, 4>(out, best);
    run<0, 16, 1, 4>(out, best);
    run<1, 16, 1, 4>(out, best);
    // producer / consumer: half the waves, so MFMA-only time is the reference
    run<0, 0, 2, 4>(out, best);
    run<0, 8, 2, 4>(out, best);
    run<0, 16, 2, 4>(out, best);
    run<0, 32, 2, 4>(out, best);
    // the VALU kind: non-packed FMA, integer ops, bf16 packing, mixed per wave
    for (int r = 0; r < 1; r++) {
        run<0, 16, 0, 4, 1>(out, best);
        run<0, 16, 0, 4, 2>(out, best);
        run<0, 16, 0, 4, 3>(out, best);
        run<0, 16, 2, 4, 1>(out, best);
        run<0, 16, 2, 4, 2>(out, best);
    }
    hipFree(out);
    return 0;
}
