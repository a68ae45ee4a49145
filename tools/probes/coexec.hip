// MFMA / VALU co-execution probe (diagnostic): does the SIMD run VALU work
// under bf16 MFMAs, and does it matter whether the MFMA accumulators live in
// the architectural VGPRs (what the compiler picks for k_scan_split: the
// kernel's "amdgpu-agpr-alloc" is inferred 0) or in the AGPRs?
//   8 waves per workgroup (2 per SIMD), per wave and iteration 8 independent
//   v_mfma_f32_32x32x16_bf16 (8 accumulators, 128 registers) and NV packed
//   FP32 FMAs on independent chains; AGPR = 1 makes the compiler take the
//   MFMAs' AGPR form (an "a"-constraint inline-asm hint).  DEP = 1: the VALU chain of iteration i
//   forms (v_cvt_pk_bf16_f32) the A operand of iteration i + 1's MFMAs, as the
//   scan's w formation feeds its products.
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

template <int AGPR, int NV, int DEP>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
k_coexec(float* out, float seed)
{
    const int lane = threadIdx.x & 63;
    // AGPR: an inline-asm operand in the AGPR class keeps the attributor from
    // inferring "amdgpu-agpr-alloc"="0", and instruction selection then takes
    // the MFMAs' AGPR form (accumulators in a[...], half the registers each)
    if (AGPR) { float h = 0.f; asm volatile("; agpr hint %0" : "+a"(h)); }
    f32x16 acc[8];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 16; j++) acc[i][j] = 0.f;
    u32x4 ab;
    for (int k = 0; k < 4; k++) ab[k] = __builtin_bit_cast(unsigned, bf16x2{(__bf16)(seed + lane), (__bf16)(seed * k)});
    bf16x8 a = __builtin_bit_cast(bf16x8, ab), b = a;
    f32x2 x[8], y = {seed, seed * 0.5f}, z = {1e-3f, 2e-3f};
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = f32x2{seed + k, seed - k};
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
#pragma unroll
            for (int v = 0; v < NV / 8; v++) {
                const int k = (i * (NV / 8) + v) & 7;
                x[k] = __builtin_elementwise_fma(x[k], y, z);
            }
        }
        if (DEP) {
            u32x4 q;
#pragma unroll
            for (int k = 0; k < 4; k++)
                q[k] = __builtin_bit_cast(unsigned, bf16x2{(__bf16)x[2 * k].x, (__bf16)x[2 * k + 1].y});
            a = __builtin_bit_cast(bf16x8, q);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 16; j++) s += acc[i][j];
#pragma unroll
    for (int k = 0; k < 8; k++) s += x[k].x + x[k].y;
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int AGPR, int NV, int DEP>
void run(float* out, double& best_mfma_rate)
{
    const int grid = 256 * 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((k_coexec<AGPR, NV, DEP>), dim3(grid), dim3(512), 0, 0, out, 1.0f);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_coexec<AGPR, NV, DEP>), dim3(grid), dim3(512), 0, 0, out, 1.0f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double mfma = (double)grid * 8 * ITERS * 8;           // wave-level MFMA instructions
    const double rate = mfma / (best * 1e-3);
    if (rate > best_mfma_rate) best_mfma_rate = rate;
    printf("{\"agpr\": %d, \"valu_per_mfma\": %.2f, \"dep\": %d, \"ms\": %.4f, \"mfma_per_s\": %.4e, "
           "\"bf16_TFLOPs\": %.1f, \"rate_vs_best\": %.3f}\n",
           AGPR, NV / 8.0, DEP, best, rate, rate * 32768.0 / 1e12, rate / best_mfma_rate);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main()
{
    float* out;
    hipMalloc(&out, sizeof(float) * 256 * 4 * 512);
    double best = 0;
    run<0, 0, 0>(out, best);
    run<1, 0, 0>(out, best);
    run<0, 0, 0>(out, best);
    run<0, 8, 0>(out, best);
    run<1, 8, 0>(out, best);
    run<0, 16, 0>(out, best);
    run<1, 16, 0>(out, best);
    run<0, 32, 0>(out, best);
    run<1, 32, 0>(out, best);
    run<0, 64, 0>(out, best);
    run<1, 64, 0>(out, best);
    run<0, 16, 1>(out, best);
    run<1, 16, 1>(out, best);
    run<0, 32, 1>(out, best);
    run<1, 32, 1>(out, best);
    hipFree(out);
    return 0;
}
