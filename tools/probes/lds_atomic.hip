// LDS float-atomic throughput probe (diagnostic): ds_add_f32 from 512-thread
// workgroups with different per-wave address patterns, against plain
// ds_read + ds_write of the same addresses.  hipcc -O3 --offload-arch=gfx950
// -munsafe-fp-atomics lds_atomic.hip -o lds_atomic && ./lds_atomic
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 4913 * 2;
constexpr int ITER = 4096;

template <int MODE, bool ATOMIC, typename V = float>
__global__ void __launch_bounds__(512) k(float* out, int seed)
{
    __shared__ V s[N];
    for (int i = threadIdx.x; i < N; i += 512) s[i] = 0.f;
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned h = (threadIdx.x + 1) * 2654435761u ^ seed;
    int a;
    for (int it = 0; it < ITER; it++) {
        if (MODE == 0) a = (wv * 64 + lane + it * 7) % N;                 // consecutive
        if (MODE == 1) a = (2 * (wv * 64 + lane) + it * 14) % N;          // stride 2
        if (MODE == 2) { h = h * 1664525u + 1013904223u; a = (h >> 8) % N; } // random
        if (MODE == 3) a = (((wv * 64 + lane) >> 2) + it * 7) % N;        // 4 lanes per address
        if (MODE == 4) a = ((4 * lane + 68 * wv) + it * 3) % N;           // stride 4
        if (ATOMIC) atomicAdd(&s[a], (V)1);
        else s[a] += (V)1;
    }
    __syncthreads();
    float v = 0.f;
    for (int i = threadIdx.x; i < N; i += 512) v += (float)s[i];
    out[blockIdx.x * 512 + threadIdx.x] = v;
}

template <int MODE, bool ATOMIC, typename V = float>
void run(const char* name, float* d)
{
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int blocks = 256 * 2 * 4;
    hipLaunchKernelGGL((k<MODE, ATOMIC, V>), dim3(blocks), dim3(512), 0, 0, d, 1);
    hipEventRecord(a);
    hipLaunchKernelGGL((k<MODE, ATOMIC, V>), dim3(blocks), dim3(512), 0, 0, d, 2);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double instr = (double)blocks * 8 * ITER;   // wave-instructions
    const double cyc = ms * 1e-3 * 2.4e9 * 256 / instr;
    printf("{\"type\": \"%s\", \"pattern\": \"%s\", \"atomic\": %d, \"ms\": %.3f, \"cu_cycles_per_wave_op\": %.2f}\n", sizeof(V) == 8 ? "u64" : ((V)0.5 == 0 ? "u32" : "f32"), name,
           (int)ATOMIC, ms, cyc);
}

int main()
{
    float* d;
    hipMalloc(&d, 256 * 2 * 4 * 512 * sizeof(float));
    run<0, true>("consecutive", d); run<0, false>("consecutive", d);
    run<1, true>("stride2", d); run<1, false>("stride2", d);
    run<4, true>("stride4", d); run<4, false>("stride4", d);
    run<2, true>("random", d); run<2, false>("random", d);
    run<3, true>("4-per-address", d); run<3, false>("4-per-address", d);
    run<0, true, unsigned>("consecutive", d); run<2, true, unsigned>("random", d);
    run<3, true, unsigned>("4-per-address", d);
    run<0, true, unsigned long long>("consecutive", d); run<2, true, unsigned long long>("random", d);
    run<3, true, unsigned long long>("4-per-address", d);
    return 0;
}
