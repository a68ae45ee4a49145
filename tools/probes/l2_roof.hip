// L2 -> L1 gather roof probe (diagnostic): how fast the chip serves loads
// from an L2-resident table (2 MB by default, the size of the local phase's
// low-resolution projectee ball) when every lane hits a different 128-B line.
//   line16  : each lane 16 B from a random line (the half-complex row piece)
//   line8   : each lane 8 B from a random line (a single voxel)
//   seg64   : each lane 64 B (4 x 16 B) from one random 64-B segment (a cell)
//   stream  : 8 lanes per line, every byte of a line used (the L2 -> L1 peak)
//   coop64  : lanes 4s .. 4s+3 read the four 16-B pieces of one random 64-B
//             segment in one instruction (does the L1 merge a quad's pieces?)
// A table that fits L1 (e.g. 0.016 MB) measures the L1 access rate alone.
// Prints one JSON line per pattern: ms, loads/s, 128-B lines/s, and the line
// bytes per second (lines x 128 B) -- the roof the local phase's L2 gathers
// are priced against (bench.py roofline).
//   hipcc -O3 --offload-arch=gfx950 l2_roof.hip -o l2_roof_bin && ./l2_roof_bin [table_MB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int ITERS = 512, UNROLL = 8, THREADS = 512;

__device__ __forceinline__ unsigned mix(unsigned h)
{
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
}

template <int PAT>
__global__ void __launch_bounds__(THREADS) k_roof(const float* __restrict__ t, unsigned nLines, float* out)
{
    const unsigned gid = blockIdx.x * THREADS + threadIdx.x;
    float acc = 0.f;
    unsigned h = mix(gid * 2654435761u + 1);
    for (int it = 0; it < ITERS; it += UNROLL) {
        f32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
            h = mix(h + u);
            const unsigned line = h % nLines;
            if (PAT == 0) {        // line16
                v[u] = *reinterpret_cast<const f32x4*>(t + (size_t)line * 32 + ((h >> 24) & 7) * 4);
            } else if (PAT == 1) { // line8
                const f32x2 w = *reinterpret_cast<const f32x2*>(t + (size_t)line * 32 + ((h >> 24) & 15) * 2);
                v[u] = f32x4{w.x, w.y, 0.f, 0.f};
            } else if (PAT == 2) { // seg64: 4 x 16 B of one 64-B segment
                const f32x4* p = reinterpret_cast<const f32x4*>(t + (size_t)line * 32 + ((h >> 24) & 1) * 16);
                v[u] = p[0] + p[1] + p[2] + p[3];
            } else if (PAT == 4) { // coop64: a quad reads one 64-B segment
                const unsigned hq = mix((gid >> 2) * 2654435761u + it * 977u + u);
                const unsigned lq = hq % nLines;
                v[u] = *reinterpret_cast<const f32x4*>(t + (size_t)lq * 32 + ((hq >> 24) & 1) * 16 +
                                                       (threadIdx.x & 3) * 4);
            } else {               // stream: lanes 8k..8k+7 share a line
                const unsigned l8 = mix((gid >> 3) * 977u + it * 31u + u) % nLines;
                v[u] = *reinterpret_cast<const f32x4*>(t + (size_t)l8 * 32 + (threadIdx.x & 7) * 4);
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; u++) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    out[gid] = acc;
}

int main(int argc, char** argv)
{
    const double mb = argc > 1 ? atof(argv[1]) : 2.0;
    const unsigned nLines = (unsigned)(mb * 1024 * 1024 / 128);
    float* t;
    float* out;
    hipMalloc(&t, (size_t)nLines * 128);
    hipMemset(t, 0, (size_t)nLines * 128);
    const int blocks = 256 * 8;
    hipMalloc(&out, (size_t)blocks * THREADS * sizeof(float));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[5] = {"line16", "line8", "seg64", "stream", "coop64"};
    const double loads = (double)blocks * THREADS * ITERS;
    for (int rep = 0; rep < 2; rep++)
        for (int p = 0; p < 5; p++) {
            hipEventRecord(a);
            if (p == 0) hipLaunchKernelGGL(k_roof<0>, dim3(blocks), dim3(THREADS), 0, 0, t, nLines, out);
            if (p == 1) hipLaunchKernelGGL(k_roof<1>, dim3(blocks), dim3(THREADS), 0, 0, t, nLines, out);
            if (p == 2) hipLaunchKernelGGL(k_roof<2>, dim3(blocks), dim3(THREADS), 0, 0, t, nLines, out);
            if (p == 3) hipLaunchKernelGGL(k_roof<3>, dim3(blocks), dim3(THREADS), 0, 0, t, nLines, out);
            if (p == 4) hipLaunchKernelGGL(k_roof<4>, dim3(blocks), dim3(THREADS), 0, 0, t, nLines, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            // distinct lines per load: 1 (line16, line8), 1 per 4 loads of a segment
            // counted as one lane-load of 64 B (seg64), 1/8 (stream)
            const double lines = p == 3 ? loads / 8 : p == 4 ? loads / 4 : loads;
            if (rep)
                printf("{\"pattern\": \"%s\", \"table_MB\": %.3f, \"ms\": %.3f, \"lane_loads_per_s\": %.4g, "
                       "\"lines_per_s\": %.4g, \"line_TBps\": %.3f}\n",
                       names[p], mb, ms, loads / ms * 1e3, lines / ms * 1e3, lines * 128 / ms / 1e9);
        }
    return hipGetLastError() != hipSuccess;
}
