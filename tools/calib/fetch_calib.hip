// fetch_calib.hip -- known-bytes read patterns for calibrating rocprofv3's
// FETCH_SIZE on gfx950 against the access shapes of the local-phase kernels.
// MI355X_MICROARCH.md calibrates FETCH_SIZE only for wide streaming reads
// (it reports exactly half of the bytes); the full-resolution phase gathers
// 64-B cells (cell layout) or 4 x 16-B row pieces (half-complex layout).
//
//   stream16  : every lane reads consecutive 16 B        (the guide's case)
//   cell64    : every lane reads one random 64-B aligned segment (4 x 16 B)
//   rows4x16  : every lane reads 4 random 16-B pieces on 4 rows (half-complex taps)
//   line128   : every lane reads one random 128-B aligned segment
// Each kernel reads exactly BYTES bytes from a buffer far larger than the
// 256 MiB Infinity Cache, so every byte is a compulsory HBM read.
// Run: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib ; durations: --kernel-trace.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

__global__ void __launch_bounds__(256) stream16(const float4* __restrict__ a, size_t n, float* out)
{
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

// n segments of 64 B (4 float4), random segment per lane
__global__ void __launch_bounds__(256) cell64(const float4* __restrict__ a, size_t nSeg,
                                              size_t nPick, float* out)
{
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < nPick; i += (size_t)gridDim.x * 256) {
        const size_t g = mix(i) % nSeg;
        const float4* p = a + 4 * g;
        const float4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
        s += v0.x + v1.y + v2.z + v3.w;
    }
    if (s == 1234.5f) out[0] = s;
}

// 4 random 16-B pieces per lane on 4 "rows" (the 4 x 2-tap rows of a trilinear cell)
__global__ void __launch_bounds__(256) rows4x16(const float4* __restrict__ a, size_t nPiece,
                                                size_t nPick, float* out)
{
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < nPick; i += (size_t)gridDim.x * 256) {
        const size_t g = mix(i);
        const size_t base = g % (nPiece - 4 * 4096);
        const float4 v0 = a[base], v1 = a[base + 1024], v2 = a[base + 2048], v3 = a[base + 3072];
        s += v0.x + v1.y + v2.z + v3.w;
    }
    if (s == 1234.5f) out[0] = s;
}

__global__ void __launch_bounds__(256) line128(const float4* __restrict__ a, size_t nSeg,
                                               size_t nPick, float* out)
{
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < nPick; i += (size_t)gridDim.x * 256) {
        const size_t g = mix(i) % nSeg;
        const float4* p = a + 8 * g;
        float4 v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = p[k];
        s += v[0].x + v[1].y + v[2].z + v[3].w + v[4].x + v[5].y + v[6].z + v[7].w;
    }
    if (s == 1234.5f) out[0] = s;
}

int main()
{
    const size_t bufBytes = 8ull << 30;         // 8 GiB table (>> 256 MiB MALL)
    const size_t readBytes = 2ull << 30;        // 2 GiB read per kernel
    float4* a;
    float* out;
    CHECK(hipMalloc(&a, bufBytes));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(a, 0, bufBytes));
    const size_t n16 = bufBytes / 16;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const dim3 grid(256 * 8 * 4), blk(256);
    for (int rep = 0; rep < 2; rep++) {
        float ms;
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(stream16, grid, blk, 0, 0, a, readBytes / 16, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("stream16 bytes=%zu ms=%.3f GBs=%.1f\n", readBytes, ms, readBytes / ms / 1e6);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(cell64, grid, blk, 0, 0, a, bufBytes / 64, readBytes / 64, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("cell64 bytes=%zu ms=%.3f GBs=%.1f\n", readBytes, ms, readBytes / ms / 1e6);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(rows4x16, grid, blk, 0, 0, a, n16, readBytes / 64, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("rows4x16 bytes=%zu ms=%.3f GBs=%.1f\n", readBytes, ms, readBytes / ms / 1e6);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(line128, grid, blk, 0, 0, a, bufBytes / 128, readBytes / 128, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("line128 bytes=%zu ms=%.3f GBs=%.1f\n", readBytes, ms, readBytes / ms / 1e6);
    }
    CHECK(hipFree(a));
    CHECK(hipFree(out));
    return 0;
}
