// Trilinear gather probe (diagnostic), as gather_layout.hip: the local
// phase's unstaged taps for random rotations from a 512^3 half-complex
// projectee, lane = (rotation slot l & 15, pixel slot l >> 4), in
//   rows   [z][y][x] complex             4 x 16-B loads on 4 lines per cell
//   ypair  [z][y][x] (v(y), v(y+1))      4 x 16-B loads on 2 lines (2x memory)
//   quad   [z][y][x] (v(y,z), v(y+1,z), v(y,z+1), v(y+1,z+1))
//                                        4 x 16-B loads on 1-2 lines (4x memory)
// Prints ms per 1.36e9 samples (one bench phase).
//   hipcc -O3 --offload-arch=gfx950 gather_pairs.hip -o gather_pairs_bin
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int VD = 512, NC = VD / 2 + 1;

__device__ __forceinline__ int wrapi(int v) { return v >= 0 ? v : v + VD; }

__device__ __forceinline__ void rot_of(unsigned s, float* m)
{
    unsigned h = s * 2654435761u;
    float q[4];
    for (int k = 0; k < 4; k++) { h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15; q[k] = (float)(h & 0xffff) / 32768.f - 1.f; }
    const float n = rsqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int k = 0; k < 4; k++) q[k] *= n;
    const float a = q[0], b = q[1], c = q[2], d = q[3];
    m[0] = a * a + b * b - c * c - d * d; m[1] = 2 * (b * c + a * d); m[2] = 2 * (b * d - a * c);
    m[3] = 2 * (b * c - a * d); m[4] = a * a - b * b + c * c - d * d; m[5] = 2 * (c * d + a * b);
}

template <int LAYOUT>
__global__ void __launch_bounds__(512) k_gather(const float4* __restrict__ vol, int nTile, float* out)
{
    float m[6];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    rot_of(blockIdx.x * 128 + wv * 16 + (lane & 15), m);
    const int g = lane >> 4;
    float acc = 0.f;
    for (int c = 0; c < nTile; c++) {
        const unsigned h = (blockIdx.x * 977u + c * 131u) * 2654435761u;
        const int pc = (int)(h % 40u) - 20, pr = (int)((h >> 8) % 40u) - 20;
        for (int s = 0; s < 4; s++) {
            const float X = 2.f * (pc + g), Y = 2.f * (pr + s);
            float x = m[0] * X + m[3] * Y, y = m[1] * X + m[4] * Y, z = m[2] * X + m[5] * Y;
            if (x < 0) { x = -x; y = -y; z = -z; }
            const int x0 = (int)floorf(x), y0 = (int)floorf(y), z0 = (int)floorf(z);
            const float dx = x - x0, dy = y - y0, dz = z - z0;
            float sre = 0.f;
            if (LAYOUT == 0) {          // rows: float4 = 2 complex along x
                const float2* v2 = reinterpret_cast<const float2*>(vol);
                for (int kz = 0; kz < 2; kz++)
                    for (int jy = 0; jy < 2; jy++) {
                        const size_t r = ((size_t)wrapi(z0 + kz) * VD + wrapi(y0 + jy)) * NC + x0;
                        const float2 a = v2[r], b = v2[r + 1];
                        sre += (a.x * (1.f - dx) + b.x * dx) * (jy ? dy : 1.f - dy) * (kz ? dz : 1.f - dz);
                    }
            } else if (LAYOUT == 1) {   // ypair: one float4 per voxel = (v(y), v(y+1))
                for (int kz = 0; kz < 2; kz++) {
                    const size_t r = ((size_t)wrapi(z0 + kz) * VD + wrapi(y0)) * NC + x0;
                    const float4 a = vol[r], b = vol[r + 1];
                    const float wz = kz ? dz : 1.f - dz;
                    sre += ((a.x * (1.f - dy) + a.z * dy) * (1.f - dx) + (b.x * (1.f - dy) + b.z * dy) * dx) * wz;
                }
            } else {                    // quad: two float4 per voxel
                const size_t r = (((size_t)wrapi(z0) * VD + wrapi(y0)) * NC + x0) * 2;
                const float4 a0 = vol[r], a1 = vol[r + 1], b0 = vol[r + 2], b1 = vol[r + 3];
                const float w00 = (1.f - dy) * (1.f - dz), w10 = dy * (1.f - dz), w01 = (1.f - dy) * dz, w11 = dy * dz;
                sre += (a0.x * w00 + a0.z * w10 + a1.x * w01 + a1.z * w11) * (1.f - dx) +
                       (b0.x * w00 + b0.z * w10 + b1.x * w01 + b1.z * w11) * dx;
            }
            acc += sre;
        }
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

int main()
{
    const size_t nv = (size_t)VD * VD * NC;
    float4* vol;
    float* out;
    hipMalloc(&vol, nv * 2 * sizeof(float4));            // room for the quad layout
    hipMemset(vol, 0, nv * 2 * sizeof(float4));
    const int nImg = 12500, nTile = 59;
    hipMalloc(&out, (size_t)nImg * 512 * sizeof(float));
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const char* names[3] = {"rows", "ypair", "quad"};
    for (int rep = 0; rep < 2; rep++)
        for (int L = 0; L < 3; L++) {
            hipEventRecord(a);
            if (L == 0) hipLaunchKernelGGL(k_gather<0>, dim3(nImg), dim3(512), 0, 0, vol, nTile, out);
            if (L == 1) hipLaunchKernelGGL(k_gather<1>, dim3(nImg), dim3(512), 0, 0, vol, nTile, out);
            if (L == 2) hipLaunchKernelGGL(k_gather<2>, dim3(nImg), dim3(512), 0, 0, vol, nTile, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("{\"layout\": \"%s\", \"ms\": %.3f}\n", names[L], ms);
        }
    return 0;
}
