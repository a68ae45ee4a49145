// Trilinear gather probe (diagnostic): the local phase's unstaged taps for
// random rotations -- lane = (rotation slot l & 15, pixel slot l >> 4), four
// pixels of a patch row 2 voxels apart, 4 steps -- from a 512^3 half-complex
// projectee in (a) the row layout [z][y][x] (four 16-B row pieces per cell)
// and (b) 4x2x2-voxel bricks (one 128-B line per brick; x-pairs inside a
// brick row are one 16-B load).  Prints ms per 1.36e9 samples (one bench
// phase).  hipcc -O3 --offload-arch=gfx950 gather_layout.hip -o gather_layout_bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

constexpr int VD = 512, NC = VD / 2 + 1;
constexpr int BX = (NC + 3) / 4, BY = VD / 2, BZ = VD / 2;   // brick grid

__device__ __forceinline__ int wrapi(int v) { return v >= 0 ? v : v + VD; }

__device__ __forceinline__ size_t brick_idx(int x, int y, int z)
{
    // y, z wrapped to [0, VD); brick (x>>2, y>>1, z>>1), inside (z&1, y&1, x&3)
    const size_t b = ((size_t)(z >> 1) * BY + (y >> 1)) * BX + (x >> 2);
    return b * 16 + ((z & 1) * 2 + (y & 1)) * 4 + (x & 3);
}

__device__ __forceinline__ void rot_of(unsigned s, float* m)
{
    // a pseudo-random rotation from a hashed unit quaternion
    unsigned h = s * 2654435761u;
    float q[4];
    for (int k = 0; k < 4; k++) { h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15; q[k] = (float)(h & 0xffff) / 32768.f - 1.f; }
    const float n = rsqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int k = 0; k < 4; k++) q[k] *= n;
    const float a = q[0], b = q[1], c = q[2], d = q[3];
    m[0] = a * a + b * b - c * c - d * d; m[1] = 2 * (b * c + a * d); m[2] = 2 * (b * d - a * c);
    m[3] = 2 * (b * c - a * d); m[4] = a * a - b * b + c * c - d * d; m[5] = 2 * (c * d + a * b);
}

template <bool BRICK>
__global__ void __launch_bounds__(512) k_gather(const float2* __restrict__ vol, int nTile, float* out)
{
    float m[6];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    rot_of(blockIdx.x * 128 + wv * 16 + (lane & 15), m);
    const int g = lane >> 4;
    float acc = 0.f;
    for (int c = 0; c < nTile; c++) {            // patches of 4x4 pixels inside radius ~24
        const unsigned h = (blockIdx.x * 977u + c * 131u) * 2654435761u;
        const int pc = (int)(h % 40u) - 20, pr = (int)((h >> 8) % 40u) - 20;
        for (int s = 0; s < 4; s++) {
            const float X = 2.f * (pc + g), Y = 2.f * (pr + s);
            float x = m[0] * X + m[3] * Y, y = m[1] * X + m[4] * Y, z = m[2] * X + m[5] * Y;
            if (x < 0) { x = -x; y = -y; z = -z; }
            const int x0 = (int)floorf(x), y0 = (int)floorf(y), z0 = (int)floorf(z);
            const float dx = x - x0, dy = y - y0, dz = z - z0;
            float sre = 0.f;
            for (int kz = 0; kz < 2; kz++)
                for (int jy = 0; jy < 2; jy++) {
                    const int yy = wrapi(y0 + jy), zz = wrapi(z0 + kz);
                    float2 a, b;
                    if (!BRICK) {
                        const float4 v = *reinterpret_cast<const float4*>(vol + ((size_t)zz * VD + yy) * NC + x0);
                        a = make_float2(v.x, v.y); b = make_float2(v.z, v.w);
                    } else if ((x0 & 3) != 3) {
                        const float4 v = *reinterpret_cast<const float4*>(vol + brick_idx(x0, yy, zz));
                        a = make_float2(v.x, v.y); b = make_float2(v.z, v.w);
                    } else {
                        a = vol[brick_idx(x0, yy, zz)]; b = vol[brick_idx(x0 + 1, yy, zz)];
                    }
                    const float wyz = (jy ? dy : 1.f - dy) * (kz ? dz : 1.f - dz);
                    sre += (a.x * (1.f - dx) + b.x * dx) * wyz;
                }
            acc += sre;
        }
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

int main()
{
    const size_t nv = (size_t)BX * 4 * BY * 2 * BZ * 2;
    float2* vol;
    float* out;
    hipMalloc(&vol, nv * sizeof(float2));
    hipMemset(vol, 0, nv * sizeof(float2));
    const int nImg = 12500, nTile = 59;   // 12 500 images x 59 patches, 128 rotations each
    hipMalloc(&out, (size_t)nImg * 512 * sizeof(float));
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int rep = 0; rep < 2; rep++) {
        for (int layout = 0; layout < 2; layout++) {
            hipEventRecord(a);
            if (layout == 0) hipLaunchKernelGGL(k_gather<false>, dim3(nImg), dim3(512), 0, 0, vol, nTile, out);
            else hipLaunchKernelGGL(k_gather<true>, dim3(nImg), dim3(512), 0, 0, vol, nTile, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("{\"layout\": \"%s\", \"ms\": %.3f}\n", layout ? "brick4x2x2" : "rows", ms);
        }
    }
    return 0;
}
