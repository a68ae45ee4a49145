// fsc.hip -- a14: Fourier shell correlation of two half-complex volumes
// (FSC(vec&, const Volume&, const Volume&), src/Functions/Spectrum.cpp:
// 302-337, over VOLUME_FOR_EACH_PIXEL_FT, include/Image/Volume.h:86-89).
#include "common.h"

// Grid-stride over the half-complex grid; per-block shell histograms in LDS
// (FP64), one FP64 atomic per shell per block into the workspace.  The grid
// is HBM-streamed once (16 B per voxel pair read).
__global__ void __launch_bounds__(256) k_fsc_accum(const float2* __restrict__ A,
                                                   const float2* __restrict__ B,
                                                   int vdim, int nShell,
                                                   double* __restrict__ acc)
{
    extern __shared__ double sh[];   // [3][nShell]
    for (int s = threadIdx.x; s < 3 * nShell; s += blockDim.x) sh[s] = 0.0;
    __syncthreads();
    const int nColFT = vdim / 2 + 1;
    const long n = (long)nColFT * vdim * vdim;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int i = (int)(q % nColFT);
        const long jk = q / nColFT;
        const int jr = (int)(jk % vdim), kr = (int)(jk / vdim);
        const int j = jr < vdim / 2 ? jr : jr - vdim;
        const int k = kr < vdim / 2 ? kr : kr - vdim;
        const int u = (int)rint(sqrt((double)(i * i + j * j + k * k)));
        if (u < nShell) {
            const float2 a = A[q], b = B[q];
            atomicAdd(&sh[u], (double)(a.x * b.x + a.y * b.y));
            atomicAdd(&sh[nShell + u], (double)(a.x * a.x + a.y * a.y));
            atomicAdd(&sh[2 * nShell + u], (double)(b.x * b.x + b.y * b.y));
        }
    }
    __syncthreads();
    for (int s = threadIdx.x; s < 3 * nShell; s += blockDim.x)
        if (sh[s] != 0.0) atomicAdd(&acc[s], sh[s]);
}

__global__ void k_fsc_final(const double* __restrict__ acc, int nShell,
                            double* __restrict__ fsc)
{
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nShell) return;
    const double ab = sqrt(acc[nShell + s] * acc[2 * nShell + s]);
    fsc[s] = ab == 0.0 ? 0.0 : acc[s] / ab;
}

extern "C" size_t thx_fsc_workspace(int nShell)
{
    return sizeof(double) * 3 * (size_t)(nShell > 0 ? nShell : 0) + 256;
}

extern "C" int thx_fsc(const float* A, const float* B, int vdim, int nShell,
                       double* fsc, void* workspace, size_t wsBytes,
                       thx_stream_t stream)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0 && nShell > 0 && nShell <= 4096,
                  "thx_fsc: bad sizes");
    THX_CHECK_ARG(workspace && wsBytes >= thx_fsc_workspace(nShell),
                  "thx_fsc: workspace too small");
    hipStream_t s = thx::as_stream(stream);
    double* acc = static_cast<double*>(workspace);
    THX_HIP(hipMemsetAsync(acc, 0, sizeof(double) * 3 * nShell, s));
    hipLaunchKernelGGL(k_fsc_accum, dim3(1024), dim3(256),
                       sizeof(double) * 3 * nShell, s,
                       reinterpret_cast<const float2*>(A),
                       reinterpret_cast<const float2*>(B), vdim, nShell, acc);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_fsc_final, dim3(thx::cdiv(nShell, 256)), dim3(256), 0, s,
                       acc, nShell, fsc);
    THX_LAUNCH_CHECK();
    return THX_OK;
}
