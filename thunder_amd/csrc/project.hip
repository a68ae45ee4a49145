// project.hip -- a6: Fourier-slice extraction (Projector::project,
// src/Projector.cpp:356-374) for a set of rotations shared by all images.
#include "common.h"

// One thread per (rotation, pixel): FP64 rotated coordinate, FP32 trilinear
// gather.  Rotation index is blockIdx.y, so the matrix loads are wave-uniform
// (scalar loads).  At the global-search radius the touched volume shell is a
// few MB and stays in L2; rotP is written once, coalesced.
__global__ void __launch_bounds__(256) k_project3d(const float2* __restrict__ vol,
                                                   int vdim, int pf,
                                                   const double* __restrict__ mat,
                                                   const int* __restrict__ iCol,
                                                   const int* __restrict__ iRow,
                                                   int nPxl,
                                                   float2* __restrict__ rotP)
{
    const int r = blockIdx.y;
    const double* m = mat + 9 * (size_t)r;
    double mm[6] = {m[0], m[1], m[2], m[3], m[4], m[5]};
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nPxl;
         i += gridDim.x * blockDim.x) {
        float x, y, z;
        rot_coord(mm, iCol[i], iRow[i], pf, x, y, z);
        rotP[(size_t)r * nPxl + i] = interp_ft(vol, vdim, x, y, z);
    }
}

extern "C" int thx_project3d(const float* vol, int vdim, int pf,
                             const double* mat, int nR, const int* iCol,
                             const int* iRow, int nPxl, float* rotP,
                             thx_stream_t stream)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0 && pf > 0 && nR >= 0 && nPxl >= 0,
                  "thx_project3d: bad sizes");
    THX_CHECK_ARG(nR <= 65535, "thx_project3d: nR > 65535 per call");
    if (nR == 0 || nPxl == 0) return THX_OK;
    const unsigned gx = thx::cdiv(nPxl, 256) > 32 ? 32 : thx::cdiv(nPxl, 256);
    hipLaunchKernelGGL(k_project3d, dim3(gx, nR), dim3(256), 0,
                       thx::as_stream(stream),
                       reinterpret_cast<const float2*>(vol), vdim, pf, mat,
                       iCol, iRow, nPxl, reinterpret_cast<float2*>(rotP));
    THX_LAUNCH_CHECK();
    return THX_OK;
}
