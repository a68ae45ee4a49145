// insert.hip -- a12: weighted trilinear back-projection into the half-map
// (Reconstructor::insertP, src/Reconstructor.cpp:782-863, driven by the CPU
// loop of src/Optimiser.cpp:7036-7241; GPU twin cuthunder::InsertFT,
// gpu/src/cuthunder.cu:5570-5826).
#include "common.h"

// Trilinear scatter of Volume::addFT (src/Image/Volume.cpp:340-375):
// Hermitian fold conjugates the complex value, 8 taps in box order, FP32
// device-scope atomics (global_atomic_add_f32) on F (re, im) and T.
THX_DEV void scatter_ft(float2* __restrict__ F, float* __restrict__ T, int vdim,
                        float x, float y, float z, float vr, float vi, float tv)
{
    if (!(x >= 0.f)) { x = -x; y = -y; z = -z; vi = -vi; }
    const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
    const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
    const float dx = x - fx, dy = y - fy, dz = z - fz;
    const float vx[2] = {1.f - dx, dx};
    const float vy[2] = {1.f - dy, dy};
    const float vz[2] = {1.f - dz, dz};
    const int nColFT = vdim / 2 + 1;
#pragma unroll
    for (int k = 0; k < 2; k++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const size_t row = ((size_t)wrap_idx(z0 + k, vdim) * vdim +
                                wrap_idx(y0 + j, vdim)) * nColFT + x0;
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const float w = vx[i] * vy[j] * vz[k];
                float* f = reinterpret_cast<float*>(F + row + i);
                atomicAdd(f, vr * w);
                atomicAdd(f + 1, vi * w);
                atomicAdd(T + row + i, tv * w);
            }
        }
}

// Workgroup = (pixel slice, sample m, image l).  The rotation comes from the
// sample's quaternion (rotate3D), the image is re-centred by -(t - off)
// (translate(dst, src, ...), src/Image/ImageFunctions.cpp:471-492), and the
// value inserted is src * ctf * w; T receives ctf^2 * w.
__global__ void __launch_bounds__(256) k_insert3d(float2* __restrict__ F,
                                                  float* __restrict__ T,
                                                  double* __restrict__ O,
                                                  int* __restrict__ counter,
                                                  int vdim, int pf,
                                                  const float2* __restrict__ dat,
                                                  const float* __restrict__ ctf,
                                                  const double* __restrict__ quat,
                                                  const double* __restrict__ trans,
                                                  const double* __restrict__ offS,
                                                  const float* __restrict__ w,
                                                  int mReco,
                                                  const int* __restrict__ iCol,
                                                  const int* __restrict__ iRow,
                                                  int nPxl, int idim)
{
    const int m = blockIdx.y, l = blockIdx.z;
    const size_t sIdx = (size_t)l * mReco + m;
    __shared__ double sMat[9];
    if (threadIdx.x == 0) {
        double q[4] = {quat[4 * sIdx], quat[4 * sIdx + 1], quat[4 * sIdx + 2],
                       quat[4 * sIdx + 3]};
        quat_to_mat(q, sMat);
    }
    __syncthreads();
    const double dx = trans[2 * sIdx] - offS[2 * l];
    const double dy = trans[2 * sIdx + 1] - offS[2 * l + 1];
    const float rCol = (float)(-dx) / idim, rRow = (float)(-dy) / idim;
    const float wl = w[l];
    const double m0 = sMat[0], m1 = sMat[1], m2 = sMat[2];
    const double m3 = sMat[3], m4 = sMat[4], m5 = sMat[5];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // insertDir(-R (t - off, 0)), src/Reconstructor.cpp:407-422
        atomicAdd(O + 0, -(m0 * dx + m3 * dy));
        atomicAdd(O + 1, -(m1 * dx + m4 * dy));
        atomicAdd(O + 2, -(m2 * dx + m5 * dy));
        atomicAdd(counter, 1);
    }
    const float2* D = dat + (size_t)l * nPxl;
    const float* C = ctf + (size_t)l * nPxl;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nPxl;
         i += gridDim.x * blockDim.x) {
        const int ic = iCol[i], ir = iRow[i];
        const float2 src = cmul(D[i], phase_shift(ic, ir, rCol, rRow));
        const float c = C[i];
        const float vr = (src.x * c) * wl, vi = (src.y * c) * wl;
        const float tv = (float)((double)c * c) * wl;
        const double nx = (double)(ic * pf), ny = (double)(ir * pf);
        scatter_ft(F, T, vdim, (float)(m0 * nx + m3 * ny), (float)(m1 * nx + m4 * ny),
                   (float)(m2 * nx + m5 * ny), vr, vi, tv);
    }
}

extern "C" int thx_insert3d(float* F, float* T, double* O, int* counter,
                            int vdim, int pf, const float* dat, const float* ctf,
                            const double* quat, const double* trans,
                            const double* offS, const float* w, int nImg,
                            int mReco, const int* iCol, const int* iRow,
                            int nPxl, int idim, thx_stream_t stream)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0 && pf > 0 && nImg >= 0 && mReco >= 0 &&
                      nPxl >= 0 && idim > 0,
                  "thx_insert3d: bad sizes");
    THX_CHECK_ARG(nImg <= 65535 && mReco <= 65535, "thx_insert3d: grid too large");
    if (nImg == 0 || mReco == 0 || nPxl == 0) return THX_OK;
    const unsigned gx = thx::cdiv(nPxl, 256) > 16 ? 16 : thx::cdiv(nPxl, 256);
    hipLaunchKernelGGL(k_insert3d, dim3(gx, mReco, nImg), dim3(256), 0,
                       thx::as_stream(stream), reinterpret_cast<float2*>(F), T, O,
                       counter, vdim, pf, reinterpret_cast<const float2*>(dat),
                       ctf, quat, trans, offS, w, mReco, iCol, iRow, nPxl, idim);
    THX_LAUNCH_CHECK();
    return THX_OK;
}
