// twod.hip -- f4: the 2D classification path (MODE_2D) on device.
//
//   a6 2D: Projector::project(Complex*, const dmat22&, ...) (src/Projector.cpp:
//     337-354) -> Image::getByInterpolationFT (src/Image/Image.cpp:345-367):
//     c = R (iCol pf, iRow pf), R = [[c, -s], [s, c]] (rotate2D,
//     src/Geometry/Euler.cpp:125-131, from the particle's (_r(i,0), _r(i,1)),
//     src/Particle.cpp:850-854); Hermitian fold when x < 0; bilinear
//     (WG_BI_INTERP_LINEAR, include/Functions/Interpolation.h:137-150) over
//     the half-complex [j][i] image (getFTHalf, rows wrapped).  GPU twins
//     kernel_Project2D / 2DL (gpu/src/Kernel.cu:750-819).
//   the global scan of every class (ExpectGlobal2D, gpu/interface/Interface.h:
//     176-197; cuthunder::expectGlobal2D, gpu/src/cuthunder.cu:905): the 2D
//     projections feed the same likelihood / marginal kernels as 3D
//     (thx_global_scan with kIdx / nK).
//   one particle-filter phase (the 2D branch of src/Optimiser.cpp:1183-1402,
//     ExpectLocalPreI2D + ExpectLocalM): per image its own mLR rotations and
//     mLT translations, direct likelihood dvp[r][t] = sum_i sigRcp |d - c T P|^2
//     with the class image staged in LDS, then the per-image marginals.
//   a12 2D: Reconstructor::insertP(const Complex*, ..., const dmat22&, ...)
//     (src/Reconstructor.cpp:708-781) / cuthunder InsertI2D (cuthunder.cu:3265,
//     kernel_InsertF2D / T2D / O2D, Kernel.cu:2276-2500 without
//     OPTIMISER_RECONSTRUCT_SIGMA_REGULARISE): per sample of class nc the
//     re-centred image src ctf w and ctf^2 w scattered bilinearly into
//     F2D[nc] / T2D[nc] at R (iCol pf, iRow pf), O2D[nc] += -R (t - off),
//     counter[nc] += 1.
// 2D half-complex images: [vdim][vdim/2 + 1], i fastest, negative rows wrapped.
#include "common.h"

namespace thx {
int launch_local_weights(const float* dvp, int nR, int nT, const double* pC, const double* pR,
                         const double* pT, float* wC, float* wR, float* wT, float* baseL, int nImg,
                         hipStream_t s, const int* act = nullptr, const int* nAct = nullptr);
int launch_local_weights_d(const float* dvp, int nR, int nT, int nD, const double* pC,
                           const double* pR, const double* pT, const double* pD, float* wC,
                           float* wR, float* wT, float* wD, float* baseL, int nImg, hipStream_t s,
                           const int* act = nullptr, const int* nAct = nullptr);
}

namespace {

// bilinear gather of Image::getByInterpolationFT (fold, floor, 4 taps in box
// order j, i of getFTHalf)
THX_DEV float2 interp2(const float2* __restrict__ img, int vdim, float x, float y)
{
    const bool conj = !(x >= 0.f);
    if (conj) { x = -x; y = -y; }
    const float fx = floorf(x), fy = floorf(y);
    const int x0 = (int)fx, y0 = (int)fy;
    const float dx = x - fx, dy = y - fy;
    const float wx[2] = {1.f - dx, dx}, wy[2] = {1.f - dy, dy};
    const int nc = vdim / 2 + 1;
    float re = 0.f, im = 0.f;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const float2* row = img + (size_t)wrap_idx(y0 + j, vdim) * nc + x0;
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const float w = wx[i] * wy[j];
            re += row[i].x * w;
            im += row[i].y * w;
        }
    }
    return make_float2(re, conj ? -im : im);
}

THX_DEV void rot2(const double* cs, int ic, int ir, int pf, float& x, float& y)
{
    const double nx = (double)(ic * pf), ny = (double)(ir * pf);
    x = (float)(cs[0] * nx - cs[1] * ny);
    y = (float)(cs[1] * nx + cs[0] * ny);
}

__global__ void __launch_bounds__(256) k_project2d(const float2* __restrict__ vol, int vdim, int pf,
                                                   const double* __restrict__ rot, int rotStride,
                                                   const int* __restrict__ iCol,
                                                   const int* __restrict__ iRow, int nPxl,
                                                   float2* __restrict__ rotP)
{
    const int r = blockIdx.y;
    const double cs[2] = {rot[(size_t)rotStride * r], rot[(size_t)rotStride * r + 1]};
    for (int i = blockIdx.x * 256 + threadIdx.x; i < nPxl; i += gridDim.x * 256) {
        float x, y;
        rot2(cs, iCol[i], iRow[i], pf, x, y);
        rotP[(size_t)r * nPxl + i] = interp2(vol, vdim, x, y);
    }
}

// One workgroup per image: the class image in LDS (when it fits), per rotation
// the projection at this thread's pixels and the direct likelihood against
// every column, accumulated per thread and reduced per (r, column).  Columns
// are the translations, or with CTF search (nD > 1) the (t, d) pairs of
// kernel_logDataVSLC (column t nD + d) with the CTF of defocus sample d from
// ctf = ctfD[nImg][nD][nPxl].
constexpr int L2D_THREADS = 256;
constexpr int L2D_TMAX = 16;                // columns per pass
constexpr int L2D_LDS_VOX = 18432;          // 144 KiB of dynamic LDS: a projectee up to vdim 190

__global__ void __launch_bounds__(L2D_THREADS) k_local2d(const float2* __restrict__ vol, int vdim,
                                                         int pf, long volStride,
                                                         const int* __restrict__ cls,
                                                         const double* __restrict__ rot, int rotStride,
                                                         int nR,
                                                         const double* __restrict__ trans, int nT,
                                                         const float2* __restrict__ dat,
                                                         const float* __restrict__ ctf,
                                                         const float* __restrict__ sig,
                                                         const int* __restrict__ iCol,
                                                         const int* __restrict__ iRow, int nPxl,
                                                         int idim, float* __restrict__ dvp,
                                                         const int* __restrict__ done, int nD)
{
    extern __shared__ __attribute__((aligned(16))) float2 sImg[];   // the class image when staged
    __shared__ float sRed[L2D_THREADS / 64][L2D_TMAX];
    __shared__ float sTr[L2D_TMAX][2];
    __shared__ int sCRow[L2D_TMAX];
    const int l = blockIdx.x;
    if (done && done[l]) return;     // stopped by the driver's vari-decrease rule
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const float2* img = vol + (cls ? (size_t)cls[l] * volStride : 0);
    const long nVox = (long)(vdim / 2 + 1) * vdim;
    const bool staged = nVox <= L2D_LDS_VOX;
    if (staged) {
        for (long q = tid; q < nVox; q += L2D_THREADS) sImg[q] = img[q];
        __syncthreads();
    }
    const float2* src = staged ? sImg : img;
    const int nCol = nT * nD;
    const float2* D = dat + (size_t)l * nPxl;
    const float* C = ctf + (size_t)l * nD * nPxl;
    const float* S = sig + (size_t)l * nPxl;
    for (int r = 0; r < nR; r++) {
        const size_t rq = ((size_t)l * nR + r) * rotStride;
        const double cs[2] = {rot[rq], rot[rq + 1]};
        for (int t0 = 0; t0 < nCol; t0 += L2D_TMAX) {
            const int nt = min(L2D_TMAX, nCol - t0);
            if (tid < nt) {
                const int t = (t0 + tid) / nD;
                sTr[tid][0] = (float)trans[((size_t)l * nT + t) * 2] / idim;
                sTr[tid][1] = (float)trans[((size_t)l * nT + t) * 2 + 1] / idim;
                sCRow[tid] = ((t0 + tid) % nD) * nPxl;
            }
            __syncthreads();
            float acc[L2D_TMAX];
#pragma unroll
            for (int t = 0; t < L2D_TMAX; t++) acc[t] = 0.f;
            for (int i = tid; i < nPxl; i += L2D_THREADS) {
                const int ic = iCol[i], ir = iRow[i];
                float x, y;
                rot2(cs, ic, ir, pf, x, y);
                const float2 P = interp2(src, vdim, x, y);
                const float2 d = D[i];
                const float c0 = C[i], s = S[i];
#pragma unroll
                for (int t = 0; t < L2D_TMAX; t++) {
                    if (t < nt) {
                        // priAllP = traP * priRotP, then logDataVSPrior_m_huabin
                        const float c = nD == 1 ? c0 : C[sCRow[t] + i];
                        const float2 Tt = phase_shift(ic, ir, sTr[t][0], sTr[t][1]);
                        const float2 p = cmul(Tt, P);
                        const float er = d.x - c * p.x, ei = d.y - c * p.y;
                        acc[t] += (er * er + ei * ei) * s;
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < L2D_TMAX; t++) {
                const float v = wave_sum(acc[t]);
                if (lane == 0) sRed[wv][t] = v;
            }
            __syncthreads();
            if (tid < nt) {
                float v = 0.f;
                for (int w = 0; w < L2D_THREADS / 64; w++) v += sRed[w][tid];
                dvp[((size_t)l * nR + r) * nCol + t0 + tid] = v;
            }
            __syncthreads();
        }
    }
}

// bilinear scatter of Image::addFT (src/Image/Image.cpp:369-409): fold
// conjugates the complex value, 4 taps, FP32 atomics
THX_DEV void scatter2(float2* __restrict__ F, float* __restrict__ T, int vdim, float x, float y,
                      float vr, float vi, float tv)
{
    if (!(x >= 0.f)) { x = -x; y = -y; vi = -vi; }
    const float fx = floorf(x), fy = floorf(y);
    const int x0 = (int)fx, y0 = (int)fy;
    const float dx = x - fx, dy = y - fy;
    const float wx[2] = {1.f - dx, dx}, wy[2] = {1.f - dy, dy};
    const int nc = vdim / 2 + 1;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const size_t row = (size_t)wrap_idx(y0 + j, vdim) * nc + x0;
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const float w = wx[i] * wy[j];
            float* f = reinterpret_cast<float*>(F + row + i);
            atomicAdd(f, vr * w);
            atomicAdd(f + 1, vi * w);
            atomicAdd(T + row + i, tv * w);
        }
    }
}

__global__ void __launch_bounds__(256) k_insert2d(float2* __restrict__ F, float* __restrict__ T,
                                                  double* __restrict__ O, int* __restrict__ counter,
                                                  int vdim, int pf, const float2* __restrict__ dat,
                                                  const float* __restrict__ ctf,
                                                  const double* __restrict__ rot,
                                                  const double* __restrict__ trans,
                                                  const double* __restrict__ offS,
                                                  const float* __restrict__ w,
                                                  const int* __restrict__ nc, int mReco,
                                                  const int* __restrict__ iCol,
                                                  const int* __restrict__ iRow, int nPxl, int idim,
                                                  const float* __restrict__ attr,
                                                  const double* __restrict__ nD)
{
    const int m = blockIdx.y, l = blockIdx.z;
    const size_t sIdx = (size_t)l * mReco + m;
    const size_t dimSize = (size_t)(vdim / 2 + 1) * vdim;
    const int k = nc ? nc[sIdx] : 0;
    float2* Fk = F + (size_t)k * dimSize;
    float* Tk = T + (size_t)k * dimSize;
    const double cs[2] = {rot[2 * sIdx], rot[2 * sIdx + 1]};
    const double dx = trans[2 * sIdx] - offS[2 * l];
    const double dy = trans[2 * sIdx + 1] - offS[2 * l + 1];
    const float rCol = (float)(-dx) / idim, rRow = (float)(-dy) / idim;
    const float wl = w[l];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // insertDir(-R (t - off)), src/Reconstructor.cpp:397-401
        atomicAdd(O + 2 * k, -(cs[0] * dx - cs[1] * dy));
        atomicAdd(O + 2 * k + 1, -(cs[1] * dx + cs[0] * dy));
        atomicAdd(counter + k, 1);
    }
    const float2* D = dat + (size_t)l * nPxl;
    const float* C = attr ? nullptr : ctf + (size_t)l * nPxl;
    // CTF search (InsertI2D with cSearch): the sample's own CTF at (dU d, dV d)
    // (kernel_CalculateCTF, gpu/src/cuthunder.cu:3753; src/Optimiser.cpp:7101-7120)
    const float* A = attr ? attr + 8 * (size_t)l : nullptr;
    const float dU = A ? (float)(A[2] * nD[sIdx]) : 0.f, dV = A ? (float)(A[3] * nD[sIdx]) : 0.f;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nPxl; i += gridDim.x * blockDim.x) {
        const int ic = iCol[i], ir = iRow[i];
        const float2 src = cmul(D[i], phase_shift(ic, ir, rCol, rRow));
        const float c = A ? ctf_at(A, dU, dV, ic, ir, idim) : C[i];
        const float vr = (src.x * c) * wl, vi = (src.y * c) * wl;
        const float tv = (float)((double)c * c) * wl;
        float x, y;
        rot2(cs, ic, ir, pf, x, y);
        scatter2(Fk, Tk, vdim, x, y, vr, vi, tv);
    }
}

}  // namespace

namespace thx {
// The 2D projection / phase with the rotations at a stride (2: (cos, sin)
// pairs of the adapters; 4: the particle layout _r of Particle, whose columns
// 0, 1 hold (cos, sin) in MODE_2D) -- the launchers of the C-ABI entry points
// below and of the MODE_2D driver (csrc/optimiser.hip).
int project2d_launch(const float* vol, int vdim, int pf, const double* rot, int rotStride, int nR,
                     const int* iCol, const int* iRow, int nPxl, float* rotP, hipStream_t s)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0 && pf > 0 && nR >= 0 && nR <= 65535 && nPxl >= 0 &&
                      rotStride >= 2,
                  "thx_project2d: bad sizes");
    if (nR == 0 || nPxl == 0) return THX_OK;
    THX_CHECK_ARG(vol && rot && iCol && iRow && rotP, "thx_project2d: null argument");
    const unsigned gx = thx::cdiv(nPxl, 256) > 32 ? 32 : thx::cdiv(nPxl, 256);
    hipLaunchKernelGGL(k_project2d, dim3(gx, nR), dim3(256), 0, s,
                       reinterpret_cast<const float2*>(vol), vdim, pf, rot, rotStride, iCol, iRow,
                       nPxl, reinterpret_cast<float2*>(rotP));
    THX_LAUNCH_CHECK();
    return THX_OK;
}

// dvp: nImg x nR x nT (x nD) scratch; done (may be NULL): images to skip.
// nD >= 1 with pD / wD: CTF search, ctf = ctfD[nImg][nD][nPxl].
int local_phase2d_launch(const float* vol, int vdim, int pf, const int* cls, const double* rot,
                         int rotStride, int nR, const double* trans, int nT, const double* pC,
                         const double* pR, const double* pT, const float* dat, const float* ctf,
                         const float* sigRcp, const int* iCol, const int* iRow, int nPxl, int idim,
                         int nImg, float* wC, float* wR, float* wT, float* baseL, float* dvp,
                         const int* done, hipStream_t s, int nD = 0, const double* pD = nullptr,
                         float* wD = nullptr, const int* act = nullptr, const int* nAct = nullptr)
{
    // act / nAct (the driver's active list, with done): the weights of the
    // images still running only, as the 3D phase
    const long nVox = (long)(vdim / 2 + 1) * vdim;
    const size_t lds = nVox <= L2D_LDS_VOX ? (size_t)nVox * sizeof(float2) : 0;
    hipLaunchKernelGGL(k_local2d, dim3(nImg), dim3(L2D_THREADS), lds, s,
                       reinterpret_cast<const float2*>(vol), vdim, pf, nVox, cls, rot, rotStride,
                       nR, trans, nT, reinterpret_cast<const float2*>(dat), ctf, sigRcp, iCol, iRow,
                       nPxl, idim, dvp, done, nD > 0 ? nD : 1);
    THX_LAUNCH_CHECK();
    if (nD > 0)
        return launch_local_weights_d(dvp, nR, nT, nD, pC, pR, pT, pD, wC, wR, wT, wD, baseL, nImg,
                                      s, act, nAct);
    return launch_local_weights(dvp, nR, nT, pC, pR, pT, wC, wR, wT, baseL, nImg, s, act, nAct);
}
}  // namespace thx

extern "C" int thx_project2d(const float* vol, int vdim, int pf, const double* rot, int nR,
                             const int* iCol, const int* iRow, int nPxl, float* rotP,
                             thx_stream_t stream)
{
    return thx::project2d_launch(vol, vdim, pf, rot, 2, nR, iCol, iRow, nPxl, rotP,
                                 thx::as_stream(stream));
}

extern "C" size_t thx_local_phase2d_workspace(int nImg, int nR, int nT)
{
    return (size_t)nImg * nR * nT * sizeof(float) + 256;
}

extern "C" int thx_local_phase2d(const float* vol, int vdim, int pf, const int* cls,
                                 const double* rot, int nR, const double* trans, int nT,
                                 const double* pC, const double* pR, const double* pT,
                                 const float* dat, const float* ctf, const float* sigRcp,
                                 const int* iCol, const int* iRow, int nPxl, int idim, int nImg,
                                 float* wC, float* wR, float* wT, float* baseL, float* dvp,
                                 void* workspace, size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0 && pf > 0 && nR > 0 && nT > 0 && nPxl > 0 &&
                      nImg >= 0 && nImg <= 0x7fffffff,
                  "thx_local_phase2d: bad sizes");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(vol && rot && trans && pC && pR && pT && dat && ctf && sigRcp && iCol && iRow &&
                      wC && wR && wT && baseL,
                  "thx_local_phase2d: null argument");
    float* d = dvp;
    if (!d) {
        THX_CHECK_ARG(workspace && wsBytes >= thx_local_phase2d_workspace(nImg, nR, nT),
                      "thx_local_phase2d: workspace too small");
        d = static_cast<float*>(workspace);
    }
    return thx::local_phase2d_launch(vol, vdim, pf, cls, rot, 2, nR, trans, nT, pC, pR, pT, dat,
                                     ctf, sigRcp, iCol, iRow, nPxl, idim, nImg, wC, wR, wT, baseL,
                                     d, nullptr, thx::as_stream(stream));
}

extern "C" size_t thx_local_phase2d_d_workspace(int nImg, int nR, int nT, int nD)
{
    return (size_t)nImg * nR * nT * (nD > 0 ? nD : 1) * sizeof(float) + 256;
}

// MODE_2D CTF search phase: columns (t, d), ctfD[nImg][nD][nPxl] (thx_ctf_search),
// priors pD / marginal wD [nImg][nD]; dvp (optional) [nImg][nR][nT][nD]
extern "C" int thx_local_phase2d_d(const float* vol, int vdim, int pf, const int* cls,
                                   const double* rot, int nR, const double* trans, int nT, int nD,
                                   const double* pC, const double* pR, const double* pT,
                                   const double* pD, const float* dat, const float* ctfD,
                                   const float* sigRcp, const int* iCol, const int* iRow, int nPxl,
                                   int idim, int nImg, float* wC, float* wR, float* wT, float* wD,
                                   float* baseL, float* dvp, void* workspace, size_t wsBytes,
                                   thx_stream_t stream)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0 && pf > 0 && nR > 0 && nT > 0 && nD > 0 && nPxl > 0 &&
                      nImg >= 0 && (long)nT * nD <= 1024,
                  "thx_local_phase2d_d: bad sizes");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(vol && rot && trans && pC && pR && pT && pD && dat && ctfD && sigRcp && iCol &&
                      iRow && wC && wR && wT && wD && baseL,
                  "thx_local_phase2d_d: null argument");
    float* d = dvp;
    if (!d) {
        THX_CHECK_ARG(workspace && wsBytes >= thx_local_phase2d_d_workspace(nImg, nR, nT, nD),
                      "thx_local_phase2d_d: workspace too small");
        d = static_cast<float*>(workspace);
    }
    return thx::local_phase2d_launch(vol, vdim, pf, cls, rot, 2, nR, trans, nT, pC, pR, pT, dat,
                                     ctfD, sigRcp, iCol, iRow, nPxl, idim, nImg, wC, wR, wT, baseL,
                                     d, nullptr, thx::as_stream(stream), nD, pD, wD);
}

static int insert2d_impl(float* F, float* T, double* O, int* counter, int vdim, int pf,
                         const float* dat, const float* ctf, const float* attr, const double* nD,
                         const double* rot, const double* trans, const double* offS,
                         const float* w, const int* nc, int nImg, int mReco, const int* iCol,
                         const int* iRow, int nPxl, int idim, thx_stream_t stream)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0 && pf > 0 && nImg >= 0 && mReco >= 0 && nPxl >= 0 &&
                      idim > 0 && nImg <= 65535 && mReco <= 65535,
                  "thx_insert2d: bad sizes");
    if (nImg == 0 || mReco == 0 || nPxl == 0) return THX_OK;
    THX_CHECK_ARG(F && T && O && counter && dat && (ctf || (attr && nD)) && rot && trans && offS &&
                      w && iCol && iRow,
                  "thx_insert2d: null argument");
    const unsigned gx = thx::cdiv(nPxl, 256) > 8 ? 8 : thx::cdiv(nPxl, 256);
    hipLaunchKernelGGL(k_insert2d, dim3(gx, mReco, nImg), dim3(256), 0, thx::as_stream(stream),
                       reinterpret_cast<float2*>(F), T, O, counter, vdim, pf,
                       reinterpret_cast<const float2*>(dat), ctf, rot, trans, offS, w, nc, mReco,
                       iCol, iRow, nPxl, idim, attr, nD);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_insert2d(float* F, float* T, double* O, int* counter, int vdim, int pf,
                            const float* dat, const float* ctf, const double* rot,
                            const double* trans, const double* offS, const float* w,
                            const int* nc, int nImg, int mReco, const int* iCol, const int* iRow,
                            int nPxl, int idim, thx_stream_t stream)
{
    THX_CHECK_ARG(ctf || nImg == 0, "thx_insert2d: null ctf");
    return insert2d_impl(F, T, O, counter, vdim, pf, dat, ctf, nullptr, nullptr, rot, trans, offS,
                         w, nc, nImg, mReco, iCol, iRow, nPxl, idim, stream);
}

extern "C" int thx_insert2d_d(float* F, float* T, double* O, int* counter, int vdim, int pf,
                              const float* dat, const float* attr, const double* nD,
                              const double* rot, const double* trans, const double* offS,
                              const float* w, const int* nc, int nImg, int mReco, const int* iCol,
                              const int* iRow, int nPxl, int idim, thx_stream_t stream)
{
    THX_CHECK_ARG((attr && nD) || nImg == 0, "thx_insert2d_d: null attr / nD");
    return insert2d_impl(F, T, O, counter, vdim, pf, dat, nullptr, attr, nD, rot, trans, offS, w,
                         nc, nImg, mReco, iCol, iRow, nPxl, idim, stream);
}
