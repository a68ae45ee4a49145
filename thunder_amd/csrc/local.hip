// local.hip -- a6 + a7 + a9: one particle-filter phase for a batch of images,
// each image with its own rotation / translation samples.
//
// The reference runs this per image with a host round trip per phase
// (ExpectLocalRTD -> ExpectLocalPreI3D -> ExpectLocalM ->
// cudaStreamSynchronize, gpu/src/cuthunder.cu:2675-3140) or, on the CPU, as
// the FOR_EACH_R / FOR_EACH_T loop of src/Optimiser.cpp:1205-1402.  Here one
// launch covers every image of the batch: a workgroup owns (image, block of
// RPB rotations, chunk of TCH translations), each thread a pixel stride.  Per
// pixel the RPB slices are gathered once (trilinear, FP64 coordinates) and
// compared against the TCH translated copies held in registers, so the gather
// bytes (the roofline of this kernel, 64 B per rotation-pixel) are read once.
#include "common.h"

namespace {

constexpr int THREADS = 256;
constexpr int RPB = 4;   // rotations per workgroup

template <int TCH>
__global__ void __launch_bounds__(THREADS) k_local_dvp(const float2* __restrict__ vol,
                                                       int vdim, int pf,
                                                       const double* __restrict__ quat,
                                                       int nR,
                                                       const double* __restrict__ trans,
                                                       int nT,
                                                       const float2* __restrict__ dat,
                                                       const float* __restrict__ ctf,
                                                       const float* __restrict__ sig,
                                                       const int* __restrict__ iCol,
                                                       const int* __restrict__ iRow,
                                                       int nPxl, int idim,
                                                       float* __restrict__ dvp)
{
    const int rb = blockIdx.x, l = blockIdx.y, t0 = blockIdx.z * TCH;
    __shared__ double sMat[RPB][6];
    __shared__ float sTr[TCH][2];
    __shared__ float sRed[THREADS / 64][RPB * TCH];
    if (threadIdx.x < RPB) {
        const int r = rb * RPB + threadIdx.x;
        double q[4] = {1, 0, 0, 0};
        if (r < nR)
            for (int k = 0; k < 4; k++) q[k] = quat[((size_t)l * nR + r) * 4 + k];
        double m[9];
        quat_to_mat(q, m);
        for (int k = 0; k < 6; k++) sMat[threadIdx.x][k] = m[k];
    }
    if (threadIdx.x < TCH) {
        const int t = t0 + threadIdx.x;
        float tx = 0.f, ty = 0.f;
        if (t < nT) {
            tx = (float)trans[((size_t)l * nT + t) * 2];
            ty = (float)trans[((size_t)l * nT + t) * 2 + 1];
        }
        sTr[threadIdx.x][0] = tx / idim;   // rCol, ImageFunctions.cpp:243
        sTr[threadIdx.x][1] = ty / idim;
    }
    __syncthreads();

    float acc[RPB][TCH];
#pragma unroll
    for (int a = 0; a < RPB; a++)
#pragma unroll
        for (int b = 0; b < TCH; b++) acc[a][b] = 0.f;

    const float2* D = dat + (size_t)l * nPxl;
    const float* C = ctf + (size_t)l * nPxl;
    const float* S = sig + (size_t)l * nPxl;
    for (int i = threadIdx.x; i < nPxl; i += THREADS) {
        const int ic = iCol[i], ir = iRow[i];
        const float2 d = D[i];
        const float c = C[i], s = S[i];
        float2 T[TCH];
#pragma unroll
        for (int b = 0; b < TCH; b++) T[b] = phase_shift(ic, ir, sTr[b][0], sTr[b][1]);
#pragma unroll
        for (int a = 0; a < RPB; a++) {
            const double m[6] = {sMat[a][0], sMat[a][1], sMat[a][2],
                                 sMat[a][3], sMat[a][4], sMat[a][5]};
            float x, y, z;
            rot_coord(m, ic, ir, pf, x, y, z);
            const float2 P = interp_ft(vol, vdim, x, y, z);
#pragma unroll
            for (int b = 0; b < TCH; b++) {
                const float2 pri = cmul(T[b], P);
                const float er = d.x - c * pri.x;
                const float ei = d.y - c * pri.y;
                acc[a][b] += (er * er + ei * ei) * s;
            }
        }
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < RPB; a++)
#pragma unroll
        for (int b = 0; b < TCH; b++) {
            const float v = wave_sum(acc[a][b]);
            if (lane == 0) sRed[wv][a * TCH + b] = v;
        }
    __syncthreads();
    if (threadIdx.x < RPB * TCH) {
        const int a = threadIdx.x / TCH, b = threadIdx.x % TCH;
        const int r = rb * RPB + a, t = t0 + b;
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < THREADS / 64; k++) v += sRed[k][threadIdx.x];
        if (r < nR && t < nT) dvp[((size_t)l * nR + r) * nT + t] = v;
    }
}

// Per-image normalisation of src/Optimiser.cpp:1383-1402 (nC = nD = 1,
// wD = 1) evaluated at the final baseline: s = exp(dvp - max),
// wC += s pR pT, wR[r] += s pC pT, wT[t] += s pC pR.
__global__ void __launch_bounds__(256) k_local_weights(const float* __restrict__ dvp,
                                                       int nR, int nT,
                                                       const double* __restrict__ pC,
                                                       const double* __restrict__ pR,
                                                       const double* __restrict__ pT,
                                                       float* __restrict__ wC,
                                                       float* __restrict__ wR,
                                                       float* __restrict__ wT,
                                                       float* __restrict__ baseL)
{
    const int l = blockIdx.x;
    const float* Dl = dvp + (size_t)l * nR * nT;
    const double* pRl = pR + (size_t)l * nR;
    const double* pTl = pT + (size_t)l * nT;
    const double c = pC[l];
    __shared__ float sm[4];
    __shared__ double sd[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float m = -INFINITY;
    for (int q = threadIdx.x; q < nR * nT; q += blockDim.x) m = fmaxf(m, Dl[q]);
    m = wave_max(m);
    if (lane == 0) sm[wv] = m;
    __syncthreads();
    const float base = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    double cacc = 0.0;
    for (int r = threadIdx.x; r < nR; r += blockDim.x) {
        double a = 0.0;
        for (int t = 0; t < nT; t++) a += (double)expf(Dl[r * nT + t] - base) * pTl[t];
        wR[(size_t)l * nR + r] = (float)(a * c);
        cacc += a * pRl[r];
    }
    for (int t = threadIdx.x; t < nT; t += blockDim.x) {
        double a = 0.0;
        for (int r = 0; r < nR; r++) a += (double)expf(Dl[r * nT + t] - base) * pRl[r];
        wT[(size_t)l * nT + t] = (float)(a * c);
    }
    cacc = wave_sum(cacc);
    if (lane == 0) sd[wv] = cacc;
    __syncthreads();
    if (threadIdx.x == 0) {
        wC[l] = (float)(sd[0] + sd[1] + sd[2] + sd[3]);
        baseL[l] = base;
    }
}

template <int TCH>
int launch_dvp(const float* vol, int vdim, int pf, const double* quat, int nR,
               const double* trans, int nT, const float* dat, const float* ctf,
               const float* sig, const int* iCol, const int* iRow, int nPxl,
               int idim, int nImg, float* dvp, hipStream_t s)
{
    dim3 grid(thx::cdiv(nR, RPB), nImg, thx::cdiv(nT, TCH));
    hipLaunchKernelGGL(k_local_dvp<TCH>, grid, dim3(THREADS), 0, s,
                       reinterpret_cast<const float2*>(vol), vdim, pf, quat, nR,
                       trans, nT, reinterpret_cast<const float2*>(dat), ctf, sig,
                       iCol, iRow, nPxl, idim, dvp);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

}  // namespace

extern "C" size_t thx_local_phase_workspace(int nImg, int nR, int nT)
{
    return (size_t)nImg * nR * nT * sizeof(float) + 256;
}

extern "C" int thx_local_phase(const float* vol, int vdim, int pf,
                               const double* quat, int nR, const double* trans,
                               int nT, const double* pC, const double* pR,
                               const double* pT, const float* dat,
                               const float* ctf, const float* sigRcp,
                               const int* iCol, const int* iRow, int nPxl,
                               int idim, int nImg, float* wC, float* wR,
                               float* wT, float* baseL, float* dvp,
                               void* workspace, size_t wsBytes,
                               thx_stream_t stream)
{
    THX_CHECK_ARG(nR > 0 && nT > 0 && nPxl > 0 && nImg >= 0 && vdim > 0 && pf > 0,
                  "thx_local_phase: bad sizes");
    THX_CHECK_ARG(nImg <= 65535, "thx_local_phase: nImg > 65535 per call");
    if (nImg == 0) return THX_OK;
    float* d = dvp;
    if (!d) {
        THX_CHECK_ARG(workspace && wsBytes >= thx_local_phase_workspace(nImg, nR, nT),
                      "thx_local_phase: workspace too small");
        d = static_cast<float*>(workspace);
    }
    hipStream_t s = thx::as_stream(stream);
    int st = nT <= 9 ? launch_dvp<9>(vol, vdim, pf, quat, nR, trans, nT, dat, ctf,
                                     sigRcp, iCol, iRow, nPxl, idim, nImg, d, s)
                     : launch_dvp<16>(vol, vdim, pf, quat, nR, trans, nT, dat, ctf,
                                      sigRcp, iCol, iRow, nPxl, idim, nImg, d, s);
    if (st != THX_OK) return st;
    hipLaunchKernelGGL(k_local_weights, dim3(nImg), dim3(256), 0, s, d, nR, nT,
                       pC, pR, pT, wC, wR, wT, baseL);
    THX_LAUNCH_CHECK();
    return THX_OK;
}
