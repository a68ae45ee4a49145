// scan.hip -- a7 + a8: global-search likelihoods and marginal weights.
//
// algo 0 (this file): direct per-pixel formulation of kernel_logDataVS
// (gpu/src/Kernel.cu:947-1004), dvp materialised in the workspace, then one
// normalisation pass per image.  Kept as the arithmetic twin of the reference
// and as the cross-check for the fused MFMA path (algo 1, scan_mfma.hip).
#include "common.h"
#include "scan_common.h"

// --------------------------------------------------------------- a7 direct
// Block = (rotation r, image l, translation chunk of TCH).  Lanes stride the
// pixels; each lane keeps TCH partial sums; wave + LDS reduction at the end.
template <int TCH>
__global__ void __launch_bounds__(256) k_dvp_direct(const float2* __restrict__ rotP,
                                                    int nR,
                                                    const float2* __restrict__ traP,
                                                    int nT,
                                                    const float2* __restrict__ dat,
                                                    const float* __restrict__ ctf,
                                                    const float* __restrict__ sig,
                                                    int nPxl,
                                                    float* __restrict__ dvp)
{
    const int r = blockIdx.x, l = blockIdx.y, t0 = blockIdx.z * TCH;
    float acc[TCH];
#pragma unroll
    for (int k = 0; k < TCH; k++) acc[k] = 0.f;
    const float2* P = rotP + (size_t)r * nPxl;
    const float2* D = dat + (size_t)l * nPxl;
    const float* C = ctf + (size_t)l * nPxl;
    const float* S = sig + (size_t)l * nPxl;
    for (int i = threadIdx.x; i < nPxl; i += blockDim.x) {
        const float2 p = P[i], d = D[i];
        const float c = C[i], s = S[i];
#pragma unroll
        for (int k = 0; k < TCH; k++) {
            const int t = t0 + k;
            if (t < nT) {
                const float2 pri = cmul(traP[(size_t)t * nPxl + i], p);
                const float er = d.x - c * pri.x;
                const float ei = d.y - c * pri.y;
                acc[k] += (er * er + ei * ei) * s;
            }
        }
    }
    __shared__ float red[4][TCH];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < TCH; k++) {
        const float v = wave_sum(acc[k]);
        if (lane == 0) red[wv][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < TCH) {
        const int t = t0 + threadIdx.x;
        if (t < nT)
            dvp[((size_t)l * nR + r) * nT + t] =
                red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                red[3][threadIdx.x];
    }
}

extern "C" int thx_dvp(const float* rotP, int nR, const float* traP, int nT,
                       const float* dat, const float* ctf, const float* sigRcp,
                       int nImg, int nPxl, float* dvp, thx_stream_t stream)
{
    THX_CHECK_ARG(nR >= 0 && nT >= 0 && nImg >= 0 && nPxl >= 0,
                  "thx_dvp: bad sizes");
    THX_CHECK_ARG(nImg <= 65535 && nR <= 0x7fffffff,
                  "thx_dvp: nImg > 65535 per call");
    if (nR == 0 || nT == 0 || nImg == 0) return THX_OK;
    constexpr int TCH = 16;
    dim3 grid(nR, nImg, thx::cdiv(nT, TCH));
    hipLaunchKernelGGL(k_dvp_direct<TCH>, grid, dim3(256), 0,
                       thx::as_stream(stream),
                       reinterpret_cast<const float2*>(rotP), nR,
                       reinterpret_cast<const float2*>(traP), nT,
                       reinterpret_cast<const float2*>(dat), ctf, sigRcp, nPxl,
                       dvp);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

// ------------------------------------------------------------ a8 weights
// One block per image over a materialised dvp[l][nR][nT].  Equivalent to the
// CPU online-baseline loop (src/Optimiser.cpp:834-894) evaluated with its
// final baseline; sums in FP64, stored as RFLOAT like the reference's host
// matrices.
__global__ void __launch_bounds__(256) k_weights_global(const float* __restrict__ dvp,
                                                        int nR, int nT,
                                                        const double* __restrict__ pR,
                                                        const double* __restrict__ pT,
                                                        int kIdx, int nK,
                                                        float* __restrict__ wC,
                                                        float* __restrict__ wR,
                                                        float* __restrict__ wT,
                                                        float* __restrict__ baseL)
{
    const int l = blockIdx.x;
    const float* D = dvp + (size_t)l * nR * nT;
    const long n = (long)nR * nT;
    __shared__ float smax[4];
    __shared__ double ssum[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float m = -INFINITY;
    for (long q = threadIdx.x; q < n; q += blockDim.x) m = fmaxf(m, D[q]);
    m = wave_max(m);
    if (lane == 0) smax[wv] = m;
    __syncthreads();
    m = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
    const float base = merge_baseline(l, m, kIdx, nK, nR, nT, wC, wR, wT, baseL);
    // wR[r] = sum_t w pT[t]; wC = sum_r pR[r] wR[r]
    double cacc = 0.0;
    float* wRl = wR + ((size_t)l * nK + kIdx) * nR;
    float* wTl = wT + ((size_t)l * nK + kIdx) * nT;
    for (int r = threadIdx.x; r < nR; r += blockDim.x) {
        double a = 0.0;
        for (int t = 0; t < nT; t++) a += (double)expf(D[(size_t)r * nT + t] - base) * pT[t];
        wRl[r] = (float)a;
        cacc += a * pR[r];
    }
    for (int t = threadIdx.x; t < nT; t += blockDim.x) {
        double a = 0.0;
        for (int r = 0; r < nR; r++) a += (double)expf(D[(size_t)r * nT + t] - base) * pR[r];
        wTl[t] = (float)a;
    }
    cacc = wave_sum(cacc);
    if (lane == 0) ssum[wv] = cacc;
    __syncthreads();
    if (threadIdx.x == 0)
        wC[(size_t)l * nK + kIdx] = (float)(ssum[0] + ssum[1] + ssum[2] + ssum[3]);
}

namespace thx {
int scan_mfma(const float* rotP, int nR, const float* traP, int nT,
              const float* dat, const float* ctf, const float* sigRcp,
              int nImg, int nPxl, const double* pR, const double* pT, int kIdx,
              int nK, float* wC, float* wR, float* wT, float* baseL,
              void* workspace, size_t wsBytes, hipStream_t stream);
size_t scan_mfma_workspace(int nImg, int nR, int nT, int nPxl);
int scan_split_algo(int algo, const float* rotP, int nR, const float* traP, int nT,
                    const float* dat, const float* ctf, const float* sigRcp, int nImg, int nPxl,
                    const double* pR, const double* pT, int kIdx, int nK, float* wC, float* wR,
                    float* wT, float* baseL, float guard, float* dvpOut, void* workspace,
                    size_t wsBytes, hipStream_t s);
size_t scan_split_workspace(int nImg, int nR, int nT, int nPxl);
float scan_guard_default();
}  // namespace thx

extern "C" size_t thx_global_scan_workspace(int nImg, int nR, int nT, int nPxl,
                                            int algo)
{
    if (algo == 1) return thx::scan_mfma_workspace(nImg, nR, nT, nPxl);
    if (algo == 2 || algo == 4) return thx::scan_split_workspace(nImg, nR, nT, nPxl);
    thx::Carver c(nullptr, 0);
    c.take<float>((size_t)nImg * nR * nT);
    return c.off + 256;
}

#define SCAN_ARGS_CHECK()                                                                    \
    THX_CHECK_ARG(nR > 0 && nT > 0 && nImg >= 0 && nPxl > 0,                                 \
                  "thx_global_scan: bad sizes nR=%d nT=%d nImg=%d nPxl=%d", nR, nT, nImg,    \
                  nPxl);                                                                     \
    THX_CHECK_ARG(nK >= 1 && kIdx >= 0 && kIdx < nK, "thx_global_scan: bad kIdx=%d nK=%d",  \
                  kIdx, nK)

extern "C" int thx_global_scan(const float* rotP, int nR, const float* traP,
                               int nT, const float* dat, const float* ctf,
                               const float* sigRcp, int nImg, int nPxl,
                               const double* pR, const double* pT, int kIdx,
                               int nK, float* wC, float* wR, float* wT,
                               float* baseL, int algo, void* workspace,
                               size_t wsBytes, thx_stream_t stream)
{
    SCAN_ARGS_CHECK();
    THX_CHECK_ARG(algo >= 0 && algo <= 4 && algo != 3,
                  "thx_global_scan: algo must be 0, 1, 2 or 4 (3, fp16x2, was retired in ABI 9)");
    THX_CHECK_ARG(wsBytes >= thx_global_scan_workspace(nImg, nR, nT, nPxl, algo),
                  "thx_global_scan: workspace too small");
    if (nImg == 0) return THX_OK;
    hipStream_t s = thx::as_stream(stream);
    if (algo == 1)
        return thx::scan_mfma(rotP, nR, traP, nT, dat, ctf, sigRcp, nImg, nPxl,
                              pR, pT, kIdx, nK, wC, wR, wT, baseL, workspace,
                              wsBytes, s);
    if (algo >= 2)
        return thx::scan_split_algo(algo, rotP, nR, traP, nT, dat, ctf, sigRcp, nImg, nPxl, pR,
                                    pT, kIdx, nK, wC, wR, wT, baseL, thx::scan_guard_default(),
                                    nullptr, workspace, wsBytes, s);
    thx::Carver c(workspace, wsBytes);
    float* dvp = c.take<float>((size_t)nImg * nR * nT);
    for (int l0 = 0; l0 < nImg; l0 += 65535) {
        const int nb = nImg - l0 < 65535 ? nImg - l0 : 65535;
        int st = thx_dvp(rotP, nR, traP, nT, dat + 2 * (size_t)l0 * nPxl,
                         ctf + (size_t)l0 * nPxl, sigRcp + (size_t)l0 * nPxl,
                         nb, nPxl, dvp + (size_t)l0 * nR * nT, stream);
        if (st != THX_OK) return st;
    }
    hipLaunchKernelGGL(k_weights_global, dim3(nImg), dim3(256), 0, s, dvp, nR,
                       nT, pR, pT, kIdx, nK, wC, wR, wT, baseL);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_global_scan_dvp(const float* rotP, int nR, const float* traP, int nT,
                                   const float* dat, const float* ctf, const float* sigRcp,
                                   int nImg, int nPxl, const double* pR, const double* pT,
                                   int kIdx, int nK, float* wC, float* wR, float* wT,
                                   float* baseL, int algo, float guard, float* dvp,
                                   void* workspace, size_t wsBytes, thx_stream_t stream)
{
    SCAN_ARGS_CHECK();
    THX_CHECK_ARG(algo == 2 || algo == 4, "thx_global_scan_dvp: algo must be 2 or 4");
    THX_CHECK_ARG(guard >= 0.f, "thx_global_scan_dvp: guard must be >= 0");
    THX_CHECK_ARG(wsBytes >= thx_global_scan_workspace(nImg, nR, nT, nPxl, algo),
                  "thx_global_scan_dvp: workspace too small");
    if (nImg == 0) return THX_OK;
    return thx::scan_split_algo(algo, rotP, nR, traP, nT, dat, ctf, sigRcp, nImg, nPxl, pR, pT,
                                kIdx, nK, wC, wR, wT, baseL, guard, dvp, workspace, wsBytes,
                                thx::as_stream(stream));
}
