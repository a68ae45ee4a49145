// geom.hip -- pixel set (a1), CTF (a2), translation table (a4), quaternion ->
// rotation (a5), and the error / version plumbing of the C-ABI.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <vector>

#include "common.h"

namespace thx {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

}  // namespace thx

extern "C" int thx_abi_version(void) { return THX_ABI_VERSION; }
extern "C" const char* thx_last_error(void) { return thx::g_err; }

// ---------------------------------------------------------------------- a1
extern "C" int thx_pixel_set(int idim, int pf, float rU, float rL, int cap,
                             int* iCol, int* iRow, int* iSig, int* iPxl,
                             int* nPxl)
{
    THX_CHECK_ARG(idim > 0 && pf > 0 && nPxl, "thx_pixel_set: bad idim/pf/nPxl");
    THX_CHECK_ARG(rU <= idim / 2 - 1,
                  "thx_pixel_set: rU=%g exceeds idim/2-1 (trilinear taps would leave the volume)",
                  (double)rU);
    // Optimiser::allocPreCalIdx, src/Optimiser.cpp:8008-8040.
    const float rU2 = (float)((double)rU * rU);
    const float rL2 = (float)((double)rL * rL);
    const float r = rU + 1;
    const long nColFT = idim / 2 + 1;
    int n = 0;
    for (long j = (long)(-r); j < r; j++)
        for (long i = 0; i <= r; i++) {
            if (i == 0 && j < 0) continue;
            const float u = (float)((double)i * i + (double)j * j);
            if (u < rU2 && u >= rL2) {
                const int v = (int)std::rint(std::hypot((double)i, (double)j));
                if (v < rU && v >= rL) {
                    if (n >= cap) {
                        thx::set_error("thx_pixel_set: cap=%d too small", cap);
                        return THX_ERR_ARG;
                    }
                    if (iCol) iCol[n] = (int)i;
                    if (iRow) iRow[n] = (int)j;
                    if (iSig) iSig[n] = v;
                    if (iPxl) iPxl[n] = (int)((j >= 0 ? j : j + idim) * nColFT + i);
                    n++;
                }
            }
        }
    *nPxl = n;
    return THX_OK;
}

extern "C" int thx_pixel_tile_order(const int* iCol, const int* iRow, int nPxl, int cap,
                                    int* order, int* nOrd)
{
    constexpr int TILE = 4, GROUP = TILE * TILE;
    THX_CHECK_ARG(iCol && iRow && nOrd && nPxl >= 0 && cap >= 0,
                  "thx_pixel_tile_order: bad arguments");
    *nOrd = 0;
    if (nPxl == 0) return THX_OK;
    int cMin = iCol[0], rMin = iRow[0], cMax = iCol[0];
    for (int i = 1; i < nPxl; i++) {
        cMin = std::min(cMin, iCol[i]);
        cMax = std::max(cMax, iCol[i]);
        rMin = std::min(rMin, iRow[i]);
    }
    const long nTc = (cMax - cMin) / TILE + 1;
    std::vector<long> key(nPxl);
    for (int i = 0; i < nPxl; i++) {
        const long tr = (iRow[i] - rMin) / TILE, tc0 = (iCol[i] - cMin) / TILE;
        const long tc = (tr & 1) ? nTc - 1 - tc0 : tc0;   // serpentine square rows
        key[i] = tr * nTc + tc;
    }
    // inside a square: its 2x2 quads in turn, so that every 4 consecutive
    // entries (one step of the local phase's lanes) are a compact quad
    std::vector<int> sub(nPxl, 0);
    for (int i = 0; i < nPxl; i++) {
        const int lc = (iCol[i] - cMin) % TILE, lr = (iRow[i] - rMin) % TILE;
        sub[i] = ((lr / 2) * 2 + lc / 2) * 4 + (lr % 2) * 2 + lc % 2;
    }
    std::vector<int> idx(nPxl);
    for (int i = 0; i < nPxl; i++) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) {
        return key[a] != key[b] ? key[a] < key[b] : sub[a] < sub[b];
    });
    // groups of <= 16: whole squares, consecutive partial squares merged
    std::vector<int> out;
    out.reserve(nPxl + GROUP);
    int fill = 0;
    for (int a = 0; a < nPxl;) {
        int b = a;
        while (b < nPxl && key[idx[b]] == key[idx[a]]) b++;
        if (fill + (b - a) > GROUP) {
            out.insert(out.end(), GROUP - fill, -1);
            fill = 0;
        }
        out.insert(out.end(), idx.begin() + a, idx.begin() + b);
        fill += b - a;
        a = b;
    }
    if (fill) out.insert(out.end(), GROUP - fill, -1);
    *nOrd = (int)out.size();
    if (order) {
        THX_CHECK_ARG((int)out.size() <= cap, "thx_pixel_tile_order: cap=%d < %d", cap,
                      (int)out.size());
        std::copy(out.begin(), out.end(), order);
    }
    return THX_OK;
}

// ---------------------------------------------------------------------- a2
// One workgroup column per image, pixels across threads.  CTF(RFLOAT*, ...),
// src/CTF.cpp:113-151 (ctf_at, common.h).
__global__ void __launch_bounds__(256) k_ctf(const float* __restrict__ attr,
                                             const int* __restrict__ iCol,
                                             const int* __restrict__ iRow,
                                             int nPxl, int idim,
                                             float* __restrict__ ctfP)
{
    const int l = blockIdx.y;
    const float* a = attr + 8 * l;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nPxl;
         i += gridDim.x * blockDim.x)
        ctfP[(size_t)l * nPxl + i] = ctf_at(a, a[2], a[3], iCol[i], iRow[i], idim);
}

extern "C" int thx_ctf(const float* attr, int nImg, const int* iCol,
                       const int* iRow, int nPxl, int idim, float* ctfP,
                       thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && nPxl >= 0 && idim > 0, "thx_ctf: bad sizes");
    if (nImg == 0 || nPxl == 0) return THX_OK;
    THX_CHECK_ARG(nImg <= 65535 * 64, "thx_ctf: nImg too large");
    dim3 grid(thx::cdiv(nPxl, 256) > 64 ? 64 : thx::cdiv(nPxl, 256), nImg);
    hipLaunchKernelGGL(k_ctf, grid, dim3(256), 0, thx::as_stream(stream), attr,
                       iCol, iRow, nPxl, idim, ctfP);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

// CTF search precalculation, the cSearch branch of allocPreCal
// (src/Optimiser.cpp:8124-8170): frequency (shared), per-pixel defocus, K1,
// K2 per image (the wavelength constant 12.2643274 of that branch, quirk q5).
__global__ void __launch_bounds__(256) k_defocus_pre(const float* __restrict__ attr,
                                                     const int* __restrict__ iCol,
                                                     const int* __restrict__ iRow, int nPxl,
                                                     int idim, float* __restrict__ freq,
                                                     float* __restrict__ defocusP,
                                                     float* __restrict__ K1,
                                                     float* __restrict__ K2)
{
    const int l = blockIdx.y;
    const float* a = attr + 8 * l;
    const float pixelSize = a[0], voltage = a[1], dU = a[2], dV = a[3], theta = a[4];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nPxl; i += gridDim.x * blockDim.x) {
        const int ic = iCol[i], ir = iRow[i];
        if (l == 0 && freq)
            freq[i] = (float)(sqrt((double)ic * ic + (double)ir * ir) / idim / pixelSize);
        const float angle = (float)(atan2((double)ir, (double)ic) - theta);
        defocusP[(size_t)l * nPxl + i] = -(dU + dV + (dU - dV) * cosf(2.f * angle)) / 2.f;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const float lambda =
            (float)(12.2643274 / sqrt((double)voltage * (1 + (double)voltage * 0.978466e-6)));
        K1[l] = (float)(M_PI * lambda);
        K2[l] = (float)(M_PI_2 * a[5] * ((double)lambda * lambda * lambda));
    }
}

// kernel_CalCTFL (gpu/src/Kernel.cu:481-515) / src/Optimiser.cpp:1252-1271:
// ctfD[l][d][i] for the image's defocus factors dD[l][d]; one workgroup
// column per (image, defocus sample).
__global__ void __launch_bounds__(256) k_ctf_search(const float* __restrict__ defocusP,
                                                    const float* __restrict__ freq,
                                                    const double* __restrict__ dD, int nD,
                                                    const float* __restrict__ K1,
                                                    const float* __restrict__ K2,
                                                    const float* __restrict__ attr, int nPxl,
                                                    float* __restrict__ ctfD)
{
    const int l = blockIdx.y / nD, iD = blockIdx.y % nD;
    const float conT = attr[8 * l + 6], ps = attr[8 * l + 7];
    const float k1 = K1[l], k2 = K2[l];
    const double d = dD[(size_t)l * nD + iD];
    const float* dfo = defocusP + (size_t)l * nPxl;
    float* out = ctfD + ((size_t)l * nD + iD) * nPxl;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nPxl; i += gridDim.x * blockDim.x)
        out[i] = ctf_search_at(k1, dfo[i], d, freq[i], k2, ps, conT);
}

extern "C" int thx_defocus_pre(const float* attr, int nImg, const int* iCol, const int* iRow,
                               int nPxl, int idim, float* freq, float* defocusP, float* K1,
                               float* K2, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && nPxl >= 0 && idim > 0, "thx_defocus_pre: bad sizes");
    if (nImg == 0 || nPxl == 0) return THX_OK;
    THX_CHECK_ARG(nImg <= 65535 * 64, "thx_defocus_pre: nImg too large");
    THX_CHECK_ARG(attr && iCol && iRow && defocusP && K1 && K2, "thx_defocus_pre: null pointer");
    dim3 grid(thx::cdiv(nPxl, 256) > 64 ? 64 : thx::cdiv(nPxl, 256), nImg);
    hipLaunchKernelGGL(k_defocus_pre, grid, dim3(256), 0, thx::as_stream(stream), attr, iCol,
                       iRow, nPxl, idim, freq, defocusP, K1, K2);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_ctf_search(const float* defocusP, const float* freq, const double* dD,
                              int nD, const float* K1, const float* K2, const float* attr,
                              int nImg, int nPxl, float* ctfD, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && nPxl >= 0 && nD > 0, "thx_ctf_search: bad sizes");
    if (nImg == 0 || nPxl == 0) return THX_OK;
    THX_CHECK_ARG((long)nImg * nD <= 65535L * 64, "thx_ctf_search: nImg * nD too large");
    THX_CHECK_ARG(defocusP && freq && dD && K1 && K2 && attr && ctfD,
                  "thx_ctf_search: null pointer");
    dim3 grid(thx::cdiv(nPxl, 256) > 16 ? 16 : thx::cdiv(nPxl, 256), nImg * nD);
    hipLaunchKernelGGL(k_ctf_search, grid, dim3(256), 0, thx::as_stream(stream), defocusP, freq,
                       dD, nD, K1, K2, attr, nPxl, ctfD);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

// ---------------------------------------------------------------------- a4
__global__ void __launch_bounds__(256) k_trans_table(const double* __restrict__ trans,
                                                     const int* __restrict__ iCol,
                                                     const int* __restrict__ iRow,
                                                     int nPxl, int idim,
                                                     float2* __restrict__ traP)
{
    const int t = blockIdx.y;
    // translate(): rCol = nTransCol / nCol in RFLOAT (ImageFunctions.cpp:243-244)
    const float rCol = (float)trans[2 * t] / idim;
    const float rRow = (float)trans[2 * t + 1] / idim;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nPxl;
         i += gridDim.x * blockDim.x)
        traP[(size_t)t * nPxl + i] = phase_shift(iCol[i], iRow[i], rCol, rRow);
}

extern "C" int thx_trans_table(const double* trans, int nT, const int* iCol,
                               const int* iRow, int nPxl, int idim,
                               float* traP, thx_stream_t stream)
{
    THX_CHECK_ARG(nT >= 0 && nPxl >= 0 && idim > 0 && nT <= 65535,
                  "thx_trans_table: bad sizes");
    if (nT == 0 || nPxl == 0) return THX_OK;
    dim3 grid(thx::cdiv(nPxl, 256) > 64 ? 64 : thx::cdiv(nPxl, 256), nT);
    hipLaunchKernelGGL(k_trans_table, grid, dim3(256), 0,
                       thx::as_stream(stream), trans, iCol, iRow, nPxl, idim,
                       reinterpret_cast<float2*>(traP));
    THX_LAUNCH_CHECK();
    return THX_OK;
}

// ---------------------------------------------------------------------- a5
__global__ void __launch_bounds__(256) k_rotmat(const double* __restrict__ quat,
                                                int n, double* __restrict__ mat)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    double q[4] = {quat[4 * r], quat[4 * r + 1], quat[4 * r + 2], quat[4 * r + 3]};
    double m[9];
    quat_to_mat(q, m);
#pragma unroll
    for (int k = 0; k < 9; k++) mat[9 * (size_t)r + k] = m[k];
}

extern "C" int thx_rotmat(const double* quat, int n, double* mat,
                          thx_stream_t stream)
{
    THX_CHECK_ARG(n >= 0, "thx_rotmat: bad n");
    if (n == 0) return THX_OK;
    hipLaunchKernelGGL(k_rotmat, dim3(thx::cdiv(n, 256)), dim3(256), 0,
                       thx::as_stream(stream), quat, n, mat);
    THX_LAUNCH_CHECK();
    return THX_OK;
}
