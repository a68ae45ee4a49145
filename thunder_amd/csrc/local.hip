// local.hip -- a6 + a7 + a9: one particle-filter phase for a batch of images,
// each image with its own rotation / translation samples.
//
// The reference runs this per image with a host round trip per phase
// (ExpectLocalRTD -> ExpectLocalPreI3D -> ExpectLocalM ->
// cudaStreamSynchronize, gpu/src/cuthunder.cu:2675-3140) or, on the CPU, as
// the FOR_EACH_R / FOR_EACH_T loop of src/Optimiser.cpp:1205-1402.  Here one
// launch covers the whole batch, one workgroup per (image, 128 rotations).
//
// Per pixel i and translation t the likelihood term expands, with |T| = 1, to
//   s|d - c T P|^2 = s|d|^2 + P.re U_t + P.im V_t + b |P|^2
//   U_t = Re(Y) T.re + Im(Y) T.im,  V_t = Im(Y) T.re - Re(Y) T.im,
//   Y = -2 s c d,  b = s c^2,
// so dvp[r][t] - A_l = sum_i [P.re, P.im, |P|^2, 0]_ri . [U, V, b, 0]_it is a
// K = 4 nPxl product of a (rotation x 4 nPxl) projection tile and a
// (4 nPxl x translation) image tile.  The workgroup gathers the projection
// tile (the HBM-bound part: 8 taps per rotation-pixel), stages it in LDS and
// reduces it against the translation tile on v_mfma_f32_16x16x4_f32, so no
// cross-lane reduction and no per-(r,t) VALU loop is left.
#include "common.h"

namespace {

constexpr int THREADS = 256;
constexpr int RT = 128;          // rotations per workgroup (8 MFMA M-tiles)
constexpr int TT = 16;           // translations per workgroup (1 MFMA N-tile)
constexpr int KC = 32;           // pixels per LDS stage
constexpr int APITCH = KC + 1;   // LDS row pitch (float2) of the [rotation][pixel] tile

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Cell-expanded projectee (thx_volume_cells): the 8 taps of the trilinear
// cell with base (x0, y0, z0) are 64 contiguous bytes, so one gather is one
// aligned 64-B segment instead of four 16-B pieces on four rows.
THX_DEV float2 interp_cells(const float4* __restrict__ cells, int vdim, float x,
                            float y, float z)
{
    const bool conj = !(x >= 0.f);
    if (conj) { x = -x; y = -y; z = -z; }
    const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
    const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
    const float dx = x - fx, dy = y - fy, dz = z - fz;
    const int nColFT = vdim / 2 + 1;
    const size_t c = (((size_t)wrap_idx(z0, vdim) * vdim + wrap_idx(y0, vdim)) * nColFT + x0) * 4;
    const float4 q0 = cells[c], q1 = cells[c + 1], q2 = cells[c + 2], q3 = cells[c + 3];
    const float ax = 1.f - dx, ay = 1.f - dy, az = 1.f - dz;
    float w, re = 0.f, im = 0.f;
    w = ax * ay * az; re += q0.x * w; im += q0.y * w;
    w = dx * ay * az; re += q0.z * w; im += q0.w * w;
    w = ax * dy * az; re += q1.x * w; im += q1.y * w;
    w = dx * dy * az; re += q1.z * w; im += q1.w * w;
    w = ax * ay * dz; re += q2.x * w; im += q2.y * w;
    w = dx * ay * dz; re += q2.z * w; im += q2.w * w;
    w = ax * dy * dz; re += q3.x * w; im += q3.y * w;
    w = dx * dy * dz; re += q3.z * w; im += q3.w * w;
    return make_float2(re, conj ? -im : im);
}

template <bool CELLS>
__global__ void __launch_bounds__(THREADS) k_local_fused(const float2* __restrict__ vol,
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
    const int l = blockIdx.x, r0 = blockIdx.y * RT, t0 = blockIdx.z * TT;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    __shared__ double sMat[RT][6];
    __shared__ float sTr[TT][2];
    __shared__ __attribute__((aligned(16))) float2 sA[RT * APITCH];      // [r][px]
    __shared__ __attribute__((aligned(16))) float sB[KC * 4 * TT];       // [px][k][t]
    __shared__ float sRed[THREADS / 64];

    if (tid < RT) {
        const int r = r0 + tid;
        double q[4] = {1, 0, 0, 0};
        if (r < nR)
            for (int k = 0; k < 4; k++) q[k] = quat[((size_t)l * nR + r) * 4 + k];
        double m[9];
        quat_to_mat(q, m);
        for (int k = 0; k < 6; k++) sMat[tid][k] = m[k];
    }
    if (tid < TT) {
        const int t = t0 + tid;
        float tx = 0.f, ty = 0.f;
        if (t < nT) {
            tx = (float)trans[((size_t)l * nT + t) * 2];
            ty = (float)trans[((size_t)l * nT + t) * 2 + 1];
        }
        sTr[tid][0] = tx / idim;   // rCol of translate(), ImageFunctions.cpp:243
        sTr[tid][1] = ty / idim;
    }

    const float2* D = dat + (size_t)l * nPxl;
    const float* C = ctf + (size_t)l * nPxl;
    const float* S = sig + (size_t)l * nPxl;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    float aConst = 0.f;
    // gather mapping: a half-wave covers 32 consecutive pixels of one rotation
    // (neighbouring pixels hit neighbouring cells of the same slice)
    const int gpx = lane & 31, grq = lane >> 5;
    // MFMA mapping: wave wv owns M-tiles 2wv, 2wv+1 (32 rotations)
    const int mm = lane & 15, kk = lane >> 4;

    __syncthreads();
    for (int i0 = 0; i0 < nPxl; i0 += KC) {
        // ---- translation / image tile: B[px][0..3][t] = (U, V, b, 0)
#pragma unroll
        for (int u = 0; u < KC * TT / THREADS; u++) {
            const int q = tid + u * THREADS;
            const int bpx = q / TT, bt = q % TT;
            const int i = i0 + bpx;
            float U = 0.f, V = 0.f, b = 0.f;
            if (i < nPxl) {
                const float2 d = D[i];
                const float c = C[i], s = S[i];
                const float k2 = -2.f * s * c;
                const float yr = k2 * d.x, yi = k2 * d.y;
                if (t0 + bt < nT) {
                    const float2 T = phase_shift(iCol[i], iRow[i], sTr[bt][0], sTr[bt][1]);
                    U = yr * T.x + yi * T.y;
                    V = yi * T.x - yr * T.y;
                    b = s * c * c;
                }
                if (bt == 0) aConst += s * (d.x * d.x + d.y * d.y);
            }
            float* B = sB + bpx * 4 * TT;
            B[0 * TT + bt] = U;
            B[1 * TT + bt] = V;
            B[2 * TT + bt] = b;
            B[3 * TT + bt] = 0.f;
        }
        // ---- projection tile: A[px][r] = P (complex)
        {
            const int i = i0 + gpx;
            const bool ok = i < nPxl;
            const int ic = ok ? iCol[i] : 0, ir = ok ? iRow[i] : 0;
            const double nx = (double)(ic * pf), ny = (double)(ir * pf);
#pragma unroll 4
            for (int p = 0; p < RT / 8; p++) {
                const int r = wv * (RT / 4) + p * 2 + grq;
                const double* m = sMat[r];
                const float x = (float)(m[0] * nx + m[3] * ny);
                const float y = (float)(m[1] * nx + m[4] * ny);
                const float z = (float)(m[2] * nx + m[5] * ny);
                float2 P = make_float2(0.f, 0.f);
                if (ok)
                    P = CELLS ? interp_cells(reinterpret_cast<const float4*>(vol), vdim, x, y, z)
                              : interp_ft(vol, vdim, x, y, z);
                sA[r * APITCH + gpx] = P;
            }
        }
        __syncthreads();
        // ---- reduce the chunk on the matrix cores: A row = (P.re, P.im, |P|^2, 0)
#pragma unroll 8
        for (int px = 0; px < KC; px++) {
            const float bv = sB[(px * 4 + kk) * TT + mm];
            const float2 p0 = sA[(wv * 32 + mm) * APITCH + px];
            const float2 p1 = sA[(wv * 32 + 16 + mm) * APITCH + px];
            const float a0 = kk == 0 ? p0.x : kk == 1 ? p0.y : kk == 2 ? p0.x * p0.x + p0.y * p0.y : 0.f;
            const float a1 = kk == 0 ? p1.x : kk == 1 ? p1.y : kk == 2 ? p1.x * p1.x + p1.y * p1.y : 0.f;
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, bv, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, bv, acc1, 0, 0, 0);
        }
        __syncthreads();
    }
    // A_l = sum_i s |d|^2 (only the bt == 0 threads accumulated)
    aConst = wave_sum(aConst);
    if (lane == 0) sRed[wv] = aConst;
    __syncthreads();
    const float Al = sRed[0] + sRed[1] + sRed[2] + sRed[3];
    // C layout of 16x16x4: col = lane & 15 (translation), row = 4 (lane >> 4) + j
    const int t = t0 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int ra = r0 + wv * 32 + 4 * (lane >> 4) + j;
        const int rb = ra + 16;
        if (t < nT) {
            if (ra < nR) dvp[((size_t)l * nR + ra) * nT + t] = Al + acc0[j];
            if (rb < nR) dvp[((size_t)l * nR + rb) * nT + t] = Al + acc1[j];
        }
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

// One thread per cell: the 8 taps (dz, dy, dx) of base voxel (i, j, k), rows
// and slices wrapped like iFTHalf, i + 1 past the half-plane edge -> 0.
__global__ void __launch_bounds__(256) k_volume_cells(const float2* __restrict__ vol,
                                                      int vdim, float2* __restrict__ cells)
{
    const int nColFT = vdim / 2 + 1;
    const long n = (long)nColFT * vdim * vdim;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int i = (int)(q % nColFT);
        const long jk = q / nColFT;
        const int j = (int)(jk % vdim), k = (int)(jk / vdim);
        const int j1 = j + 1 == vdim ? 0 : j + 1, k1 = k + 1 == vdim ? 0 : k + 1;
        float2 v[8];
        const int zz[2] = {k, k1}, yy[2] = {j, j1};
#pragma unroll
        for (int dz = 0; dz < 2; dz++)
#pragma unroll
            for (int dy = 0; dy < 2; dy++)
#pragma unroll
                for (int dx = 0; dx < 2; dx++) {
                    const int x = i + dx;
                    v[dz * 4 + dy * 2 + dx] =
                        x < nColFT ? vol[((size_t)zz[dz] * vdim + yy[dy]) * nColFT + x]
                                   : make_float2(0.f, 0.f);
                }
        float4* o = reinterpret_cast<float4*>(cells + 8 * (size_t)q);
#pragma unroll
        for (int u = 0; u < 4; u++) o[u] = make_float4(v[2 * u].x, v[2 * u].y, v[2 * u + 1].x, v[2 * u + 1].y);
    }
}

}  // namespace

extern "C" int thx_volume_cells(const float* vol, int vdim, float* cells,
                                thx_stream_t stream)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0, "thx_volume_cells: bad vdim");
    hipLaunchKernelGGL(k_volume_cells, dim3(4096), dim3(256), 0, thx::as_stream(stream),
                       reinterpret_cast<const float2*>(vol), vdim,
                       reinterpret_cast<float2*>(cells));
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" size_t thx_local_phase_workspace(int nImg, int nR, int nT)
{
    return (size_t)nImg * nR * nT * sizeof(float) + 256;
}

extern "C" int thx_local_phase(const float* vol, int volLayout, int vdim, int pf,
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
    THX_CHECK_ARG(volLayout == 0 || volLayout == 1, "thx_local_phase: volLayout must be 0 or 1");
    THX_CHECK_ARG(nImg <= 0x7fffffff && (nR + RT - 1) / RT <= 65535 && (nT + TT - 1) / TT <= 65535,
                  "thx_local_phase: grid too large");
    if (nImg == 0) return THX_OK;
    float* d = dvp;
    if (!d) {
        THX_CHECK_ARG(workspace && wsBytes >= thx_local_phase_workspace(nImg, nR, nT),
                      "thx_local_phase: workspace too small");
        d = static_cast<float*>(workspace);
    }
    hipStream_t s = thx::as_stream(stream);
    dim3 grid(nImg, thx::cdiv(nR, RT), thx::cdiv(nT, TT));
    if (volLayout == 1)
        hipLaunchKernelGGL(k_local_fused<true>, grid, dim3(THREADS), 0, s,
                           reinterpret_cast<const float2*>(vol), vdim, pf, quat, nR, trans, nT,
                           reinterpret_cast<const float2*>(dat), ctf, sigRcp, iCol, iRow, nPxl,
                           idim, d);
    else
        hipLaunchKernelGGL(k_local_fused<false>, grid, dim3(THREADS), 0, s,
                           reinterpret_cast<const float2*>(vol), vdim, pf, quat, nR, trans, nT,
                           reinterpret_cast<const float2*>(dat), ctf, sigRcp, iCol, iRow, nPxl,
                           idim, d);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_local_weights, dim3(nImg), dim3(256), 0, s, d, nR, nT, pC, pR, pT, wC,
                       wR, wT, baseL);
    THX_LAUNCH_CHECK();
    return THX_OK;
}
