// insert.hip -- a12: weighted trilinear back-projection into the half-map
// (Reconstructor::insertP, src/Reconstructor.cpp:782-863, driven by the CPU
// loop of src/Optimiser.cpp:7036-7241; GPU twin cuthunder::InsertFT,
// gpu/src/cuthunder.cu:5570-5826).
#include <climits>

#include "common.h"
#include "patch.h"

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
                                                  const int* __restrict__ nC,
                                                  int mReco,
                                                  const int* __restrict__ iCol,
                                                  const int* __restrict__ iRow,
                                                  int nPxl, int idim)
{
    const int m = blockIdx.y, l = blockIdx.z;
    if (nC && m >= nC[l]) return;      // K-class call: image l drew this class nC[l] times
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
                            const double* offS, const float* w, const int* nC, int nImg,
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
                       ctf, quat, trans, offS, w, nC, mReco, iCol, iRow, nPxl, idim);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

namespace {

constexpr int INS_THREADS = 512;
constexpr int INS_WAVES = INS_THREADS / 64;
constexpr int INS_CAP = 5120;    // LDS voxels: F (8 B) + T (4 B) = 60 KiB, two workgroups per CU
constexpr int KC = thx::PATCH_KC;
constexpr int RT = thx::PATCH_RT;
constexpr int REC = thx::PATCH_REC;
static_assert(INS_CAP <= thx::PATCH_BOX_CAP, "records carry LDS offsets up to PATCH_BOX_CAP");

// One workgroup per (patch c, sample tile ry, image l): the samples
// m0 .. m0 + nM - 1 of image l scattered at the KC pixels of patch c.
// Memory-side float atomics with 64 lanes in 64 rows run at ~0.08 TB/s
// (MI355X_MICROARCH.md, global float atomics), so the patch's neighbourhood
// (the k_patch_boxes record, the same boxes as the local phase) is
// accumulated in LDS with ds_add_f32 and flushed once, one box row per
// wave pass, skipping untouched voxels.  A box larger than INS_CAP is swept
// in z-chunks of whole slices (both Hermitian sides), the samples re-run per
// chunk and keeping only their taps inside it; a box whose single slice
// pair exceeds INS_CAP scatters straight to HBM (scatter_ft).  The F / T
// values and coordinates are those of k_insert3d; only the FP32 summation
// order differs.
__global__ void __launch_bounds__(INS_THREADS) k_insert_patches(float2* __restrict__ F,
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
                                                                const int* __restrict__ nCnt,
                                                                int mReco,
                                                                const int* __restrict__ iCol,
                                                                const int* __restrict__ iRow,
                                                                const int* __restrict__ order,
                                                                int nVisit, int nPxl, int idim,
                                                                const int* __restrict__ rec)
{
    __shared__ __attribute__((aligned(16))) float2 sF[INS_CAP];
    __shared__ float sT[INS_CAP];
    __shared__ double sM[RT][6];           // first two columns of R per sample
    __shared__ float sSh[RT][2];           // (rCol, rRow) of the re-centring shift
    __shared__ float sPx[KC][4];           // dat.re, dat.im, ctf of the patch's pixels
    __shared__ int sIc[KC][2];             // (iCol, iRow), INT_MIN row for padding
    __shared__ double sO[INS_WAVES][3];
    const int c = blockIdx.x, ry = blockIdx.y, l = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nC = (nVisit + KC - 1) / KC, nRT = (mReco + RT - 1) / RT;
    const int m0 = ry * RT;
    // samples of this tile (the K-class call inserts only the first nC[l])
    const int nM = max(0, min(RT, (nCnt ? min(nCnt[l], mReco) : mReco) - m0));
    if (nM == 0) return;
    const int* R = rec + (((size_t)l * nRT + ry) * nC + c) * REC;
    int rv[REC];
#pragma unroll
    for (int k = 0; k < REC; k++) rv[k] = R[k];
    const float wl = w[l];
    const double offx = offS[2 * l], offy = offS[2 * l + 1];

    // per-sample rotation and shift; insertDir(-R (t - off, 0)) once per image
    double o0 = 0.0, o1 = 0.0, o2 = 0.0;
    if (tid < nM) {
        const size_t sIdx = (size_t)l * mReco + m0 + tid;
        double q[4] = {quat[4 * sIdx], quat[4 * sIdx + 1], quat[4 * sIdx + 2], quat[4 * sIdx + 3]};
        double m[9];
        quat_to_mat(q, m);
        for (int k = 0; k < 6; k++) sM[tid][k] = m[k];
        const double dx = trans[2 * sIdx] - offx, dy = trans[2 * sIdx + 1] - offy;
        sSh[tid][0] = (float)(-dx) / idim;
        sSh[tid][1] = (float)(-dy) / idim;
        o0 = -(m[0] * dx + m[3] * dy);
        o1 = -(m[1] * dx + m[4] * dy);
        o2 = -(m[2] * dx + m[5] * dy);
    }
    if (c == 0) {        // src/Reconstructor.cpp:407-422, one workgroup per sample tile
        o0 = wave_sum(o0); o1 = wave_sum(o1); o2 = wave_sum(o2);
        if (lane == 0) { sO[wv][0] = o0; sO[wv][1] = o1; sO[wv][2] = o2; }
    }
    if (tid < KC) {
        const int p = patch_pixel(order, nVisit, c * KC + tid);
        if (p >= 0) {
            const float2 d = dat[(size_t)l * nPxl + p];
            sPx[tid][0] = d.x; sPx[tid][1] = d.y; sPx[tid][2] = ctf[(size_t)l * nPxl + p];
            sIc[tid][0] = iCol[p]; sIc[tid][1] = iRow[p];
        } else {
            sIc[tid][0] = 0; sIc[tid][1] = INT_MIN;
        }
    }
    __syncthreads();
    if (c == 0 && tid == 0) {
        double a0 = 0.0, a1 = 0.0, a2 = 0.0;
        for (int k = 0; k < INS_WAVES; k++) { a0 += sO[k][0]; a1 += sO[k][1]; a2 += sO[k][2]; }
        atomicAdd(O + 0, a0);
        atomicAdd(O + 1, a1);
        atomicAdd(O + 2, a2);
        atomicAdd(counter, nM);
    }

    // box geometry and z-chunking
    const int nx = rv[6], sp = rv[7], ny = rv[8];
    const int nv0 = rv[9], nv1 = rv[10] - rv[9];
    const int nSides = (nv0 > 0) + (nv1 > 0);
    const int nz = max(nv0, nv1) / sp;
    const int zc = nSides ? min(nz, INS_CAP / (sp * nSides)) : 0;   // slices per chunk

    // sample q -> (folded coordinate, conj flag, values)
    auto sample = [&](int q, float& x, float& y, float& z, float& vr, float& vi, float& tv) {
        const int m = q / KC, k = q % KC;
        const int ic = sIc[k][0], ir = sIc[k][1];
        if (ir == INT_MIN) return false;
        const float2 src = cmul(make_float2(sPx[k][0], sPx[k][1]),
                                phase_shift(ic, ir, sSh[m][0], sSh[m][1]));
        const float cf = sPx[k][2];
        vr = (src.x * cf) * wl;
        vi = (src.y * cf) * wl;
        tv = (float)((double)cf * cf) * wl;
        const double X = (double)(ic * pf), Y = (double)(ir * pf);
        x = (float)(sM[m][0] * X + sM[m][3] * Y);
        y = (float)(sM[m][1] * X + sM[m][4] * Y);
        z = (float)(sM[m][2] * X + sM[m][5] * Y);
        return true;
    };

    if (zc == 0) {       // not even one slice pair fits: scatter to HBM
        for (int q = tid; q < nM * KC; q += INS_THREADS) {
            float x, y, z, vr, vi, tv;
            if (sample(q, x, y, z, vr, vi, tv)) scatter_ft(F, T, vdim, x, y, z, vr, vi, tv);
        }
        return;
    }

    const int nColFT = vdim / 2 + 1;
    float* Ff = reinterpret_cast<float*>(F);
    const float* sFf = reinterpret_cast<const float*>(sF);
    for (int zk = 0; zk < nz; zk += zc) {
        const int zn = min(zc, nz - zk);
        const int base1 = nv0 > 0 ? zn * sp : 0;          // LDS offset of side 1
        const int nvox = base1 + (nv1 > 0 ? zn * sp : 0);
        for (int v = tid; v < nvox; v += INS_THREADS) { sF[v] = make_float2(0.f, 0.f); sT[v] = 0.f; }
        __syncthreads();
        for (int q = tid; q < nM * KC; q += INS_THREADS) {
            float x, y, z, vr, vi, tv;
            if (!sample(q, x, y, z, vr, vi, tv)) continue;
            const bool conj = !(x >= 0.f);
            if (conj) { x = -x; y = -y; z = -z; vi = -vi; }
            const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
            const float dx = x - fx, dy = y - fy, dz = z - fz;
            const float wx[2] = {1.f - dx, dx}, wy[2] = {1.f - dy, dy}, wz[2] = {1.f - dz, dz};
            // box-local cell corner; side s origin rv[3 s .. 3 s + 2], chunk from slice zk
            const int lx = (int)fx - rv[conj ? 3 : 0];
            const int ly = (int)fy - rv[conj ? 4 : 1];
            const int lz = (int)fz - rv[conj ? 5 : 2] - zk;
            const int a = (conj ? base1 : 0) + lz * sp + ly * nx + lx;
#pragma unroll
            for (int kz = 0; kz < 2; kz++) {
                if (lz + kz < 0 || lz + kz >= zn) continue;
#pragma unroll
                for (int jy = 0; jy < 2; jy++)
#pragma unroll
                    for (int ix = 0; ix < 2; ix++) {
                        const float wt = wx[ix] * wy[jy] * wz[kz];
                        const int v = a + kz * sp + jy * nx + ix;
                        atomicAdd(&sF[v].x, vr * wt);
                        atomicAdd(&sF[v].y, vi * wt);
                        atomicAdd(&sT[v], tv * wt);
                    }
            }
        }
        __syncthreads();
        // flush: one box row per wave pass, lanes over the row's floats
        const int rowsSide = zn * ny;
        const int rows0 = nv0 > 0 ? rowsSide : 0, rows = rows0 + (nv1 > 0 ? rowsSide : 0);
        for (int row = wv; row < rows; row += INS_WAVES) {
            const bool s1 = row >= rows0;
            const int rr = s1 ? row - rows0 : row;
            const int z = rr / ny, y = rr - z * ny;
            const int base = (s1 ? base1 : 0) + z * sp + y * nx;
            const int gx0 = s1 ? rv[3] : rv[0];
            const int gy = wrap_idx((s1 ? rv[4] : rv[1]) + y, vdim);
            const int gz = wrap_idx((s1 ? rv[5] : rv[2]) + zk + z, vdim);
            const size_t g = ((size_t)gz * vdim + gy) * nColFT + gx0;
            for (int j = lane; j < 2 * nx; j += 64) {
                const float v = sFf[2 * base + j];
                if (v != 0.f && gx0 + (j >> 1) < nColFT) atomicAdd(Ff + 2 * g + j, v);
            }
            for (int j = lane; j < nx; j += 64) {
                const float v = sT[base + j];
                if (v != 0.f && gx0 + j < nColFT) atomicAdd(T + g + j, v);
            }
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" size_t thx_insert3d_workspace(int nImg, int mReco, int nOrd)
{
    return thx::patch_rec_bytes(nImg, mReco, nOrd) + 256;
}

extern "C" int thx_insert3d_tiled(float* F, float* T, double* O, int* counter, int vdim, int pf,
                                  const float* dat, const float* ctf, const double* quat,
                                  const double* trans, const double* offS, const float* w,
                                  const int* nC, int nImg, int mReco, const int* iCol, const int* iRow,
                                  const int* pxOrder, int nOrd, int nPxl, int idim,
                                  void* workspace, size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0 && pf > 0 && nImg >= 0 && mReco >= 0 &&
                      nPxl >= 0 && idim > 0,
                  "thx_insert3d_tiled: bad sizes");
    THX_CHECK_ARG(pxOrder && nOrd > 0 && nOrd % KC == 0,
                  "thx_insert3d_tiled: pxOrder from thx_pixel_tile_order required");
    THX_CHECK_ARG(nImg <= 65535 && (mReco + RT - 1) / RT <= 65535 && nOrd / KC <= 0x7fffffff,
                  "thx_insert3d_tiled: grid too large");
    if (nImg == 0 || mReco == 0 || nPxl == 0) return THX_OK;
    THX_CHECK_ARG(workspace && wsBytes >= thx_insert3d_workspace(nImg, mReco, nOrd),
                  "thx_insert3d_tiled: workspace too small");
    hipStream_t s = thx::as_stream(stream);
    int* rec = static_cast<int*>(workspace);
    int st = thx::launch_patch_boxes(quat, mReco, iCol, iRow, pxOrder, nOrd, pf, vdim, nImg, rec, s);
    if (st != THX_OK) return st;
    hipLaunchKernelGGL(k_insert_patches, dim3(nOrd / KC, thx::cdiv(mReco, RT), nImg),
                       dim3(INS_THREADS), 0, s, reinterpret_cast<float2*>(F), T, O, counter, vdim,
                       pf, reinterpret_cast<const float2*>(dat), ctf, quat, trans, offS, w, nC,
                       mReco, iCol, iRow, pxOrder, nOrd, nPxl, idim, rec);
    THX_LAUNCH_CHECK();
    return THX_OK;
}
