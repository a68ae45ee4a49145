/*
 * thunder_oracle.c -- CPU restatement of THUNDER's expectation / insert hot path.
 *
 * TEST INFRASTRUCTURE ONLY -- see thunder_oracle.h for the usage rule and the
 * "parity unpinned" status.  Built with -ffp-contract=off so that float
 * products round exactly as in the reference's non-FMA (-mavx) build.
 *
 * Every function restates the reference routine cited in its comment; types
 * follow the reference single-precision build (RFLOAT = float, rotation
 * matrices / quaternions / particle weights double).
 */
#include "thunder_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define M_2X_PI_REF 6.28318530717959 /* include/Macro.h:14 */

/* ---------------------------------------------------------------- a1 ---- */
int orc_pixel_set(int N, int pf, float rU, float rL, int cap, int* iCol,
                  int* iRow, int* iSig, int* iPxl, int* iColPad, int* iRowPad)
{
    /* src/Optimiser.cpp:8008-8040; IMAGE_FOR_PIXEL_R_FT(rU + 1)
     * (include/Image/Image.h:68-70): j outer, i inner. */
    const float rU2 = (float)((double)rU * (double)rU); /* TSGSL_pow_2 */
    const float rL2 = (float)((double)rL * (double)rL);
    const float r = rU + 1;
    const long nColFT = N / 2 + 1;
    int n = 0;
    for (long j = (long)(-r); j < r; j++)
        for (long i = 0; i <= r; i++) {
            if ((i == 0) && (j < 0)) continue;
            float u = (float)((double)i * (double)i + (double)j * (double)j);
            if ((u < rU2) && (u >= rL2)) {
                int v = (int)rint(hypot((double)i, (double)j)); /* AROUND(NORM) */
                if ((v < rU) && (v >= rL)) {
                    if (n >= cap) return -1;
                    if (iPxl) iPxl[n] = (int)((j >= 0 ? j : j + N) * nColFT + i);
                    if (iCol) iCol[n] = (int)i;
                    if (iRow) iRow[n] = (int)j;
                    if (iSig) iSig[n] = v;
                    if (iColPad) iColPad[n] = (int)i * pf;
                    if (iRowPad) iRowPad[n] = (int)j * pf;
                    n++;
                }
            }
        }
    return n;
}

/* ---------------------------------------------------------------- a2 ---- */
void orc_ctf(float* dst, float pixelSize, float voltage, float defocusU,
             float defocusV, float theta, float Cs, float amplitudeContrast,
             float phaseShift, int nCol, int nRow, const int* iCol,
             const int* iRow, int nPxl)
{
    /* src/CTF.cpp:113-151 (wavelength constant 12.2643247, quirk q5). */
    float lambda = (float)(12.2643247 / sqrt((double)voltage *
                                            (1 + (double)voltage * 0.978466e-6)));
    float w1 = sqrtf(1 - (float)((double)amplitudeContrast * amplitudeContrast));
    float w2 = amplitudeContrast;
    float K1 = (float)(M_PI * lambda);
    float K2 = (float)(M_PI_2 * Cs * (float)((double)lambda * lambda * lambda));
    for (int i = 0; i < nPxl; i++) {
        float a = iCol[i] / (pixelSize * nCol);
        float b = iRow[i] / (pixelSize * nRow);
        float u = (float)hypot((double)a, (double)b);
        float angle = (float)(atan2((double)iRow[i], (double)iCol[i]) - theta);
        float defocus = -(defocusU + defocusV +
                          (defocusU - defocusV) * cosf(2 * angle)) / 2;
        float u2 = (float)((double)u * u);
        float u4 = (float)((double)u * u * u * u);
        float ki = K1 * defocus * u2 + K2 * u4 - phaseShift;
        dst[i] = -w1 * sinf(ki) + w2 * cosf(ki);
    }
}

/* a2, CTF search: allocPreCal's cSearch branch (src/Optimiser.cpp:8124-8170)
 * for one image: frequency, per-pixel defocus, K1, K2 (its wavelength
 * constant 12.2643274, quirk q5). */
void orc_defocus_pre(const float* attr, const int* iCol, const int* iRow, int nPxl,
                     int idim, float* freq, float* defocusP, float* K1, float* K2)
{
    const float pixelSize = attr[0], voltage = attr[1], dU = attr[2], dV = attr[3];
    const float theta = attr[4], Cs = attr[5];
    for (int i = 0; i < nPxl; i++) {
        /* NORM(iCol, iRow) / size / pixelSize (:8138-8142) */
        freq[i] = (float)(sqrt((double)iCol[i] * iCol[i] + (double)iRow[i] * iRow[i]) / idim /
                          pixelSize);
        float angle = (float)(atan2((double)iRow[i], (double)iCol[i]) - theta); /* :8149-8151 */
        defocusP[i] = -(dU + dV + (dU - dV) * cosf(2 * angle)) / 2;             /* :8153-8157 */
    }
    float lambda = (float)(12.2643274 / sqrt((double)voltage * (1 + (double)voltage * 0.978466e-6)));
    *K1 = (float)(M_PI * lambda);                                              /* :8167 */
    *K2 = (float)(M_PI_2 * Cs * ((double)lambda * lambda * lambda));           /* :8168 */
}

/* a2, CTF search: the per-defocus-sample CTF of a local phase,
 * src/Optimiser.cpp:1252-1271 (GPU twin kernel_CalCTFL, gpu/src/Kernel.cu:
 * 481-515): ctfD[iD][i] for the image's defocus factors d[nD]. */
void orc_ctf_search(float* ctfD, const float* defocusP, const float* freq, const double* d,
                    int nD, float K1, float K2, float phaseShift, float conT, int nPxl)
{
    const float w1 = sqrtf(1 - (float)((double)conT * conT));
    for (int iD = 0; iD < nD; iD++)
        for (int i = 0; i < nPxl; i++) {
            const double f2 = (double)freq[i] * freq[i];
            const float ki = (float)((double)(K1 * defocusP[i]) * d[iD] * f2 + K2 * (f2 * f2) -
                                     phaseShift);
            ctfD[(size_t)iD * nPxl + i] = -w1 * sinf(ki) + conT * cosf(ki);
        }
}

/* ---------------------------------------------------------------- a4 ---- */
void orc_translate(float* dst, float nTransCol, float nTransRow, int nCol,
                   int nRow, const int* iCol, const int* iRow, int nPxl)
{
    /* src/Image/ImageFunctions.cpp:233-252 */
    float rCol = nTransCol / nCol;
    float rRow = nTransRow / nRow;
    for (int i = 0; i < nPxl; i++) {
        float phase = (float)(M_2X_PI_REF * (iCol[i] * rCol + iRow[i] * rRow));
        dst[2 * i] = cosf(-phase); /* COMPLEX_POLAR, include/Complex.h:33-39 */
        dst[2 * i + 1] = sinf(-phase);
    }
}

void orc_translate_src(float* dst, const float* src, float nTransCol,
                       float nTransRow, int nCol, int nRow, const int* iCol,
                       const int* iRow, int nPxl)
{
    /* src/Image/ImageFunctions.cpp:471-492: dst = src * POLAR(-phase) */
    float rCol = nTransCol / nCol;
    float rRow = nTransRow / nRow;
    for (int i = 0; i < nPxl; i++) {
        float phase = (float)(M_2X_PI_REF * (iCol[i] * rCol + iRow[i] * rRow));
        float pr = cosf(-phase), pi = sinf(-phase);
        float sr = src[2 * i], si = src[2 * i + 1];
        dst[2 * i] = sr * pr - si * pi; /* operator*, include/Complex.h:195-203 */
        dst[2 * i + 1] = sr * pi + si * pr;
    }
}

/* ---------------------------------------------------------------- a5 ---- */
void orc_rotate3d(double* mat, const double* q)
{
    /* src/Geometry/Euler.cpp:181-189: R = I + 2 q0 A + 2 A A */
    double A[3][3] = {{0, -q[3], q[2]}, {q[3], 0, -q[1]}, {-q[2], q[1], 0}};
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            double aa = 0;
            for (int k = 0; k < 3; k++) aa += (2 * A[r][k]) * A[k][c];
            double v = (r == c ? 1.0 : 0.0) + (2 * q[0]) * A[r][c] + aa;
            mat[c * 3 + r] = v; /* column-major */
        }
}

/* ------------------------------------------------------------- a6 ------- */
static inline long wrapi(long v, long n) { return v >= 0 ? v : v + n; }

/* Volume::getByInterpolationFT (src/Image/Volume.cpp:314-338) at a float
 * coordinate; result in out[2]. */
static void interp_ft(float* out, const float* vol, int vdim, float x, float y,
                      float z)
{
    int conj = 0;
    if (!(x >= 0)) { /* conjHalf, include/Image/Volume.h:135-147 */
        x = -x; y = -y; z = -z;
        conj = 1;
    }
    /* WG_TRI_INTERP_LINEAR, include/Functions/Interpolation.h:187-200 */
    float c[3] = {x, y, z};
    long x0[3];
    float v[3][2];
    for (int d = 0; d < 3; d++) {
        x0[d] = (long)floorf(c[d]);
        float xd = c[d] - (float)x0[d];
        v[d][0] = 1 - xd;
        v[d][1] = xd;
    }
    const long nColFT = vdim / 2 + 1;
    float re = 0, im = 0;
    /* getFTHalf (src/Image/Volume.cpp:491-563): order box[k][j][i], i fastest;
     * per-tap wrap is what both the unfolded fast path and the x0 == -1 slow
     * path compute for every reachable coordinate. */
    for (int k = 0; k < 2; k++)
        for (int j = 0; j < 2; j++)
            for (int i = 0; i < 2; i++) {
                float w = v[0][i] * v[1][j] * v[2][k];
                size_t idx = (size_t)(wrapi(x0[2] + k, vdim) * vdim +
                                      wrapi(x0[1] + j, vdim)) * nColFT +
                             (size_t)(x0[0] + i);
                re += vol[2 * idx] * w;
                im += vol[2 * idx + 1] * w;
            }
    out[0] = re;
    out[1] = conj ? -im : im;
}

void orc_project3d(float* dst, const float* vol, int vdim, int pf,
                   const double* mat, const int* iCol, const int* iRow,
                   int nPxl)
{
    /* src/Projector.cpp:356-374: oldCor = mat * (iCol*pf, iRow*pf, 0) in
     * double, cast to RFLOAT at the getByInterpolationFT call. */
    for (int i = 0; i < nPxl; i++) {
        double nx = (double)(iCol[i] * pf), ny = (double)(iRow[i] * pf), nz = 0;
        double ox = mat[0] * nx + mat[3] * ny + mat[6] * nz;
        double oy = mat[1] * nx + mat[4] * ny + mat[7] * nz;
        double oz = mat[2] * nx + mat[5] * ny + mat[8] * nz;
        interp_ft(dst + 2 * i, vol, vdim, (float)ox, (float)oy, (float)oz);
    }
}

/* ---------------------------------------------------------------- a7 ---- */
float orc_logdatavs(const float* dat, const float* pri, const float* ctf,
                    const float* sigRcp, int m)
{
    /* src/Optimiser.cpp:9187-9213 */
    float result2 = 0;
    for (int i = 0; i < m; i++) {
        float tmpReal = ctf[i] * pri[2 * i];
        float tmpImag = ctf[i] * pri[2 * i + 1];
        float tmp1Real = dat[2 * i] - tmpReal;
        float tmp1Imag = dat[2 * i + 1] - tmpImag;
        float tmp2 = tmp1Real * tmp1Real + tmp1Imag * tmp1Imag;
        result2 += (tmp2 * sigRcp[i]);
    }
    return result2;
}

static void cmul(float* dst, const float* a, const float* b, int n)
{
    for (int i = 0; i < n; i++) {
        float ar = a[2 * i], ai = a[2 * i + 1], br = b[2 * i], bi = b[2 * i + 1];
        dst[2 * i] = ar * br - ai * bi;
        dst[2 * i + 1] = ar * bi + ai * br;
    }
}

void orc_dvp_global(float* dvp, const float* vol, int vdim, int pf,
                    const double* quat, int nR, const double* trans, int nT,
                    const float* dat, const float* ctf, const float* sigRcp,
                    int nImg, const int* iCol, const int* iRow, int nPxl,
                    int idim, int nThreads)
{
    /* translation table, src/Optimiser.cpp:708-724 */
    float* traP = (float*)malloc(sizeof(float) * 2 * (size_t)nT * nPxl);
    for (int n = 0; n < nT; n++)
        orc_translate(traP + 2 * (size_t)n * nPxl, (float)trans[2 * n],
                      (float)trans[2 * n + 1], idim, idim, iCol, iRow, nPxl);
#ifdef _OPENMP
    if (nThreads > 0) omp_set_num_threads(nThreads);
#else
    (void)nThreads;
#endif
    /* src/Optimiser.cpp:756-826: OpenMP over rotations m, translations n inner,
     * likelihood over all images per (m, n). */
#pragma omp parallel
    {
        float* priRotP = (float*)malloc(sizeof(float) * 2 * nPxl);
        float* priAllP = (float*)malloc(sizeof(float) * 2 * nPxl);
#pragma omp for schedule(dynamic)
        for (int m = 0; m < nR; m++) {
            double mat[9];
            orc_rotate3d(mat, quat + 4 * m);
            orc_project3d(priRotP, vol, vdim, pf, mat, iCol, iRow, nPxl);
            for (int n = 0; n < nT; n++) {
                cmul(priAllP, traP + 2 * (size_t)n * nPxl, priRotP, nPxl);
                for (int l = 0; l < nImg; l++)
                    dvp[((size_t)l * nR + m) * nT + n] = orc_logdatavs(
                        dat + 2 * (size_t)l * nPxl, priAllP,
                        ctf + (size_t)l * nPxl, sigRcp + (size_t)l * nPxl, nPxl);
            }
        }
        free(priRotP);
        free(priAllP);
    }
    free(traP);
}

/* ---------------------------------------------------------------- a8 ---- */
void orc_weights_global(const float* dvp, int nImg, int nR, int nT,
                        const double* pR, const double* pT, int kIdx, int nK,
                        float* wC, float* wR, float* wT, float* baseL)
{
    /* src/Optimiser.cpp:834-894 */
    for (int l = 0; l < nImg; l++) {
        float* wCl = wC + (size_t)l * nK;
        float* wRl = wR + (size_t)l * nK * nR;
        float* wTl = wT + (size_t)l * nK * nT;
        for (int m = 0; m < nR; m++)
            for (int n = 0; n < nT; n++) {
                float d = dvp[((size_t)l * nR + m) * nT + n];
                if (isnan(baseL[l]))
                    baseL[l] = d;
                else if (d > baseL[l]) {
                    float offset = d - baseL[l];
                    float nf = expf(-offset);
                    for (int c = 0; c < nK; c++) wCl[c] *= nf;
                    for (size_t q = 0; q < (size_t)nK * nR; q++) wRl[q] *= nf;
                    for (size_t q = 0; q < (size_t)nK * nT; q++) wTl[q] *= nf;
                    baseL[l] += offset;
                }
                float w = expf(d - baseL[l]);
                wCl[kIdx] = (float)(wCl[kIdx] + w * (pR[m] * pT[n]));
                wRl[(size_t)kIdx * nR + m] =
                    (float)(wRl[(size_t)kIdx * nR + m] + w * pT[n]);
                wTl[(size_t)kIdx * nT + n] =
                    (float)(wTl[(size_t)kIdx * nT + n] + w * pR[m]);
            }
    }
}

/* ---------------------------------------------------------------- a9 ---- */
void orc_local_phase(const float* vol, int vdim, int pf, const double* quat,
                     int nR, const double* trans, int nT, double pC,
                     const double* pR, const double* pT, const float* dat,
                     const float* ctf, const float* sigRcp, const int* iCol,
                     const int* iRow, int nPxl, int idim, float* wC,
                     float* wR, float* wT, float* baseL, float* dvp)
{
    /* src/Optimiser.cpp:1205-1402 with nC = nD = 1, wD = 1 */
    float* traP = (float*)malloc(sizeof(float) * 2 * (size_t)nT * nPxl);
    float* priRotP = (float*)malloc(sizeof(float) * 2 * nPxl);
    float* priAllP = (float*)malloc(sizeof(float) * 2 * nPxl);
    for (int t = 0; t < nT; t++)
        orc_translate(traP + 2 * (size_t)t * nPxl, (float)trans[2 * t],
                      (float)trans[2 * t + 1], idim, idim, iCol, iRow, nPxl);
    const double pD = 1.0;
    float baseLine = NAN;
    wC[0] = 0;
    for (int r = 0; r < nR; r++) wR[r] = 0;
    for (int t = 0; t < nT; t++) wT[t] = 0;
    for (int r = 0; r < nR; r++) {
        double mat[9];
        orc_rotate3d(mat, quat + 4 * r);
        orc_project3d(priRotP, vol, vdim, pf, mat, iCol, iRow, nPxl);
        for (int t = 0; t < nT; t++) {
            cmul(priAllP, traP + 2 * (size_t)t * nPxl, priRotP, nPxl);
            float w = orc_logdatavs(dat, priAllP, ctf, sigRcp, nPxl);
            if (dvp) dvp[(size_t)r * nT + t] = w;
            baseLine = isnan(baseLine) ? w : baseLine;
            if (w > baseLine) {
                float nf = expf(baseLine - w);
                wC[0] *= nf;
                for (int q = 0; q < nR; q++) wR[q] *= nf;
                for (int q = 0; q < nT; q++) wT[q] *= nf;
                baseLine = w;
            }
            float s = expf(w - baseLine);
            wC[0] = (float)(wC[0] + s * (pR[r] * pT[t] * pD));
            wR[r] = (float)(wR[r] + s * (pC * pT[t] * pD));
            wT[t] = (float)(wT[t] + s * (pC * pR[r] * pD));
        }
    }
    *baseL = baseLine;
    free(traP);
    free(priRotP);
    free(priAllP);
}

/* a9, CTF search: the same phase over (r, t, d) with one CTF per defocus
 * sample (ctfD[nD][nPxl], orc_ctf_search) and the defocus priors pD --
 * src/Optimiser.cpp:1225-1427 with nC = 1; dvp[r][t][d] (the layout of
 * kernel_logDataVSLC, gpu/src/Kernel.cu:889-939). */
void orc_project2d(float* dst, const float* img, int vdim, int pf, const double* cs,
                   const int* iCol, const int* iRow, int nPxl);

/* twoD: the projection of the 2D branch (orc_project2d of the class image
 * at rotation rows (cos, sin), stride 2) instead of orc_project3d */
static void local_phase_d_impl(int twoD, const float* vol, int vdim, int pf, const double* quat,
                               int nR, const double* trans, int nT, int nD, double pC,
                               const double* pR, const double* pT, const double* pD,
                               const float* dat, const float* ctfD, const float* sigRcp,
                               const int* iCol, const int* iRow, int nPxl, int idim, float* wC,
                               float* wR, float* wT, float* wD, float* baseL, float* dvp)
{
    float* traP = (float*)malloc(sizeof(float) * 2 * (size_t)nT * nPxl);
    float* priRotP = (float*)malloc(sizeof(float) * 2 * nPxl);
    float* priAllP = (float*)malloc(sizeof(float) * 2 * nPxl);
    for (int t = 0; t < nT; t++)
        orc_translate(traP + 2 * (size_t)t * nPxl, (float)trans[2 * t],
                      (float)trans[2 * t + 1], idim, idim, iCol, iRow, nPxl);
    float baseLine = NAN;
    wC[0] = 0;
    for (int r = 0; r < nR; r++) wR[r] = 0;
    for (int t = 0; t < nT; t++) wT[t] = 0;
    for (int d = 0; d < nD; d++) wD[d] = 0;
    for (int r = 0; r < nR; r++) {
        if (twoD) {
            orc_project2d(priRotP, vol, vdim, pf, quat + 2 * r, iCol, iRow, nPxl);
        } else {
            double mat[9];
            orc_rotate3d(mat, quat + 4 * r);
            orc_project3d(priRotP, vol, vdim, pf, mat, iCol, iRow, nPxl);
        }
        for (int t = 0; t < nT; t++) {
            cmul(priAllP, traP + 2 * (size_t)t * nPxl, priRotP, nPxl);
            for (int d = 0; d < nD; d++) {
                float w = orc_logdatavs(dat, priAllP, ctfD + (size_t)d * nPxl, sigRcp, nPxl);
                if (dvp) dvp[((size_t)r * nT + t) * nD + d] = w;
                baseLine = isnan(baseLine) ? w : baseLine;
                if (w > baseLine) {
                    float nf = expf(baseLine - w);
                    wC[0] *= nf;
                    for (int q = 0; q < nR; q++) wR[q] *= nf;
                    for (int q = 0; q < nT; q++) wT[q] *= nf;
                    for (int q = 0; q < nD; q++) wD[q] *= nf;
                    baseLine = w;
                }
                float s = expf(w - baseLine);
                wC[0] = (float)(wC[0] + s * (pR[r] * pT[t] * pD[d]));
                wR[r] = (float)(wR[r] + s * (pC * pT[t] * pD[d]));
                wT[t] = (float)(wT[t] + s * (pC * pR[r] * pD[d]));
                wD[d] = (float)(wD[d] + s * (pC * pR[r] * pT[t]));
            }
        }
    }
    *baseL = baseLine;
    free(traP);
    free(priRotP);
    free(priAllP);
}

void orc_local_phase_d(const float* vol, int vdim, int pf, const double* quat, int nR,
                       const double* trans, int nT, int nD, double pC, const double* pR,
                       const double* pT, const double* pD, const float* dat,
                       const float* ctfD, const float* sigRcp, const int* iCol,
                       const int* iRow, int nPxl, int idim, float* wC, float* wR, float* wT,
                       float* wD, float* baseL, float* dvp)
{
    local_phase_d_impl(0, vol, vdim, pf, quat, nR, trans, nT, nD, pC, pR, pT, pD, dat, ctfD,
                       sigRcp, iCol, iRow, nPxl, idim, wC, wR, wT, wD, baseL, dvp);
}

/* f4 with CTF search: the 2D phase over (r, t, d) (the MODE_2D projection of
 * src/Optimiser.cpp:1277-1300 in the SEARCH_TYPE_CTF loop); rot: nR rows
 * (cos, sin) */
void orc_local_phase2d_d(const float* img, int vdim, int pf, const double* rot, int nR,
                         const double* trans, int nT, int nD, double pC, const double* pR,
                         const double* pT, const double* pD, const float* dat,
                         const float* ctfD, const float* sigRcp, const int* iCol,
                         const int* iRow, int nPxl, int idim, float* wC, float* wR, float* wT,
                         float* wD, float* baseL, float* dvp)
{
    local_phase_d_impl(1, img, vdim, pf, rot, nR, trans, nT, nD, pC, pR, pT, pD, dat, ctfD,
                       sigRcp, iCol, iRow, nPxl, idim, wC, wR, wT, wD, baseL, dvp);
}

/* --------------------------------------------------------------- a10 ---- */
int orc_resample(int nIn, const double* w, const double* u, int nOut,
                 double u0, int* ancestor, double* wOut)
{
    /* src/Particle.cpp:1343-1383 (PAR_R branch; PAR_T/PAR_C identical) */
    int maxIdx = 0; /* iMax: first index of the maximum of u */
    for (int i = 1; i < nIn; i++)
        if (u[i] > u[maxIdx]) maxIdx = i;
    double* ww = (double*)malloc(sizeof(double) * nIn);
    double* cdf = (double*)malloc(sizeof(double) * nIn);
    double sum = 0;
    for (int i = 0; i < nIn; i++) ww[i] = w[i] * u[i];
    for (int i = 0; i < nIn; i++) sum += ww[i];
    for (int i = 0; i < nIn; i++) ww[i] /= sum;
    double acc = 0;
    for (int i = 0; i < nIn; i++) { acc += ww[i]; cdf[i] = acc; } /* d_cumsum */
    double last = cdf[nIn - 1];
    for (int i = 0; i < nIn; i++) cdf[i] /= last;
    int i = 0;
    double s = 0;
    for (int j = 0; j < nOut; j++) {
        double uj = u0 + j * 1.0 / nOut;
        while (uj > cdf[i]) i++;
        ancestor[j] = i;
        wOut[j] = 1.0 / u[i]; /* PARTICLE_PRIOR_ONE */
    }
    for (int j = 0; j < nOut; j++) s += wOut[j];
    for (int j = 0; j < nOut; j++) wOut[j] /= s; /* normW */
    free(ww);
    free(cdf);
    return maxIdx;
}

/* --------------------------------------------------------------- a12 ---- */
static void add_ft_half(float* vol, int vdim, int ncomp, const float* value,
                        float x, float y, float z, int is_complex)
{
    /* Volume::addFT (src/Image/Volume.cpp:340-375) + addFTHalf (:565-712) */
    int conj = 0;
    if (!(x >= 0)) {
        x = -x; y = -y; z = -z;
        conj = 1;
    }
    float c[3] = {x, y, z};
    long x0[3];
    float v[3][2];
    for (int d = 0; d < 3; d++) {
        x0[d] = (long)floorf(c[d]);
        float xd = c[d] - (float)x0[d];
        v[d][0] = 1 - xd;
        v[d][1] = xd;
    }
    float vr = value[0];
    float vi = is_complex ? (conj ? -value[1] : value[1]) : 0;
    const long nColFT = vdim / 2 + 1;
    for (int k = 0; k < 2; k++)
        for (int j = 0; j < 2; j++)
            for (int i = 0; i < 2; i++) {
                float w = v[0][i] * v[1][j] * v[2][k];
                size_t idx = (size_t)(wrapi(x0[2] + k, vdim) * vdim +
                                      wrapi(x0[1] + j, vdim)) * nColFT +
                             (size_t)(x0[0] + i);
                vol[ncomp * idx] += vr * w;
                if (is_complex) vol[ncomp * idx + 1] += vi * w;
            }
}

void orc_insert3d(float* F, float* T, int vdim, const float* src,
                  const float* ctf, const double* mat, float w,
                  const int* iColPad, const int* iRowPad, int nPxl)
{
    /* src/Reconstructor.cpp:782-863 */
    for (int i = 0; i < nPxl; i++) {
        int iCol = iColPad[i], iRow = iRowPad[i];
        double ox = mat[0] * iCol + mat[3] * iRow;
        double oy = mat[1] * iCol + mat[4] * iRow;
        double oz = mat[2] * iCol + mat[5] * iRow;
        float val[2];
        val[0] = ((src[2 * i] * ctf[i]) * 1.0f) * w;
        val[1] = ((src[2 * i + 1] * ctf[i]) * 1.0f) * w;
        add_ft_half(F, vdim, 2, val, (float)ox, (float)oy, (float)oz, 1);
        float tv = ((float)((double)ctf[i] * ctf[i]) * 1.0f) * w;
        add_ft_half(T, vdim, 1, &tv, (float)ox, (float)oy, (float)oz, 0);
    }
}

void orc_insert_batch(float* F, float* T, double* O, long* counter, int vdim,
                      int pf, const float* dat, const float* ctf,
                      const double* quat, const double* trans,
                      const double* offS, const float* w, int nImg, int mReco,
                      const int* iCol, const int* iRow, int nPxl, int idim)
{
    /* src/Optimiser.cpp:7036-7241 (3D, OPTIMISER_RECENTRE_IMAGE_EACH_ITERATION) */
    float* tr = (float*)malloc(sizeof(float) * 2 * nPxl);
    int* iColPad = (int*)malloc(sizeof(int) * nPxl);
    int* iRowPad = (int*)malloc(sizeof(int) * nPxl);
    for (int i = 0; i < nPxl; i++) {
        iColPad[i] = iCol[i] * pf;
        iRowPad[i] = iRow[i] * pf;
    }
    for (int l = 0; l < nImg; l++)
        for (int m = 0; m < mReco; m++) {
            const double* q = quat + 4 * ((size_t)l * mReco + m);
            const double* t = trans + 2 * ((size_t)l * mReco + m);
            double dx = t[0] - offS[2 * l], dy = t[1] - offS[2 * l + 1];
            double mat[9];
            orc_rotate3d(mat, q);
            orc_translate_src(tr, dat + 2 * (size_t)l * nPxl, (float)(-dx),
                              (float)(-dy), idim, idim, iCol, iRow, nPxl);
            orc_insert3d(F, T, vdim, tr, ctf + (size_t)l * nPxl, mat, w[l],
                         iColPad, iRowPad, nPxl);
            /* insertDir(-rot3D * (dx, dy, 0)), src/Reconstructor.cpp:407-422 */
            O[0] += -(mat[0] * dx + mat[3] * dy);
            O[1] += -(mat[1] * dx + mat[4] * dy);
            O[2] += -(mat[2] * dx + mat[5] * dy);
            *counter += 1;
        }
    free(tr);
    free(iColPad);
    free(iRowPad);
}

/* a12 with CTF search: every sample (l, m) inserts with its own CTF,
 * CTF(defocusU * d, defocusV * d) of the image's attributes (src/Optimiser.cpp:
 * 7101-7120; GPU kernel_CalculateCTF, gpu/src/Kernel.cu:2206-2270); attr:
 * nImg x 8 as thx_ctf, nD: nImg x mReco defocus factors. */
void orc_insert_batch_d(float* F, float* T, double* O, long* counter, int vdim, int pf,
                        const float* dat, const float* attr, const double* nD,
                        const double* quat, const double* trans, const double* offS,
                        const float* w, int nImg, int mReco, const int* iCol, const int* iRow,
                        int nPxl, int idim)
{
    float* tr = (float*)malloc(sizeof(float) * 2 * nPxl);
    float* ctf = (float*)malloc(sizeof(float) * nPxl);
    int* iColPad = (int*)malloc(sizeof(int) * nPxl);
    int* iRowPad = (int*)malloc(sizeof(int) * nPxl);
    for (int i = 0; i < nPxl; i++) {
        iColPad[i] = iCol[i] * pf;
        iRowPad[i] = iRow[i] * pf;
    }
    for (int l = 0; l < nImg; l++)
        for (int m = 0; m < mReco; m++) {
            const size_t s = (size_t)l * mReco + m;
            const double* q = quat + 4 * s;
            const double* t = trans + 2 * s;
            const float* a = attr + 8 * (size_t)l;
            const double d = nD[s];
            double dx = t[0] - offS[2 * l], dy = t[1] - offS[2 * l + 1];
            double mat[9];
            orc_rotate3d(mat, q);
            orc_translate_src(tr, dat + 2 * (size_t)l * nPxl, (float)(-dx), (float)(-dy), idim,
                              idim, iCol, iRow, nPxl);
            orc_ctf(ctf, a[0], a[1], (float)(a[2] * d), (float)(a[3] * d), a[4], a[5], a[6], a[7],
                    idim, idim, iCol, iRow, nPxl);
            orc_insert3d(F, T, vdim, tr, ctf, mat, w[l], iColPad, iRowPad, nPxl);
            O[0] += -(mat[0] * dx + mat[3] * dy);
            O[1] += -(mat[1] * dx + mat[4] * dy);
            O[2] += -(mat[2] * dx + mat[5] * dy);
            *counter += 1;
        }
    free(tr);
    free(ctf);
    free(iColPad);
    free(iRowPad);
}

/* ------------------------------------------------------------ f4 (2D) --- */
void orc_project2d(float* dst, const float* img, int vdim, int pf, const double* cs,
                   const int* iCol, const int* iRow, int nPxl)
{
    /* Projector::project(Complex*, const dmat22&, ...) (src/Projector.cpp:337-354),
     * R = rotate2D(cs) (src/Geometry/Euler.cpp:125-131), then
     * Image::getByInterpolationFT (src/Image/Image.cpp:345-367): conjHalf,
     * WG_BI_INTERP_LINEAR (include/Functions/Interpolation.h:137-150), getFTHalf
     * summing the 2 x 2 taps row by row */
    const long nColFT = vdim / 2 + 1;
    for (int i = 0; i < nPxl; i++) {
        const double nx = (double)(iCol[i] * pf), ny = (double)(iRow[i] * pf);
        float x = (float)(cs[0] * nx - cs[1] * ny);
        float y = (float)(cs[1] * nx + cs[0] * ny);
        int conj = 0;
        if (!(x >= 0)) { x = -x; y = -y; conj = 1; }
        const float fx = floorf(x), fy = floorf(y);
        const int x0 = (int)fx, y0 = (int)fy;
        const float dx = x - fx, dy = y - fy;
        const float wx[2] = {1 - dx, dx}, wy[2] = {1 - dy, dy};
        float re = 0, im = 0;
        for (int j = 0; j < 2; j++) {
            int yy = y0 + j;
            if (yy < 0) yy += vdim;
            for (int a = 0; a < 2; a++) {
                const float w = wx[a] * wy[j];
                const float* v = img + 2 * ((size_t)yy * nColFT + x0 + a);
                re += v[0] * w;
                im += v[1] * w;
            }
        }
        dst[2 * i] = re;
        dst[2 * i + 1] = conj ? -im : im;
    }
}

void orc_insert2d_batch(float* F, float* T, double* O, long* counter, int vdim, int pf,
                        const float* dat, const float* ctf, const double* rot,
                        const double* trans, const double* offS, const float* w, const int* nc,
                        int nImg, int mReco, const int* iCol, const int* iRow, int nPxl, int idim)
{
    /* the 2D insert of src/Optimiser.cpp:6752-6850 (samples (cls, rot, tran)
     * from Particle::rand) -> Reconstructor::insertP(const Complex*, ...,
     * const dmat22&, ...) (src/Reconstructor.cpp:708-781, trilinear-kernel
     * branch = bilinear Image::addFT, src/Image/Image.cpp:369-409);
     * insertDir(-R (t - off)) (:397-401) */
    const long img = (long)(vdim / 2 + 1) * vdim;
    const long nColFT = vdim / 2 + 1;
    float* tr = (float*)malloc(sizeof(float) * 2 * nPxl);
    for (int l = 0; l < nImg; l++)
        for (int m = 0; m < mReco; m++) {
            const size_t sIdx = (size_t)l * mReco + m;
            const double* cs = rot + 2 * sIdx;
            const int k = nc ? nc[sIdx] : 0;
            float* Fk = F + 2 * img * k;
            float* Tk = T + img * k;
            const double dx = trans[2 * sIdx] - offS[2 * l], dy = trans[2 * sIdx + 1] - offS[2 * l + 1];
            orc_translate_src(tr, dat + 2 * (size_t)l * nPxl, (float)(-dx), (float)(-dy), idim,
                              idim, iCol, iRow, nPxl);
            for (int i = 0; i < nPxl; i++) {
                const double nx = (double)(iCol[i] * pf), ny = (double)(iRow[i] * pf);
                float x = (float)(cs[0] * nx - cs[1] * ny);
                float y = (float)(cs[1] * nx + cs[0] * ny);
                const float c = ctf[(size_t)l * nPxl + i];
                float vr = tr[2 * i] * c * w[l], vi = tr[2 * i + 1] * c * w[l];
                const float tv = (float)((double)c * c) * w[l];
                if (!(x >= 0)) { x = -x; y = -y; vi = -vi; }
                const float fx = floorf(x), fy = floorf(y);
                const int x0 = (int)fx, y0 = (int)fy;
                const float ddx = x - fx, ddy = y - fy;
                const float wx[2] = {1 - ddx, ddx}, wy[2] = {1 - ddy, ddy};
                for (int j = 0; j < 2; j++) {
                    int yy = y0 + j;
                    if (yy < 0) yy += vdim;
                    for (int a = 0; a < 2; a++) {
                        const float ww = wx[a] * wy[j];
                        const size_t q = (size_t)yy * nColFT + x0 + a;
                        Fk[2 * q] += vr * ww;
                        Fk[2 * q + 1] += vi * ww;
                        Tk[q] += tv * ww;
                    }
                }
            }
            O[2 * k] += -(cs[0] * dx - cs[1] * dy);
            O[2 * k + 1] += -(cs[1] * dx + cs[0] * dy);
            counter[k] += 1;
        }
    free(tr);
}

/* --------------------------------------------------------------- a14 ---- */
void orc_fsc(double* fsc, int nShell, const float* A, const float* B, int vdim)
{
    /* src/Functions/Spectrum.cpp:302-337 over VOLUME_FOR_EACH_PIXEL_FT
     * (include/Image/Volume.h:86-89); sums kept in double here (the reference
     * accumulates float with omp atomics in a dynamic order). */
    double* S = (double*)calloc(nShell, sizeof(double));
    double* SA = (double*)calloc(nShell, sizeof(double));
    double* SB = (double*)calloc(nShell, sizeof(double));
    const long nColFT = vdim / 2 + 1;
    for (long k = -vdim / 2; k < vdim / 2; k++)
        for (long j = -vdim / 2; j < vdim / 2; j++)
            for (long i = 0; i <= vdim / 2; i++) {
                double rr = sqrt((double)(i * i + j * j + k * k));
                int u = (int)rint(rr);
                if (u < nShell) {
                    size_t idx = (size_t)(wrapi(k, vdim) * vdim + wrapi(j, vdim)) *
                                     nColFT + (size_t)i;
                    float ar = A[2 * idx], ai = A[2 * idx + 1];
                    float br = B[2 * idx], bi = B[2 * idx + 1];
                    S[u] += (double)(ar * br - ai * (-bi));
                    SA[u] += (double)(ar * ar + ai * ai);
                    SB[u] += (double)(br * br + bi * bi);
                }
            }
    for (int i = 0; i < nShell; i++) {
        double AB = sqrt(SA[i] * SB[i]);
        fsc[i] = (AB == 0) ? 0 : S[i] / AB;
    }
    free(S);
    free(SA);
    free(SB);
}
