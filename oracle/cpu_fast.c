/*
 * cpu_fast.c -- the CPU baseline of bench.py ("FFTW/OpenMP CPU path" of
 * BASELINE.json, timed on the GPU node's host cores).
 *
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY: loaded by bench.py's cpu_baseline
 * leg (and its CPU test), never by the product package thunder_amd.
 *
 * The same workload as one bench step per image, organised like the
 * reference's CPU expectation (src/Optimiser.cpp:622-1681) and built
 * -O3 -march=native -fopenmp (oracle/Makefile):
 *   global scan: OpenMP over rotations (:756-759); per rotation the slice is
 *     extracted (Projector::project, src/Projector.cpp:356-374), then per
 *     translation priAllP = traP * priRotP (:793) and the likelihood of ALL
 *     images at once from pixel-major data (logDataVSPrior_m_n_huabin and its
 *     SIMD256 twin, :9931-9973 / :9222-9306: the inner loop runs over
 *     images, vectorised by the compiler); the online baseline and marginals
 *     of :834-894 accumulate per thread and merge at the end (the reference
 *     takes a per-image lock instead -- same sums, less contention);
 *   local phases: OpenMP over images (:1162); per phase and rotation the
 *     slice, per translation the likelihood over pixels
 *     (logDataVSPrior_m_huabin, :9187-9213, vectorised) and the online
 *     baseline + marginals (:1383-1402).
 * FP32 arithmetic as the reference's single-precision build; rotations FP64.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { float re, im; } cpx;

/* OpenMP threads of the parallel regions below (the caller's CPU share). */
void cpu_set_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

static void rotmat(const double* q, double* m)
{
    /* rotate3D, src/Geometry/Euler.cpp:181-189 (column-major) */
    const double A[3][3] = {{0, -q[3], q[2]}, {q[3], 0, -q[1]}, {-q[2], q[1], 0}};
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            double aa = 0;
            for (int k = 0; k < 3; k++) aa += (2 * A[r][k]) * A[k][c];
            m[c * 3 + r] = (r == c ? 1.0 : 0.0) + (2 * q[0]) * A[r][c] + aa;
        }
}

static inline int wrapi(int v, int n) { return v >= 0 ? v : v + n; }

/* Projector::project -> Volume::getByInterpolationFT (trilinear, Hermitian fold) */
static void project(const cpx* vol, int vdim, int pf, const double* m, const int* iCol,
                    const int* iRow, int nPxl, cpx* out)
{
    const int nc = vdim / 2 + 1;
    for (int i = 0; i < nPxl; i++) {
        const double nx = iCol[i] * pf, ny = iRow[i] * pf;
        float x = (float)(m[0] * nx + m[3] * ny);
        float y = (float)(m[1] * nx + m[4] * ny);
        float z = (float)(m[2] * nx + m[5] * ny);
        int conj = 0;
        if (!(x >= 0)) { x = -x; y = -y; z = -z; conj = 1; }
        const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
        const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
        const float dx = x - fx, dy = y - fy, dz = z - fz;
        const float wx[2] = {1 - dx, dx}, wy[2] = {1 - dy, dy}, wz[2] = {1 - dz, dz};
        float re = 0, im = 0;
        for (int k = 0; k < 2; k++)
            for (int j = 0; j < 2; j++) {
                const cpx* row = vol + ((size_t)wrapi(z0 + k, vdim) * vdim + wrapi(y0 + j, vdim)) * nc + x0;
                for (int a = 0; a < 2; a++) {
                    const float w = wx[a] * wy[j] * wz[k];
                    re += row[a].re * w;
                    im += row[a].im * w;
                }
            }
        out[i].re = re;
        out[i].im = conj ? -im : im;
    }
}

/* translate(Complex*, tx, ty, N, N, iCol, iRow, nPxl), ImageFunctions.cpp:233-252 */
static void trans_table(const double* t, int idim, const int* iCol, const int* iRow, int nPxl,
                        cpx* out)
{
    const float rCol = (float)t[0] / idim, rRow = (float)t[1] / idim;
    for (int i = 0; i < nPxl; i++) {
        const float ph = -2.f * (float)M_PI * (iCol[i] * rCol + iRow[i] * rRow);
        out[i].re = cosf(ph);
        out[i].im = sinf(ph);
    }
}

/*
 * One bench step for nImg images:
 *   scan over nR x nT (pixel set nPxl), then nPhase local phases of mR x mT
 *   samples per image (lquat: nImg x nPhase x mR x 4, ltrans: nImg x nPhase x
 *   mT x 2).  dat image-major Complex, ctf / sig image-major.
 * Outputs the scan baselines base[nImg] and the last phase's baselines
 * lbase[nImg] (returned so the work cannot be optimised away).
 */
void cpu_step(const float* volf, int vdim, int pf, const double* quat, int nR, const double* trans,
              int nT, const double* pR, const double* pT, const float* datf, const float* ctf,
              const float* sig, int nImg, const int* iCol, const int* iRow, int nPxl, int idim,
              const double* lquat, int mR, const double* ltrans, int mT, int nPhase,
              float* base, float* lbase)
{
    const cpx* vol = (const cpx*)volf;
    const cpx* dat = (const cpx*)datf;
    /* pixel-major copies for the scan (allocPreCal(pixelMajor = true), :636) */
    cpx* datP = malloc(sizeof(cpx) * (size_t)nPxl * nImg);
    float* ctfP = malloc(sizeof(float) * (size_t)nPxl * nImg);
    float* sigP = malloc(sizeof(float) * (size_t)nPxl * nImg);
    for (int l = 0; l < nImg; l++)
        for (int i = 0; i < nPxl; i++) {
            datP[(size_t)i * nImg + l] = dat[(size_t)l * nPxl + i];
            ctfP[(size_t)i * nImg + l] = ctf[(size_t)l * nPxl + i];
            sigP[(size_t)i * nImg + l] = sig[(size_t)l * nPxl + i];
        }
    cpx* traP = malloc(sizeof(cpx) * (size_t)nT * nPxl);
    for (int t = 0; t < nT; t++) trans_table(trans + 2 * t, idim, iCol, iRow, nPxl, traP + (size_t)t * nPxl);

    int nth = 1;
#ifdef _OPENMP
    nth = omp_get_max_threads();
#endif
    /* per-thread online accumulators: base, wC, wR (nR), wT (nT) per image */
    float* tBase = malloc(sizeof(float) * (size_t)nth * nImg);
    double* tC = calloc((size_t)nth * nImg, sizeof(double));
    double* tR = calloc((size_t)nth * nImg * nR, sizeof(double));
    double* tT = calloc((size_t)nth * nImg * nT, sizeof(double));
    for (size_t k = 0; k < (size_t)nth * nImg; k++) tBase[k] = NAN;

#pragma omp parallel
    {
        int th = 0;
#ifdef _OPENMP
        th = omp_get_thread_num();
#endif
        cpx* rot = malloc(sizeof(cpx) * nPxl);
        cpx* all = malloc(sizeof(cpx) * nPxl);
        float* res = malloc(sizeof(float) * nImg);
        float* B = tBase + (size_t)th * nImg;
        double* C = tC + (size_t)th * nImg;
        double* R = tR + (size_t)th * nImg * nR;
        double* Tt = tT + (size_t)th * nImg * nT;
#pragma omp for schedule(dynamic)
        for (int r = 0; r < nR; r++) {
            double m[9];
            rotmat(quat + 4 * r, m);
            project(vol, vdim, pf, m, iCol, iRow, nPxl, rot);
            for (int t = 0; t < nT; t++) {
                const cpx* tr = traP + (size_t)t * nPxl;
                for (int i = 0; i < nPxl; i++) {
                    all[i].re = tr[i].re * rot[i].re - tr[i].im * rot[i].im;
                    all[i].im = tr[i].re * rot[i].im + tr[i].im * rot[i].re;
                }
                memset(res, 0, sizeof(float) * nImg);
                /* logDataVSPrior_m_n_huabin: pixel-major, vectorised over images */
                for (int i = 0; i < nPxl; i++) {
                    const float pr = all[i].re, pi = all[i].im;
                    const cpx* d = datP + (size_t)i * nImg;
                    const float* c = ctfP + (size_t)i * nImg;
                    const float* s = sigP + (size_t)i * nImg;
#pragma omp simd
                    for (int l = 0; l < nImg; l++) {
                        const float er = d[l].re - c[l] * pr, ei = d[l].im - c[l] * pi;
                        res[l] += (er * er + ei * ei) * s[l];
                    }
                }
                for (int l = 0; l < nImg; l++) {
                    const float w = res[l];
                    if (isnan(B[l])) B[l] = w;
                    if (w > B[l]) {
                        const double nf = exp((double)(B[l] - w));
                        C[l] *= nf;
                        for (int k = 0; k < nR; k++) R[(size_t)l * nR + k] *= nf;
                        for (int k = 0; k < nT; k++) Tt[(size_t)l * nT + k] *= nf;
                        B[l] = w;
                    }
                    const double sx = exp((double)(w - B[l]));
                    C[l] += sx * pR[r] * pT[t];
                    R[(size_t)l * nR + r] += sx * pT[t];
                    Tt[(size_t)l * nT + t] += sx * pR[r];
                }
            }
        }
        free(rot); free(all); free(res);
    }
    /* merge the per-thread accumulators onto the common baseline */
    double* mR_ = calloc((size_t)nR, sizeof(double));
    double* mT_ = calloc((size_t)nT, sizeof(double));
    for (int l = 0; l < nImg; l++) {
        float b = NAN;
        for (int th = 0; th < nth; th++) {
            const float v = tBase[(size_t)th * nImg + l];
            if (!isnan(v) && (isnan(b) || v > b)) b = v;
        }
        base[l] = b;
        memset(mR_, 0, sizeof(double) * nR);
        memset(mT_, 0, sizeof(double) * nT);
        for (int th = 0; th < nth; th++) {
            const float v = tBase[(size_t)th * nImg + l];
            if (isnan(v)) continue;
            const double f = exp((double)(v - b));
            for (int k = 0; k < nR; k++) mR_[k] += f * tR[((size_t)th * nImg + l) * nR + k];
            for (int k = 0; k < nT; k++) mT_[k] += f * tT[((size_t)th * nImg + l) * nT + k];
        }
    }
    free(mR_); free(mT_);
    free(datP); free(ctfP); free(sigP); free(traP);
    free(tBase); free(tC); free(tR); free(tT);

    /* local phases: OpenMP over images (src/Optimiser.cpp:1162) */
#pragma omp parallel
    {
        cpx* rot = malloc(sizeof(cpx) * nPxl);
        cpx* all = malloc(sizeof(cpx) * nPxl);
        cpx* ltr = malloc(sizeof(cpx) * (size_t)mT * nPxl);
        double* wR = malloc(sizeof(double) * mR);
        double* wT = malloc(sizeof(double) * mT);
#pragma omp for schedule(dynamic)
        for (int l = 0; l < nImg; l++) {
            const cpx* d = dat + (size_t)l * nPxl;
            const float* c = ctf + (size_t)l * nPxl;
            const float* s = sig + (size_t)l * nPxl;
            float bl = NAN;
            for (int ph = 0; ph < nPhase; ph++) {
                const double* q = lquat + ((size_t)l * nPhase + ph) * mR * 4;
                const double* tt = ltrans + ((size_t)l * nPhase + ph) * mT * 2;
                for (int t = 0; t < mT; t++) trans_table(tt + 2 * t, idim, iCol, iRow, nPxl, ltr + (size_t)t * nPxl);
                float b = NAN;
                double wC = 0;
                memset(wR, 0, sizeof(double) * mR);
                memset(wT, 0, sizeof(double) * mT);
                for (int r = 0; r < mR; r++) {
                    double m[9];
                    rotmat(q + 4 * r, m);
                    project(vol, vdim, pf, m, iCol, iRow, nPxl, rot);
                    for (int t = 0; t < mT; t++) {
                        const cpx* tr = ltr + (size_t)t * nPxl;
                        float w = 0;
                        /* logDataVSPrior_m_huabin, vectorised over pixels */
#pragma omp simd reduction(+ : w)
                        for (int i = 0; i < nPxl; i++) {
                            const float pr = tr[i].re * rot[i].re - tr[i].im * rot[i].im;
                            const float pi = tr[i].re * rot[i].im + tr[i].im * rot[i].re;
                            const float er = d[i].re - c[i] * pr, ei = d[i].im - c[i] * pi;
                            w += (er * er + ei * ei) * s[i];
                        }
                        if (isnan(b)) b = w;
                        if (w > b) {
                            const double nf = exp((double)(b - w));
                            wC *= nf;
                            for (int k = 0; k < mR; k++) wR[k] *= nf;
                            for (int k = 0; k < mT; k++) wT[k] *= nf;
                            b = w;
                        }
                        const double sx = exp((double)(w - b));
                        wC += sx / ((double)mR * mT);
                        wR[r] += sx / mT;
                        wT[t] += sx / mR;
                    }
                }
                bl = b;
            }
            lbase[l] = bl;
        }
        free(rot); free(all); free(ltr); free(wR); free(wT);
    }
}
