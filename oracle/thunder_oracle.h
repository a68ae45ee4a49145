/*
 * thunder_oracle.h -- CPU restatement of THUNDER's expectation / insert hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product path (thunder_amd/) never links, loads or calls it.
 *
 * PARITY STATUS: "parity unpinned".  The reference (Low-power/THUNDER v1.4.14)
 * ships no golden vectors or known-answer tests for this path (its unit tests are
 * empty stubs), and its CPU path cannot be built here under this
 * round's rules: every hot-path translation unit includes include/Precision.h,
 * which pulls GSL 2.4 + FFTW 3.3.7 headers (vendored only as source packages,
 * i.e. external libraries) and Boost 1.60 (absent: .MISSING_LARGE_BLOBS).
 * Each function below therefore restates the reference algorithm line by line,
 * citing the file:line it follows, and is cross-checked in tests/ against
 * independent known answers (analytic Fourier transforms, closed-form CTF,
 * float64 re-derivations) rather than against reference outputs.
 *
 * Conventions (reference single-precision build, include/Precision.h:64-106):
 *   RFLOAT = float; Complex = float[2] interleaved (re, im);
 *   rotation matrices are double, column-major 3x3 (Eigen default, as used by
 *   src/Reconstructor.cpp:808-815); quaternions are double[4] (w, x, y, z).
 *   Half-complex volumes are [k][j][i] with i in [0, vdim/2] fastest, negative
 *   j/k wrapped by +vdim (include/Image/Volume.h:567-575).
 */
#ifndef THUNDER_ORACLE_H
#define THUNDER_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* a1: Optimiser::allocPreCalIdx (src/Optimiser.cpp:7991-8041).  Returns nPxl,
 * or -1 if cap is too small.  Any output pointer may be NULL. */
int orc_pixel_set(int N, int pf, float rU, float rL, int cap,
                  int* iCol, int* iRow, int* iSig, int* iPxl,
                  int* iColPad, int* iRowPad);

/* a2: CTF(RFLOAT* dst, ...) (src/CTF.cpp:113-151). */
void orc_ctf(float* dst, float pixelSize, float voltage, float defocusU,
             float defocusV, float theta, float Cs, float amplitudeContrast,
             float phaseShift, int nCol, int nRow, const int* iCol,
             const int* iRow, int nPxl);

/* a2, CTF search: allocPreCal's cSearch branch (src/Optimiser.cpp:8124-8170)
 * for one image (attr as thx_ctf), and the per-defocus-sample CTF of a local
 * phase (src/Optimiser.cpp:1252-1271, kernel_CalCTFL gpu/src/Kernel.cu:481). */
void orc_defocus_pre(const float* attr, const int* iCol, const int* iRow, int nPxl,
                     int idim, float* freq, float* defocusP, float* K1, float* K2);
void orc_ctf_search(float* ctfD, const float* defocusP, const float* freq, const double* d,
                    int nD, float K1, float K2, float phaseShift, float conT, int nPxl);

/* a9, CTF search: local phase over (r, t, d), dvp[r][t][d]
 * (src/Optimiser.cpp:1225-1427, nC = 1). */
void orc_local_phase_d(const float* vol, int vdim, int pf, const double* quat, int nR,
                       const double* trans, int nT, int nD, double pC, const double* pR,
                       const double* pT, const double* pD, const float* dat,
                       const float* ctfD, const float* sigRcp, const int* iCol,
                       const int* iRow, int nPxl, int idim, float* wC, float* wR, float* wT,
                       float* wD, float* baseL, float* dvp);
void orc_local_phase2d_d(const float* img, int vdim, int pf, const double* rot, int nR,
                       const double* trans, int nT, int nD, double pC, const double* pR,
                       const double* pT, const double* pD, const float* dat,
                       const float* ctfD, const float* sigRcp, const int* iCol,
                       const int* iRow, int nPxl, int idim, float* wC, float* wR, float* wT,
                       float* wD, float* baseL, float* dvp);

/* a12, CTF search: insert with a per-sample CTF(defocus x d)
 * (src/Optimiser.cpp:7101-7120). */
void orc_insert_batch_d(float* F, float* T, double* O, long* counter, int vdim, int pf,
                        const float* dat, const float* attr, const double* nD,
                        const double* quat, const double* trans, const double* offS,
                        const float* w, int nImg, int mReco, const int* iCol, const int* iRow,
                        int nPxl, int idim);

/* a4: translate(Complex* dst, tx, ty, ...) (src/Image/ImageFunctions.cpp:233-252). */
void orc_translate(float* dst, float nTransCol, float nTransRow, int nCol,
                   int nRow, const int* iCol, const int* iRow, int nPxl);

/* a4/a12: translate(Complex* dst, const Complex* src, ...)
 * (src/Image/ImageFunctions.cpp:471-492). */
void orc_translate_src(float* dst, const float* src, float nTransCol,
                       float nTransRow, int nCol, int nRow, const int* iCol,
                       const int* iRow, int nPxl);

/* a5: rotate3D(dmat33&, const dvec4&) (src/Geometry/Euler.cpp:181-189);
 * mat is column-major. */
void orc_rotate3d(double* mat, const double* quat);

/* a6: Projector::project(Complex*, const dmat33&, iCol, iRow, nPxl)
 * (src/Projector.cpp:356-374) over Volume::getByInterpolationFT
 * (src/Image/Volume.cpp:314-338) and getFTHalf (:491-563). */
void orc_project3d(float* dst, const float* vol, int vdim, int pf,
                   const double* mat, const int* iCol, const int* iRow,
                   int nPxl);

/* a7: logDataVSPrior_m_huabin (src/Optimiser.cpp:9187-9213). */
float orc_logdatavs(const float* dat, const float* pri, const float* ctf,
                    const float* sigRcp, int m);

/* a6+a7: dvp[l][r][t] for nImg images against nR rotations x nT translations,
 * the reference CPU global-scan arithmetic (src/Optimiser.cpp:756-826):
 * project per rotation, priAllP = traP * priRotP, then the likelihood. */
void orc_dvp_global(float* dvp, const float* vol, int vdim, int pf,
                    const double* quat, int nR, const double* trans, int nT,
                    const float* dat, const float* ctf, const float* sigRcp,
                    int nImg, const int* iCol, const int* iRow, int nPxl,
                    int idim, int nThreads);

/* a8: online baseline + weight accumulation of the CPU global scan
 * (src/Optimiser.cpp:834-894), class kIdx of nK, visiting (r, t) in order.
 * wC[nImg*nK], wR[nImg*nK*nR], wT[nImg*nK*nT], baseL[nImg] are read-modify-
 * write (baseL NaN = unset), exactly as the reference accumulates across
 * classes. */
void orc_weights_global(const float* dvp, int nImg, int nR, int nT,
                        const double* pR, const double* pT, int kIdx, int nK,
                        float* wC, float* wR, float* wT, float* baseL);

/* a6+a7+a9: one particle-filter phase of one image (src/Optimiser.cpp:
 * 1205-1402) with C = D = 1 (no CTF search).  quat[nR*4], trans[nT*2] are the
 * particle's own samples; pC, pR[nR], pT[nT] its current weights.  Outputs the
 * un-normalised likelihood marginals wC[1], wR[nR], wT[nT], the baseline and
 * (optionally) dvp[nR*nT]. */
void orc_local_phase(const float* vol, int vdim, int pf, const double* quat,
                     int nR, const double* trans, int nT, double pC,
                     const double* pR, const double* pT, const float* dat,
                     const float* ctf, const float* sigRcp, const int* iCol,
                     const int* iRow, int nPxl, int idim, float* wC,
                     float* wR, float* wT, float* baseL, float* dvp);

/* a10: systematic resampling of Particle::resample (src/Particle.cpp:
 * 1343-1383) applied to an already-shuffled set: w <- w*u, normalise, CDF,
 * u_j = u0 + j/nOut.  PARTICLE_PRIOR_ONE (include/Config.h:63): new prior
 * 1/u(ancestor), then normW() (src/Particle.cpp:815-821).  Returns the index of
 * max u (iMax, src/Particle.cpp:1880-1891). */
int orc_resample(int nIn, const double* w, const double* u, int nOut,
                 double u0, int* ancestor, double* wOut);

/* a12: Reconstructor::insertP(const Complex*, const RFLOAT*, const dmat33&,
 * RFLOAT w) (src/Reconstructor.cpp:782-863) with RECONSTRUCTOR_TRILINEAR_KERNEL
 * and RECONSTRUCTOR_ADD_T_DURING_INSERT; Volume::addFT (src/Image/Volume.cpp:
 * 340-375) and addFTHalf (:565-712).  F is complex (2 floats / voxel), T real. */
void orc_insert3d(float* F, float* T, int vdim, const float* src,
                  const float* ctf, const double* mat, float w,
                  const int* iColPad, const int* iRowPad, int nPxl);

/* a12 driver: the CPU insert loop of Optimiser::reconstructRef
 * (src/Optimiser.cpp:7036-7241, 3D branch, cSearch off): for each image and
 * each of mReco samples (quat, trans), translate by -(t - off), insertP with
 * w[l], insertDir(-R (t - off, 0)).  O[3] and counter accumulate. */
void orc_insert_batch(float* F, float* T, double* O, long* counter, int vdim,
                      int pf, const float* dat, const float* ctf,
                      const double* quat, const double* trans,
                      const double* offS, const float* w, int nImg, int mReco,
                      const int* iCol, const int* iRow, int nPxl, int idim);

/* a14: FSC(vec&, const Volume& A, const Volume& B) (src/Functions/
 * Spectrum.cpp:302-337); vdim = real-space box of A and B. */
void orc_fsc(double* fsc, int nShell, const float* A, const float* B,
             int vdim);

#ifdef __cplusplus
}
#endif
/* f4 (2D): Projector::project (2D) and the 2D insert */
void orc_project2d(float* dst, const float* img, int vdim, int pf, const double* cs,
                   const int* iCol, const int* iRow, int nPxl);
void orc_insert2d_batch(float* F, float* T, double* O, long* counter, int vdim, int pf,
                        const float* dat, const float* ctf, const double* rot,
                        const double* trans, const double* offS, const float* w, const int* nc,
                        int nImg, int mReco, const int* iCol, const int* iRow, int nPxl, int idim);

#endif
