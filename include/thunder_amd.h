/*
 * thunder_amd.h -- C-ABI of the MI355X (gfx950) expectation / insert engine.
 *
 * This is the drop-in boundary for THUNDER's GPU plugin surface
 * (gpu/interface/Interface.h:16-530, C++ free functions wrapping cuthunder::*).
 * Every entry point is extern "C", takes plain pointers and sizes, returns an
 * int status (THX_OK == 0) and never exits the process: the reference's
 * cudaCheckErrors -> exit(1) convention (gpu/config/Device.cuh.in:27-58)
 * becomes THX_ERR_* + thx_last_error().
 *
 * Two layers:
 *   1. Device-pointer kernels (thx_*): all array arguments are device pointers
 *      on the current HIP device, work is enqueued on `stream` (a hipStream_t,
 *      NULL = default stream) and nothing synchronises, allocates or frees, so
 *      callers may capture them into a HIP graph.  Scratch comes from a
 *      caller-provided workspace sized by the matching *_workspace() query.
 *   2. Reference-shaped host adapters (thx_Expect*, thx_InsertFT): the same
 *      argument lists and host-pointer ownership as Interface.h, stateless
 *      (allocate, copy, run, copy back, free), so gpu/interface/Interface.cpp can
 *      be replaced by one-line forwards.
 *
 * Data conventions (reference single-precision build, include/Precision.h):
 *   Complex = float[2] (re, im) interleaved; RFLOAT = float; rotations are
 *   double column-major 3x3 (Eigen, gpu/src/util/Mat33.cu:88-103);
 *   quaternions double[4] (w, x, y, z); translations double[2] in pixels.
 *   Half-complex volumes: [k][j][i], i in [0, vdim/2] fastest, negative j/k
 *   wrapped by +vdim (include/Image/Volume.h:567-575); dimSize =
 *   (vdim/2+1)*vdim*vdim.  Per-image arrays are image-major [l*nPxl + i]
 *   (allocPreCal(pixelMajor=false), src/Optimiser.cpp:8043-8083).
 */
#ifndef THUNDER_AMD_H
#define THUNDER_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define THX_ABI_VERSION 9

enum {
    THX_OK = 0,
    THX_ERR_ARG = 1,   /* invalid shape / argument / too-small workspace */
    THX_ERR_HIP = 2,   /* a HIP runtime call failed */
    THX_ERR_NOMEM = 3, /* host or device allocation failed (host adapters) */
};

typedef void* thx_stream_t; /* hipStream_t */

int thx_abi_version(void);
const char* thx_last_error(void);

/* ------------------------------------------------------------------ a1 ---
 * Pixel index set of Optimiser::allocPreCalIdx (src/Optimiser.cpp:
 * 7991-8041): half-plane pixels (i >= 0, skipping i == 0 && j < 0) with
 * rL^2 <= i^2+j^2 < rU^2 and rL <= round(|(i,j)|) < rU, in the loop order of
 * IMAGE_FOR_PIXEL_R_FT (include/Image/Image.h:68-70).  Host function.
 * Outputs (any may be NULL) need `cap` entries; *nPxl receives the count. */
int thx_pixel_set(int idim, int pf, float rU, float rL, int cap, int* iCol,
                  int* iRow, int* iSig, int* iPxl, int* nPxl);

/* Visiting order of the pixel set for the local phases (no reference
 * counterpart; the reference walks the set in allocPreCalIdx order): the
 * set is cut into 4 x 4 squares of (iCol, iRow), squares in serpentine row
 * order, inside a square its four 2 x 2 quads in turn, consecutive partial
 * squares (the disc edge) merged while they fit in 16 entries, every group
 * padded to 16 with -1.  Each 16-entry group of
 * `order` is then a compact patch whose slice neighbourhood fits in LDS
 * (thx_local_phase).  Host function; order: cap ints, *nOrd receives the
 * length (a multiple of 16; every pixel index appears exactly once). */
int thx_pixel_tile_order(const int* iCol, const int* iRow, int nPxl, int cap,
                         int* order, int* nOrd);

/* ------------------------------------------------------------------ a2 ---
 * Per-image CTF over the pixel set: CTF(RFLOAT* dst, ...) (src/CTF.cpp:
 * 113-151), computed on device instead of on the host in allocPreCal
 * (src/Optimiser.cpp:8088-8121).  attr: nImg x 8 floats {pixelSize, voltage,
 * defocusU, defocusV, defocusTheta, Cs, amplitudeContrast, phaseShift}
 * (CTFAttr, include/Database.h:302).  ctfP: nImg x nPxl. */
int thx_ctf(const float* attr, int nImg, const int* iCol, const int* iRow,
            int nPxl, int idim, float* ctfP, thx_stream_t stream);

/* ------------------------------------------------------------------ a3 ---
 * The global-search sample set.  thx_global_sample_sizes (host): the 3D
 * clamp mS >= 1500 (1 + nSymElem) (src/Optimiser.cpp:170-175), nR = mS /
 * (1 + nSymElem) in 3D (mode 1) or mS in 2D (mode 0), nT = max(30,
 * AROUND(pi (transS chi2Qinv(0.5, 2))^2 transSearchFactor)) (:1724-1745).
 * thx_global_sample_set (device): Particle::reset (src/Particle.cpp:87-169)
 * for 3D, C1 -- quat[nR*4] uniform on S^3 (sampleACG with the identity),
 * trans[nT*2] ~ N(0, transS^2 I), pR = 1/nR, pT = balanceWeight(PAR_T)
 * normalised; counter RNG (seed). */
int thx_global_sample_sizes(int mode, int mS, int nSymElem, double transS,
                            double transSearchFactor, int* mSOut, int* nR, int* nT);
int thx_global_sample_set(int nR, int nT, double transS, unsigned long long seed,
                          double* quat, double* trans, double* pR, double* pT,
                          thx_stream_t stream);

/* ------------------------------------------------------------------ a4 ---
 * Translation phase table traP[t][i] = exp(-2 pi i (iCol tx + iRow ty)/idim)
 * (translate(), src/Image/ImageFunctions.cpp:233-252; kernel_Translate,
 * gpu/src/Kernel.cu:443-473).  trans: nT x 2; traP: nT x nPxl Complex. */
int thx_trans_table(const double* trans, int nT, const int* iCol,
                    const int* iRow, int nPxl, int idim, float* traP,
                    thx_stream_t stream);

/* ------------------------------------------------------------------ a5 ---
 * Quaternion -> rotation matrix, rotate3D (src/Geometry/Euler.cpp:181-189;
 * kernel_getRotMat, gpu/src/Kernel.cu:572-617).  quat: n x 4; mat: n x 9. */
int thx_rotmat(const double* quat, int n, double* mat, thx_stream_t stream);

/* ------------------------------------------------------------------ a6 ---
 * Fourier-slice extraction, Projector::project(Complex*, const dmat33&, ...)
 * (src/Projector.cpp:356-374; kernel_Project3D, gpu/src/Kernel.cu:661-697):
 * rotP[r][i] = trilinear(vol, R_r (iCol*pf, iRow*pf, 0)).
 * vol: dimSize Complex; mat: nR x 9; rotP: nR x nPxl Complex. */
int thx_project3d(const float* vol, int vdim, int pf, const double* mat,
                  int nR, const int* iCol, const int* iRow, int nPxl,
                  float* rotP, thx_stream_t stream);

/* ------------------------------------------------------------------ a7 ---
 * Materialised log-likelihoods of the global scan, the arithmetic of
 * kernel_logDataVS (gpu/src/Kernel.cu:947-1004) and logDataVSPrior_m_huabin
 * (src/Optimiser.cpp:9187-9213):
 *   dvp[l][r][t] = sum_i sigRcp_li |dat_li - ctf_li (traP_ti * rotP_ri)|^2.
 * dat: nImg x nPxl Complex, ctf/sigRcp: nImg x nPxl, dvp: nImg x nR x nT. */
int thx_dvp(const float* rotP, int nR, const float* traP, int nT,
            const float* dat, const float* ctf, const float* sigRcp, int nImg,
            int nPxl, float* dvp, thx_stream_t stream);

/* ------------------------------------------------------------- a7 + a8 ---
 * Global scan of ExpectGlobal3D (gpu/interface/Interface.h:221-237;
 * cuthunder::expectGlobal3D, gpu/src/cuthunder.cu:1842-2198): likelihood of
 * every image against every (rotation, translation) sample of class kIdx and
 * the normalised marginals of the CPU online-baseline loop
 * (src/Optimiser.cpp:834-894):
 *   base_l   = max over visited classes, r, t of dvp
 *   wC[l][k] = sum_rt exp(dvp - base_l) pR[r] pT[t]
 *   wR[l][k][r] = sum_t exp(dvp - base_l) pT[t]
 *   wT[l][k][t] = sum_r exp(dvp - base_l) pR[r]
 * kIdx == 0 initialises wC/wR/wT/baseL; kIdx > 0 merges, rescaling earlier
 * classes when the baseline rises (kernel_setBaseLine, Kernel.cu:1096-1128).
 * algo: 0 = direct per-pixel formulation, materialised dvp;
 *       1 = fused FP32 MFMA formulation;
 *       2 = bf16 MFMA, three-product split (bf16x3, ~2^-16 per product);
 *       4 = bf16 MFMA, exact three-way split of both FP32 operands and six
 *           products (bf16x6: the dropped m l and l m are <= 2^-24 |w||T|
 *           each, about 2^-23 together -- comparable to the FP32 rounding of
 *           a product) -- the expectation driver's default;
 *       (3, fp16x2, was retired in ABI 9);
 *       2 and 4 run the cancellation guard (samples whose expanded form
 *       A + B + X cancels by more than 4x are recomputed in the direct form)
 *       and fall back to 1 when nT > 160.
 * workspace: >= thx_global_scan_workspace(...) bytes of device memory. */
size_t thx_global_scan_workspace(int nImg, int nR, int nT, int nPxl, int algo);
int thx_global_scan(const float* rotP, int nR, const float* traP, int nT,
                    const float* dat, const float* ctf, const float* sigRcp,
                    int nImg, int nPxl, const double* pR, const double* pT,
                    int kIdx, int nK, float* wC, float* wR, float* wT,
                    float* baseL, int algo, void* workspace, size_t wsBytes,
                    thx_stream_t stream);

/* thx_global_scan for algo 2 or 4 with two debug controls (ABI 9): dvp
 * [nImg][nR][nT] (optional, NULL = no dump) receives every sample's final
 * log-likelihood (the value the marginals are formed from), for the
 * element-wise dump-compare of gpu/src/cuthunder.cu:2247-2271; guard = the
 * cancellation ratio above which a sample is recomputed in the direct form
 * (thx_global_scan uses 4; 0 turns the guard off).  A dump needs nT <= 160. */
int thx_global_scan_dvp(const float* rotP, int nR, const float* traP, int nT,
                        const float* dat, const float* ctf, const float* sigRcp,
                        int nImg, int nPxl, const double* pR, const double* pT,
                        int kIdx, int nK, float* wC, float* wR, float* wT,
                        float* baseL, int algo, float guard, float* dvp,
                        void* workspace, size_t wsBytes, thx_stream_t stream);

/* --------------------------------------------------------- a6 + a7 + a9 ---
 * One particle-filter phase for a batch of images, each with its own
 * rotation / translation samples: fused projection + likelihood + per-image
 * normalisation (src/Optimiser.cpp:1205-1402; ExpectLocalPreI3D +
 * ExpectLocalM, gpu/src/cuthunder.cu:2834-3140, kernel_Project3DL,
 * kernel_logDataVSL, kernel_getMaxBaseL, kernel_UpdateWL).
 *   quat: nImg x nR x 4, trans: nImg x nT x 2, pC: nImg, pR: nImg x nR,
 *   pT: nImg x nT (double priors, as Particle::wC/wR/wT).
 * Outputs wC[nImg], wR[nImg x nR], wT[nImg x nT], baseL[nImg] (float, like
 * the reference's RFLOAT vec) and, if dvp != NULL, dvp[nImg x nR x nT].
 * volLayout 0: `vol` is the half-complex projectee; 1: `vol` is its
 * cell-expanded copy from thx_volume_cells (8x the bytes, one aligned 64-B
 * segment per trilinear gather -- the layout for HBM-bound full-resolution
 * phases); 2: `vol` is its y-pair copy from thx_volume_ypair (2x the bytes,
 * two 32-B pieces per gather, read by lane pairs -- the layout for wide
 * clouds on an L2-resident ball).  (ABI 6 retired the bricked layout and the
 * quad form of the y-pair gather, volLayout 2 / 3 of ABI 5.)
 * pxOrder (device, nOrd ints, may be NULL = set order, nOrd ignored): the
 * pixel visiting order from thx_pixel_tile_order (-1 entries skipped).
 * Pixels are taken 16 at a time; when the
 * Hermitian-folded neighbourhood of a 16-pixel patch under the workgroup's
 * 128 rotations fits in LDS it is staged there once and the 8 taps of every
 * sample are read from LDS, otherwise straight from `vol`.  The order only
 * changes the FP32 summation order over pixels, not which taps are summed.
 * workspace (required): >= thx_local_phase_workspace(nImg, nR, nT, nVisit)
 * bytes, nVisit = nOrd with pxOrder, nPxl without. */
size_t thx_local_phase_workspace(int nImg, int nR, int nT, int nVisit);
int thx_local_phase(const float* vol, int volLayout, int vdim, int pf,
                    const double* quat,
                    int nR, const double* trans, int nT, const double* pC,
                    const double* pR, const double* pT, const float* dat,
                    const float* ctf, const float* sigRcp, const int* iCol,
                    const int* iRow, const int* pxOrder, int nOrd, int nPxl,
                    int idim, int nImg, float* wC,
                    float* wR, float* wT, float* baseL, float* dvp,
                    void* workspace, size_t wsBytes, thx_stream_t stream);

/* Image selection for the same phase (the expectation driver's own use, and
 * a C++ host's): `active` / `nActive` (device; both or neither) restrict the
 * launch to images active[0 .. *nActive) -- the grid is sized by nImg and
 * slots past the count exit at once, so the host never reads the count -- and
 * `cls` (device, nImg, may be NULL) makes image l project class cls[l]'s
 * volume, vol + cls[l] * volStride float2 elements (K-class classification:
 * the phases run on the class the reseed drew, src/Optimiser.cpp:1957-1965).
 * Per-image arrays keep their nImg-row layout. */
typedef struct thx_local_sel {
    const int* active;
    const int* nActive;
    const int* cls;
    long long volStride;
} thx_local_sel;
int thx_local_phase_sel(const thx_local_sel* sel, const float* vol, int volLayout,
                        int vdim, int pf, const double* quat, int nR,
                        const double* trans, int nT, const double* pC,
                        const double* pR, const double* pT, const float* dat,
                        const float* ctf, const float* sigRcp, const int* iCol,
                        const int* iRow, const int* pxOrder, int nOrd, int nPxl,
                        int idim, int nImg, float* wC, float* wR, float* wT,
                        float* baseL, float* dvp, void* workspace, size_t wsBytes,
                        thx_stream_t stream);

/* The phase on the device route (what thx_expectation runs for half-complex
 * phases without CTF search): a sample of every 16th image's patch records
 * picks, on the device, the LDS-staged half-complex kernel where the patch
 * boxes of the clouds fit (>= 50 %) and otherwise the pair-form y-pair kernel
 * on `ypair` (thx_volume_ypair of vol), or the box-less half-complex kernel
 * when ypair is NULL; no host round trip.  route (device int, may be NULL)
 * receives the choice: 0 staged, 1 box-less, 2 y-pair, -1 not routed (the
 * large-box full-resolution phases, pf sqrt(2 nPxl / pi) >= 300, run the
 * big-box staged kernel).  pxOrder is required; the rest as
 * thx_local_phase_sel with volLayout 0. */
int thx_local_phase_routed(const thx_local_sel* sel, const float* vol,
                           const float* ypair, int vdim, int pf, const double* quat,
                           int nR, const double* trans, int nT, const double* pC,
                           const double* pR, const double* pT, const float* dat,
                           const float* ctf, const float* sigRcp, const int* iCol,
                           const int* iRow, const int* pxOrder, int nOrd, int nPxl,
                           int idim, int nImg, float* wC, float* wR, float* wT,
                           float* baseL, float* dvp, int* route, void* workspace,
                           size_t wsBytes, thx_stream_t stream);

/* The compact y-pair ball the expectation driver gathers from (ABI 9; the
 * copy every bench phase reads): elements (x, y, z), 0 <= x < R + 2,
 * -R <= y, z < R + 2, each (v(x, y, z), v(x, y+1, z)) without wrap, the
 * slices z, z+1 (z + R even) interleaved element by element; R = ceil(pf
 * r_max) + 2 for a pixel ring of radius r_max (max sqrt(iCol^2 + iRow^2)).
 * thx_ypair_ball_elems(R): float4 elements of the ball (0 for R <= 0). */
size_t thx_ypair_ball_elems(int R);
int thx_volume_ypair_ball(const float* vol, int vdim, int R, float* ball, thx_stream_t stream);
/* thx_local_phase_routed with the ball as its y-pair copy (the driver's
 * call); checks on the device's pixel set that pf r_max + 2 <= ballR (one
 * read-back, so not graph-capturable) before any gather. */
int thx_local_phase_routed_ball(const thx_local_sel* sel, const float* vol,
                                const float* ball, int ballR, int vdim, int pf,
                                const double* quat, int nR, const double* trans, int nT,
                                const double* pC, const double* pR, const double* pT,
                                const float* dat, const float* ctf, const float* sigRcp,
                                const int* iCol, const int* iRow, const int* pxOrder,
                                int nOrd, int nPxl, int idim, int nImg, float* wC,
                                float* wR, float* wT, float* baseL, float* dvp,
                                int* route, void* workspace, size_t wsBytes,
                                thx_stream_t stream);

/* The image order thx_expectation's 3D phases use (the active list of
 * thx_local_phase_sel): images stably sorted by the Hilbert index (16-bit
 * cells) of the octahedral map of their slice normal n = R(q) e_z, q = the first
 * particle quat[l][0] of the cloud, n and -n one plane (n_z >= 0).  The
 * workgroups in flight then gather from one slab of the projectee, which
 * stays in an XCD's L2; per-image results do not depend on the order.
 * ord (device, nImg ints) receives the permutation; workspace >=
 * thx_view_order_workspace(nImg) bytes. */
size_t thx_view_order_workspace(int nImg);
int thx_view_order(int nImg, int mLR, const double* quat, int* ord, void* workspace,
                   size_t wsBytes, thx_stream_t stream);

/* ---------------------------------------------------- CTF search (a2/a9) ---
 * SEARCH_TYPE_CTF: the local phase over nD defocus samples per image.
 * thx_defocus_pre -- allocPreCal's cSearch branch (src/Optimiser.cpp:
 *   8124-8170) on device: freq[nPxl] (may be NULL), defocusP[nImg][nPxl],
 *   K1[nImg], K2[nImg] from attr (nImg x 8, as thx_ctf).
 * thx_ctf_search -- kernel_CalCTFL (gpu/src/Kernel.cu:481-515; CPU
 *   src/Optimiser.cpp:1252-1271): ctfD[nImg][nD][nPxl] for the defocus
 *   factors dD[nImg][nD]; phase shift and amplitude contrast from attr.
 * thx_local_phase_d -- thx_local_phase_sel over (r, t, d) triples
 *   (kernel_logDataVSLC + kernel_UpdateWLC, gpu/src/Kernel.cu:889-939,
 *   1459-1554; CPU src/Optimiser.cpp:1225-1427): ctfD as above, pD[nImg][nD]
 *   the defocus priors, wD[nImg][nD] their marginals; dvp (optional)
 *   [nImg][nR][nT][nD]; nT * nD <= 1024; workspace
 *   thx_local_phase_workspace(nImg, nR, nT * nD, nVisit); sel may be NULL. */
int thx_defocus_pre(const float* attr, int nImg, const int* iCol, const int* iRow,
                    int nPxl, int idim, float* freq, float* defocusP, float* K1,
                    float* K2, thx_stream_t stream);
int thx_ctf_search(const float* defocusP, const float* freq, const double* dD,
                   int nD, const float* K1, const float* K2, const float* attr,
                   int nImg, int nPxl, float* ctfD, thx_stream_t stream);
int thx_local_phase_d(const thx_local_sel* sel, const float* vol, int volLayout,
                      int vdim, int pf, const double* quat, int nR,
                      const double* trans, int nT, int nD, const double* pC,
                      const double* pR, const double* pT, const double* pD,
                      const float* dat, const float* ctfD, const float* sigRcp,
                      const int* iCol, const int* iRow, const int* pxOrder, int nOrd,
                      int nPxl, int idim, int nImg, float* wC, float* wR, float* wT,
                      float* wD, float* baseL, float* dvp, void* workspace,
                      size_t wsBytes, thx_stream_t stream);

/* Cell-expanded copy of a half-complex volume: cells[(k*vdim + j)*(vdim/2+1)
 * + i] holds the 8 Complex taps v(i+dx, j+dy, k+dz), (dz, dy, dx) in the box
 * order of getFTHalf (src/Image/Volume.cpp:491-563), rows / slices wrapped,
 * i + 1 past the half plane zero.  cells: 8 * dimSize Complex. */
int thx_volume_cells(const float* vol, int vdim, float* cells,
                     thx_stream_t stream);

/* The y-pair copy of a half-complex projectee (thx_local_phase volLayout 2):
 * element (x, y, z) holds v(x, y, z) and v(x, (y + 1) mod vdim, z) (16 B), so
 * a trilinear cell is two 32-B pieces; the slices z, z + 1 of each even z are
 * interleaved element by element -- element (x, y, z) sits at index
 * ((z / 2 * vdim + y) * (vdim / 2 + 1) + x) * 2 + z % 2 -- so for even z0 a
 * cell is one contiguous 64-B piece.  ypair: 4 dimSize floats (ABI 8). */
int thx_volume_ypair(const float* vol, int vdim, float* ypair, thx_stream_t stream);

/* ----------------------------------------------------------------- a10 ---
 * Systematic resampling of Particle::resample (src/Particle.cpp:1291-1478)
 * for nImg particles at once, on an already shuffled support: w <- w*u,
 * normalise, CDF, u_j = u0 + j/nOut; ancestor[j]; new prior 1/u[ancestor]
 * (PARTICLE_PRIOR_ONE, include/Config.h:63) normalised (normW,
 * src/Particle.cpp:815-821); iMax = first argmax of u.
 *   w: nImg x nIn double, u: nImg x nIn float, u0: nImg double,
 *   ancestor: nImg x nOut int, wOut: nImg x nOut double, iMax: nImg int. */
int thx_resample(int nImg, int nIn, const double* w, const float* u,
                 int nOut, const double* u0, int* ancestor, double* wOut,
                 int* iMax, thx_stream_t stream);

/* The expectation driver's resampling step (k_pf_resample, used by
 * thx_expectation): Particle::resample (src/Particle.cpp:1291-1478) for nImg
 * images at once, one wave per image -- shuffle(pt) first when `shuffle`
 * (src/Particle.cpp:1298, 2202-2300; a uniform permutation from the counter
 * RNG keyed by (seed, image, stream_id)), then iMax = first maximum of u in
 * shuffled order, the CDF of w*u in shuffled order and the systematic draw
 * u_j = u0 + j/nOut, u0 ~ U(0, 1/nOut).  Outputs are element indices of the
 * unshuffled support.  w: nImg rows at stride ldw (0 = one row shared by all
 * images), u: float rows at stride ldu; w and wOut may alias (ldw == nOut ==
 * nIn).  perm (optional, nImg x nIn): the permutation, position i of the
 * shuffled support holds element perm[i]; u0 (optional, nImg): the draws.
 * workspace: >= thx_pf_resample_workspace(nImg, nIn) bytes. */
size_t thx_pf_resample_workspace(int nImg, int nIn);
int thx_pf_resample(int nImg, int nIn, int nOut, const double* w, int ldw,
                    const float* u, int ldu, unsigned long long seed,
                    unsigned stream_id, int shuffle, int* anc, double* wOut,
                    int* iMax, int* perm, double* u0, void* workspace,
                    size_t wsBytes, thx_stream_t stream);

/* Particle statistics of the particle filter, one image per wave, nImg at a
 * time (device pointers; FP64 particles, FP32 marginals):
 * thx_pf_calvari -- Particle::calVari, 3D (src/Particle.cpp:1004-1121):
 *   k[3 l + j-1] = max(kFloor, A(j,j)/A(0,0)) of inferACG
 *   (src/Geometry/DirectionalStat.cpp:93-222) on the cloud de-meaned by its
 *   ACG principal axis; sd[2 l + c] = max(sFloor, gsl_stats_sd(t_c)).
 *   quat: nImg x mR x 4, trans: nImg x mT x 2.  The de-meaned fixed point is
 *   the first one's iterates replayed through the de-meaning rotation (equal
 *   in exact arithmetic); their history takes 20 KB per image of
 *   stream-ordered scratch (hipMallocAsync on `stream`) for the call.
 * thx_pf_balance_rot -- Particle::balanceWeight(PAR_R), 3D
 *   (src/Particle.cpp:2330-2340): pR = 1/pdfACG(q, inferACG(Q)), normalised.
 * thx_pf_peak -- Particle::setPeakFactor(PAR_R) (src/Particle.cpp:1920-1925,
 *   when setFactor) and keepHalfHeightPeak (:1964-1984) on u in place:
 *   u: nImg rows of n floats at stride ldu, peak: nImg doubles (out / in). */
int thx_pf_calvari(int nImg, int mR, const double* quat, int mT, const double* trans,
                   double kFloor, double sFloor, double* k, double* sd, thx_stream_t stream);
int thx_pf_balance_rot(int nImg, int mR, const double* quat, double* pR, thx_stream_t stream);
/* Defocus particles of a CTF search (nImg x mD, one image per 16 lanes):
 * op 0 initD (src/Particle.cpp:281-310): d = 1 + N(0, arg), pD =
 * balanceWeight(PAR_D) (:2374-2409); op 1 perturb(arg, PAR_D) (:1278-1288):
 * d += N(0, sd[l]) arg, pD as op 0; op 2 calVari(PAR_D) (:1120-1141): sd[l]
 * = sample standard deviation (0 for mD = 1).  Counter RNG (seed, stream_id). */
int thx_pf_defocus(int nImg, int mD, int op, double arg, unsigned long long seed,
                   unsigned stream_id, double* d, double* pD, double* sd,
                   thx_stream_t stream);
int thx_pf_peak(int nImg, int n, float* u, int ldu, double* peak, int setFactor,
                thx_stream_t stream);

/* ----------------------------------------------------------------- a12 ---
 * Weighted trilinear Fourier-space back-projection of the CPU insert loop
 * (src/Optimiser.cpp:7036-7241 -> Reconstructor::insertP, src/Reconstructor.
 * cpp:782-863 -> Volume::addFT, src/Image/Volume.cpp:340-375) and of
 * cuthunder::InsertFT (gpu/src/cuthunder.cu:5249-5826; kernel_Translate
 * :2088, kernel_InsertT :2959, kernel_InsertF :3000, kernel_InsertO3D :3048):
 * for image l, sample m: src = dat_l * exp(+2 pi i (i (tx-offx) + j (ty-offy))/idim),
 * F += src ctf w_l and T += ctf^2 w_l scattered trilinearly at
 * R_m (iCol*pf, iRow*pf, 0) (Hermitian fold conjugates the F value),
 * O += -R_m (t - off, 0) and counter += 1 (insertDir, src/Reconstructor.cpp:
 * 407-422).  F: dimSize Complex, T: dimSize float, O: 3 double, counter: 1
 * int (all accumulated, not cleared).  quat: nImg x mReco x 4,
 * trans: nImg x mReco x 2, offS: nImg x 2, w: nImg.  nC (device, nImg, may
 * be NULL): image l inserts only its first nC[l] samples -- the K-class call
 * of InsertFT (gpu/interface/Interface.h:267-292, cuthunder.cu:4115), where
 * each class's reconstructor receives mReco = the largest per-image count of
 * samples that drew it and nC[l] = image l's count (src/Optimiser.cpp:
 * 6852-6950); O and counter see only the inserted samples. */
int thx_insert3d(float* F, float* T, double* O, int* counter, int vdim,
                 int pf, const float* dat, const float* ctf,
                 const double* quat, const double* trans, const double* offS,
                 const float* w, const int* nC, int nImg, int mReco, const int* iCol,
                 const int* iRow, int nPxl, int idim, thx_stream_t stream);

/* Same insert, pixels visited in thx_pixel_tile_order patches (pxOrder:
 * device, nOrd ints): per (image, patch) the samples are accumulated in an
 * LDS copy of the patch's neighbourhood (the local phase's patch boxes) and
 * flushed row by row, so the memory-side atomics run on contiguous rows
 * instead of one row per lane.  Values and coordinates as thx_insert3d; the
 * FP32 summation order differs.  workspace: >= thx_insert3d_workspace bytes
 * of device memory. */
size_t thx_insert3d_workspace(int nImg, int mReco, int nOrd);
int thx_insert3d_tiled(float* F, float* T, double* O, int* counter, int vdim,
                       int pf, const float* dat, const float* ctf,
                       const double* quat, const double* trans,
                       const double* offS, const float* w, const int* nC, int nImg, int mReco,
                       const int* iCol, const int* iRow, const int* pxOrder,
                       int nOrd, int nPxl, int idim, void* workspace,
                       size_t wsBytes, thx_stream_t stream);

/* Same insert as a binned deposition (the default of the host front end):
 * samples of an image with bitwise-identical quaternions are merged (their
 * taps coincide), every (group, pixel) entry is binned to a 16^3 tile of the
 * half-map, and each tile is summed in LDS and flushed once per chunk of
 * entries.  rMax: bound on the pixel radius sqrt(iCol^2 + iRow^2) (rU of the
 * pixel set; pixels beyond it are still inserted, by direct atomics).
 * Requires mReco <= 1024 and (pf rMax + 2) <= vdim/2 - 1; the tile grid
 * (2 pf rMax / 16)^2 (pf rMax / 16) must stay within 16384 tiles.  Values and
 * coordinates as thx_insert3d; the FP32 summation order differs.
 * workspace: >= thx_insert3d_binned_workspace bytes (entries of at most
 * 2^28 per image batch, 24 B each). */
size_t thx_insert3d_binned_workspace(int nImg, int mReco, int nOrd, int pf, int rMax);
int thx_insert3d_binned(float* F, float* T, double* O, int* counter, int vdim, int pf,
                        const float* dat, const float* ctf, const double* quat,
                        const double* trans, const double* offS, const float* w,
                        const int* nC, int nImg, int mReco, const int* iCol, const int* iRow,
                        const int* pxOrder, int nOrd, int nPxl, int idim, int rMax,
                        void* workspace, size_t wsBytes, thx_stream_t stream);
/* The same with CTF search (InsertFT's cSearch, src/Optimiser.cpp:7101-7120;
 * kernel_CalculateCTF gpu/src/Kernel.cu:2206-2270): sample (l, m) inserts with
 * CTF(defocusU nD[l][m], defocusV nD[l][m]) of image l's attributes attr
 * (nImg x 8, as thx_ctf) instead of a per-image ctf row. */
int thx_insert3d_binned_d(float* F, float* T, double* O, int* counter, int vdim,
                          int pf, const float* dat, const float* attr,
                          const double* nD, const double* quat, const double* trans,
                          const double* offS, const float* w, const int* nC, int nImg,
                          int mReco, const int* iCol, const int* iRow,
                          const int* pxOrder, int nOrd, int nPxl, int idim, int rMax,
                          void* workspace, size_t wsBytes, thx_stream_t stream);

/* ----------------------------------------------------------------- a13 ---
 * The per-hemisphere half-map reduction of cuthunder::InsertFT
 * (gpu/src/cuthunder.cu:5294-5324 communicator setup, :5903-5993 the
 * all-reduces; CPU twin Reconstructor::allReduceF/T/O,
 * src/Reconstructor.cpp:2350-2520) over RCCL.  One process per GPU: the
 * communicator spans the ranks of one hemisphere.  The host moves the
 * THX_RCCL_ID_BYTES unique id from the hemisphere's first rank to the others
 * (MPI_Bcast over `hemi` in THUNDER, as the reference does).
 * thx_halfmap_allreduce sums in place, as one RCCL group on `stream`:
 * F (2 dimSize nK floats), T (dimSize nK floats), O (3 nK doubles, may be
 * NULL) and counter (nK int32, may be NULL; the reference's ncclInt64 on an
 * int, quirk q2, is not replicated). */
#define THX_RCCL_ID_BYTES 128
int thx_rccl_unique_id(void* id);
int thx_rccl_comm_init(int nranks, const void* id, int rank, void** comm);
int thx_rccl_comm_destroy(void* comm);
int thx_halfmap_allreduce(void* comm, float* F, float* T, double* O, int* counter,
                          long long dimSize, int nK, thx_stream_t stream);
/* The hemispheres' hand-over for the FSC of Model::compareTwoHemispheres
 * (src/Model.cpp:307-852, MPI_Recv_Large of the A and B maps on the master):
 * send nSend floats to rank peerSend and receive nRecv floats from rank
 * peerRecv of `comm` (a communicator over both hemispheres' leads), one RCCL
 * group on `stream`; either side may be NULL. */
int thx_halfmap_sendrecv(void* comm, const float* send, long long nSend, int peerSend,
                         float* recv, long long nRecv, int peerRecv, thx_stream_t stream);

/* ------------------------------------------------------------------ f4 ---
 * The 2D classification path (MODE_2D).  2D projectees / half-maps are
 * half-complex images [vdim][vdim/2+1]; a 2D rotation is (cos, sin) (the
 * particle's (_r(i,0), _r(i,1)) -> rotate2D, src/Geometry/Euler.cpp:125-131).
 * thx_project2d -- Projector::project(Complex*, const dmat22&, ...)
 *   (src/Projector.cpp:337-354; kernel_Project2D, gpu/src/Kernel.cu:786):
 *   rotP[r][i] = bilinear(vol, R_r (iCol pf, iRow pf)).  rot: nR x 2.
 * thx_local_phase2d -- one particle-filter phase of the 2D branch of
 *   src/Optimiser.cpp:1183-1402 for a batch (per image mR rotations [nImg][mR][2],
 *   mT translations, priors as thx_local_phase; cls (device, may be NULL):
 *   image l projects class cls[l] of the nK images at vol); direct likelihood,
 *   per-image marginals; dvp optional (else workspace >=
 *   thx_local_phase2d_workspace).
 * thx_insert2d -- the 2D insert (Reconstructor::insertP, src/Reconstructor.cpp:
 *   708-781; kernel_InsertF2D / T2D / O2D, gpu/src/Kernel.cu:2276-2500): F, T
 *   hold nK class half-maps back to back, O nK x 2, counter nK; rot / trans:
 *   nImg x mReco x 2; nc (may be NULL = class 0): nImg x mReco class of each
 *   sample. */
int thx_project2d(const float* vol, int vdim, int pf, const double* rot, int nR,
                  const int* iCol, const int* iRow, int nPxl, float* rotP,
                  thx_stream_t stream);
size_t thx_local_phase2d_workspace(int nImg, int nR, int nT);
int thx_local_phase2d(const float* vol, int vdim, int pf, const int* cls, const double* rot,
                      int nR, const double* trans, int nT, const double* pC, const double* pR,
                      const double* pT, const float* dat, const float* ctf, const float* sigRcp,
                      const int* iCol, const int* iRow, int nPxl, int idim, int nImg, float* wC,
                      float* wR, float* wT, float* baseL, float* dvp, void* workspace,
                      size_t wsBytes, thx_stream_t stream);
/* thx_local_phase2d_d -- the 2D phase with CTF search (ExpectLocalPreI2D +
 *   ExpectLocalM with cSearch; kernel_logDataVSLC / kernel_UpdateWLC,
 *   gpu/src/Kernel.cu:889-939, 1459-1554, on the 2D projections): columns are
 *   the nT x nD (t, d) pairs, ctfD [nImg][nD][nPxl] (thx_ctf_search), priors
 *   pD / marginal wD [nImg][nD]; dvp (optional) [nImg][nR][nT][nD]. */
size_t thx_local_phase2d_d_workspace(int nImg, int nR, int nT, int nD);
int thx_local_phase2d_d(const float* vol, int vdim, int pf, const int* cls, const double* rot,
                        int nR, const double* trans, int nT, int nD, const double* pC,
                        const double* pR, const double* pT, const double* pD, const float* dat,
                        const float* ctfD, const float* sigRcp, const int* iCol, const int* iRow,
                        int nPxl, int idim, int nImg, float* wC, float* wR, float* wT, float* wD,
                        float* baseL, float* dvp, void* workspace, size_t wsBytes,
                        thx_stream_t stream);
int thx_insert2d(float* F, float* T, double* O, int* counter, int vdim, int pf,
                 const float* dat, const float* ctf, const double* rot, const double* trans,
                 const double* offS, const float* w, const int* nc, int nImg, int mReco,
                 const int* iCol, const int* iRow, int nPxl, int idim, thx_stream_t stream);
/* The 2D insert with CTF search (InsertI2D's cSearch, kernel_CalculateCTF per
 * sample, gpu/src/cuthunder.cu:3753): sample (l, m) inserts with the CTF of
 * attr[l] (nImg x 8, as thx_ctf) at defocus factor nD[l*mReco + m]. */
int thx_insert2d_d(float* F, float* T, double* O, int* counter, int vdim, int pf,
                   const float* dat, const float* attr, const double* nD, const double* rot,
                   const double* trans, const double* offS, const float* w, const int* nc,
                   int nImg, int mReco, const int* iCol, const int* iRow, int nPxl, int idim,
                   thx_stream_t stream);

/* ------------------------------------------------------------------ f2 ---
 * Image preprocessing of Optimiser::initImg (src/Optimiser.cpp:4608-5024),
 * the re-mask of reMaskImg / ReMask (:6093-6190; gpu/src/cuthunder.cu:9406)
 * and GCTFinit's CTF images (cuthunder.cu:9641), for a device stack of nImg
 * real-space idim x idim float images.
 * thx_img_stats -- substractBgImg + the per-image terms of statImg: img in
 *   (centred = 1: as stored in an MRC stack; 0: the reference's corner-origin
 *   Image layout), out (corner origin) = (x - bgMean) / bgSd over the pixels
 *   outside rMask (pixels); stats[nImg][5] = {bgMean, bgSd, bgStddev(0)
 *   after, stddev(0) after, mean inside rMask after}.  stdN = the mean of
 *   stats[.][2] over the hemisphere's images (the caller's all-reduce).
 * thx_img_finish -- maskImg + normaliseImg + fwImg: ori (optional) = img /
 *   stdN; img = softMask(img, rMask, edge = EDGE_WIDTH_RL 6) / stdN with a zero
 *   background (zeroMask) or N(0, stdN) noise; imgFT / oriFT = forward r2c
 *   FFTs (unnormalised), [nImg][idim][idim/2+1] Complex.  img is overwritten.
 * thx_remask -- imgFT in place: backward FFT / idim^2, x soft mask, forward;
 *   rl: nImg x idim^2 floats of scratch.
 * thx_img_gather -- allocPreCal's datP[l][i] = imgFT_l[iPxl[i]] (a1's iPxl).
 * thx_ctf_image -- ctf[nImg][idim][idim/2+1] over the whole half-complex grid. */
int thx_img_stats(const float* img, int centred, int nImg, int idim, float rMask, float* out,
                  float* stats, thx_stream_t stream);
int thx_img_finish(float* img, int nImg, int idim, float rMask, float edge, int zeroMask,
                   float stdN, unsigned long long seed, float* imgFT, float* ori, float* oriFT,
                   thx_stream_t stream);
int thx_remask(float* imgFT, int nImg, int idim, float rMask, float edge, float* rl,
               thx_stream_t stream);
int thx_img_gather(const float* imgFT, int nImg, int idim, const int* iPxl, int nPxl,
                   float* datP, thx_stream_t stream);
int thx_ctf_image(const float* attr, int nImg, int idim, float* ctf, thx_stream_t stream);

/* ------------------------------------------------------------------ f1 ---
 * The reconstruction solve of one half-map, Reconstructor::reconstruct
 * (src/Reconstructor.cpp:1129-1831; GPU twin reconstructG :1835), 3D,
 * trilinear kernel, on device with hipFFT: optional MAP Wiener factor from the
 * half-map FSC (fsc[nFsc] per shell of the unpadded box, joinHalf), W = 1
 * in the sphere |k| < maxRadius pf, T = max(T, 1e-25), gridCorr: W balanced
 * against the MKB(a, alpha) real-space kernel until max||C| - 1| < 1e-2 (or
 * the MIN / MAX / no-decrease rules), else W = 1 / max(|T|, 1e-6); then
 * F W -> inverse FFT (1/size) -> the central N^3 box divided by
 * j0(pi |r| / (pf N))^2.
 *   F: dimSize Complex (read), T: dimSize float (modified in place),
 *   dst: N^3 float real space, origin at [0][0][0], negatives wrapped
 *   (Volume RL storage); dstFT (may be NULL): its forward transform,
 *   (N/2+1) N N Complex, for thx_fsc; maxRadius <= 0: N/2 - ceil(a);
 *   nIter / diffOut (may be NULL; diffOut >= 30 floats): balancing iterations
 *   run and max||C| - 1| after each.
 * Host-synchronous (one 4-byte read per balancing iteration); workspace >=
 * thx_reconstruct_workspace(N, pf) device bytes (W, C, the real-space pad,
 * the kernel table and hipFFT's work area). */
size_t thx_reconstruct_workspace(int N, int pf);
int thx_reconstruct(const float* F, float* T, int N, int pf, float a, float alpha,
                    int gridCorr, int maxRadius, int map, const double* fsc, int nFsc,
                    int joinHalf, float* dst, float* dstFT, int* nIter, float* diffOut,
                    void* workspace, size_t wsBytes, thx_stream_t stream);

/* MODE_2D: the 2D branches of Reconstructor::reconstruct (src/Reconstructor.cpp:
 * 1136-1589, 1669-1818; GPU ExposePT2D / ExposeWT2D / ExposePF2D /
 * ExposeCorrF2D) for nK class images at once, each with its own balancing
 * iterations and stopping rule (OPTIMISER_2D_GRID_CORR, include/Config.h:206):
 *   F [nK][vdim][vdim/2+1] Complex (read), T [nK][vdim][vdim/2+1] float
 *   (modified in place), vdim = pf N; fsc (device, may be NULL: no MAP)
 *   [nK][nFsc]; dst [nK][N][N] real space, origin at [0][0], negatives
 *   wrapped; nIter (host, may be NULL) [nK].  Host-synchronous.
 * thx_prepare_tf2d -- prepareTF's MODE_2D part: F_k, T_k *= 1 / T_k[0] per class
 *   (RECONSTRUCTOR_NORMALISE_T_F, src/Reconstructor.cpp:2459-2466). */
int thx_prepare_tf2d(float* F, float* T, int vdim, int nK, thx_stream_t stream);
size_t thx_reconstruct2d_workspace(int N, int pf, int nK);
int thx_reconstruct2d(const float* F, float* T, int nK, int N, int pf, float a, float alpha,
                      int gridCorr, int maxRadius, const double* fsc, int nFsc, int joinHalf,
                      float* dst, int* nIter, void* workspace, size_t wsBytes,
                      thx_stream_t stream);

/* FFT::fw / FFT::bw (src/FFT.cpp) of one volume of box vdim, unnormalised:
 * inverse 0: rl [vdim^3] real -> C [vdim][vdim][vdim/2+1] complex; inverse 1:
 * C -> rl (C overwritten).  method 0: the reconstruction's own choice, 1:
 * hipFFT's 3D plans, 2: LDS column passes along y / z + hipFFT's batched 1D
 * transform along x (power-of-two vdim <= 1024).  Host-synchronous. */
size_t thx_fft3d_workspace(int vdim);
int thx_fft3d(float* C, float* rl, int vdim, int inverse, int method, void* workspace,
              size_t wsBytes, thx_stream_t stream);

/* ------------------------------------------------- f1 / a3 / a10: symmetry ---
 * thx_symmetry (host) -- the non-identity elements of a point group, as
 *   Symmetry(const char*) builds them (src/Geometry/Symmetry.cpp:104-278,
 *   SymmetryFunctions.cpp:13-152): "C<n>", "D<n>", "T", "O", "I1".."I4";
 *   R[cap][3][3] row-major, quat[cap][4] (quaternion(dvec4&, dmat33&)); cap 0
 *   only counts.  *nSymElem = group order - 1 (C1: 0).
 * thx_symmetrize_ft -- SYMMETRIZE_FT (include/Geometry/Transformation.h:
 *   170-194) of a half-complex volume (complex: F, 2 floats per voxel; real: T):
 *   dst(v) = src(v) + sum_i [|R_i v|^2 < r^2] trilinear(src, R_i v); R
 *   (device) nSymElem x 9 row-major; dst != src.
 * thx_prepare_tf -- Reconstructor::prepareTF's device part (src/Reconstructor.cpp:
 *   1056-1091, 2455-2479, 2676-2690; GPU PrepareTF, gpu/src/cuthunder.cu:6176):
 *   F, T *= 1 / T[0], then both symmetrized with r = maxRadius pf + 1;
 *   nSymElem 0 normalises only.  workspace >= thx_prepare_tf_workspace(vdim).
 * thx_pf_symmetrise -- Particle::symmetrise (src/Particle.cpp:2445-2471) of
 *   nImg clouds quat[nImg][mR][4] in place: each particle -> the symmetry
 *   counterpart closest to the anchor (symmetryCounterpart, Symmetry.cpp:
 *   309-335); anchorMode 0: (1, 0, 0, 0) (Particle::reset, the global sample
 *   set); 1: anchor[nImg][4] (the perturbation mean); 2: a particle of the
 *   cloud drawn with the counter RNG (seed, streamId) (calVari).  symQuat
 *   (device) nSymElem x 4. */
int thx_symmetry(const char* sym, int cap, double* R, double* quat, int* nSymElem);
int thx_symmetrize_ft(const float* src, float* dst, int isComplex, int vdim, const double* R,
                      int nSymElem, double r, thx_stream_t stream);
size_t thx_prepare_tf_workspace(int vdim);
int thx_prepare_tf(float* F, float* T, int vdim, const double* R, int nSymElem, int maxRadius,
                   int pf, void* workspace, size_t wsBytes, thx_stream_t stream);
int thx_pf_symmetrise(int nImg, int mR, double* quat, int anchorMode, const double* anchor,
                      const double* symQuat, int nSymElem, unsigned long long seed,
                      unsigned streamId, thx_stream_t stream);

/* ----------------------------------------------------------------- a14 ---
 * Fourier shell correlation FSC(vec&, const Volume& A, const Volume& B)
 * (src/Functions/Spectrum.cpp:302-337) of two half-complex volumes of real
 * box vdim; shell u = rint(|(i,j,k)|), fsc[u] = sum Re(A conj B) /
 * sqrt(sum|A|^2 sum|B|^2) for u < nShell.  fsc: nShell double (device).
 * workspace: >= thx_fsc_workspace(nShell) bytes. */
size_t thx_fsc_workspace(int nShell);
int thx_fsc(const float* A, const float* B, int vdim, int nShell, double* fsc,
            void* workspace, size_t wsBytes, thx_stream_t stream);

/* ------------------------------------------------- a3..a11 expectation ---
 * Device-resident Optimiser::expectationG (src/Optimiser.cpp:1684-3403) for
 * one image batch, 3D (CTF search: thx_expectation_ctf below).
 *
 * searchType 0 (SEARCH_TYPE_GLOBAL): global scan of every class k < nK over
 * the shared sample set (gQuat[nR*4], gTrans[nT*2], priors gPR[nR], gPT[nT];
 * a3) with the running baseline across classes (src/Optimiser.cpp:834-894);
 * reseed (src/Optimiser.cpp:1930-2131): class marginals -> PEAK_FACTOR_C
 * keepHalfHeightPeak -> resample(K, PAR_C) -> rand(cls), then the drawn
 * class's rotation / translation marginals -> setPeakFactor +
 * keepHalfHeightPeak -> resample to mLR / mLT -> calVari with the scan floors;
 * then particle-filter phases 1, 2, ... on the drawn class's volume.
 * searchType 1 (SEARCH_TYPE_LOCAL): no scan; the phases 0, 1, ... start from
 * the caller's particle state (quat, trans, pR, pT and, for nK > 1, cls) --
 * phase 0 perturbs by perturbFactorL, the rest by perturbFactor.
 * Each phase (src/Optimiser.cpp:1183-1616, GPU twin :2422-2750): perturb +
 * balanceWeight -> fused projection + likelihood + marginals ->
 * keepHalfHeightPeak(R) -> calRank1st -> calVari -> resample R and T.
 * converge 0: exactly nPhase phases.  converge 1: the per-image stopping rule
 * of OPTIMISER_COMPRESS_CRITERIA -- from phase minPhase on, an image stops
 * after the first phase in which neither variR = (k1 k2 k3)^(1/6) nor
 * variT = s0 s1 fell below 0.95 (PARTICLE_FILTER_DECREASE_FACTOR) of its
 * smallest value so far (N_PHASE_WITH_NO_VARI_DECREASE = 1), at the latest
 * after phase maxPhase - 1; stopped images drop out of every later launch
 * (an active-image list).  In this mode the host reads the active count once
 * per phase (a 4-byte copy + stream sync), so it is not graph-capturable;
 * converge 0 enqueues only.
 * Outputs the particle sets quat[nImg*mLR*4], trans[nImg*mLT*2] with priors
 * pR[nImg*mLR], pT[nImg*mLT], score[nImg] (last baseline), and optionally
 * cls[nImg] (the drawn class; input for searchType 1, nK > 1) and
 * nPhaseOut[nImg] (phases run; the reference's _nP). */
typedef struct thx_expect_cfg {
    int idim, pf, vdim;       /* image box, padding factor, vdim = pf*idim */
    int nR, nT;               /* global sample set sizes */
    int mLR, mLT;             /* particle-filter set sizes (125, 9) */
    int nPhase;               /* phases when converge == 0 (10) */
    int algo;                 /* global-scan algorithm (thx_global_scan) */
    double perturbFactor;     /* perturbFactorSGlobal / perturbFactorSLocal (0.5) */
    double kMin, sMin;        /* reseed floors of k1..k3 and s0, s1 (src/Optimiser.cpp:1033-1079,
                                 OPTIMISER_SCAN_SET_MIN_STD_WITH_PERTURB):
                                 (mS^-1/3 / perturbFactor)^2 and
                                 1/chi2Qinv(.5,2)/sqrt(tsf pi) / perturbFactor */
    double transS, transM;    /* translation prior width, reCentre radius */
    unsigned long long seed;  /* counter-RNG seed */
    int shuffle;              /* 1: shuffle the support before every resampling, as
                                 Particle::resample does (src/Particle.cpp:1298,
                                 2202-2300); 0: resample in support order */
    /* ABI 3 */
    int nK;                   /* classes; vol holds nK projectees of dimSize Complex back to back */
    int searchType;           /* 0 global, 1 local */
    int converge;             /* 0 fixed nPhase, 1 vari-decrease stopping rule */
    int minPhase, maxPhase;   /* MIN_N_PHASE_PER_ITER_GLOBAL / _LOCAL (10 / 3), MAX_N_PHASE_PER_ITER (100) */
    int perturbMean;          /* 0: top particle; 1: inferACG mean of the cloud
                                 (PARTICLE_ROT_MEAN_USING_STAT_PERTURB, include/Config.h:79) */
    int acgIters;             /* iteration cap of inferACG's fixed point (the reference loops
                                 until sum|A - B| <= 1e-3 without a cap) */
    double perturbFactorL;    /* perturbFactorL (2): phase 0 of a local search; also phase 1 of a
                                 global search when largeFirst */
    int largeFirst;           /* OPTIMISER_GLOBAL_PERTURB_LARGE (off in include/Config.h, so 0 is
                                 the reference): 1 perturbs the first global phase by
                                 perturbFactorL (src/Optimiser.cpp:1185-1186, 2424-2425) */
    void* phaseEvents;        /* optional hipEvent_t[2 * phases]: events recorded on `stream`
                                 around every phase's k_local_fused launch (begin, end), for
                                 in-process kernel timing (bench.py); NULL: none */
    /* ABI 4 */
    const float* volCells;    /* optional cell-expanded copy of vol (thx_volume_cells, nK == 1):
                                 the phases gather one 64-B cell per sample instead of four row
                                 pieces -- the layout for large boxes at full resolution, where
                                 the projectee is far beyond L2 / MALL and the patch boxes do not
                                 fit LDS; NULL: the half-complex projectee */
    /* ABI 5 */
    int nPhaseEvents;         /* event pairs phaseEvents holds: phases past it are not timed */
    /* ABI 6 */
    int* phaseRoute;          /* optional device int[nPhaseRoute]: the kernel the device route
                                 picked in each phase (as thx_local_phase_routed's route: 0
                                 staged, 1 box-less, 2 y-pair, -1 not routed); NULL: none */
    int nPhaseRoute;
    const double* symQuat;    /* device nSymElem x 4 (thx_symmetry), 3D: Particle::symmetrise
                                 after every perturbation (anchor: the perturbation mean) and
                                 before every calVari (anchor: a drawn particle), as the
                                 reference does for non-C1 groups; NULL / 0: C1 */
    int nSymElem;
} thx_expect_cfg;

/* nOrd: length of pxOrder (<= 0 when pxOrder is NULL). */
size_t thx_expectation_workspace(const thx_expect_cfg* cfg, int nImg, int nPxl,
                                 int nOrd);
int thx_expectation(const thx_expect_cfg* cfg, const float* vol,
                    const double* gQuat, const double* gTrans,
                    const double* gPR, const double* gPT, const float* dat,
                    const float* ctf, const float* sigRcp, const int* iCol,
                    const int* iRow, const int* pxOrder, int nOrd, int nPxl,
                    int nImg, double* quat,
                    double* trans, double* pR, double* pT, float* score,
                    int* cls, int* nPhaseOut,
                    void* workspace, size_t wsBytes, thx_stream_t stream);

/* SEARCH_TYPE_CTF (cfg->searchType == 2): a local search from the caller's
 * particle state whose phases also sample mLD defocus factors per image --
 * initD at phase 0, perturb(perturbFactorSCTF, PAR_D) after, the CTF per
 * defocus sample from the images' CTF attributes (allocPreCal's cSearch
 * branch + kernel_CalCTFL), the (r, t, d) likelihood, calVari / resample of
 * the defocus set and variD in the stopping rule (src/Optimiser.cpp:
 * 1159-1616, the SEARCH_TYPE_CTF branches; src/Particle.cpp:281-310,
 * 1120-1141, 1278-1288, 2374-2409).  d / pD (device, nImg x mLD) receive
 * the final defocus particles and their priors. */
typedef struct thx_ctf_search_cfg {
    int mLD;                   /* defocus samples per particle ("Number of Sampling Points of
                                  Defocus in Local Search", 9 in script/demo.json) */
    double ctfRefineS;         /* initD spread ("CTF Refine Standard Deviation", 0.01) */
    double perturbFactorSCTF;  /* "Perturbation Factor (Small, CTF)" (0.5) */
    const float* attr;         /* device, nImg x 8 CTF attributes (as thx_ctf) */
    double* d;                 /* device, nImg x mLD: out */
    double* pD;                /* device, nImg x mLD: out */
} thx_ctf_search_cfg;
size_t thx_expectation_ctf_workspace(const thx_expect_cfg* cfg,
                                     const thx_ctf_search_cfg* cs, int nImg,
                                     int nPxl, int nOrd);
int thx_expectation_ctf(const thx_expect_cfg* cfg, const thx_ctf_search_cfg* cs,
                        const float* vol, const float* dat, const float* sigRcp,
                        const int* iCol, const int* iRow, const int* pxOrder, int nOrd,
                        int nPxl, int nImg, double* quat, double* trans, double* pR,
                        double* pT, float* score, int* cls, int* nPhaseOut,
                        void* workspace, size_t wsBytes, thx_stream_t stream);

/* MODE_2D (the _para.mode == MODE_2D branches of Optimiser::expectationG,
 * src/Optimiser.cpp:646-1079, 1183-1616, 1726-2131): the same driver with
 *   vol      nK half-complex class images [nK][vdim][vdim/2+1] Complex;
 *   gRot     the global rotations as Particle::_r rows (cos, sin, 0, 0)
 *            (nR x 4; thx_global_sample_set2d), gTrans / gPR / gPT as 3D;
 *   rot      the particles' rotations, nImg x mLR x 4 rows (cos, sin, 0, 0);
 *   kMin     the reseed floor of k1 ((1 / perturbFactor) MIN_STD_FACTOR / mS,
 *            :2032-2044);
 * particle statistics of von Mises rotations (src/Particle.cpp:87-169,
 * 1013-1016, 1160-1178, 1920-1921, 2317-2329; src/Geometry/DirectionalStat.cpp:
 * 252-384): calVari k1 = 1 - R (inferVMS), perturb r_i <- r_i d_i with
 * d_i ~ sampleVMS(k = min(1, k1 pf)), pR = 1 / pdfVMS, peak factor from the
 * (n / 2)-th largest weight, the stopping rule on variR = k1.  perturbMean
 * and volCells do not apply (ignored / NULL); pxOrder is not used (the 2D
 * phase is direct, thx_local_phase2d).  thx_expectation2d_ctf: the
 * SEARCH_TYPE_CTF local search of thx_expectation_ctf in MODE_2D (the 2D
 * phase over (r, t, d) columns, thx_local_phase2d_d). */
size_t thx_expectation2d_workspace(const thx_expect_cfg* cfg, int nImg, int nPxl);
int thx_expectation2d(const thx_expect_cfg* cfg, const float* vol, const double* gRot,
                      const double* gTrans, const double* gPR, const double* gPT,
                      const float* dat, const float* ctf, const float* sigRcp, const int* iCol,
                      const int* iRow, int nPxl, int nImg, double* rot, double* trans,
                      double* pR, double* pT, float* score, int* cls, int* nPhaseOut,
                      void* workspace, size_t wsBytes, thx_stream_t stream);
size_t thx_expectation2d_ctf_workspace(const thx_expect_cfg* cfg, const thx_ctf_search_cfg* cs,
                                       int nImg, int nPxl);
int thx_expectation2d_ctf(const thx_expect_cfg* cfg, const thx_ctf_search_cfg* cs,
                          const float* vol, const float* dat, const float* sigRcp,
                          const int* iCol, const int* iRow, int nPxl, int nImg, double* rot,
                          double* trans, double* pR, double* pT, float* score, int* cls,
                          int* nPhaseOut, void* workspace, size_t wsBytes, thx_stream_t stream);
/* The perturbation mean of PARTICLE_ROT_MEAN_USING_STAT_PERTURB (inferACG's
 * principal axis, src/Geometry/DirectionalStat.cpp:93-145, 224-251; at most
 * acgIters fixed-point iterations): meanQ nImg x 4, iters (may be NULL) the
 * iterations each image took. */
int thx_pf_acg_mean(int nImg, int mR, const double* quat, int acgIters, double* meanQ,
                    int* iters, thx_stream_t stream);
/* MODE_2D particle statistics one image at a time (rows (cos, sin, 0, 0)):
 * thx_global_sample_set2d -- Particle::reset's 2D rotations (sampleVMS with
 *   k = 1: uniform angles, src/Particle.cpp:101-103), translations / priors as
 *   thx_global_sample_set;
 * thx_pf_calvari2d -- calVari: k[3l..3l+2] = max(kFloor, 1 - R), sd as
 *   thx_pf_calvari;
 * thx_pf_balance_rot2d -- balanceWeight(PAR_R): pR = 1 / pdfVMS normalised;
 * thx_pf_perturb2d -- perturb(pf, PAR_R / PAR_T) + balanceWeight with the
 *   spreads k / sd of thx_pf_calvari2d (counter RNG: seed, stream_id). */
int thx_global_sample_set2d(int nR, int nT, double transS, unsigned long long seed, double* rot,
                            double* trans, double* pR, double* pT, thx_stream_t stream);
int thx_pf_calvari2d(int nImg, int mR, const double* rot, int mT, const double* trans,
                     double kFloor, double sFloor, double* k, double* sd, thx_stream_t stream);
int thx_pf_balance_rot2d(int nImg, int mR, const double* rot, double* pR, thx_stream_t stream);
int thx_pf_perturb2d(int nImg, int mR, int mT, double* rot, double* trans, double* pR,
                     double* pT, const double* k, const double* sd, double pf, double transS,
                     double transM, unsigned long long seed, unsigned stream_id,
                     thx_stream_t stream);

/* HIP event pairs for thx_expect_cfg.phaseEvents: create n (begin, end)
 * pairs, read back ms[i] per pair (-1: not recorded), destroy. */
int thx_event_pairs_create(int n, void** events);
int thx_event_pairs_elapsed(void* events, int n, float* ms);
int thx_event_pairs_destroy(void* events, int n);

/* ====================================================================== *
 * Reference-shaped host adapters (host pointers, stateless, synchronous).  *
 * ====================================================================== */

/* The batch adapters (ExpectGlobal3D / 2D, InsertFT*, InsertI2D) deal their
 * images out over several GPUs in contiguous blocks, one host thread per
 * device, as cuthunder deals batches round-robin over every visible GPU
 * (gpu/src/cuthunder.cu:2002-2198, 5570-5826); insert partial half-maps are
 * summed onto the first device.  The devices (also what thx_getAviDevice
 * reports to the per-image local path), THX_DEVICES unset: every visible
 * GPU, as the reference's getAviDevice -- except when the launcher's
 * environment puts at least as many processes on the node as there are GPUs
 * (LOCAL_WORLD_SIZE / OMPI_COMM_WORLD_LOCAL_SIZE / MPI_LOCALNRANKS /
 * SLURM_NTASKS_PER_NODE >= the GPU count, with LOCAL_RANK /
 * OMPI_COMM_WORLD_LOCAL_RANK / MPI_LOCALRANKID / SLURM_LOCALID): then one
 * device per process, (local rank % GPU count) (ABI 9; THUNDER's master +
 * two hemisphere ranks on an 8-GPU node keep all eight); THX_DEVICES=all /
 * local / current (the caller's current device) / a list ("0,2,5") forces
 * one.  A hemisphere communicator passed to the insert adapters must live on
 * the first of these devices (checked: THX_ERR_ARG otherwise).  This returns
 * the list (devs may be NULL when cap is 0). */
int thx_adapter_devices(int* devs, int cap, int* n);
/* The same policy as a pure function of its inputs (no device call): nVisible
 * GPUs, current device cur, THX_DEVICES value env (NULL = unset), the
 * launcher's local process count / local rank (-1 = unknown). */
int thx_adapter_device_policy(int nVisible, int cur, const char* env, int localSize,
                              int localRank, int* devs, int cap, int* n);
/* hipSetDevice for C++ callers without HIP headers (e.g. before
 * thx_rccl_comm_init, whose communicator lives on the current device). */
int thx_set_device(int dev);

/* gpu/interface/Interface.h:199-208 ExpectRotran: traP[nT][npxl] and
 * rotMat[nR][9] from trans[nT*2] and rot[nR*4]. */
int thx_ExpectRotran(float* traP, const double* trans, const double* rot,
                     double* rotMat, const int* iCol, const int* iRow, int nR,
                     int nT, int idim, int npxl);

/* gpu/interface/Interface.h:210-219 ExpectProject: rotP[nR][npxl] from the
 * half-complex projectee `vol` (vdim box).  interp must be LINEAR_INTERP (1),
 * the only mode the search uses (include/Model.h:90-93). */
int thx_ExpectProject(const float* vol, float* rotP, const double* rotMat,
                      const int* iCol, const int* iRow, int nR, int pf,
                      int interp, int vdim, int npxl);

/* gpu/interface/Interface.h:221-237 ExpectGlobal3D.  pR[nR], pT[nT]; wC
 * [imgNum*nK], wR[imgNum*nK*nR], wT[imgNum*nK*nT], baseL[imgNum] in/out
 * (kIdx > 0 merges into them). */
int thx_ExpectGlobal3D(const float* rotP, const float* traP, const float* datP,
                       const float* ctfP, const float* sigRcpP, float* wC,
                       float* wR, float* wT, const double* pR,
                       const double* pT, float* baseL, int kIdx, int nK,
                       int nR, int nT, int npxl, int imgNum);

/* ---- the per-image local-search surface, gpu/interface/Interface.h:16-164
 * (called from the OpenMP image loop of Optimiser::expectationG,
 * src/Optimiser.cpp:2160-2750).  Complex arrays are float[2]; the device
 * pointers these return are owned by the caller and freed by the matching
 * *Fin / *FreeIdx call.  The ManagedArrayTexture / ManagedCalPoint objects
 * become opaque handles: thx_tex_create / thx_calpoint_create mirror their
 * Init(mode, vdim, gpu) / Init(mode, searchType, gpu, mLR, mLT, mLD, nPxl).
 * MODE_3D, and MODE_2D through thx_ExpectLocalV2D / thx_ExpectLocalPreI2D (the
 * class image of thx_tex_create(0, vdim, ...); the 2D calpoint takes (cos,
 * sin) = the first two entries of each particle's 4-double rotation row, as
 * Optimiser packs them; no 2D CTF search).  CTF search (searchType 2 / cSearch): ExpectLocalIn also
 * allocates devdefO, ExpectLocalP copies defO (the image's per-pixel defocus,
 * thx_defocus_pre), ExpectLocalRTD takes dpara (mLD defocus factors) and oldD
 * (their priors), ExpectLocalPreI3D builds the CTF per defocus sample from
 * devdefO + datShift * npxl, devfreQ, phaseShift, conT, k1, k2, and
 * ExpectLocalM returns wD[mLD]. */
int thx_getAviDevice(int* gpus, int cap, int* n);   /* :16 -- the adapter devices */
int thx_ExpectPreidx(int gpuIdx, int** deviCol, int** deviRow, const int* iCol,
                     const int* iRow, int npxl);                                  /* :18 */
int thx_ExpectPrefre(int gpuIdx, float** devfreQ, const float* freQ, int npxl); /* :26 */
int thx_ExpectLocalIn(int gpuIdx, float** devdatP, float** devctfP, float** devdefO,
                      float** devsigP, int nPxl, int cpyNumL, int searchType);   /* :31 */
int thx_tex_create(int mode, int vdim, int gpuIdx, void** mgr);
int thx_tex_destroy(void* mgr);
int thx_ExpectLocalV3D(int gpuIdx, void* mgr, const float* volume, int vdim);   /* :44 */
int thx_ExpectLocalV2D(int gpuIdx, void* mgr, const float* volume, int dimSize); /* :40 */
int thx_ExpectLocalP(int gpuIdx, float* devdatP, float* devctfP, float* devdefO,
                     float* devsigP, const float* datP, const float* ctfP,
                     const float* defO, const float* sigP, int threadId, int imgId,
                     int npxl, int cSearch);                                      /* :49 */
int thx_ExpectLocalHostA(int gpuIdx, float** wC, float** wR, float** wT, float** wD,
                         double** oldR, double** oldT, double** oldD, double** trans,
                         double** rot, double** dpara, int mR, int mT, int mD,
                         int cSearch);                                            /* :63 */
int thx_calpoint_create(int mode, int searchType, int gpuIdx, int mR, int mT, int mD,
                        int npxl, void** mcp);
int thx_calpoint_destroy(void* mcp);
int thx_ExpectLocalRTD(int gpuIdx, void* mcp, const double* oldR, const double* oldT,
                       const double* oldD, const double* trans, const double* rot,
                       const double* dpara);                                      /* :79 */
int thx_ExpectLocalPreI3D(int gpuIdx, int datShift, void* mgr, void* mcp,
                          const float* devdefO, const float* devfreQ, const int* deviCol,
                          const int* deviRow, float phaseShift, float conT, float k1,
                          float k2, int pf, int idim, int vdim, int npxl, int interp); /* :106 */
int thx_ExpectLocalPreI2D(int gpuIdx, int datShift, void* mgr, void* mcp,
                          const float* devdefO, const float* devfreQ, const int* deviCol,
                          const int* deviRow, float phaseShift, float conT, float k1,
                          float k2, int pf, int idim, int vdim, int npxl, int interp); /* :89 */
int thx_ExpectLocalM(int gpuIdx, int datShift, void* mcp, const float* devdatP,
                     const float* devctfP, const float* devsigP, float* wC, float* wR,
                     float* wT, float* wD, double oldC, int npxl);                /* :124 */
int thx_ExpectLocalHostF(int gpuIdx, float** wC, float** wR, float** wT, float** wD,
                         double** oldR, double** oldT, double** oldD, double** trans,
                         double** rot, double** dpara, int cSearch);              /* :140 */
int thx_ExpectLocalFin(int gpuIdx, float** devdatP, float** devctfP, float** devdefO,
                       float** devfreQ, float** devsigP, int cSearch);            /* :153 */
int thx_ExpectFreeIdx(int gpuIdx, int** deviCol, int** deviRow);                /* :161 */

/* gpu/interface/Interface.h:176-197 ExpectGlobal2D: the global scan of all
 * nK 2D classes (vol: nK half-complex images) over the shared rotations
 * rot[nR*2] (cos, sin) and translations trans[nT*2]; outputs as
 * thx_ExpectGlobal3D with the running baseline across classes kept inside. */
int thx_ExpectGlobal2D(const float* vol, const float* datP, const float* ctfP,
                       const float* sigRcpP, const double* trans, float* wC, float* wR,
                       float* wT, const double* pR, const double* pT, const double* rot,
                       const int* iCol, const int* iRow, int nK, int nR, int nT, int pf,
                       int interp, int idim, int vdim, int npxl, int imgNum);

/* gpu/interface/Interface.h:239-265 InsertI2D, argument for argument: F2D[nk
 * images], T2D, O2D[nk*2], counter[nk] read-modify-write host buffers;
 * nC[imgNum*mReco] the sample classes, nR / nT[imgNum*mReco*2] (cos, sin) /
 * translations; iCol / iRow the padded pixel set.  The reference's (hemi,
 * slav) MPI pair becomes `comm`: the hemisphere's RCCL communicator
 * (thx_rccl_comm_init; NULL = no reduction).  cSearch: sample (l, m) inserts
 * with the CTF of ctfaData[l] (CTFAttr, 7 floats) at defocus factor
 * nD[l*mReco + m] and pixelSize (kernel_CalculateCTF); else ctfP[imgNum*npxl].
 * sigRcpP is unused (OPTIMISER_RECONSTRUCT_SIGMA_REGULARISE is off). */
int thx_InsertI2D(float* F2D, float* T2D, double* O2D, int* counter, void* comm,
                  const float* datP, const float* ctfP, const float* sigRcpP, const float* w,
                  const double* offS, const int* nC, const double* nR, const double* nT,
                  const double* nD, const float* ctfaData, const int* iCol, const int* iRow,
                  float pixelSize, int cSearch, int nk, int opf, int npxl, int mReco, int idim,
                  int vdim, int imgNum);

/* gpu/interface/Interface.h:294-318 InsertFT (K = 1, cSearch off): F3D
 * [dimSize*2], T3D[dimSize] (real), O3D[3], counter[1] are read-modify-write
 * host buffers; nR[imgNum*mReco*4], nT[imgNum*mReco*2], offS[imgNum*2],
 * w[imgNum]; iCol/iRow the Reconstructor's padded pixel set (i*opf, j*opf,
 * as passed by Reconstructor::insertI, src/Reconstructor.cpp:928-985).
 * The MPI/NCCL hemisphere reduction of the reference call is the caller's
 * (thunder_amd.halfmap_allreduce over RCCL). */
int thx_InsertFT(float* F3D, float* T3D, double* O3D, int* counter,
                 const float* datP, const float* ctfP, const double* offS,
                 const float* w, const double* nR, const double* nT,
                 const int* iCol, const int* iRow, int opf, int npxl,
                 int mReco, int idim, int vdim, int imgNum);

/* gpu/interface/Interface.h:267-292 InsertFT with nC (the K-class call, one
 * per class reconstructor): as thx_InsertFT, image l inserting only its first
 * nC[l] (host, imgNum ints) of the mReco samples. */
int thx_InsertFTC(float* F3D, float* T3D, double* O3D, int* counter,
                  const float* datP, const float* ctfP, const double* offS,
                  const float* w, const double* nR, const double* nT, const int* nC,
                  const int* iCol, const int* iRow, int opf, int npxl,
                  int mReco, int idim, int vdim, int imgNum);

/* gpu/interface/Interface.h:267-318 InsertFT with cSearch = true: sample
 * (l, m) inserts with the CTF of image l at defocus factor nD[l*mReco + m]
 * (kernel_CalculateCTF, gpu/src/Kernel.cu:2206-2270; CPU src/Optimiser.cpp:
 * 7101-7120); ctfaData: CTFAttr[imgNum] as 7 floats each {voltage, defocusU,
 * defocusV, defocusTheta, Cs, amplitudeContrast, phaseShift}
 * (include/Database.h:302-327); nC and comm may be NULL (then as
 * thx_InsertFT / thx_InsertFTC / thx_InsertFTComm). */
int thx_InsertFTCS(float* F3D, float* T3D, double* O3D, int* counter,
                   const float* datP, const float* ctfaData, const double* offS,
                   const float* w, const double* nR, const double* nT,
                   const double* nD, const int* nC, const int* iCol, const int* iRow,
                   float pixelSize, int opf, int npxl, int mReco, int idim, int vdim,
                   int imgNum, void* comm);

/* Either of the two with the reference call's hemisphere reduction inside
 * (nC may be NULL): after the insert, thx_halfmap_allreduce of the device
 * F / T / O / counter over `comm` (a communicator from thx_rccl_comm_init
 * spanning the hemisphere's ranks; collective), then the copy back. */
int thx_InsertFTComm(float* F3D, float* T3D, double* O3D, int* counter,
                     const float* datP, const float* ctfP, const double* offS,
                     const float* w, const double* nR, const double* nT, const int* nC,
                     const int* iCol, const int* iRow, int opf, int npxl,
                     int mReco, int idim, int vdim, int imgNum, void* comm);

/* ------------------------------------------ reconstruction host adapters ---
 * gpu/interface/Interface.h:320-528 (ABI 7): the reconstruction and
 * preprocessing entry points Reconstructor::reconstructG / prepareTFG
 * (src/Reconstructor.cpp:1021-1052, 1835-2346) and Optimiser (src/
 * Optimiser.cpp:5059, 6185, 7402-7425) call, host pointers in and out as the
 * cuthunder bodies take them (gpu/src/cuthunder.cu:6176-9819), Complex as
 * float[2], RFLOAT as float.  Half-complex arrays [k][j][i], (dim/2+1) x dim
 * (x dim); real-space arrays dim x dim (x dim), origin at index 0.  gpuIdx:
 * the device the call runs on.  Device-resident equivalents: thx_prepare_tf,
 * thx_reconstruct, thx_reconstruct2d.  All return THX_OK or an error code. */

/* PrepareTF (:320): F and T scaled by 1 / T[0], then symmetrised with
 * r = maxRadius pf + 1 (SYMMETRIZE_FT); T = max(T, 1e-25).  T3D: the real
 * parts of T (the forward converts the complex Volume).  symMat: nSymElem 3x3
 * matrices as prepareTFG packs them (Eigen column-major). */
int thx_PrepareTF(int gpuIdx, float* F3D, float* T3D, const double* symMat, int nSymElem,
                  int maxRadius, int pf, int dim);

/* ExposePT / ExposePT2D (:328-344): the MAP step, T /= FSC' on wienerF pf <=
 * |k| < maxRadius pf (kernel_CalculateFSC), then T = max(T, 1e-25); fsc:
 * nFsc values of the FSC per shell (the RFLOAT vec _FSC). */
int thx_ExposePT(int gpuIdx, float* T3D, int maxRadius, int pf, int dim, const float* fsc,
                 int nFsc, int joinHalf, int wienerF);
int thx_ExposePT2D(int gpuIdx, float* T2D, int maxRadius, int pf, int dim, const float* fsc,
                   int nFsc, int joinHalf, int wienerF);

/* ExposeWT / ExposeWT2D with the kernel table (:346-356, 438-448): the
 * grid-correction balancing loop, W = 1 inside |k| < maxRadius pf, then
 * C = T W -> C2R -> / size x tab(|r|^2 / (pf size)^2) / nf -> R2C -> W /=
 * max(|C|, 1e-6) until max | |C| - 1 | < 1e-2 or (m >= minIter and two
 * iterations in a row not below 0.95 of the previous) or maxIter.  tab:
 * tabSize entries at spacing step (TabFunction::getData / getStep); the
 * index is clamped into the table.  nIter (may be NULL): iterations run. */
int thx_ExposeWT(int gpuIdx, const float* T3D, float* W3D, const float* tab, float step,
                 int tabSize, float nf, int maxRadius, int pf, int dim, int maxIter, int minIter,
                 int size, int* nIter);
int thx_ExposeWT2D(int gpuIdx, const float* T2D, float* W2D, const float* tab, float step,
                   int tabSize, float nf, int maxRadius, int pf, int dim, int maxIter,
                   int minIter, int size, int* nIter);
/* ExposeWT / ExposeWT2D without grid correction (:450-462): W = 1 /
 * max(|T|, 1e-6) inside |k| < maxRadius pf, W untouched outside. */
int thx_ExposeWT_T(int gpuIdx, const float* T3D, float* W3D, int maxRadius, int pf, int dim);
int thx_ExposeWT2D_T(int gpuIdx, const float* T2D, float* W2D, int maxRadius, int pf, int dim);

/* The split-step 3D balancing reconstructG drives with its own host FFTs
 * between the steps (:358-436).  thx_AllocDevicePoint: device C (room for the
 * dim^3 real C too), W, T, table and the max cell on gpuIdx, and one HIP
 * stream in stream[0] (stream[1..streamNum) = NULL; devDiff / devCount =
 * NULL: RECONSTRUCTOR_CHECK_C_AVERAGE is off).  thx_HostDeviceInit: uploads
 * T and the table, W = 1 inside the sphere.  thx_ExposeC: C3D (host,
 * half-complex) = T W.  thx_ExposeForConvC: C3D (host, real dim^3, after the
 * caller's scaled backward FFT) x tab(|r|^2 / (pf size)^2) / nf.
 * thx_ExposeWC: C3D (host, after the forward FFT) -> W /= max(|C|, 1e-6)
 * inside, *diffC = max | |C| - 1 | inside.  thx_FreeDevHostPoint: volumeW =
 * W, then frees everything and destroys the stream. */
int thx_AllocDevicePoint(int gpuIdx, float** dev_C, float** dev_W, float** dev_T, float** dev_tab,
                         float** devDiff, float** devMax, int** devCount, void** stream,
                         int streamNum, int tabSize, int dim);
int thx_HostDeviceInit(int gpuIdx, const float* T3D, const float* tab, float* dev_W, float* dev_T,
                       float* dev_tab, void** stream, int streamNum, int tabSize, int maxRadius,
                       int pf, int dim);
int thx_ExposeC(int gpuIdx, float* C3D, float* dev_C, const float* dev_T, const float* dev_W,
                void** stream, int streamNum, int dim);
int thx_ExposeForConvC(int gpuIdx, float* C3D, float* dev_C, const float* dev_tab, void** stream,
                       float step, int tabSize, float nf, int streamNum, int pf, int size, int dim);
int thx_ExposeWC(int gpuIdx, const float* C3D, float* dev_C, float* dev_W, float* devMax,
                 void** stream, float* diffC, int streamNum, int maxRadius, int pf, int dim);
int thx_FreeDevHostPoint(int gpuIdx, float** dev_C, float** dev_W, float** dev_T, float** dev_tab,
                         float** devDiff, float** devMax, int** devCount, void** stream,
                         float* volumeW, int streamNum, int dim);

/* ExposePFW (:472): padDst (pdim half-complex) = F W inside |k| < maxRadius
 * pf, zero elsewhere.  ExposePF / ExposePF2D (:464-485): the same padded
 * array back-transformed and divided by its size into padDstR (pdim^3 /
 * pdim^2 real). */
int thx_ExposePFW(int gpuIdx, float* padDst, const float* F3D, const float* W3D, int maxRadius,
                  int pf, int pdim, int fdim);
int thx_ExposePF(int gpuIdx, float* padDstR, const float* F3D, const float* W3D, int maxRadius,
                 int pf, int pdim, int fdim);
int thx_ExposePF2D(int gpuIdx, float* padDstR, const float* F2D, const float* W2D, int maxRadius,
                   int pf, int pdim, int fdim);

/* ExposeCorrF (:493-502) / ExposeCorrF2D (:487): the real-space kernel
 * correction, x / mkbRL(|i|, |j|, |k|) (x nf when nf != 0: the MKB-kernel
 * build; reconstructG passes nf = 0 with the trilinear kernel); mkbRL:
 * (dim/2+1)^3 (2D: ^2) values, i fastest.  thx_ExposeCorrF: dst (dim^3 real)
 * in place.  thx_ExposeCorrFT (the two-volume overload): dstN corrected and
 * forward-transformed into dst (half-complex).  thx_ExposeCorrF2D: imgDst
 * (dim^2 real) corrected and forward-transformed into dst. */
int thx_ExposeCorrF(int gpuIdx, float* dst, const float* mkbRL, float nf, int dim);
int thx_ExposeCorrFT(int gpuIdx, const float* dstN, float* dst, const float* mkbRL, float nf,
                     int dim);
int thx_ExposeCorrF2D(int gpuIdx, const float* imgDst, float* dst, const float* mkbRL, float nf,
                      int dim);

/* TranslateI / TranslateI2D (:504-515): the half-complex volume / image x
 * exp(-2 pi i (i ox + j oy + k oz) / dim) inside i^2 + j^2 + k^2 < r^2. */
int thx_TranslateI(int gpuIdx, float* ref, double ox, double oy, double oz, int r, int dim);
int thx_TranslateI2D(int gpuIdx, float* img, double ox, double oy, int r, int dim);

/* ReMask (:517): each image's transform (img[l]: idim x (idim/2+1) Complex)
 * back-transformed / idim^2, soft-masked at maskRadius / pixelSize with edge
 * ew, forward-transformed, in place.  GCTFinit (:524): img[l] = (CTF, 0) of
 * ctfAttr[l] (7 floats, CTFAttr) over the whole half-complex grid.  Images
 * are dealt over thx_adapter_devices(). */
int thx_ReMask(float* const* img, float maskRadius, float pixelSize, float ew, int idim,
               int imgNum);
int thx_GCTFinit(float* const* img, const float* ctfAttr, float pixelSize, int idim, int imgNum);

#ifdef __cplusplus
}
#endif
#endif /* THUNDER_AMD_H */
