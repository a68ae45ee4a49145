// optimiser.hip -- device-resident expectation driver (host orchestration in
// C++ over the device kernels), the MI355X counterpart of
// Optimiser::expectationG (src/Optimiser.cpp:1684-3403) for 3D, K >= 1
// classes, global or local search, no CTF search:
//
//   global scan (a4-a8) -> reseed every particle from the scan marginals
//   (keepHalfHeightPeak, resample nR -> mLR, nT -> mLT, calVari with the scan
//   floors; src/Optimiser.cpp:1966-2079) -> nPhase particle-filter phases,
//   each: perturb + balanceWeight (R, T) -> fused projection + likelihood +
//   marginals (a6+a7+a9) -> keepHalfHeightPeak (R) -> calVari -> resample
//   (a10; src/Optimiser.cpp:1183-1500).
//
// The reference leaves the particle filter on the host and round-trips to the
// GPU once per image per phase (gpu/src/cuthunder.cu:2675-3140 with a stream
// sync at :3140); here every step runs for the whole batch on device and the
// host only enqueues kernels.  The host waits on the device at two points
// only: one 4-byte read-back per call (the pixel ring's radius, which sizes
// the compact y-pair ball) and, with the stopping rule on, the count of
// images left after each phase from minPhase on.  So the phase loop with
// converge == 0 is stream-ordered end to end, but a whole call is not
// capturable into a HIP graph (the read-back would have to move into the
// caller's configuration first).
//
// The particle statistics follow Particle / DirectionalStat with the
// reference's Config.h switches: ACG spreads by inferACG's fixed point,
// 1/pdfACG rotation priors, the 3D peak factor, the support shuffle before
// every systematic resampling (a bitonic sort of counter-RNG keys, see
// k_pf_resample).  Not replicated: the generator -- sampling is counter-based
// (Philox4x32-10), so a run is reproducible for a given seed, where the
// reference draws from an urandom-seeded GSL mt19937.
#include <cmath>
#include <map>
#include <mutex>
#include <cstdlib>
#include <string>
#include <utility>

#include "common.h"
#include "symmetry.h"


namespace thx {
int project2d_launch(const float* vol, int vdim, int pf, const double* rot, int rotStride, int nR,
                     const int* iCol, const int* iRow, int nPxl, float* rotP, hipStream_t s);
int local_phase2d_launch(const float* vol, int vdim, int pf, const int* cls, const double* rot,
                         int rotStride, int nR, const double* trans, int nT, const double* pC,
                         const double* pR, const double* pT, const float* dat, const float* ctf,
                         const float* sigRcp, const int* iCol, const int* iRow, int nPxl, int idim,
                         int nImg, float* wC, float* wR, float* wT, float* baseL, float* dvp,
                         const int* done, hipStream_t s, int nD = 0, const double* pD = nullptr,
                         float* wD = nullptr, const int* act = nullptr, const int* nAct = nullptr);
int local_phase_timed(const thx_local_sel* sel, hipEvent_t evBeg, hipEvent_t evEnd,
                      const float* vol, int volLayout, int vdim, int pf, const double* quat, int nR,
                      const double* trans, int nT, const double* pC, const double* pR,
                      const double* pT, const float* dat, const float* ctf, const float* sigRcp,
                      const int* iCol, const int* iRow, const int* pxOrder, int nOrd, int nPxl,
                      int idim, int nImg, float* wC, float* wR, float* wT, float* baseL,
                      void* workspace, size_t wsBytes, thx_stream_t stream, int nD = 0,
                      const double* pD = nullptr, float* wD = nullptr,
                      const float* ypair = nullptr, int* routeOut = nullptr,
                      const int* const* routeSample = nullptr, int ypairR = 0);
size_t ypair_ball_elems(int R);
int volume_ypair_ball(const float* vol, int vdim, int R, float* ypair, hipStream_t s);
bool phase_routed(int volLayout, int pf, int nPxl, int nD);
int pf_symmetrise_launch(int nImg, int mR, double* quat, int anchorMode, const double* anchor,
                         const double* symQ, int nSym, uint64_t seed, uint32_t stream,
                         const int* done, hipStream_t s);
size_t view_order_tmp_bytes(int nImg);
int view_order(int nImg, int mLR, const double* quat, unsigned* keys, unsigned* keysOut, int* idx,
               int* ord, void* tmp, size_t tmpBytes, hipStream_t s);
}

// max iCol^2 + iRow^2 over the pixel set (one workgroup)
__global__ void __launch_bounds__(256) k_max_r2(const int* __restrict__ iCol,
                                                const int* __restrict__ iRow, int nPxl,
                                                int* __restrict__ out)
{
    __shared__ int sm[4];
    int m = 0;
    for (int i = threadIdx.x; i < nPxl; i += 256) m = max(m, iCol[i] * iCol[i] + iRow[i] * iRow[i]);
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) *out = max(max(sm[0], sm[1]), max(sm[2], sm[3]));
}

// the 3D phases visit the images in view order (order.hip) and gather from
// the compact y-pair ball; THX_VIEW_ORDER=0 / THX_YPAIR_BALL=0 in the
// environment turn either off per call (the tests that they leave every
// image's result unchanged compare both)
static bool env_on(const char* name)
{
    const char* e = std::getenv(name);
    return !(e && e[0] == '0');
}
static bool view_order_on() { return env_on("THX_VIEW_ORDER"); }

namespace {

THX_DEV void qmul(const double* a, const double* b, double* o)
{
    // quaternion_mul (src/Geometry/Euler.cpp), Hamilton product
    const double w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    const double x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    const double y = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    const double z = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
    o[0] = w; o[1] = x; o[2] = y; o[3] = z;
}

// ------------------------------------------------- particle statistics (a10)
// Angular central Gaussian estimates of src/Geometry/DirectionalStat.cpp on
// one wave per image: lanes stride over the particles, every lane holds the
// 4x4 matrices (FP64) and repeats the tiny dense algebra.

// Inverse of a symmetric 4x4 matrix (every A of the ACG estimates is built
// symmetric): the adjugate from the six 2x2 minors of the top and bottom row
// pairs (Laplace expansion), upper triangle only, mirrored; det == 0 or a
// non-finite input gives NaNs (the reference's Eigen inverse of a singular A
// does too).  ~90 FP64 operations instead of the ~300 of 16 full cofactors.
// 1 / x from v_rcp_f64 and two Newton steps (within an ulp of the IEEE
// quotient, a third of its instructions: the fixed-point chains below are
// latency-bound).  Outside 2^-1021 <= |x| <= 2^1021 -- zero, infinities, NaN
// and the operands whose reciprocal leaves the normal range -- the IEEE
// quotient itself (1 / 0 = inf, 1 / inf = 0, where the Newton steps would
// give NaN), so degenerate clouds see the reference's division.
THX_DEV double rcp_nr(double x)
{
    const double ax = __builtin_fabs(x);
    if (!(ax >= 0x1p-1021 && ax <= 0x1p1021)) return 1.0 / x;
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    return fma(r, fma(-x, r, 1.0), r);
}

THX_DEV double inv4(const double* m, double* o)
{
    const double s0 = m[0] * m[5] - m[4] * m[1], s1 = m[0] * m[6] - m[4] * m[2];
    const double s2 = m[0] * m[7] - m[4] * m[3], s3 = m[1] * m[6] - m[5] * m[2];
    const double s4 = m[1] * m[7] - m[5] * m[3], s5 = m[2] * m[7] - m[6] * m[3];
    const double c5 = m[10] * m[15] - m[14] * m[11], c4 = m[9] * m[15] - m[13] * m[11];
    const double c3 = m[9] * m[14] - m[13] * m[10], c2 = m[8] * m[15] - m[12] * m[11];
    const double c1 = m[8] * m[14] - m[12] * m[10], c0 = m[8] * m[13] - m[12] * m[9];
    const double det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0;
    const double r = det != 0.0 ? rcp_nr(det) : __builtin_nan("");
    o[0] = (m[5] * c5 - m[6] * c4 + m[7] * c3) * r;
    o[1] = (-m[1] * c5 + m[2] * c4 - m[3] * c3) * r;
    o[2] = (m[13] * s5 - m[14] * s4 + m[15] * s3) * r;
    o[3] = (-m[9] * s5 + m[10] * s4 - m[11] * s3) * r;
    o[5] = (m[0] * c5 - m[2] * c2 + m[3] * c1) * r;
    o[6] = (-m[12] * s5 + m[14] * s2 - m[15] * s1) * r;
    o[7] = (m[8] * s5 - m[10] * s2 + m[11] * s1) * r;
    o[10] = (m[12] * s4 - m[13] * s2 + m[15] * s0) * r;
    o[11] = (-m[8] * s4 + m[9] * s2 - m[11] * s0) * r;
    o[15] = (m[8] * s3 - m[9] * s1 + m[10] * s0) * r;
    o[4] = o[1]; o[8] = o[2]; o[12] = o[3];
    o[9] = o[6]; o[13] = o[7]; o[14] = o[11];
    return det;
}

// inv4 with every 2x2 minor compensated (Kahan's a d - b c: the product b c
// and its FMA residual): the minors of a near-rank-1 A cancel by about the
// ratio of its eigenvalues, and the plain products leave the small
// eigen-directions of A^-1 -- the ones a de-meaning rotation exposes --
// with ~1e-6 relative error on a cloud of 1e-4 spread, the compensated ones
// with ~1e-8.  Used by calvari_acg_impl, whose second fixed point reads them.
THX_DEV double dop2(double a, double d, double b, double c)
{
    const double w = b * c;
    const double e = fma(-b, c, w);
    return fma(a, d, -w) + e;
}

THX_DEV double inv4_acc(const double* m, double* o)
{
    const double s0 = dop2(m[0], m[5], m[4], m[1]), s1 = dop2(m[0], m[6], m[4], m[2]);
    const double s2 = dop2(m[0], m[7], m[4], m[3]), s3 = dop2(m[1], m[6], m[5], m[2]);
    const double s4 = dop2(m[1], m[7], m[5], m[3]), s5 = dop2(m[2], m[7], m[6], m[3]);
    const double c5 = dop2(m[10], m[15], m[14], m[11]), c4 = dop2(m[9], m[15], m[13], m[11]);
    const double c3 = dop2(m[9], m[14], m[13], m[10]), c2 = dop2(m[8], m[15], m[12], m[11]);
    const double c1 = dop2(m[8], m[14], m[12], m[10]), c0 = dop2(m[8], m[13], m[12], m[9]);
    const double det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0;
    const double r = det != 0.0 ? rcp_nr(det) : __builtin_nan("");
    o[0] = (m[5] * c5 - m[6] * c4 + m[7] * c3) * r;
    o[1] = (-m[1] * c5 + m[2] * c4 - m[3] * c3) * r;
    o[2] = (m[13] * s5 - m[14] * s4 + m[15] * s3) * r;
    o[3] = (-m[9] * s5 + m[10] * s4 - m[11] * s3) * r;
    o[5] = (m[0] * c5 - m[2] * c2 + m[3] * c1) * r;
    o[6] = (-m[12] * s5 + m[14] * s2 - m[15] * s1) * r;
    o[7] = (m[8] * s5 - m[10] * s2 + m[11] * s1) * r;
    o[10] = (m[12] * s4 - m[13] * s2 + m[15] * s0) * r;
    o[11] = (-m[8] * s4 + m[9] * s2 - m[11] * s0) * r;
    o[15] = (m[8] * s3 - m[9] * s1 + m[10] * s0) * r;
    o[4] = o[1]; o[8] = o[2]; o[12] = o[3];
    o[9] = o[6]; o[13] = o[7]; o[14] = o[11];
    return det;
}

// A symmetric matrix packed as its upper triangle with the off-diagonal
// entries doubled, so q^T M q = sum_j q_j sum_{k >= j} Mp_jk q_k (14 FMAs).
THX_DEV void pack10(const double* M, double* Mp)
{
    int t = 0;
    for (int j = 0; j < 4; j++)
        for (int k = j; k < 4; k++) Mp[t++] = (j == k ? 1.0 : 2.0) * M[4 * j + k];
}
THX_DEV double quad10(const double* Mp, const double* q)
{
    double s = 0.0;
    int t = 0;
    for (int j = 0; j < 4; j++) {
        double a = 0.0;
        for (int k = j; k < 4; k++) a += Mp[t++] * q[k];
        s += q[j] * a;
    }
    return s;
}

// Particle statistics run one image per GROUP lanes (8 images per wave): the
// 4x4 algebra is repeated by every lane anyway, so narrower groups mean
// fewer waves for the same latency-bound FP64 chains, and each lane's 16
// register-resident particles give the fixed point's quadratic forms ILP.
// Measured on 12 500 x 125 (tools/pf_bench.py, profiles/r02_pf_group_ab.jsonl):
// calVari 0.145 / 0.105 ms at GROUP 16 / 8 on 3-degree clouds, 32 and 64 slower.
constexpr int GROUP = 8;

// v from another lane of the row by DPP (both 32-bit halves)
template <int CTRL>
THX_DEV double dpp_d(double v)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    // every lane's source lies inside its row: no 'old' operand to initialise
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Sum over the GROUP lanes of an image, the same value in every lane.  For
// GROUP 8 by DPP (quad pairs, quad halves, then the row's half mirror pairs
// the two quads): VALU moves instead of three dependent ds_bpermute rounds
// per value, 11 values per fixed-point pass.
THX_DEV double group_sum(double v)
{
    if constexpr (GROUP == 8) {
        v += dpp_d<0xb1>(v);    // quad_perm [1, 0, 3, 2]
        v += dpp_d<0x4e>(v);    // quad_perm [2, 3, 0, 1]
        v += dpp_d<0x141>(v);   // row_half_mirror: lane i <-> 7 - i of its 8
        return v;
    }
#pragma unroll
    for (int o = GROUP / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// inferACG(dmat44&, const dmat4&), DirectionalStat.cpp:93-145: Tyler's fixed
// point B = 4/nf sum q q^T / (q^T A^-1 q) from B = I while sum|A - B| > 1e-3
// (a NaN criterion ends the loop, as in the reference's `while`); returns the
// last A.  Particle q_i is read as pre q_i (pre = conj(mean) de-means).
// Clouds of up to GROUP * QREG particles keep this lane's (de-meaned)
// particles in registers across the iterations -- the loop is a serial
// chain, and re-reading them from L2 every iteration was its latency.  Each
// lane then holds a block of QREG consecutive particles as runs of equal
// ones: a resampled cloud stores an ancestor's copies next to each other, so
// the term of a run is taken once with its multiplicity.  The degenerate
// clouds that run the fixed point to its cap are the ones with a few
// ancestors, so their iterations cost one or two terms per lane instead of
// QREG.  The sum is the reference's up to rounding (multiplicity x term for
// repeated additions, block for strided order).
constexpr int QREG = 128 / GROUP;

// idx (optional): particle i is Q[idx[i]] -- a resampled cloud read through
// its ancestors, in the gathered order, without the gather
template <bool REG>
THX_DEV int infer_acg_impl(const double* Q, int m, const double* pre, int lane, double* A,
                           int maxIt, const int* idx = nullptr)
{
    auto at = [&](int i) { return Q + 4 * (idx ? idx[i] : i); };
    double qr[REG ? QREG : 1][4];
    int nd = 0, nIn = 0;                          // runs, particles this lane holds
    unsigned runs = 0;                            // bit p: block particle p starts a run
    if (REG) {
        const int i0 = lane * QREG;
        nIn = max(0, min(QREG, m - i0));
        unsigned starts = 0;
        double prev[4] = {0, 0, 0, 0};
#pragma unroll
        for (int p = 0; p < QREG; p++) {
            if (p < nIn) {
                const double* c = at(i0 + p);
                const double c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
                if (p == 0 || c0 != prev[0] || c1 != prev[1] || c2 != prev[2] || c3 != prev[3])
                    starts |= 1u << p;
                prev[0] = c0; prev[1] = c1; prev[2] = c2; prev[3] = c3;
            }
        }
        runs = starts;
        nd = __builtin_popcount(starts);
#pragma unroll
        for (int p = 0; p < QREG; p++) {
            if (starts) {
                const double* c = at(i0 + __builtin_ctz(starts));
                starts &= starts - 1;
                if (pre) qmul(pre, c, qr[p]);
                else for (int k = 0; k < 4; k++) qr[p][k] = c[k];
            }
        }
    }
    double B[16];
    for (int k = 0; k < 16; k++) B[k] = (k % 5 == 0) ? 1.0 : 0.0;
    for (int it = 0; it < maxIt; it++) {
        for (int k = 0; k < 16; k++) A[k] = B[k];
        double Ai[16], Mp[10];
        inv4(A, Ai);
        pack10(Ai, Mp);
        double b[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, nf = 0.0;
        auto term = [&](const double* q, double w) {
            const double r = w * rcp_nr(quad10(Mp, q));
            int t = 0;
            for (int j = 0; j < 4; j++) {
                const double qj = q[j] * r;
                for (int k = j; k < 4; k++) b[t++] += qj * q[k];
            }
            nf += r;
        };
        if (REG) {
            unsigned rs = runs;
#pragma unroll
            for (int p = 0; p < QREG; p++) {
                if (p < nd) {
                    const int s0 = __builtin_ctz(rs);
                    rs &= rs - 1;
                    term(qr[p], (double)((rs ? __builtin_ctz(rs) : nIn) - s0));
                }
            }
        } else {
            for (int i = lane; i < m; i += GROUP) {
                double q[4];
                const double* c = at(i);
                if (pre) qmul(pre, c, q);
                else for (int k = 0; k < 4; k++) q[k] = c[k];
                term(q, 1.0);
            }
        }
        for (int t = 0; t < 10; t++) b[t] = group_sum(b[t]);
        nf = group_sum(nf);
        int t = 0;
        for (int j = 0; j < 4; j++)
            for (int k = j; k < 4; k++, t++) B[4 * j + k] = B[4 * k + j] = b[t] * (4.0 * rcp_nr(nf));
        double crit = 0.0;
        for (int k = 0; k < 16; k++) crit += fabs(A[k] - B[k]);
        if (!(crit > 1e-3)) return it + 1;
    }
    return maxIt;
}

THX_DEV int infer_acg(const double* Q, int m, const double* pre, int lane, double* A,
                      int maxIt = 256, const int* idx = nullptr)
{
    return m <= GROUP * QREG ? infer_acg_impl<true>(Q, m, pre, lane, A, maxIt, idx)
                             : infer_acg_impl<false>(Q, m, pre, lane, A, maxIt, idx);
}

// Unit eigenvector of the largest eigenvalue of a symmetric 4x4 (cyclic
// Jacobi), the mean of inferACG(dvec4&, ...), DirectionalStat.cpp:224-251.
THX_DEV void principal_axis(const double* A0, double* v)
{
    double a[16], V[16];
    for (int k = 0; k < 16; k++) { a[k] = A0[k]; V[k] = (k % 5 == 0) ? 1.0 : 0.0; }
    for (int sweep = 0; sweep < 32; sweep++) {
        double off = 0.0, dia = 0.0;
        for (int p = 0; p < 4; p++)
            for (int q = 0; q < 4; q++) (p == q ? dia : off) += a[4 * p + q] * a[4 * p + q];
        if (!(off > 1e-30 * dia)) break;
        for (int p = 0; p < 3; p++)
            for (int q = p + 1; q < 4; q++) {
                const double apq = a[4 * p + q];
                if (apq == 0.0) continue;
                const double th = (a[4 * q + q] - a[4 * p + p]) / (2.0 * apq);
                const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 4; k++) {      // a <- a J
                    const double x = a[4 * k + p], y = a[4 * k + q];
                    a[4 * k + p] = c * x - s * y;
                    a[4 * k + q] = s * x + c * y;
                }
                for (int k = 0; k < 4; k++) {      // a <- J^T a
                    const double x = a[4 * p + k], y = a[4 * q + k];
                    a[4 * p + k] = c * x - s * y;
                    a[4 * q + k] = s * x + c * y;
                }
                for (int k = 0; k < 4; k++) {      // V <- V J
                    const double x = V[4 * k + p], y = V[4 * k + q];
                    V[4 * k + p] = c * x - s * y;
                    V[4 * k + q] = s * x + c * y;
                }
            }
    }
    int best = 0;
    for (int k = 1; k < 4; k++)
        if (a[5 * k] > a[5 * best]) best = k;
    double n = 0.0;
    for (int k = 0; k < 4; k++) n += V[4 * k + best] * V[4 * k + best];
    n = sqrt(n);
    for (int k = 0; k < 4; k++) v[k] = V[4 * k + best] / n;
}

// calVari's two fixed points from one (k_pf_calvari with a history buffer).
// The de-meaned cloud q' = c q (c = conj(mean), a unit quaternion) is the
// cloud under the orthogonal map M: q -> c q, and Tyler's map commutes with
// it (q'^T (M A M^T)^-1 q' = q^T A^-1 q, so F(M A M^T) = M F(A) M^T): from
// B'_0 = I = M I M^T the second fixed point's iterates are B'_k = M B_k M^T,
// B_k the first's.  The first pass keeps its iterates in hist (10 doubles
// each, lane 0 of the group); the second pass's stopping rule (sum |A' - B'|,
// not invariant under M, so it may stop before or after the first) is then
// evaluated on the replayed iterates, GROUP iterations at a time, one per
// lane, and the first recurrence is continued when the second needs more
// iterates than the first pass made.  Equal to the two passes in exact
// arithmetic; the rounding differs from iterating on c q, as any summation
// order does.  Returns the second fixed point's A in A2 (every lane).
constexpr int ACG_HIST_MAX = 256;      // infer_acg's cap, the history's length per image
constexpr int ACG_HIST = 10 * ACG_HIST_MAX;

// B' = M B M^T of a symmetric B given as its upper triangle u (row-major j <= k)
THX_DEV void acg_conj(const double* M, const double* u, double* P)
{
    double B[16];
    int t = 0;
    for (int j = 0; j < 4; j++)
        for (int k = j; k < 4; k++, t++) B[4 * j + k] = B[4 * k + j] = u[t];
    double T[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            T[4 * i + j] = M[4 * i] * B[j] + M[4 * i + 1] * B[4 + j] + M[4 * i + 2] * B[8 + j] +
                           M[4 * i + 3] * B[12 + j];
    for (int i = 0; i < 4; i++)
        for (int j = i; j < 4; j++)
            P[4 * i + j] = P[4 * j + i] = T[4 * i] * M[4 * j] + T[4 * i + 1] * M[4 * j + 1] +
                                          T[4 * i + 2] * M[4 * j + 2] + T[4 * i + 3] * M[4 * j + 3];
}

THX_DEV void acg_conj_hist(const double* M, const double* h, double* P)
{
    const double2* h2 = reinterpret_cast<const double2*>(h);
    double u[10];
    for (int t = 0; t < 5; t++) {
        const double2 v = h2[t];
        u[2 * t] = v.x; u[2 * t + 1] = v.y;
    }
    acg_conj(M, u, P);
}

template <bool REG>
THX_DEV void calvari_acg_impl(const double* Q, int m, int lane, double* __restrict__ hist,
                              double* A2)
{
    constexpr int maxIt = ACG_HIST_MAX;
    double qr[REG ? QREG : 1][4];
    int nd = 0, nIn = 0;
    unsigned runs = 0;
    if (REG) {                                     // as infer_acg_impl
        const int i0 = lane * QREG;
        nIn = max(0, min(QREG, m - i0));
        unsigned starts = 0;
        double prev[4] = {0, 0, 0, 0};
#pragma unroll
        for (int p = 0; p < QREG; p++) {
            if (p < nIn) {
                const double* c = Q + 4 * (i0 + p);
                const double c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
                if (p == 0 || c0 != prev[0] || c1 != prev[1] || c2 != prev[2] || c3 != prev[3])
                    starts |= 1u << p;
                prev[0] = c0; prev[1] = c1; prev[2] = c2; prev[3] = c3;
            }
        }
        runs = starts;
        nd = __builtin_popcount(starts);
#pragma unroll
        for (int p = 0; p < QREG; p++) {
            if (starts) {
                const double* c = Q + 4 * (i0 + __builtin_ctz(starts));
                starts &= starts - 1;
                for (int k = 0; k < 4; k++) qr[p][k] = c[k];
            }
        }
    }
    double A[16], B[16];
    for (int k = 0; k < 16; k++) B[k] = (k % 5 == 0) ? 1.0 : 0.0;
    // one pass of the fixed point (infer_acg_impl's): A <- B, B <- F(A); sum
    // |A - B|.  fromMem: the particles re-read from Q (the continuation past
    // the history, so that the register cloud is dead during the replay)
    auto step = [&](bool fromMem) -> double {
        for (int k = 0; k < 16; k++) A[k] = B[k];
        double Ai[16], Mp[10];
        inv4_acc(A, Ai);
        pack10(Ai, Mp);
        double b[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, nf = 0.0;
        auto term = [&](const double* q, double w) {
            const double r = w * rcp_nr(quad10(Mp, q));
            int t = 0;
            for (int j = 0; j < 4; j++) {
                const double qj = q[j] * r;
                for (int k = j; k < 4; k++) b[t++] += qj * q[k];
            }
            nf += r;
        };
        if (REG && !fromMem) {
            unsigned rs = runs;
#pragma unroll
            for (int p = 0; p < QREG; p++) {
                if (p < nd) {
                    const int s0 = __builtin_ctz(rs);
                    rs &= rs - 1;
                    term(qr[p], (double)((rs ? __builtin_ctz(rs) : nIn) - s0));
                }
            }
        } else {
            for (int i = lane; i < m; i += GROUP) term(Q + 4 * i, 1.0);
        }
        for (int t = 0; t < 10; t++) b[t] = group_sum(b[t]);
        nf = group_sum(nf);
        int t = 0;
        for (int j = 0; j < 4; j++)
            for (int k = j; k < 4; k++, t++) B[4 * j + k] = B[4 * k + j] = b[t] * (4.0 * rcp_nr(nf));
        double crit = 0.0;
        for (int k = 0; k < 16; k++) crit += fabs(A[k] - B[k]);
        return crit;
    };
    // first fixed point, its iterates B_1 .. B_it1 kept
    int it1 = maxIt;
    for (int it = 0; it < maxIt; it++) {
        const double crit = step(false);
        if (lane == 0) {
            double2* h2 = reinterpret_cast<double2*>(hist + 10 * it);
            h2[0] = make_double2(B[0], B[1]);
            h2[1] = make_double2(B[2], B[3]);
            h2[2] = make_double2(B[5], B[6]);
            h2[3] = make_double2(B[7], B[10]);
            h2[4] = make_double2(B[11], B[15]);
        }
        if (!(crit > 1e-3)) { it1 = it + 1; break; }
    }
    double mean[4];
    principal_axis(A, mean);
    // M: q -> qmul(c, q), c = conj(mean)
    const double ca = mean[0], cb = -mean[1], cc = -mean[2], cd = -mean[3];
    const double M[16] = {ca, -cb, -cc, -cd, cb, ca, -cd, cc, cc, cd, ca, -cb, cd, -cc, cb, ca};
    // the group's lane 0 wrote the history: make it visible to the group's lanes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // replay: iteration k of the second pass compares B'_k with B'_{k+1}
    // (B'_k = M hist[k - 1] M^T, B'_0 = I) and stops at the first k where
    // !(sum |B'_k - B'_{k+1}| > 1e-3), returning B'_k
    const int gBase = (int)(threadIdx.x & 63) & ~(GROUP - 1);
    int kStop = -1;
    for (int k0 = 0; k0 < it1 && kStop < 0; k0 += GROUP) {
        const int k = k0 + lane;
        bool stop = false;
        if (k < it1) {
            double Pk[16], Pn[16];
            if (k == 0) for (int t = 0; t < 16; t++) Pk[t] = (t % 5 == 0) ? 1.0 : 0.0;
            else acg_conj_hist(M, hist + 10 * (k - 1), Pk);
            acg_conj_hist(M, hist + 10 * k, Pn);
            double crit = 0.0;
            for (int t = 0; t < 16; t++) crit += fabs(Pk[t] - Pn[t]);
            stop = !(crit > 1e-3);
        }
        const unsigned bits = (unsigned)(__ballot(stop) >> gBase) & ((1u << GROUP) - 1);
        if (bits) kStop = k0 + __builtin_ctz(bits);
    }
    if (kStop == 0) {
        for (int t = 0; t < 16; t++) A2[t] = (t % 5 == 0) ? 1.0 : 0.0;
        return;
    }
    if (kStop > 0 || it1 == maxIt) {               // stopped in the history, or ran to the cap
        acg_conj_hist(M, hist + 10 * ((kStop > 0 ? kStop : maxIt) - 1), A2);
        return;
    }
    // the second pass needs iterates past the first's: continue the first
    // recurrence from (B_{it1 - 1}, B_it1)
    double P[16];
    {
        double u[10];
        int t = 0;
        for (int j = 0; j < 4; j++)
            for (int k = j; k < 4; k++, t++) u[t] = B[4 * j + k];
        acg_conj(M, u, P);                         // B'_it1
    }
    for (int k = it1; k < maxIt; k++) {
        for (int t = 0; t < 16; t++) A2[t] = P[t];
        step(true);
        double u[10], Pn[16];
        int t = 0;
        for (int j = 0; j < 4; j++)
            for (int i = j; i < 4; i++, t++) u[t] = B[4 * j + i];
        acg_conj(M, u, Pn);
        double crit = 0.0;
        for (int q = 0; q < 16; q++) crit += fabs(A2[q] - Pn[q]);
        if (!(crit > 1e-3)) return;
        for (int q = 0; q < 16; q++) P[q] = Pn[q];
    }
}

// Particle::calVari (src/Particle.cpp:1004-1121), 3D: R -- de-mean by the
// ACG principal axis (PARTICLE_ROT_MEAN_USING_STAT_CAL_VARI), k_j =
// A(j, j) / A(0, 0) of inferACG on the de-meaned cloud (:184-222), floored at
// kFloor; T -- sample standard deviations (gsl_stats_sd), floored at sFloor
// (the reseed floors of src/Optimiser.cpp:1033-1079).
__global__ void __launch_bounds__(256) k_pf_calvari(int nImg, int mR, const double* __restrict__ quat,
                                                    int mT, const double* __restrict__ trans,
                                                    double kFloor, double sFloor,
                                                    double* __restrict__ kOut,
                                                    double* __restrict__ sOut,
                                                    const int* __restrict__ done = nullptr,
                                                    double* __restrict__ hist = nullptr)
{
    const int l = (blockIdx.x * 256 + threadIdx.x) / GROUP;
    const int lane = threadIdx.x % GROUP;
    if (l >= nImg || (done && done[l])) return;
    const double* Q = quat + (size_t)l * mR * 4;
    double A[16];
    if (hist) {
        // both fixed points from one (calvari_acg_impl)
        double* h = hist + (size_t)l * ACG_HIST;
        if (mR <= GROUP * QREG) calvari_acg_impl<true>(Q, mR, lane, h, A);
        else calvari_acg_impl<false>(Q, mR, lane, h, A);
    } else {
        double mean[4], cm[4];
        infer_acg(Q, mR, nullptr, lane, A);
        principal_axis(A, mean);
        cm[0] = mean[0]; cm[1] = -mean[1]; cm[2] = -mean[2]; cm[3] = -mean[3];
        infer_acg(Q, mR, cm, lane, A);
    }
    const double* Tr = trans + (size_t)l * mT * 2;
    double sx = 0, sy = 0;
    for (int i = lane; i < mT; i += GROUP) { sx += Tr[2 * i]; sy += Tr[2 * i + 1]; }
    sx = group_sum(sx) / mT; sy = group_sum(sy) / mT;
    double vx = 0, vy = 0;
    for (int i = lane; i < mT; i += GROUP) {
        vx += (Tr[2 * i] - sx) * (Tr[2 * i] - sx);
        vy += (Tr[2 * i + 1] - sy) * (Tr[2 * i + 1] - sy);
    }
    vx = group_sum(vx); vy = group_sum(vy);
    if (lane == 0) {
        for (int j = 1; j < 4; j++) kOut[3 * l + j - 1] = fmax(kFloor, A[5 * j] / A[0]);
        sOut[2 * l] = fmax(sFloor, mT > 1 ? sqrt(vx / (mT - 1)) : 0.0);
        sOut[2 * l + 1] = fmax(sFloor, mT > 1 ? sqrt(vy / (mT - 1)) : 0.0);
    }
}

// Particle::balanceWeight(PAR_R), 3D (src/Particle.cpp:2330-2340):
// w_i = 1 / pdfACG(q_i, inferACG(Q)), pdfACG = det(A)^-1/2 (q^T A^-1 q)^-2
// (DirectionalStat.cpp:19-24), normalised to sum 1 (the scale cancels in
// resample's w u / sum).
THX_DEV void balance_rot(const double* Q, int m, int lane, double* w)
{
    double A[16], Ai[16], Mp[10];
    infer_acg(Q, m, nullptr, lane, A);
    const double det = inv4(A, Ai);
    pack10(Ai, Mp);
    const double sd = sqrt(det);
    double tot = 0.0;
    for (int i = lane; i < m; i += GROUP) {
        const double u = quad10(Mp, Q + 4 * i);
        const double x = sd * u * u;
        w[i] = x;
        tot += x;
    }
    tot = group_sum(tot);
    for (int i = lane; i < m; i += GROUP) w[i] /= tot;
}

// Particle::setPeakFactor(PAR_R) (src/Particle.cpp:1920-1925) when
// setFactor: peak = clamp(u_(n/rankDiv) / u_max, 1e-3, 0.5) -- rankDiv =
// PEAK_FACTOR_BASE^3 = 8 in 3D, PEAK_FACTOR_BASE = 2 in 2D -- with u_(k) the k-th
// largest (0-based); then keepHalfHeightPeak (:1964-1984) in place:
// u <- u < hh ? 0 : u - hh, hh = u_max peak.  u >= 0, so the k-th largest is
// found by a bisection over the ordered float bit patterns.
__global__ void __launch_bounds__(256) k_pf_peak(int nImg, int n, float* __restrict__ u, int ldu,
                                                 double* __restrict__ peak, int setFactor,
                                                 const int* __restrict__ cls = nullptr, int ldc = 0,
                                                 const int* __restrict__ done = nullptr,
                                                 int rankDiv = 8)
{
    const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (l >= nImg || (done && done[l])) return;
    float* ul = u + (size_t)l * ldu + (cls ? (size_t)cls[l] * ldc : 0);
    // up to PEAK_REG x 64 values stay in registers for the bisection (the
    // global scan's 2000 rotations: each of its ~32 passes re-read them from
    // L2, 0.47 ms per 12 500-image call)
    constexpr int PEAK_REG = 32;
    const bool reg = n <= 64 * PEAK_REG;
    uint32_t v[PEAK_REG];
    float mx = 0.f;
    if (reg) {
#pragma unroll
        for (int q = 0; q < PEAK_REG; q++) {
            const int i = lane + 64 * q;
            v[q] = i < n ? __float_as_uint(ul[i]) : 0u;   // (u >= 0: 0 counts below any mid > 0)
            if (i < n) mx = fmaxf(mx, __uint_as_float(v[q]));
        }
    } else {
        for (int i = lane; i < n; i += 64) mx = fmaxf(mx, ul[i]);
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    double pk;
    if (setFactor) {
        const int k = n / rankDiv;
        // largest bit pattern v with count(u >= v) >= k + 1
        uint32_t lo = 0, hi = __float_as_uint(mx);
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo + 1) / 2;
            int c = 0;
            if (reg) {
#pragma unroll
                for (int q = 0; q < PEAK_REG; q++) c += v[q] >= mid;
            } else {
                for (int i = lane; i < n; i += 64) c += __float_as_uint(ul[i]) >= mid;
            }
            for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
            if (c >= k + 1) lo = mid; else hi = mid - 1;
        }
        const double r = mx > 0.f ? (double)__uint_as_float(lo) / (double)mx : 0.0;
        pk = fmax(1e-3, fmin(0.5, r));
        if (lane == 0) peak[l] = pk;
    } else {
        pk = peak[l];
    }
    const double hh = (double)mx * pk;
    for (int i = lane; i < n; i += 64) {
        const double v = ul[i];
        ul[i] = v < hh ? 0.f : (float)(v - hh);
    }
}

__global__ void __launch_bounds__(256) k_pf_balance_rot(int nImg, int mR,
                                                        const double* __restrict__ quat,
                                                        double* __restrict__ pR)
{
    const int l = (blockIdx.x * 256 + threadIdx.x) / GROUP;
    if (l >= nImg) return;
    balance_rot(quat + (size_t)l * mR * 4, mR, threadIdx.x % GROUP, pR + (size_t)l * mR);
}

// --------------------------------------------------------------- resample
constexpr int RESAMPLE_KMAX = 2048;

// Dynamic LDS of a k_pf_resample launch (keys of the bitonic shuffle).
size_t resample_lds(int nIn, bool shuffle)
{
    if (!shuffle || nIn > RESAMPLE_KMAX) return 0;
    int n = 1;
    while (n < nIn) n <<= 1;
    return (size_t)4 * n * sizeof(uint64_t);
}


// Bitonic sort of one wave's 64 KPL distinct 64-bit keys held in registers:
// position p = KPL lane + r is kv[r] of lane `lane`.  Pairs (p, p ^ j) with
// j < KPL sit in one lane (BitonicIn); the others are lanes lane ^ (j / KPL)
// at the same r, exchanged by ds_bpermute (__shfl_xor).  The keys are
// distinct, so the sorted sequence -- the only thing the caller reads -- is
// that of any other correct sort (the LDS network it replaces).
template <int J, int KPL>
THX_DEV void bitonic_in(uint64_t (&kv)[KPL], int lane, int k)
{
#pragma unroll
    for (int r = 0; r < KPL; r++) {
        if (r & J) continue;
        const bool asc = ((KPL * lane + r) & k) == 0;
        const uint64_t a = kv[r], b = kv[r | J];
        // ascending pairs put the minimum first, descending ones the maximum
        const bool sw = (a > b) == asc;
        kv[r] = sw ? b : a;
        kv[r | J] = sw ? a : b;
    }
}

template <int KPL>
THX_DEV void wave_bitonic(uint64_t (&kv)[KPL], int lane)
{
    constexpr int N = 64 * KPL;
    for (int k = 2; k <= N; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= KPL) {
                const int lm = j / KPL;
                const bool upper = (lane & lm) != 0;
                // every partner first (the exchanges in flight together), then
                // the compare-exchanges
                uint64_t o[KPL];
#pragma unroll
                for (int r = 0; r < KPL; r++) {
                    const uint32_t lo = __shfl_xor((uint32_t)kv[r], lm, 64);
                    const uint32_t hi = __shfl_xor((uint32_t)(kv[r] >> 32), lm, 64);
                    o[r] = ((uint64_t)hi << 32) | lo;
                }
#pragma unroll
                for (int r = 0; r < KPL; r++) {
                    const bool asc = ((KPL * lane + r) & k) == 0;
                    // the lower position of an ascending pair keeps the minimum
                    const bool keepMin = upper != asc;
                    kv[r] = (o[r] < kv[r]) == keepMin ? o[r] : kv[r];
                }
            } else if (KPL >= 2 && j == 1) {
                bitonic_in<1, KPL>(kv, lane, k);
            } else if (KPL >= 4 && j == 2) {
                bitonic_in<2, KPL>(kv, lane, k);
            } else if (KPL >= 8 && j == 4) {
                bitonic_in<4, KPL>(kv, lane, k);
            } else if (KPL >= 16 && j == 8) {
                bitonic_in<8, KPL>(kv, lane, k);
            } else if (KPL >= 32 && j == 16) {
                bitonic_in<16, KPL>(kv, lane, k);
            }
        }
}

// The shuffle's keys of one image, sorted in registers: lane `lane` draws the
// keys of entries i = lane + 64 m (the LDS network's draws, same Philox
// stream and order), the wave sorts them, and position p's index half goes
// to k32[p] for p < nIn.
template <int KPL>
THX_DEV void shuffle_keys_reg(Philox& sh, int nIn, int lane, uint32_t* k32)
{
    uint64_t kv[KPL];
    uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int m = 0; m < KPL; m++) {
        if ((m & 3) == 0) v = sh.next();
        const uint32_t x = (m & 3) == 0 ? v.x : (m & 3) == 1 ? v.y : (m & 3) == 2 ? v.z : v.w;
        const int i = lane + 64 * m;
        kv[m] = i < nIn ? ((uint64_t)x << 32) | (uint64_t)i : ~0ull;
    }
    wave_bitonic<KPL>(kv, lane);
#pragma unroll
    for (int r = 0; r < KPL; r++) {
        const int p = KPL * lane + r;
        if (p < nIn) k32[p] = (uint32_t)kv[r];
    }
}

// The reseed's shuffle on its own (one wave per image): the permutation of a
// support of 64 KPL / 2 < nIn <= 64 KPL entries, sorted in registers, into
// perm[l][.] -- k_pf_resample<.., true> then reads it, so the resampling
// proper keeps its low register count and occupancy
template <int KPL>
__global__ void __launch_bounds__(256) k_pf_shuffle_perm(int nImg, int nIn, uint64_t seed,
                                                         uint32_t stream, int* __restrict__ perm,
                                                         const int* __restrict__ done)
{
    const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (l >= nImg || (done && done[l])) return;
    Philox sh(seed, (uint32_t)l, stream, 0x5f1e0000u | (uint32_t)lane);
    uint64_t kv[KPL];
    uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int m = 0; m < KPL; m++) {
        if ((m & 3) == 0) v = sh.next();
        const uint32_t x = (m & 3) == 0 ? v.x : (m & 3) == 1 ? v.y : (m & 3) == 2 ? v.z : v.w;
        const int i = lane + 64 * m;
        kv[m] = i < nIn ? ((uint64_t)x << 32) | (uint64_t)i : ~0ull;
    }
    wave_bitonic<KPL>(kv, lane);
    int* pl = perm + (size_t)l * nIn;
#pragma unroll
    for (int r = 0; r < KPL; r++) {
        const int p = KPL * lane + r;
        if (p < nIn) pl[p] = (int)(uint32_t)kv[r];
    }
}

// One wave per image: systematic resampling (src/Particle.cpp:1343-1383) of
// (w, u) -> ancestors and 1/u priors; w may be shared by all images (ldw = 0).
// u0 ~ U(0, 1/nOut) is drawn from the counter RNG.  w and wOut may alias (the
// in-phase resamples overwrite the priors in place: every read of w comes
// before the barrier that precedes the first store to wOut), so neither is
// __restrict__.  permOut / u0Out (optional) expose the support permutation
// and the draw for thx_pf_resample's parity tests.
// REGKPL: supports of 64 .. 64 REGKPL entries (next power of two) sort in
// registers (wave_bitonic), the rest in LDS; the reseed's 2000-entry support
// uses 32 keys per lane (the LDS network took ~1.0 ms of its 1.26 ms per
// 12 500-image call), the phases' supports 4 (fewer VGPRs, more waves)
template <int REGKPL, bool PRE = false>
__global__ void __launch_bounds__(256) k_pf_resample(int nImg, int nIn, int nOut,
                                                     const double* w, int ldw,
                                                     const float* __restrict__ u, int ldu,
                                                     uint64_t seed, uint32_t stream,
                                                     int* __restrict__ anc,
                                                     double* wOut,
                                                     int* __restrict__ top,
                                                     double* __restrict__ cdfWs,
                                                     int* __restrict__ permWs,
                                                     int* __restrict__ permOut,
                                                     double* __restrict__ u0Out,
                                                     const int* __restrict__ cls = nullptr,
                                                     int ldc = 0,
                                                     const int* __restrict__ done = nullptr)
{
    const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (l >= nImg || (done && done[l])) return;
    const double* wl = w + (size_t)l * ldw;
    const float* ul = u + (size_t)l * ldu + (cls ? (size_t)cls[l] * ldc : 0);
    double* cdf = cdfWs + (size_t)l * nIn;
    // Particle::shuffle before resampling (src/Particle.cpp:1298, 2202-2300):
    // a uniform random permutation of the support (gsl_ran_shuffle); position
    // i of the shuffled support holds element pm[i], so the CDF, the top
    // particle (iMax, first maximum in shuffled order) and the systematic
    // draw all run in shuffled order.  Up to 2048 entries the wave sorts
    // 64-bit (32 random bits | index) keys with a bitonic network in LDS --
    // all 64 lanes work; the index half makes the keys distinct, so the sorted
    // indices are a permutation, and two entries tie on their random halves
    // (and keep their index order) with probability ~nIn^2 / 2^33 per shuffle
    // (a one-lane Fisher-Yates took 1.4 ms per 12 500-image call at 2000
    // entries, a rank count 7 ms).  Larger supports fall back to Fisher-Yates
    // by lane 0 in global memory.
    // The keys live in dynamic LDS sized by the launch (resample_lds): 4 waves
    // x the next power of two >= nIn keys, so small supports (the phases'
    // mLR, mLT) do not pin 64 KiB per workgroup.
    constexpr int KMAX = RESAMPLE_KMAX;
    extern __shared__ __attribute__((aligned(16))) uint64_t sKeyDyn[];
    int* pm = permWs ? permWs + (size_t)l * nIn : nullptr;
    int regN = 1;
    while (regN < nIn) regN <<= 1;
    const bool regSort = !PRE && pm && regN >= 64 && regN <= 64 * REGKPL;
    if (PRE && pm && nIn <= KMAX) {
        // k_pf_shuffle_perm left the permutation in pm: into this wave's LDS row
        int* k32 = reinterpret_cast<int*>(sKeyDyn + (size_t)(threadIdx.x >> 6) * regN);
        for (int i = lane; i < nIn; i += 64) k32[i] = pm[i];
        pm = k32;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else if (PRE && pm) {
        // (larger supports read the permutation where it lies)
    } else if (regSort) {
        uint32_t* k32 = reinterpret_cast<uint32_t*>(sKeyDyn + (size_t)(threadIdx.x >> 6) * regN);
        Philox sh(seed, (uint32_t)l, stream, 0x5f1e0000u | (uint32_t)lane);
        const int kpl = regN / 64;
        if (REGKPL >= 32 && kpl == 32) shuffle_keys_reg<(REGKPL >= 32 ? 32 : 1)>(sh, nIn, lane, k32);
        else if (REGKPL >= 16 && kpl == 16) shuffle_keys_reg<(REGKPL >= 16 ? 16 : 1)>(sh, nIn, lane, k32);
        else if (REGKPL >= 8 && kpl == 8) shuffle_keys_reg<(REGKPL >= 8 ? 8 : 1)>(sh, nIn, lane, k32);
        else if (REGKPL >= 4 && kpl == 4) shuffle_keys_reg<(REGKPL >= 4 ? 4 : 1)>(sh, nIn, lane, k32);
        else if (REGKPL >= 2 && kpl == 2) shuffle_keys_reg<(REGKPL >= 2 ? 2 : 1)>(sh, nIn, lane, k32);
        else shuffle_keys_reg<1>(sh, nIn, lane, k32);
        pm = reinterpret_cast<int*>(k32);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else if (pm && nIn <= KMAX) {
        int ib = 0;
        while ((1 << ib) < nIn) ib++;
        const int N = 1 << ib;
        uint64_t* kk = sKeyDyn + (size_t)(threadIdx.x >> 6) * N;
        Philox sh(seed, (uint32_t)l, stream, 0x5f1e0000u | (uint32_t)lane);
        uint4 v = make_uint4(0, 0, 0, 0);
        for (int i = lane, k = 0; i < N; i += 64, k = (k + 1) & 3) {
            if (k == 0) v = sh.next();
            const uint32_t x = k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
            // padding (i >= nIn) is all ones and sorts last: a real key has an
            // index half < 2048
            kk[i] = i < nIn ? ((uint64_t)x << 32) | (uint64_t)i : ~0ull;
        }
        // one stage: the N/2 disjoint pairs (i, i + j), four per lane loaded
        // before any is compared and stored (a quarter of the LDS round trips
        // of pair-at-a-time)
        constexpr int PPL = 4;
        for (int k = 2; k <= N; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                for (int p0 = 0; p0 < (N >> 1); p0 += 64 * PPL) {
                    uint64_t x[PPL], y[PPL];
#pragma unroll
                    for (int u = 0; u < PPL; u++) {
                        const int p = p0 + lane + 64 * u;
                        const int i = ((p & ~(j - 1)) << 1) | (p & (j - 1));
                        if (p < (N >> 1)) { x[u] = kk[i]; y[u] = kk[i + j]; }
                    }
#pragma unroll
                    for (int u = 0; u < PPL; u++) {
                        const int p = p0 + lane + 64 * u;
                        const int i = ((p & ~(j - 1)) << 1) | (p & (j - 1));
                        if (p < (N >> 1) && (x[u] > y[u]) == ((i & k) == 0)) {
                            kk[i] = y[u];
                            kk[i + j] = x[u];
                        }
                    }
                }
            }
        // compact the index halves into the first 4 nIn bytes of the same LDS
        // row: every lane holds its (<= 32) indices in registers across the
        // barrier, so no word is overwritten before it has been read
        uint32_t idx[KMAX / 64];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
        for (int q = 0; q < KMAX / 64; q++) {
            const int i = lane + 64 * q;
            idx[q] = i < nIn ? (uint32_t)kk[i] : 0u;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        uint32_t* k32 = reinterpret_cast<uint32_t*>(kk);
#pragma unroll
        for (int q = 0; q < KMAX / 64; q++) {
            const int i = lane + 64 * q;
            if (i < nIn) k32[i] = idx[q];
        }
        pm = reinterpret_cast<int*>(k32);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else if (pm) {
        for (int i = lane; i < nIn; i += 64) pm[i] = i;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (lane == 0) {
            Philox sh(seed, (uint32_t)l, stream, 0x5f1e);
            uint4 v = make_uint4(0, 0, 0, 0);
            for (int i = nIn - 1, k = 0; i > 0; i--, k = (k + 1) & 3) {
                if (k == 0) v = sh.next();
                const uint32_t x = k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
                const int j = (int)(((uint64_t)x * (uint64_t)(i + 1)) >> 32);   // U{0..i}
                const int a = pm[i], b = pm[j];
                pm[i] = b;
                pm[j] = a;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    auto at = [&](int i) { return pm ? pm[i] : i; };
    if (permOut)
        for (int i = lane; i < nIn; i += 64) permOut[(size_t)l * nIn + i] = at(i);
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = lane; i < nIn; i += 64) {
        const float v = ul[at(i)];
        if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (bi >= nIn) bi = 0;   // every u NaN: no comparison held (keep the index in range)
    if (top && lane == 0) top[l] = at(bi);
    // CDF by a wave prefix scan in FP64
    double tot = 0.0;
    for (int i = lane; i < nIn; i += 64) tot += wl[at(i)] * (double)ul[at(i)];
    tot = wave_sum(tot);
    double carry = 0.0;
    for (int b = 0; b < nIn; b += 64) {
        const int i = b + lane;
        double v = i < nIn ? wl[at(i)] * (double)ul[at(i)] / tot : 0.0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const double y = __shfl_up(v, o, 64);
            if (lane >= o) v += y;
        }
        if (i < nIn) cdf[i] = carry + v;
        carry += __shfl(v, 63, 64);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const double last = carry;
    Philox rng(seed, (uint32_t)l, stream, 0x5e5a);
    const double u0 = rng.uniform() / nOut;
    if (u0Out && lane == 0) u0Out[l] = u0;
    double s = 0.0;
    for (int j = lane; j < nOut; j += 64) {
        const double uj = (u0 + j * 1.0 / nOut) * last;
        int lo = 0, hi = nIn - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (uj > cdf[mid]) lo = mid + 1; else hi = mid;
        }
        const int src = at(lo);
        const float ua = ul[src];
        anc[(size_t)l * nOut + j] = src;
        const double x = ua > 0.f ? 1.0 / (double)ua : 0.0;
        wOut[(size_t)l * nOut + j] = x;
        s += x;
    }
    s = wave_sum(s);
    for (int j = lane; j < nOut; j += 64)
        wOut[(size_t)l * nOut + j] = s > 0.0 ? wOut[(size_t)l * nOut + j] / s : 1.0 / nOut;
}

using ResampleKernel = decltype(&k_pf_resample<4>);
// supports up to 256 entries sort in the resampling kernel's registers; the
// reseed's 2000 go through k_pf_shuffle_perm first (resample_launch)
ResampleKernel resample_kernel(int nIn, bool shuffle)
{
    return shuffle && nIn > 256 && nIn <= RESAMPLE_KMAX ? &k_pf_resample<4, true> : &k_pf_resample<4>;
}

// The shuffle's permutation ahead of k_pf_resample<4, true> for supports of
// 257 .. 2048 entries (nothing for smaller ones or without a shuffle)
void shuffle_perm_launch(int nImg, int nIn, bool shuffle, uint64_t seed, uint32_t stream, int* perm,
                         const int* done, hipStream_t s)
{
    if (!shuffle || nIn <= 256 || nIn > RESAMPLE_KMAX) return;
    auto k = nIn <= 512 ? &k_pf_shuffle_perm<8> : nIn <= 1024 ? &k_pf_shuffle_perm<16>
                                                               : &k_pf_shuffle_perm<32>;
    hipLaunchKernelGGL(k, dim3(thx::cdiv(nImg, 4)), dim3(256), 0, s, nImg, nIn, seed, stream, perm, done);
}

// gather ancestors: dst[l][j][:] = src[l (or shared)][anc[l][j]][:]
// keepDone: a done image's particles are copied unchanged (src and dst are
// the two buffers of the phases' ping-pong, lds = nOut * width)
__global__ void __launch_bounds__(256) k_gather(int nImg, int nOut, int width,
                                                const double* __restrict__ src, long lds,
                                                int nIn, const int* __restrict__ anc,
                                                double* __restrict__ dst,
                                                const int* __restrict__ done = nullptr,
                                                int keepDone = 0)
{
    const long n = (long)nImg * nOut * width;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int c = (int)(q % width);
        const long lj = q / width;
        const int l = (int)(lj / nOut);
        if (done && done[l]) {
            if (keepDone) dst[q] = src[q];
            continue;
        }
        const int a = anc[lj];
        dst[q] = src[(size_t)l * lds + (size_t)a * width + c];
        (void)nIn;
    }
}

// The perturbation mean of PARTICLE_ROT_MEAN_USING_STAT_PERTURB
// (include/Config.h:79): inferACG(mean, _r) of the current (resampled) cloud
// -- Tyler's fixed point from B = I until sum|A - B| <= 1e-3
// (DirectionalStat.cpp:93-145), capped at acgIters iterations -- then its
// principal axis (:224-251).  Its own launch so the fixed point can keep the
// cloud in registers (in k_pf_perturb they would push past 256 VGPRs).
// itOut (optional): fixed-point iterations per image.  anc (optional): the
// cloud is quat[l][anc[l][j]] -- the pre-resample cloud read through the
// resampling's ancestors, so the mean need not wait for the gather (the same
// particles in the same order as the gathered cloud: the same result).
__global__ void __launch_bounds__(256) k_pf_mean(int nImg, int mR, const double* __restrict__ quat,
                                                 int acgIters, const int* __restrict__ done,
                                                 double* __restrict__ meanQ,
                                                 int* __restrict__ itOut,
                                                 const int* __restrict__ anc = nullptr)
{
    const int l = (blockIdx.x * 256 + threadIdx.x) / GROUP;
    const int lane = threadIdx.x % GROUP;
    if (l >= nImg || (done && done[l])) return;
    double A[16], mean[4];
    const int it = infer_acg(quat + (size_t)l * mR * 4, mR, nullptr, lane, A, acgIters,
                             anc ? anc + (size_t)l * mR : nullptr);
    principal_axis(A, mean);
    if (lane == 0) {
        for (int k = 0; k < 4; k++) meanQ[4 * l + k] = mean[k];
        if (itOut) itOut[l] = it;
    }
}

// Translation half of Particle::perturb + balanceWeight (3D and 2D alike):
// t_i += pf N(0, s) (src/Particle.cpp:1232-1262), reCentre beyond transM
// (:2473-2495), pT = 1/pdf of the perturbed set normalised (balanceWeight(PAR_T),
// :2342-2375).
THX_DEV void perturb_trans(double* Tr, double* pTl, int mT, double s0, double s1, double pf,
                           double transS, double transM, Philox& rng, int lane)
{
    double sx, sy, vx, vy;
    for (int i = lane; i < mT; i += GROUP) {
        const double2 g = rng.gauss2();
        double x = Tr[2 * i] + g.x * s0 * pf, y = Tr[2 * i + 1] + g.y * s1 * pf;
        if (sqrt(x * x + y * y) > transM) {
            const double2 h = rng.gauss2();
            x = h.x * transS; y = h.y * transS;
        }
        Tr[2 * i] = x; Tr[2 * i + 1] = y;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    sx = 0; sy = 0;
    for (int i = lane; i < mT; i += GROUP) { sx += Tr[2 * i]; sy += Tr[2 * i + 1]; }
    sx = group_sum(sx) / mT; sy = group_sum(sy) / mT;
    vx = 0; vy = 0;
    for (int i = lane; i < mT; i += GROUP) {
        vx += (Tr[2 * i] - sx) * (Tr[2 * i] - sx);
        vy += (Tr[2 * i + 1] - sy) * (Tr[2 * i + 1] - sy);
    }
    vx = group_sum(vx); vy = group_sum(vy);
    const double b0 = fmax(1e-6, mT > 1 ? sqrt(vx / (mT - 1)) : 1.0);
    const double b1 = fmax(1e-6, mT > 1 ? sqrt(vy / (mT - 1)) : 1.0);
    double tot = 0.0;
    for (int i = lane; i < mT; i += GROUP) {
        const double u = (Tr[2 * i] - sx) / b0, v = (Tr[2 * i + 1] - sy) / b1;
        const double p = exp(-(u * u + v * v) / 2) / (2 * M_PI * b0 * b1);
        const double x = 1.0 / fmax(p, 1e-300);
        pTl[i] = x;
        tot += x;
    }
    tot = group_sum(tot);
    for (int i = lane; i < mT; i += GROUP) pTl[i] /= tot;
}

// Particle::perturb + balanceWeight for one image per GROUP lanes
// (src/Particle.cpp:1149-1289, 2309-2375), with k / s from k_pf_calvari:
//   R: mean = inferACG(mean, _r) of the current (resampled) cloud -- the
//      reference's compiled switch PARTICLE_ROT_MEAN_USING_STAT_PERTURB
//      (include/Config.h:79): Tyler's fixed point from B = I until
//      sum|A - B| <= 1e-3 (DirectionalStat.cpp:93-145), here capped at
//      acgIters iterations, then the principal axis (:224-251) -- when
//      meanMode == 1 (k_pf_mean); the top particle (calRank1st's _topR, the branch without
//      the switch) when meanMode == 0.  r_i <- mean d_i mean^-1 r_i with
//      d ~ ACG(diag(1, pf^2 min(1,k1), pf^2 min(1,k2), pf^2 min(1,k3)))
//      (sampleACG: normalised N(0, diag)), then pR = 1 / pdfACG on the
//      perturbed cloud (balanceWeight(PAR_R)).
//   T: t_i += pf N(0, s) (:1232-1262), reCentre beyond transM (:2473-2495),
//      pT = 1/pdf normalised (balanceWeight(PAR_T), :2342-2375).
// meanMode 1 reads the mean k_pf_mean left in meanQ.

__global__ void __launch_bounds__(256) k_pf_perturb(int nImg, int mR, int mT,
                                                    double* __restrict__ quat,
                                                    double* __restrict__ trans,
                                                    double* __restrict__ pR,
                                                    double* __restrict__ pT,
                                                    const double* __restrict__ topQ,
                                                    const double* __restrict__ kIn,
                                                    const double* __restrict__ sIn,
                                                    double pf, double transS, double transM,
                                                    uint64_t seed, uint32_t stream,
                                                    int meanMode,
                                                    const double* __restrict__ meanQ,
                                                    const int* __restrict__ done,
                                                    const double* __restrict__ symQ = nullptr,
                                                    int nSym = 0)
{
    const int l = (blockIdx.x * 256 + threadIdx.x) / GROUP;
    const int lane = threadIdx.x % GROUP;
    if (l >= nImg || (done && done[l])) return;
    double* Q = quat + (size_t)l * mR * 4;
    double* Tr = trans + (size_t)l * mT * 2;
    Philox rng(seed, (uint32_t)l, stream, (uint32_t)lane);

    // ---- rotation
    double mean[4], cm[4];
    const double* mq = meanMode == 1 ? meanQ : topQ;
    for (int k = 0; k < 4; k++) mean[k] = mq[4 * l + k];
    cm[0] = mean[0]; cm[1] = -mean[1]; cm[2] = -mean[2]; cm[3] = -mean[3];
    const double sd1 = pf * sqrt(fmin(1.0, kIn[3 * l]));       // PERTURB_K_MAX = 1
    const double sd2 = pf * sqrt(fmin(1.0, kIn[3 * l + 1]));
    const double sd3 = pf * sqrt(fmin(1.0, kIn[3 * l + 2]));
    for (int i = lane; i < mR; i += GROUP) {
        const double2 g0 = rng.gauss2(), g1 = rng.gauss2();
        double d[4] = {g0.x, g0.y * sd1, g1.x * sd2, g1.y * sd3};
        const double nn = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]);
        for (int k = 0; k < 4; k++) d[k] /= nn;
        double a[4], b[4], c[4];
        qmul(cm, Q + 4 * i, a);        // conj(mean) * r
        qmul(d, a, b);                 // pert * .
        qmul(mean, b, c);              // mean * .
        const double cn = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2] + c[3] * c[3]);
        for (int k = 0; k < 4; k++) c[k] /= cn;
        // symmetrise(&mean) (src/Particle.cpp:1234): the counterpart nearest the mean
        if (nSym) thx::sym_counterpart(c, mean, symQ, nSym);
        for (int k = 0; k < 4; k++) Q[4 * i + k] = c[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    balance_rot(Q, mR, lane, pR + (size_t)l * mR);

    perturb_trans(Tr, pT + (size_t)l * mT, mT, sIn[2 * l], sIn[2 * l + 1], pf, transS, transM, rng,
                  lane);
}

// ---- MODE_2D particle statistics (von Mises rotations).  A 2D rotation is
// the particle row (cos, sin, 0, 0) of Particle::_r (sampleVMS(dmat4&),
// src/Geometry/DirectionalStat.cpp:320-332); composition is quaternion_mul of
// such rows, i.e. the angle sum.

// gsl_sf_bessel_I0 by its power series (the argument stays below 5 where
// pdfVMS uses it)
THX_DEV double bessel_i0_dev(double x)
{
    double s = 1.0, t = 1.0;
    for (int k = 1; k < 64; k++) {
        t *= (x * x * 0.25) / ((double)k * k);
        s += t;
        if (t < 1e-17 * s) break;
    }
    return s;
}

// the concentration of sampleVMS / pdfVMS from the dispersion k = 1 - R
// (DirectionalStat.cpp:256, 269)
THX_DEV double vms_kappa(double k)
{
    return (1.0 - k) * (1.0 + 2.0 * k - k * k) / k / (2.0 - k);
}

// inferVMS(dvec2& mu, double& k, src) (DirectionalStat.cpp:334-357): mu = the
// normalised resultant, k = 1 - |resultant| / n
THX_DEV void infer_vms(const double* Q, int m, int lane, double& mu0, double& mu1, double& k)
{
    double a = 0.0, b = 0.0;
    for (int i = lane; i < m; i += GROUP) { a += Q[4 * i]; b += Q[4 * i + 1]; }
    a = group_sum(a);
    b = group_sum(b);
    const double n = sqrt(a * a + b * b);
    k = 1.0 - n / m;
    mu0 = a / n;
    mu1 = b / n;
}

// Particle::balanceWeight(PAR_R), MODE_2D (src/Particle.cpp:2317-2329):
// w_i = 1 / pdfVMS(r_i; inferVMS(r)) (pdfVMS, DirectionalStat.cpp:252-262:
// exp(kappa x.mu) / (2 pi I0(kappa)) for kappa < 5, else the Gaussian pdf of
// |x - mu| with sd 1/sqrt(kappa)), normalised to sum 1.
THX_DEV void balance_rot2d(const double* Q, int m, int lane, double* w)
{
    double mu0, mu1, k;
    infer_vms(Q, m, lane, mu0, mu1, k);
    const double kappa = vms_kappa(k);
    const bool small = kappa < 5.0;
    const double c = small ? 1.0 / (2.0 * M_PI * bessel_i0_dev(kappa)) : 0.0;
    const double sd = small ? 0.0 : sqrt(1.0 / kappa);
    double tot = 0.0;
    for (int i = lane; i < m; i += GROUP) {
        const double x0 = Q[4 * i], x1 = Q[4 * i + 1];
        double p;
        if (small) {
            p = exp(kappa * (x0 * mu0 + x1 * mu1)) * c;
        } else {
            const double d0 = x0 - mu0, d1 = x1 - mu1;
            const double r2 = d0 * d0 + d1 * d1;
            p = exp(-r2 / (2.0 * sd * sd)) / (sqrt(2.0 * M_PI) * sd);
        }
        const double x = 1.0 / p;
        w[i] = x;
        tot += x;
    }
    tot = group_sum(tot);
    for (int i = lane; i < m; i += GROUP) w[i] /= tot;
}

// sampleVMS(dmat2&, mu = (1, 0), k, n) (DirectionalStat.cpp:264-318): a
// uniform direction when kappa < 0.1, else Best & Fisher's rejection sampler
// for the cosine f and a fair sign for the sine.
THX_DEV void sample_vms(double kappa, Philox& rng, double& c, double& s)
{
    if (!(kappa >= 1e-1)) {
        // gsl_ran_dir_2d: a uniform angle
        const double th = 2.0 * M_PI * rng.uniform();
        c = cos(th);
        s = sin(th);
        return;
    }
    const double a = 1.0 + sqrt(1.0 + 4.0 * kappa * kappa);
    const double b = (a - sqrt(2.0 * a)) / (2.0 * kappa);
    const double r = (1.0 + b * b) / (2.0 * b);
    double f;
    for (int it = 0; it < 1000; it++) {
        const double z = cos(M_PI * rng.uniform());
        f = (1.0 + r * z) / (r + z);
        const double cc = kappa * (r - f);
        const double u2 = rng.uniform();
        if (cc * (2.0 - cc) > u2) break;
        if (log(cc / u2) + 1.0 - cc >= 0.0) break;
    }
    const double d = sqrt((1.0 - f) * (f + 1.0));
    c = f;
    s = rng.uniform() > 0.5 ? -d : d;
}

// Particle::calVari, MODE_2D (src/Particle.cpp:1013-1016, 1098-1119): k1 =
// inferVMS's 1 - R, floored at kFloor (the reseed floor of
// src/Optimiser.cpp:2032-2044, (1 / perturbFactor) MIN_STD_FACTOR / mS; 0 in
// the phases), written to all three k slots; T as in 3D.
__global__ void __launch_bounds__(256) k_pf_calvari2d(int nImg, int mR, const double* __restrict__ quat,
                                                      int mT, const double* __restrict__ trans,
                                                      double kFloor, double sFloor,
                                                      double* __restrict__ kOut,
                                                      double* __restrict__ sOut,
                                                      const int* __restrict__ done = nullptr,
                                                      double* __restrict__ = nullptr)   // k_pf_calvari's hist
{
    const int l = (blockIdx.x * 256 + threadIdx.x) / GROUP;
    const int lane = threadIdx.x % GROUP;
    if (l >= nImg || (done && done[l])) return;
    double mu0, mu1, k;
    infer_vms(quat + (size_t)l * mR * 4, mR, lane, mu0, mu1, k);
    const double* Tr = trans + (size_t)l * mT * 2;
    double sx = 0, sy = 0;
    for (int i = lane; i < mT; i += GROUP) { sx += Tr[2 * i]; sy += Tr[2 * i + 1]; }
    sx = group_sum(sx) / mT; sy = group_sum(sy) / mT;
    double vx = 0, vy = 0;
    for (int i = lane; i < mT; i += GROUP) {
        vx += (Tr[2 * i] - sx) * (Tr[2 * i] - sx);
        vy += (Tr[2 * i + 1] - sy) * (Tr[2 * i + 1] - sy);
    }
    vx = group_sum(vx); vy = group_sum(vy);
    if (lane == 0) {
        const double k1 = fmax(kFloor, k);
        kOut[3 * l] = k1; kOut[3 * l + 1] = k1; kOut[3 * l + 2] = k1;
        sOut[2 * l] = fmax(sFloor, mT > 1 ? sqrt(vx / (mT - 1)) : 0.0);
        sOut[2 * l + 1] = fmax(sFloor, mT > 1 ? sqrt(vy / (mT - 1)) : 0.0);
    }
}

__global__ void __launch_bounds__(256) k_pf_balance_rot2d(int nImg, int mR,
                                                          const double* __restrict__ quat,
                                                          double* __restrict__ pR)
{
    const int l = (blockIdx.x * 256 + threadIdx.x) / GROUP;
    if (l >= nImg) return;
    balance_rot2d(quat + (size_t)l * mR * 4, mR, threadIdx.x % GROUP, pR + (size_t)l * mR);
}

// Particle::perturb(pf, PAR_R), MODE_2D (src/Particle.cpp:1160-1178):
// d_i ~ sampleVMS(mu = (1, 0), k = min(PERTURB_K_MAX = 1, k1 pf)), r_i <-
// quaternion_mul(r_i, d_i), balanceWeight(PAR_R); then T as in 3D.
__global__ void __launch_bounds__(256) k_pf_perturb2d(int nImg, int mR, int mT,
                                                      double* __restrict__ quat,
                                                      double* __restrict__ trans,
                                                      double* __restrict__ pR,
                                                      double* __restrict__ pT,
                                                      const double* __restrict__ kIn,
                                                      const double* __restrict__ sIn,
                                                      double pf, double transS, double transM,
                                                      uint64_t seed, uint32_t stream,
                                                      const int* __restrict__ done)
{
    const int l = (blockIdx.x * 256 + threadIdx.x) / GROUP;
    const int lane = threadIdx.x % GROUP;
    if (l >= nImg || (done && done[l])) return;
    double* Q = quat + (size_t)l * mR * 4;
    double* Tr = trans + (size_t)l * mT * 2;
    Philox rng(seed, (uint32_t)l, stream, 0x2d00u | (uint32_t)lane);
    const double kappa = vms_kappa(fmin(1.0, kIn[3 * l] * pf));
    for (int i = lane; i < mR; i += GROUP) {
        double d[4] = {0.0, 0.0, 0.0, 0.0}, o[4];
        sample_vms(kappa, rng, d[0], d[1]);
        qmul(Q + 4 * i, d, o);
        for (int k = 0; k < 4; k++) Q[4 * i + k] = o[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    balance_rot2d(Q, mR, lane, pR + (size_t)l * mR);
    perturb_trans(Tr, pT + (size_t)l * mT, mT, sIn[2 * l], sIn[2 * l + 1], pf, transS, transM, rng,
                  lane);
}

// Reseed of the class for K > 1 (src/Optimiser.cpp:1933-1965), one thread
// per image: u_c = wC[l][c] -> keepHalfHeightPeak(PAR_C) with the fixed
// PEAK_FACTOR_C = 1 - 1e-2 (PARTICLE_PEAK_FACTOR_C, include/Particle.h:55,
// setPeakFactor src/Particle.cpp:1907-1910) -> resample(K, PAR_C): shuffle,
// w u with the reset prior w = 1/K, systematic draw -> rand(cls): a uniform
// entry of the resampled set (src/Particle.cpp:2109-2118).
constexpr int KMAX_CLASS = 64;

__global__ void __launch_bounds__(256) k_pf_class(int nImg, int K, const float* __restrict__ wC,
                                                  uint64_t seed, uint32_t stream,
                                                  int* __restrict__ cls)
{
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= nImg) return;
    const float* u = wC + (size_t)l * K;
    float mx = 0.f;
    for (int c = 0; c < K; c++) mx = fmaxf(mx, u[c]);
    const double hh = (double)mx * (1.0 - 1e-2);
    int pm[KMAX_CLASS];
    for (int c = 0; c < K; c++) pm[c] = c;
    Philox sh(seed, (uint32_t)l, stream, 0x5f1e);
    for (int i = K - 1; i > 0; i--) {
        const uint32_t x = sh.next().x;
        const int j = (int)(((uint64_t)x * (uint64_t)(i + 1)) >> 32);
        const int t = pm[i]; pm[i] = pm[j]; pm[j] = t;
    }
    double tot = 0.0;
    for (int i = 0; i < K; i++) {
        const double v = u[pm[i]];
        tot += (v < hh ? 0.0 : v - hh) / K;
    }
    Philox rng(seed, (uint32_t)l, stream, 0x5e5a);
    const double u0 = rng.uniform() / K;
    const int j = (int)(((uint64_t)rng.next().x * (uint64_t)K) >> 32);   // rand(cls): U{0..K-1}
    const double uj = (u0 + j * 1.0 / K) * tot;
    double acc = 0.0;
    int pick = pm[K - 1];
    for (int i = 0; i < K; i++) {
        const double v = u[pm[i]];
        acc += (v < hh ? 0.0 : v - hh) / K;
        if (!(uj > acc)) { pick = pm[i]; break; }
    }
    cls[l] = pick;
}

// The stopping rule of the phase loop with OPTIMISER_COMPRESS_CRITERIA
// (src/Optimiser.cpp:1510-1615): from phase minPhase on, variR =
// (k1 k2 k3)^(1/6) (Particle::variR, src/Particle.cpp:611-627) and variT =
// sqrt of the eigenvalue product of [[s0^2, rho], [rho, s1^2]] = s0 s1 (rho =
// 0: PARTICLE_RHO is off) of this phase's calVari are compared with the
// smallest values so far.  All three bests start at DBL_MAX, so the first
// check always finds "room" (variD = _s never changes without CTF search);
// afterwards one phase without a 5 % decrease of either ends the image
// (N_PHASE_WITH_NO_VARI_DECREASE = 1) and _nP = phase.  lastPhase: the loop's
// end (MAX_N_PHASE_PER_ITER - 1).
// sdD / bestD (CTF search, else NULL): variD = _s (src/Particle.cpp:642-645)
// joins the criterion (src/Optimiser.cpp:1557-1559, 1591).
__global__ void k_pf_converge(int nImg, int phase, int minPhase, int lastPhase,
                              const double* __restrict__ kv, const double* __restrict__ sv,
                              double* __restrict__ bestR, double* __restrict__ bestT,
                              int* __restrict__ done, int* __restrict__ nP,
                              const double* __restrict__ sdD = nullptr,
                              double* __restrict__ bestD = nullptr, int twoD = 0)
{
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= nImg || done[l]) return;
    bool stop = phase >= lastPhase;
    if (phase >= minPhase) {
        // Particle::variR: k1 in MODE_2D, (k1 k2 k3)^(1/6) in 3D
        const double vR = twoD ? kv[3 * l] : pow(kv[3 * l] * kv[3 * l + 1] * kv[3 * l + 2], 1.0 / 6);
        const double vT = sv[2 * l] * sv[2 * l + 1];
        const bool first = phase == minPhase;
        bool room = first || vR < bestR[l] * 0.95 || vT < bestT[l] * 0.95;
        bestR[l] = first ? vR : fmin(bestR[l], vR);
        bestT[l] = first ? vT : fmin(bestT[l], vT);
        if (sdD) {
            const double vD = sdD[l];
            room = room || vD < bestD[l] * 0.95;
            bestD[l] = first ? vD : fmin(bestD[l], vD);
        }
        stop = stop || !room;
    }
    if (stop) {
        done[l] = 1;
        nP[l] = phase;
    }
}

// Active-image list: act[0 .. *nAct) = the images with done == 0, in order
// (ord: in the order ord lists them; one workgroup, ballot prefix per wave).
__global__ void __launch_bounds__(1024) k_compact(int nImg, const int* __restrict__ done,
                                                  int* __restrict__ act, int* __restrict__ nAct,
                                                  const int* __restrict__ ord = nullptr)
{
    __shared__ int sW[16];
    __shared__ int sBase;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) sBase = 0;
    __syncthreads();
    for (int b = 0; b < nImg; b += 1024) {
        const int i = b + tid;
        const int img = i < nImg ? (ord ? ord[i] : i) : 0;
        const bool f = i < nImg && !(done && done[img]);
        const unsigned long long m = __ballot(f);
        const int pre = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) sW[wv] = __popcll(m);
        __syncthreads();
        int off = sBase;
        for (int w = 0; w < wv; w++) off += sW[w];
        if (f) act[off + pre] = img;
        __syncthreads();
        if (tid == 0)
            for (int w = 0; w < 16; w++) sBase += sW[w];
        __syncthreads();
    }
    if (tid == 0) *nAct = sBase;
}

// topQ[l] = the particle of largest prior pR (calRank1st on the caller's
// state, for a local search that starts from it).
__global__ void k_top_by_weight(int nImg, int mR, const double* __restrict__ quat,
                                const double* __restrict__ pR, double* __restrict__ topQ)
{
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= nImg) return;
    int best = 0;
    for (int i = 1; i < mR; i++)
        if (pR[(size_t)l * mR + i] > pR[(size_t)l * mR + best]) best = i;
    for (int k = 0; k < 4; k++) topQ[4 * l + k] = quat[((size_t)l * mR + best) * 4 + k];
}

// ---- defocus particles (PAR_D) of a CTF search, one image per GROUP lanes.
// balanceWeight(PAR_D) (src/Particle.cpp:2374-2409): w_i = 1 / N(d_i - m; s)
// with the sample mean m and s = gsl_stats_sd_m (n - 1), 1 when s == 0
// (one sample, or all equal); normW.
THX_DEV void balance_d(const double* D, int mD, int lane, double* pD)
{
    double m = 0.0;
    for (int i = lane; i < mD; i += GROUP) m += D[i];
    m = group_sum(m) / mD;
    double v = 0.0;
    for (int i = lane; i < mD; i += GROUP) v += (D[i] - m) * (D[i] - m);
    v = group_sum(v);
    const double sd = mD > 1 ? sqrt(v / (mD - 1)) : 0.0;
    double tot = 0.0;
    for (int i = lane; i < mD; i += GROUP) {
        const double u = (D[i] - m) / sd;
        const double x = sd == 0.0 ? 1.0 : 1.0 / (exp(-0.5 * u * u) / (sd * sqrt(2 * M_PI)));
        pD[i] = x;
        tot += x;
    }
    tot = group_sum(tot);
    for (int i = lane; i < mD; i += GROUP) pD[i] /= tot;
}

// op 0: initD (src/Particle.cpp:281-310, PARTICLE_DEFOCUS_INIT_GAUSSIAN):
//       d_i = 1 + N(0, arg), balanceWeight;
// op 1: perturb(arg, PAR_D) (:1278-1288): d_i += N(0, sd[l]) arg, balanceWeight;
// op 2: calVari(PAR_D) (:1120-1141): sd[l] = gsl_stats_sd(d), 0 for one sample.
__global__ void __launch_bounds__(256) k_pf_defocus(int nImg, int mD, int op, double arg,
                                                    uint64_t seed, uint32_t stream,
                                                    double* __restrict__ d,
                                                    double* __restrict__ pD,
                                                    double* __restrict__ sd,
                                                    const int* __restrict__ done)
{
    const int l = (blockIdx.x * 256 + threadIdx.x) / GROUP;
    const int lane = threadIdx.x % GROUP;
    if (l >= nImg || (done && done[l])) return;
    double* D = d + (size_t)l * mD;
    if (op == 2) {
        double m = 0.0;
        for (int i = lane; i < mD; i += GROUP) m += D[i];
        m = group_sum(m) / mD;
        double v = 0.0;
        for (int i = lane; i < mD; i += GROUP) v += (D[i] - m) * (D[i] - m);
        v = group_sum(v);
        if (lane == 0) sd[l] = mD > 1 ? sqrt(v / (mD - 1)) : 0.0;
        return;
    }
    Philox rng(seed, (uint32_t)l, stream, 0xde00u | (uint32_t)lane);
    const double scale = op == 0 ? arg : sd[l] * arg;
    for (int i = lane; i < mD; i += GROUP) {
        const double g = rng.gauss2().x;
        D[i] = (op == 0 ? 1.0 : D[i]) + g * scale;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    balance_d(D, mD, lane, pD + (size_t)l * mD);
}

// ---- a3: the global sample set of Particle::reset (src/Particle.cpp:87-169)
// for 3D, C1: rotations from sampleACG with the identity (a normalised 4D
// Gaussian: uniform on S^3), translations from a bivariate Gaussian of width
// transS (PARTICLE_TRANS_INIT_GAUSSIAN), pR = 1/nR, pT = balanceWeight(PAR_T)
// (:2342-2375: 1 / N2(t - m; s0, s1, rho = 0) with the sample mean and
// gsl_stats_sd_m, normalised).  Counter RNG; one workgroup does T.  twoD:
// MODE_2D rotations (:101-103), uniform angles as rows (cos, sin, 0, 0).
__global__ void __launch_bounds__(256) k_sample_set(int nR, int nT, double transS, uint64_t seed,
                                                    double* __restrict__ quat,
                                                    double* __restrict__ trans,
                                                    double* __restrict__ pR,
                                                    double* __restrict__ pT, int twoD)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < nR && twoD) {
        // MODE_2D: sampleVMS(_r, (1, 0, 0, 0), k = 1) -- kappa 0, gsl_ran_dir_2d
        Philox rng(seed, (uint32_t)i, 0x5a3u, 2u);
        const double th = 2.0 * M_PI * rng.uniform();
        quat[4 * (size_t)i] = cos(th);
        quat[4 * (size_t)i + 1] = sin(th);
        quat[4 * (size_t)i + 2] = 0.0;
        quat[4 * (size_t)i + 3] = 0.0;
        pR[i] = 1.0 / nR;
    } else if (i < nR) {
        Philox rng(seed, (uint32_t)i, 0x5a3u, 0u);
        const double2 g0 = rng.gauss2(), g1 = rng.gauss2();
        const double n = sqrt(g0.x * g0.x + g0.y * g0.y + g1.x * g1.x + g1.y * g1.y);
        quat[4 * (size_t)i] = g0.x / n;
        quat[4 * (size_t)i + 1] = g0.y / n;
        quat[4 * (size_t)i + 2] = g1.x / n;
        quat[4 * (size_t)i + 3] = g1.y / n;
        pR[i] = 1.0 / nR;
    }
    if (blockIdx.x != 0) return;
    __shared__ double sRed[4][4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    auto block_sum2 = [&](double a, double b, double& ra, double& rb) {
        a = wave_sum(a);
        b = wave_sum(b);
        __syncthreads();
        if (lane == 0) { sRed[wv][0] = a; sRed[wv][1] = b; }
        __syncthreads();
        ra = sRed[0][0] + sRed[1][0] + sRed[2][0] + sRed[3][0];
        rb = sRed[0][1] + sRed[1][1] + sRed[2][1] + sRed[3][1];
    };
    double sx = 0.0, sy = 0.0;
    for (int t = threadIdx.x; t < nT; t += 256) {
        Philox rng(seed, (uint32_t)t, 0x5a4u, 0u);
        const double2 g = rng.gauss2();
        trans[2 * (size_t)t] = g.x * transS;
        trans[2 * (size_t)t + 1] = g.y * transS;
        sx += g.x * transS;
        sy += g.y * transS;
    }
    double m0, m1;
    block_sum2(sx, sy, m0, m1);
    m0 /= nT;
    m1 /= nT;
    double vx = 0.0, vy = 0.0;
    for (int t = threadIdx.x; t < nT; t += 256) {
        vx += (trans[2 * (size_t)t] - m0) * (trans[2 * (size_t)t] - m0);
        vy += (trans[2 * (size_t)t + 1] - m1) * (trans[2 * (size_t)t + 1] - m1);
    }
    double v0, v1;
    block_sum2(vx, vy, v0, v1);
    const double s0 = sqrt(v0 / (nT - 1)), s1 = sqrt(v1 / (nT - 1));
    double tot = 0.0;
    for (int t = threadIdx.x; t < nT; t += 256) {
        const double u = (trans[2 * (size_t)t] - m0) / s0, v = (trans[2 * (size_t)t + 1] - m1) / s1;
        const double x = 1.0 / (exp(-(u * u + v * v) / 2) / (2 * M_PI * s0 * s1));
        pT[t] = x;
        tot += x;
    }
    double tt, unused;
    block_sum2(tot, 0.0, tt, unused);
    for (int t = threadIdx.x; t < nT; t += 256) pT[t] /= tt;
}


struct Plan {
    // carve of the driver workspace
    float* rotP; double* gMat; float* traP;
    float* gWC; float* gWR; float* gWT; float* gBase;
    void* scanWs; size_t scanWsBytes;
    int* anc; double* cdf; int* perm; int* topR; int* topT;
    int* ancR;                           // the phases' rotation ancestors (read by the side-stream mean)
    double* tmpQ; double* tmpT;
    double* kv; double* sv; double* peakR;   // calVari k1..k3, s0 s1; setPeakFactor(R)
    double* topQ;                            // calRank1st _topR
    double* meanQ;                           // k_pf_mean's perturbation mean
    double* acgHist;                         // calVari's fixed-point iterates (calvari_acg_impl)
    float* wC; float* wR; float* wT; float* base; double* pC;
    int* cls; int* nP; int* done; int* act; int* nAct;   // classes, phases run, active list
    int* doneSnap;                       // done as of a side-stream fork (k_pf_mean on s2)
    int* actIdx; int* nActIdx;           // the active list in index order (route samples)
    int* maxR2;                          // max iCol^2 + iRow^2 of the pixel set
    unsigned* ordKey; unsigned* ordKeyOut; int* ordIdx; int* ord;   // view order (order.hip)
    void* ordTmp; size_t ordTmpBytes;
    double* bestR; double* bestT;                        // convergence: smallest variR / variT
    void* localWs; size_t localWsBytes;
    float* ypair;                        // y-pair projectees (thx_volume_ypair), per class
    // CTF search: defocus precalculation, per-phase CTF table, D statistics
    float* freq; float* dfo; float* K1; float* K2; float* ctfD; float* wD;
    double* sdD; double* bestD; double* tmpD; int* topD;
    size_t bytes;
};


// mLD > 0: the workspace of a CTF search over mLD defocus samples
Plan plan(void* base, const thx_expect_cfg& c, int nImg, int nPxl, int nVisit, int mLD = 0,
          bool twoD = false)
{
    thx::Carver k(base, ~size_t(0));
    Plan p;
    const int nK = c.nK > 0 ? c.nK : 1;
    int nMax = c.nR > c.nT ? c.nR : c.nT;           // every resampled support size
    if (c.mLR > nMax) nMax = c.mLR;
    if (c.mLT > nMax) nMax = c.mLT;
    if (mLD > nMax) nMax = mLD;
    const bool scan = c.searchType == 0;
    p.rotP = k.take<float>(scan ? (size_t)2 * c.nR * nPxl : 0);
    p.gMat = k.take<double>(scan && !twoD ? (size_t)9 * c.nR : 0);
    p.traP = k.take<float>(scan ? (size_t)2 * c.nT * nPxl : 0);
    p.gWC = k.take<float>((size_t)nImg * nK);
    p.gWR = k.take<float>(scan ? (size_t)nImg * nK * c.nR : 0);
    p.gWT = k.take<float>(scan ? (size_t)nImg * nK * c.nT : 0);
    p.gBase = k.take<float>(nImg);
    p.scanWsBytes = scan ? thx_global_scan_workspace(nImg, c.nR, c.nT, nPxl, c.algo) : 0;
    p.scanWs = k.take<char>(p.scanWsBytes);
    p.anc = k.take<int>((size_t)nImg * (c.mLR > c.mLT ? (c.mLR > mLD ? c.mLR : mLD)
                                                      : (c.mLT > mLD ? c.mLT : mLD)));
    p.ancR = k.take<int>((size_t)nImg * c.mLR);
    p.cdf = k.take<double>((size_t)nImg * nMax);
    p.perm = k.take<int>((size_t)nImg * nMax);
    p.topR = k.take<int>(nImg);
    p.topT = k.take<int>(nImg);
    p.tmpQ = k.take<double>((size_t)nImg * c.mLR * 4);
    p.tmpT = k.take<double>((size_t)nImg * c.mLT * 2);
    p.kv = k.take<double>((size_t)nImg * 3);
    p.sv = k.take<double>((size_t)nImg * 2);
    p.peakR = k.take<double>(nImg);
    p.topQ = k.take<double>((size_t)nImg * 4);
    p.meanQ = k.take<double>((size_t)nImg * 4);
    p.acgHist = k.take<double>(!twoD ? (size_t)nImg * ACG_HIST : 0);
    p.wC = k.take<float>(nImg);
    p.wR = k.take<float>((size_t)nImg * c.mLR);
    p.wT = k.take<float>((size_t)nImg * c.mLT);
    p.base = k.take<float>(nImg);
    p.pC = k.take<double>(nImg);
    p.cls = k.take<int>(nImg);
    p.nP = k.take<int>(nImg);
    p.done = k.take<int>(nImg);
    p.doneSnap = k.take<int>(nImg);
    p.act = k.take<int>(nImg);
    p.nAct = k.take<int>(1);
    p.actIdx = k.take<int>(nImg);
    p.maxR2 = k.take<int>(1);
    p.nActIdx = k.take<int>(1);
    const size_t nOrd = !twoD ? (size_t)nImg : 0;
    p.ordKey = k.take<unsigned>(nOrd);
    p.ordKeyOut = k.take<unsigned>(nOrd);
    p.ordIdx = k.take<int>(nOrd);
    p.ord = k.take<int>(nOrd);
    p.ordTmpBytes = nOrd ? thx::view_order_tmp_bytes(nImg) : 0;
    p.ordTmp = k.take<char>(p.ordTmpBytes);
    p.bestR = k.take<double>(nImg);
    p.bestT = k.take<double>(nImg);
    p.localWsBytes = twoD ? thx_local_phase2d_d_workspace(nImg, c.mLR, c.mLT, mLD)
                          : thx_local_phase_workspace(nImg, c.mLR, c.mLT * (mLD > 0 ? mLD : 1),
                                                      nVisit);
    p.localWs = k.take<char>(p.localWsBytes);
    const size_t nd = mLD > 0 ? (size_t)mLD : 0, on = mLD > 0 ? 1 : 0;
    p.freq = k.take<float>(on * nPxl);
    p.dfo = k.take<float>(on * nImg * nPxl);
    p.K1 = k.take<float>(on * nImg);
    p.K2 = k.take<float>(on * nImg);
    p.ctfD = k.take<float>(nd * nImg * nPxl);
    p.wD = k.take<float>(nd * nImg);
    p.sdD = k.take<double>(on * nImg);
    p.bestD = k.take<double>(on * nImg);
    p.tmpD = k.take<double>(nd * nImg);
    p.topD = k.take<int>(on * nImg);
    // the y-pair copy of every class's projectee for the device route's
    // pair-form kernel (phases whose LDS boxes do not pay)
    const bool yp = !c.volCells && !twoD && mLD == 0 && thx::phase_routed(0, c.pf, nPxl, 0);
    // A/B control of the compact ball's placement (THX_YPAIR_OFFSET = B: the
    // copy starts B bytes past a 2 MiB boundary of the address space; unset:
    // right after the buffers before it).  The local phases' speed depends
    // on it by a few per cent (profiles/r06_ball_placement_ab.jsonl).
    if (yp) {
        const char* e = std::getenv("THX_YPAIR_OFFSET");
        const size_t A2 = size_t(2) << 20;
        if (!k.base) {
            k.off += 2 * A2;      // the size query: room for any placement
        } else if (e) {
            const uintptr_t a = (uintptr_t)k.base + k.off;
            k.off += (A2 - a % A2) % A2 + ((size_t)std::strtoull(e, nullptr, 10) % A2 & ~size_t(255));
        }
    }
    p.ypair = yp ? k.take<float>((size_t)4 * (c.vdim / 2 + 1) * c.vdim * c.vdim * nK) : nullptr;
    p.bytes = k.off + 256;
    return p;
}

// topQ[l] = src[l (or shared)][top[l]] -- Particle::_topR after calRank1st
__global__ void k_top_copy(int nImg, const double* __restrict__ src, long lds,
                           const int* __restrict__ top, double* __restrict__ topQ,
                           const int* __restrict__ done = nullptr)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nImg * 4) return;
    const int l = q / 4, k = q % 4;
    if (done && done[l]) return;
    topQ[q] = src[(size_t)l * lds + (size_t)top[l] * 4 + k];
}

__global__ void k_fill(double* p, long n, double v)
{
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x)
        p[q] = v;
}

__global__ void k_fill_int(int* p, long n, int v)
{
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x)
        p[q] = v;
}

}  // namespace

extern "C" int thx_pf_calvari(int nImg, int mR, const double* quat, int mT, const double* trans,
                              double kFloor, double sFloor, double* k, double* sd,
                              thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && mR > 0 && mT > 0, "thx_pf_calvari: bad sizes");
    THX_CHECK_ARG(nImg == 0 || (quat && trans && k && sd), "thx_pf_calvari: null argument");
    if (nImg == 0) return THX_OK;
    // the fixed points' history (calvari_acg_impl), stream-ordered scratch
    hipStream_t s = thx::as_stream(stream);
    double* hist = nullptr;
    THX_HIP(hipMallocAsync(reinterpret_cast<void**>(&hist), sizeof(double) * nImg * ACG_HIST, s));
    hipLaunchKernelGGL(k_pf_calvari, dim3(thx::cdiv(nImg * GROUP, 256)), dim3(256), 0, s, nImg, mR,
                       quat, mT, trans, kFloor, sFloor, k, sd, nullptr, hist);
    const hipError_t e = hipGetLastError();
    THX_HIP(hipFreeAsync(hist, s));
    THX_HIP(e);
    return THX_OK;
}

// the perturbation mean of k_pf_mean (inferACG's principal axis, capped at
// acgIters fixed-point iterations) with the iterations each image took
extern "C" int thx_pf_acg_mean(int nImg, int mR, const double* quat, int acgIters, double* meanQ,
                               int* iters, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && mR > 0 && acgIters > 0, "thx_pf_acg_mean: bad sizes");
    THX_CHECK_ARG(nImg == 0 || (quat && meanQ), "thx_pf_acg_mean: null argument");
    if (nImg == 0) return THX_OK;
    hipLaunchKernelGGL(k_pf_mean, dim3(thx::cdiv(nImg * GROUP, 256)), dim3(256), 0,
                       thx::as_stream(stream), nImg, mR, quat, acgIters, nullptr, meanQ, iters);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_pf_balance_rot(int nImg, int mR, const double* quat, double* pR,
                                  thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && mR > 0, "thx_pf_balance_rot: bad sizes");
    THX_CHECK_ARG(nImg == 0 || (quat && pR), "thx_pf_balance_rot: null argument");
    if (nImg == 0) return THX_OK;
    hipLaunchKernelGGL(k_pf_balance_rot, dim3(thx::cdiv(nImg * GROUP, 256)), dim3(256), 0,
                       thx::as_stream(stream), nImg, mR, quat, pR);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_global_sample_sizes(int mode, int mS, int nSymElem, double transS,
                                       double transSearchFactor, int* mSOut, int* nR, int* nT)
{
    THX_CHECK_ARG((mode == 0 || mode == 1) && mS > 0 && nSymElem >= 0 && transS > 0.0 &&
                      transSearchFactor > 0.0 && nR && nT,
                  "thx_global_sample_sizes: bad arguments");
    // the 3D clamp of Optimiser::init (src/Optimiser.cpp:170-175, MIN_M_S = 1500)
    const int m = mode == 1 ? (mS > 1500 * (1 + nSymElem) ? mS : 1500 * (1 + nSymElem)) : mS;
    if (mSOut) *mSOut = m;
    *nR = mode == 1 ? m / (1 + nSymElem) : m;                       // :1724-1738
    // nT = max(30, AROUND(pi (transS chi2Qinv(0.5, 2))^2 tsf)), chi2Qinv(0.5, 2) = 2 ln 2
    const double r = transS * (2.0 * std::log(2.0));
    const int t = (int)std::floor(M_PI * r * r * transSearchFactor + 0.5);
    *nT = t > 30 ? t : 30;
    return THX_OK;
}

extern "C" int thx_global_sample_set(int nR, int nT, double transS, unsigned long long seed,
                                     double* quat, double* trans, double* pR, double* pT,
                                     thx_stream_t stream)
{
    THX_CHECK_ARG(nR > 0 && nT > 1 && transS > 0.0 && quat && trans && pR && pT,
                  "thx_global_sample_set: bad arguments");
    hipLaunchKernelGGL(k_sample_set, dim3(thx::cdiv(nR, 256)), dim3(256), 0,
                       thx::as_stream(stream), nR, nT, transS, (uint64_t)seed, quat, trans, pR,
                       pT, 0);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_global_sample_set2d(int nR, int nT, double transS, unsigned long long seed,
                                       double* rot, double* trans, double* pR, double* pT,
                                       thx_stream_t stream)
{
    THX_CHECK_ARG(nR > 0 && nT > 1 && transS > 0.0 && rot && trans && pR && pT,
                  "thx_global_sample_set2d: bad arguments");
    hipLaunchKernelGGL(k_sample_set, dim3(thx::cdiv(nR, 256)), dim3(256), 0,
                       thx::as_stream(stream), nR, nT, transS, (uint64_t)seed, rot, trans, pR,
                       pT, 1);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_pf_calvari2d(int nImg, int mR, const double* rot, int mT, const double* trans,
                                double kFloor, double sFloor, double* k, double* sd,
                                thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && mR > 0 && mT > 0, "thx_pf_calvari2d: bad sizes");
    THX_CHECK_ARG(nImg == 0 || (rot && trans && k && sd), "thx_pf_calvari2d: null argument");
    if (nImg == 0) return THX_OK;
    hipLaunchKernelGGL(k_pf_calvari2d, dim3(thx::cdiv(nImg * GROUP, 256)), dim3(256), 0,
                       thx::as_stream(stream), nImg, mR, rot, mT, trans, kFloor, sFloor, k, sd);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_pf_balance_rot2d(int nImg, int mR, const double* rot, double* pR,
                                    thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && mR > 0, "thx_pf_balance_rot2d: bad sizes");
    THX_CHECK_ARG(nImg == 0 || (rot && pR), "thx_pf_balance_rot2d: null argument");
    if (nImg == 0) return THX_OK;
    hipLaunchKernelGGL(k_pf_balance_rot2d, dim3(thx::cdiv(nImg * GROUP, 256)), dim3(256), 0,
                       thx::as_stream(stream), nImg, mR, rot, pR);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_pf_perturb2d(int nImg, int mR, int mT, double* rot, double* trans, double* pR,
                                double* pT, const double* k, const double* sd, double pf,
                                double transS, double transM, unsigned long long seed,
                                unsigned stream_id, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && mR > 0 && mT > 0 && pf > 0.0, "thx_pf_perturb2d: bad arguments");
    THX_CHECK_ARG(nImg == 0 || (rot && trans && pR && pT && k && sd),
                  "thx_pf_perturb2d: null argument");
    if (nImg == 0) return THX_OK;
    hipLaunchKernelGGL(k_pf_perturb2d, dim3(thx::cdiv(nImg * GROUP, 256)), dim3(256), 0,
                       thx::as_stream(stream), nImg, mR, mT, rot, trans, pR, pT, k, sd, pf, transS,
                       transM, (uint64_t)seed, (uint32_t)stream_id, nullptr);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_pf_defocus(int nImg, int mD, int op, double arg, unsigned long long seed,
                              unsigned stream_id, double* d, double* pD, double* sd,
                              thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && mD > 0 && op >= 0 && op <= 2, "thx_pf_defocus: bad arguments");
    THX_CHECK_ARG(nImg == 0 || (d && (op == 2 || pD) && (op == 0 || sd)),
                  "thx_pf_defocus: null argument");
    if (nImg == 0) return THX_OK;
    hipLaunchKernelGGL(k_pf_defocus, dim3(thx::cdiv(nImg * GROUP, 256)), dim3(256), 0,
                       thx::as_stream(stream), nImg, mD, op, arg, (uint64_t)seed,
                       (uint32_t)stream_id, d, pD, sd, nullptr);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_pf_peak(int nImg, int n, float* u, int ldu, double* peak, int setFactor,
                           thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && n > 0 && ldu >= n, "thx_pf_peak: bad sizes");
    THX_CHECK_ARG(nImg == 0 || (u && peak), "thx_pf_peak: null argument");
    if (nImg == 0) return THX_OK;
    hipLaunchKernelGGL(k_pf_peak, dim3(thx::cdiv(nImg, 4)), dim3(256), 0,
                       thx::as_stream(stream), nImg, n, u, ldu, peak, setFactor);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" size_t thx_pf_resample_workspace(int nImg, int nIn)
{
    if (nImg <= 0 || nIn <= 0) return 256;
    thx::Carver k(nullptr, ~size_t(0));
    k.take<double>((size_t)nImg * nIn);
    k.take<int>((size_t)nImg * nIn);
    return k.off + 256;
}

extern "C" int thx_pf_resample(int nImg, int nIn, int nOut, const double* w, int ldw,
                               const float* u, int ldu, unsigned long long seed,
                               unsigned stream_id, int shuffle, int* anc, double* wOut,
                               int* iMax, int* perm, double* u0, void* workspace,
                               size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && nIn > 0 && nOut > 0 && (ldw == 0 || ldw >= nIn) && ldu >= nIn,
                  "thx_pf_resample: bad sizes");
    THX_CHECK_ARG(nImg == 0 || (w && u && anc && wOut && workspace), "thx_pf_resample: null argument");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(wsBytes >= thx_pf_resample_workspace(nImg, nIn), "thx_pf_resample: workspace too small");
    thx::Carver k(workspace, wsBytes);
    double* cdf = k.take<double>((size_t)nImg * nIn);
    int* pw = k.take<int>((size_t)nImg * nIn);
    shuffle_perm_launch(nImg, nIn, shuffle, (uint64_t)seed, (uint32_t)stream_id, pw, nullptr,
                        thx::as_stream(stream));
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(resample_kernel(nIn, shuffle), dim3(thx::cdiv(nImg, 4)), dim3(256), resample_lds(nIn, shuffle),
                       thx::as_stream(stream),
                       nImg, nIn, nOut, w, ldw, u, ldu, (uint64_t)seed, (uint32_t)stream_id, anc,
                       wOut, iMax, cdf, shuffle ? pw : nullptr, perm, u0, nullptr, 0, nullptr);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

// calVari of a phase reads the pre-resample cloud and is only needed by the
// next perturbation and the stopping rule, so it runs on a side stream
// beside the resampling, the gathers and the next phase's inferACG mean --
// two latency-bound, low-occupancy kernels side by side.  One side stream
// and a fork / join event pair per (device, caller stream), made once; the
// side stream only ever waits on events recorded on the caller's stream (a
// fork / join pattern, the shape HIP graph capture accepts).
namespace {
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    // the second side stream: the next phase's inferACG mean, forked once the
    // rotations are resampled, beside the translations' resampling
    hipStream_t s2 = nullptr;
    hipEvent_t fork2 = nullptr, join2 = nullptr;
    std::mutex mu;      // calls on one caller stream are ordered anyway
};

int side_stream(hipStream_t main, SideStream** out)
{
    static std::mutex mu;
    static auto* tab = new std::map<std::pair<int, hipStream_t>, SideStream*>;
    int dev = 0;
    THX_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    SideStream*& e = (*tab)[std::make_pair(dev, main)];
    if (!e) {
        SideStream* n = new SideStream;
        THX_HIP(hipStreamCreateWithFlags(&n->s, hipStreamNonBlocking));
        THX_HIP(hipEventCreateWithFlags(&n->fork, hipEventDisableTiming));
        THX_HIP(hipEventCreateWithFlags(&n->join, hipEventDisableTiming));
        THX_HIP(hipStreamCreateWithFlags(&n->s2, hipStreamNonBlocking));
        THX_HIP(hipEventCreateWithFlags(&n->fork2, hipEventDisableTiming));
        THX_HIP(hipEventCreateWithFlags(&n->join2, hipEventDisableTiming));
        e = n;
    }
    *out = e;
    return THX_OK;
}
}  // namespace

extern "C" size_t thx_expectation_workspace(const thx_expect_cfg* cfg, int nImg, int nPxl,
                                            int nOrd)
{
    if (!cfg) return 0;
    return plan(nullptr, *cfg, nImg, nPxl, nOrd > 0 ? nOrd : nPxl).bytes;
}

extern "C" size_t thx_expectation_ctf_workspace(const thx_expect_cfg* cfg,
                                                const thx_ctf_search_cfg* cs, int nImg,
                                                int nPxl, int nOrd)
{
    if (!cfg || !cs || cs->mLD <= 0) return 0;
    return plan(nullptr, *cfg, nImg, nPxl, nOrd > 0 ? nOrd : nPxl, cs->mLD).bytes;
}

// cs != NULL: SEARCH_TYPE_CTF (searchType 2) -- a local search whose phases
// also sample nD = cs->mLD defocus factors per image (src/Optimiser.cpp:
// 1183-1616 with the _searchType == SEARCH_TYPE_CTF branches).
static int expectation_impl(const thx_expect_cfg* cfg, const thx_ctf_search_cfg* cs,
                            const float* vol, const double* gQuat, const double* gTrans,
                            const double* gPR, const double* gPT, const float* dat,
                            const float* ctf, const float* sigRcp, const int* iCol,
                            const int* iRow, const int* pxOrder, int nOrd, int nPxl, int nImg,
                            double* quat, double* trans, double* pR, double* pT, float* score,
                            int* cls, int* nPhaseOut, void* workspace, size_t wsBytes,
                            thx_stream_t stream, bool twoD = false)
{
    THX_CHECK_ARG(cfg && vol && dat && (ctf || cs) && sigRcp && iCol && iRow && quat && trans &&
                      pR && pT,
                  "thx_expectation: null argument");
    const thx_expect_cfg& c = *cfg;
    THX_CHECK_ARG(!twoD || !c.volCells, "thx_expectation2d: no cell projectee in MODE_2D");
    const bool global = c.searchType == 0;
    if (cs) {
        THX_CHECK_ARG(c.searchType == 2, "thx_expectation_ctf: searchType must be 2 (SEARCH_TYPE_CTF)");
        THX_CHECK_ARG(cs->mLD > 0 && cs->attr && cs->d && cs->pD && cs->ctfRefineS >= 0.0 &&
                          (long)c.mLT * cs->mLD <= 1024,
                      "thx_expectation_ctf: bad CTF-search configuration");
    } else {
        THX_CHECK_ARG(c.searchType == 0 || c.searchType == 1,
                      "thx_expectation: searchType must be 0 or 1");
    }
    const int mLD = cs ? cs->mLD : 0;
    THX_CHECK_ARG(!global || (gQuat && gTrans && gPR && gPT),
                  "thx_expectation: a global search needs the global sample set");
    THX_CHECK_ARG(c.mLR > 0 && c.mLT > 0 && c.vdim == c.pf * c.idim && nImg >= 0 && nImg <= 65535 &&
                      nPxl > 0 && (!global || (c.nR > 0 && c.nT > 0)),
                  "thx_expectation: bad configuration");
    THX_CHECK_ARG(c.nK >= 1 && c.nK <= KMAX_CLASS, "thx_expectation: nK must be in [1, 64]");
    THX_CHECK_ARG(!c.volCells || c.nK == 1, "thx_expectation: volCells needs nK == 1");
    THX_CHECK_ARG(global || c.nK == 1 || cls,
                  "thx_expectation: a K-class local search needs the particles' classes (cls)");
    THX_CHECK_ARG(c.converge ? (c.minPhase >= 0 && c.maxPhase > c.minPhase && c.maxPhase <= 1000)
                             : (c.nPhase >= 0),
                  "thx_expectation: bad phase counts");
    THX_CHECK_ARG(c.perturbMean == 0 || c.perturbMean == 1, "thx_expectation: perturbMean must be 0 or 1");
    THX_CHECK_ARG(c.perturbMean == 0 || c.acgIters > 0, "thx_expectation: acgIters must be > 0");
    THX_CHECK_ARG(!global || c.nR <= 65535, "thx_expectation: nR > 65535");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(!pxOrder || (nOrd > 0 && nOrd % 16 == 0),
                  "thx_expectation: nOrd must be a positive multiple of 16");
    THX_CHECK_ARG(c.nSymElem >= 0 && c.nSymElem <= thx::SYM_MAX && (c.nSymElem == 0 || c.symQuat),
                  "thx_expectation: nSymElem 0 .. 64 with symQuat");
    const Plan p = plan(workspace, c, nImg, nPxl, pxOrder ? nOrd : nPxl, mLD, twoD);
    THX_CHECK_ARG(workspace && p.bytes <= wsBytes, "thx_expectation: workspace too small");
    hipStream_t s = thx::as_stream(stream);
    SideStream* side = nullptr;
    THX_RET(side_stream(s, &side));
    std::lock_guard<std::mutex> sideLock(side->mu);
    bool sidePending = false;      // a calVari on the side stream not yet joined
    // every exit, error paths included, leaves no side-stream work behind the
    // caller's stream: the caller may free or reuse the workspace right after
    struct SideGuard {
        SideStream* side;
        hipStream_t s;
        bool open = false;         // forked and not yet joined into s
        bool open2 = false;        // the same for the second side stream
        ~SideGuard()
        {
            if (open) {
                (void)hipEventRecord(side->join, side->s);
                (void)hipStreamWaitEvent(s, side->join, 0);
                (void)hipStreamSynchronize(side->s);
            }
            if (open2) {
                (void)hipEventRecord(side->join2, side->s2);
                (void)hipStreamWaitEvent(s, side->join2, 0);
                (void)hipStreamSynchronize(side->s2);
            }
        }
    } sideGuard{side, s};
    // the next phase's perturbation mean, already running on s2
    bool meanAhead = false;
    auto join2 = [&]() -> int {
        if (sideGuard.open2) {
            THX_HIP(hipEventRecord(side->join2, side->s2));
            THX_HIP(hipStreamWaitEvent(s, side->join2, 0));
            sideGuard.open2 = false;
        }
        return THX_OK;
    };
    auto fork = [&]() -> int {
        sideGuard.open = true;
        THX_HIP(hipEventRecord(side->fork, s));
        THX_HIP(hipStreamWaitEvent(side->s, side->fork, 0));
        return THX_OK;
    };
    auto join_rec = [&]() -> int {
        THX_HIP(hipEventRecord(side->join, side->s));
        sidePending = true;
        return THX_OK;
    };
    auto join = [&]() -> int {
        if (sidePending) THX_HIP(hipStreamWaitEvent(s, side->join, 0));
        sidePending = false;
        sideGuard.open = false;
        return THX_OK;
    };
    const unsigned gImg = thx::cdiv(nImg, 4);
    const unsigned gPf = thx::cdiv(nImg * GROUP, 256);
    const unsigned gOne = thx::cdiv(nImg, 256);
    const int nK = c.nK;
    const int nSym = twoD ? 0 : c.nSymElem;     // point-group symmetry: MODE_3D only
    // one class's projectee: a half-complex volume, or a half-complex image in 2D
    const size_t dimSize = (size_t)(c.vdim / 2 + 1) * c.vdim * (twoD ? 1 : c.vdim);
    const int rankDiv = twoD ? 2 : 8;      // setPeakFactor(PAR_R): PEAK_FACTOR_BASE (^3 in 3D)
    int* clsD = cls ? cls : p.cls;
    int* nPD = nPhaseOut ? nPhaseOut : p.nP;
    const int* clsSel = nK > 1 ? clsD : nullptr;    // rows / volumes picked per image
    // the y-pair copy: the compact ball around the pixel ring (radius pf
    // r_max + 2 voxels, no wrap, a few MB instead of the whole 2x volume:
    // its pages stay in the TLBs and its lines in one region), or the whole
    // copy when the ball is the volume
    int ypairR = 0;
    if (p.ypair) {
        if (env_on("THX_YPAIR_BALL")) {
            hipLaunchKernelGGL(k_max_r2, dim3(1), dim3(256), 0, s, iCol, iRow, nPxl, p.maxR2);
            THX_LAUNCH_CHECK();
            int r2 = 0;
            THX_HIP(hipMemcpyAsync(&r2, p.maxR2, sizeof(int), hipMemcpyDeviceToHost, s));
            THX_HIP(hipStreamSynchronize(s));
            const int R = (int)std::ceil(c.pf * std::sqrt((double)r2)) + 2;
            if (R + 2 <= c.vdim / 2 + 1 && thx::ypair_ball_elems(R) <= dimSize) ypairR = R;
        }
        for (int k = 0; k < nK; k++) {
            if (ypairR > 0)
                THX_RET(thx::volume_ypair_ball(vol + 2 * dimSize * k, c.vdim, ypairR,
                                               p.ypair + 4 * thx::ypair_ball_elems(ypairR) * k, s));
            else
                THX_RET(thx_volume_ypair(vol + 2 * dimSize * k, c.vdim, p.ypair + 4 * dimSize * k,
                                         stream));
        }
    }

    if (global) {
        // ---- global scan of every class (ExpectRotran + ExpectProject + ExpectGlobal3D
        // with kIdx = class, src/Optimiser.cpp:1815-1847)
        if (!twoD) THX_RET(thx_rotmat(gQuat, c.nR, p.gMat, stream));
        THX_RET(thx_trans_table(gTrans, c.nT, iCol, iRow, nPxl, c.idim, p.traP, stream));
        for (int k = 0; k < nK; k++) {
            if (twoD)   // ExpectGlobal2D: the class image at the (cos, sin) rows of gQuat
                THX_RET(thx::project2d_launch(vol + 2 * dimSize * k, c.vdim, c.pf, gQuat, 4, c.nR,
                                              iCol, iRow, nPxl, p.rotP, s));
            else
                THX_RET(thx_project3d(vol + 2 * dimSize * k, c.vdim, c.pf, p.gMat, c.nR, iCol,
                                      iRow, nPxl, p.rotP, stream));
            THX_RET(thx_global_scan(p.rotP, c.nR, p.traP, c.nT, dat, ctf, sigRcp, nImg, nPxl, gPR,
                                    gPT, k, nK, p.gWC, p.gWR, p.gWT, p.gBase, c.algo, p.scanWs,
                                    p.scanWsBytes, stream));
        }
        // ---- reseed (src/Optimiser.cpp:1930-2131): the class draw, then
        // setPeakFactor + keepHalfHeightPeak (R), resample R and T of the drawn
        // class, calVari with the scan floors (OPTIMISER_SCAN_SET_MIN_STD_WITH_PERTURB)
        if (nK > 1) {
            hipLaunchKernelGGL(k_pf_class, dim3(gOne), dim3(256), 0, s, nImg, nK, p.gWC, c.seed,
                               999u, clsD);
            THX_LAUNCH_CHECK();
        } else {
            THX_HIP(hipMemsetAsync(clsD, 0, sizeof(int) * nImg, s));
        }
        hipLaunchKernelGGL(k_pf_peak, dim3(gImg), dim3(256), 0, s, nImg, c.nR, p.gWR, nK * c.nR,
                           p.peakR, 1, clsSel, c.nR, nullptr, rankDiv);
        THX_LAUNCH_CHECK();
        shuffle_perm_launch(nImg, c.nR, c.shuffle, c.seed, 1000u, p.perm, nullptr, s);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(resample_kernel(c.nR, c.shuffle), dim3(gImg), dim3(256), resample_lds(c.nR, c.shuffle), s,
                           nImg, c.nR, c.mLR, gPR, 0,
                           p.gWR, nK * c.nR, c.seed, 1000u, p.anc, pR, p.topR, p.cdf,
                           c.shuffle ? p.perm : nullptr, nullptr, nullptr, clsSel, c.nR, nullptr);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, nImg, c.mLR, 4, gQuat, 0L, c.nR,
                           p.anc, quat, nullptr);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_top_copy, dim3(thx::cdiv(4 * nImg, 256)), dim3(256), 0, s, nImg, gQuat,
                           0L, p.topR, p.topQ, nullptr);
        THX_LAUNCH_CHECK();
        shuffle_perm_launch(nImg, c.nT, c.shuffle, c.seed, 1001u, p.perm, nullptr, s);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(resample_kernel(c.nT, c.shuffle), dim3(gImg), dim3(256), resample_lds(c.nT, c.shuffle), s,
                           nImg, c.nT, c.mLT, gPT, 0,
                           p.gWT, nK * c.nT, c.seed, 1001u, p.anc, pT, p.topT, p.cdf,
                           c.shuffle ? p.perm : nullptr, nullptr, nullptr, clsSel, c.nT, nullptr);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, nImg, c.mLT, 2, gTrans, 0L, c.nT,
                           p.anc, trans, nullptr);
        THX_LAUNCH_CHECK();
        // calVari with the scan floors, beside phase 1's inferACG mean (both only
        // read the reseeded cloud); its symmetrise (src/Particle.cpp:1028-1036)
        // first, on the stream both read from
        if (!twoD)
            THX_RET(thx::pf_symmetrise_launch(nImg, c.mLR, quat, 2, nullptr, c.symQuat, nSym, c.seed,
                                              1002u, nullptr, s));
        THX_RET(fork());
        hipLaunchKernelGGL(twoD ? k_pf_calvari2d : k_pf_calvari, dim3(gPf), dim3(256), 0, side->s,
                           nImg, c.mLR, quat, c.mLT, trans, c.kMin, c.sMin, p.kv, p.sv, nullptr,
                           p.acgHist);
        THX_LAUNCH_CHECK();
        THX_RET(join_rec());
    } else {
        // ---- local search from the caller's particle state: its spreads
        // (calVari on the given cloud) and, for the top-particle mean, calRank1st
        if (nK == 1 && !cls) THX_HIP(hipMemsetAsync(clsD, 0, sizeof(int) * nImg, s));
        if (!twoD)
            THX_RET(thx::pf_symmetrise_launch(nImg, c.mLR, quat, 2, nullptr, c.symQuat, nSym, c.seed,
                                              1002u, nullptr, s));
        hipLaunchKernelGGL(twoD ? k_pf_calvari2d : k_pf_calvari, dim3(gPf), dim3(256), 0, s, nImg,
                           c.mLR, quat, c.mLT, trans, 0.0, 0.0, p.kv, p.sv, nullptr, p.acgHist);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_top_by_weight, dim3(gOne), dim3(256), 0, s, nImg, c.mLR, quat, pR, p.topQ);
        THX_LAUNCH_CHECK();
        // the rotation peak factor a fresh particle carries (resetPeakFactor,
        // src/Particle.cpp:1957-1962: PEAK_FACTOR_MIN); a global search sets it
        // in the reseed
        hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, s, p.peakR, (long)nImg, 1e-3);
        THX_LAUNCH_CHECK();
    }
    if (cs) {
        // allocPreCal's cSearch branch (src/Optimiser.cpp:8124-8170), once per call
        THX_RET(thx_defocus_pre(cs->attr, nImg, iCol, iRow, nPxl, c.idim, p.freq, p.dfo, p.K1,
                                p.K2, stream));
    }
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, s, p.pC, (long)nImg, 1.0);
    THX_LAUNCH_CHECK();

    // ---- particle-filter phases (src/Optimiser.cpp:1183-1616): perturb +
    // balanceWeight, likelihood + marginals, keepHalfHeightPeak (R),
    // calRank1st, calVari (pre-resample cloud), resample, stopping rule
    const int phase0 = global ? 1 : 0;
    const int nPh = c.converge ? c.maxPhase - phase0 : c.nPhase;
    const int* done = nullptr;
    // the phases' volume: the caller's cell copy or vol (with the y-pair copy
    // for the device route)
    const float* phaseVol = c.volCells ? c.volCells : vol;
    const int phaseLayout = c.volCells ? 1 : 0;
    thx_local_sel sel{nullptr, nullptr, clsSel, (long long)dimSize};
    // 3D phases visit the images in view order (order.hip), through the
    // active list; results per image are unchanged
    const int* ord = nullptr;
    if (!twoD && nPh > 0 && view_order_on()) {
        THX_RET(thx::view_order(nImg, c.mLR, quat, p.ordKey, p.ordKeyOut, p.ordIdx, p.ord, p.ordTmp,
                                p.ordTmpBytes, s));
        ord = p.ord;
    }
    // the route samples images in index order whatever the visiting order
    // (the kernel a phase runs must not depend on it): every image without
    // the stopping rule, the index-ordered active list with it
    const int* sampleNone[2] = {nullptr, nullptr};
    const int* sampleIdx[2] = {p.actIdx, p.nActIdx};
    const int* const* routeSample = ord ? (c.converge ? sampleIdx : sampleNone) : nullptr;
    if (c.converge || ord) {
        THX_HIP(hipMemsetAsync(p.done, 0, sizeof(int) * nImg, s));
        hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, nImg, p.done, p.act, p.nAct, ord);
        THX_LAUNCH_CHECK();
        if (ord && c.converge) {
            hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, nImg, p.done, p.actIdx, p.nActIdx,
                               nullptr);
            THX_LAUNCH_CHECK();
        }
        if (c.converge) done = p.done;
        sel.active = p.act;
        sel.nActive = p.nAct;
    }
    // the particle clouds ping-pong between the caller's buffers and
    // tmpQ / tmpT: a phase reads the current pair and the resampling gathers
    // into the other (the pre-resample cloud stays readable for calVari and
    // the mean without a copy); the caller's buffers get the last one
    double* cq = quat;
    double* ct = trans;
    double* nq = p.tmpQ;
    double* nt = p.tmpT;
    for (int phase = phase0; phase < phase0 + nPh; phase++) {
        const bool large = phase == phase0 && (!global || c.largeFirst);
        if (twoD) {
            // MODE_2D perturb (von Mises, no mean) + balanceWeight (R, T)
            THX_RET(join());
            hipLaunchKernelGGL(k_pf_perturb2d, dim3(gPf), dim3(256), 0, s, nImg, c.mLR, c.mLT, cq,
                               ct, pR, pT, p.kv, p.sv,
                               large ? c.perturbFactorL : c.perturbFactor, c.transS, c.transM,
                               c.seed, (uint32_t)(2000 + phase), done);
            THX_LAUNCH_CHECK();
        } else if (c.perturbMean == 1) {
            if (meanAhead) {
                THX_RET(join2());      // forked after the last phase's rotation resampling
                meanAhead = false;
            } else {
                hipLaunchKernelGGL(k_pf_mean, dim3(gPf), dim3(256), 0, s, nImg, c.mLR, cq,
                                   c.acgIters, done, p.meanQ, nullptr);
                THX_LAUNCH_CHECK();
            }
        }
        if (!twoD) {
            THX_RET(join());     // the spreads of the previous calVari
            hipLaunchKernelGGL(k_pf_perturb, dim3(gPf), dim3(256), 0, s, nImg, c.mLR, c.mLT, cq,
                               ct, pR, pT, p.topQ, p.kv, p.sv,
                               large ? c.perturbFactorL : c.perturbFactor, c.transS, c.transM,
                               c.seed, (uint32_t)(2000 + phase), c.perturbMean, p.meanQ, done,
                               c.symQuat, nSym);
            THX_LAUNCH_CHECK();
        }
        if (cs) {
            // phase 0: initD(mLD, ctfRefineS); later: perturb(perturbFactorSCTF,
            // PAR_D) (src/Optimiser.cpp:1194-1195, 1208-1209); then the phase's
            // CTF per defocus sample (:1248-1273)
            hipLaunchKernelGGL(k_pf_defocus, dim3(gPf), dim3(256), 0, s, nImg, mLD,
                               phase == phase0 ? 0 : 1,
                               phase == phase0 ? cs->ctfRefineS : cs->perturbFactorSCTF, c.seed,
                               (uint32_t)(6000 + phase), cs->d, cs->pD, p.sdD, done);
            THX_LAUNCH_CHECK();
            THX_RET(thx_ctf_search(p.dfo, p.freq, cs->d, mLD, p.K1, p.K2, cs->attr, nImg, nPxl,
                                   p.ctfD, stream));
        }
        const int pi = phase - phase0;
        // phases past the caller's event pairs run untimed
        hipEvent_t* ev = pi < c.nPhaseEvents ? static_cast<hipEvent_t*>(c.phaseEvents) : nullptr;
        if (twoD) {
            if (ev) THX_HIP(hipEventRecord(ev[2 * pi], s));
            THX_RET(thx::local_phase2d_launch(vol, c.vdim, c.pf, clsSel, cq, 4, c.mLR, ct,
                                              c.mLT, p.pC, pR, pT, dat, cs ? p.ctfD : ctf, sigRcp,
                                              iCol, iRow, nPxl, c.idim, nImg, p.wC, p.wR, p.wT,
                                              p.base, static_cast<float*>(p.localWs), done, s,
                                              mLD, cs ? cs->pD : nullptr, p.wD, sel.active,
                                              sel.nActive));
            if (ev) THX_HIP(hipEventRecord(ev[2 * pi + 1], s));
        } else
        THX_RET(thx::local_phase_timed(&sel, ev ? ev[2 * pi] : nullptr, ev ? ev[2 * pi + 1] : nullptr,
                                       phaseVol, phaseLayout, c.vdim,
                                       c.pf, cq, c.mLR, ct, c.mLT, p.pC, pR, pT,
                                       dat, cs ? p.ctfD : ctf, sigRcp, iCol, iRow, pxOrder, nOrd,
                                       nPxl, c.idim, nImg, p.wC, p.wR, p.wT, p.base, p.localWs,
                                       p.localWsBytes, stream, mLD, cs ? cs->pD : nullptr, p.wD,
                                       p.ypair, pi < c.nPhaseRoute ? c.phaseRoute + pi : nullptr,
                                       routeSample, ypairR));
        hipLaunchKernelGGL(k_pf_peak, dim3(gImg), dim3(256), 0, s, nImg, c.mLR, p.wR, c.mLR,
                           p.peakR, 0, nullptr, 0, done, rankDiv);
        THX_LAUNCH_CHECK();
        // calVari's symmetrise (a drawn particle as the anchor) on the cloud the
        // resampling gathers from, then the pre-resample cloud, kept for calVari
        // and the gathers
        if (!twoD)
            THX_RET(thx::pf_symmetrise_launch(nImg, c.mLR, cq, 2, nullptr, c.symQuat, nSym, c.seed,
                                              (uint32_t)(5000 + phase), done, s));
        // calVari of the pre-resample cloud on the side stream (needed by the next
        // perturbation and the stopping rule only)
        THX_RET(fork());
        hipLaunchKernelGGL(twoD ? k_pf_calvari2d : k_pf_calvari, dim3(gPf), dim3(256), 0, side->s,
                           nImg, c.mLR, cq, c.mLT, ct, 0.0, 0.0, p.kv, p.sv, done,
                           p.acgHist);
        THX_LAUNCH_CHECK();
        THX_RET(join_rec());
        // resample R and T by the phase marginals; ancestors gathered in place
        shuffle_perm_launch(nImg, c.mLR, c.shuffle, c.seed, (uint32_t)(3000 + phase), p.perm, done, s);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(resample_kernel(c.mLR, c.shuffle), dim3(gImg), dim3(256), resample_lds(c.mLR, c.shuffle), s,
                           nImg, c.mLR, c.mLR, pR,
                           c.mLR, p.wR, c.mLR, c.seed, (uint32_t)(3000 + phase), p.ancR, pR,
                           p.topR, p.cdf, c.shuffle ? p.perm : nullptr, nullptr, nullptr, nullptr,
                           0, done);
        THX_LAUNCH_CHECK();
        // the next phase's perturbation mean needs only the resampled
        // rotations: it runs on s2 beside the gathers and the translations'
        // resampling, reading the pre-resample cloud through the ancestors (an
        // image the stopping rule retires below gets a mean nothing reads).
        // It reads the done mask as of the fork (a snapshot), never the
        // buffer k_pf_converge / k_compact write on s after it.
        if (!twoD && c.perturbMean == 1 && phase + 1 < phase0 + nPh) {
            if (done)
                THX_HIP(hipMemcpyAsync(p.doneSnap, done, sizeof(int) * nImg,
                                       hipMemcpyDeviceToDevice, s));
            THX_HIP(hipEventRecord(side->fork2, s));
            THX_HIP(hipStreamWaitEvent(side->s2, side->fork2, 0));
            sideGuard.open2 = true;
            hipLaunchKernelGGL(k_pf_mean, dim3(gPf), dim3(256), 0, side->s2, nImg, c.mLR, cq,
                               c.acgIters, done ? p.doneSnap : nullptr, p.meanQ, nullptr, p.ancR);
            THX_LAUNCH_CHECK();
            meanAhead = true;
        }
        hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, nImg, c.mLR, 4, (const double*)cq,
                           (long)c.mLR * 4, c.mLR, p.ancR, nq, done, 1);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_top_copy, dim3(thx::cdiv(4 * nImg, 256)), dim3(256), 0, s, nImg,
                           cq, (long)c.mLR * 4, p.topR, p.topQ, done);
        THX_LAUNCH_CHECK();
        shuffle_perm_launch(nImg, c.mLT, c.shuffle, c.seed, (uint32_t)(4000 + phase), p.perm, done, s);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(resample_kernel(c.mLT, c.shuffle), dim3(gImg), dim3(256), resample_lds(c.mLT, c.shuffle), s,
                           nImg, c.mLT, c.mLT, pT,
                           c.mLT, p.wT, c.mLT, c.seed, (uint32_t)(4000 + phase), p.anc, pT,
                           p.topT, p.cdf, c.shuffle ? p.perm : nullptr, nullptr, nullptr, nullptr,
                           0, done);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, nImg, c.mLT, 2, (const double*)ct,
                           (long)c.mLT * 2, c.mLT, p.anc, nt, done, 1);
        THX_LAUNCH_CHECK();
        // the resampled clouds are current from here
        std::swap(cq, nq);
        std::swap(ct, nt);
        if (cs) {
            // calRank1st, calVari, resample (mLD, PAR_D) (src/Optimiser.cpp:1483-1488);
            // no peak factor (OPTIMISER_PEAK_FACTOR_D is off, include/Config.h:220)
            hipLaunchKernelGGL(k_pf_defocus, dim3(gPf), dim3(256), 0, s, nImg, mLD, 2, 0.0, c.seed,
                               0u, cs->d, cs->pD, p.sdD, done);
            THX_LAUNCH_CHECK();
            shuffle_perm_launch(nImg, mLD, c.shuffle, c.seed, (uint32_t)(5000 + phase), p.perm, done, s);
            THX_LAUNCH_CHECK();
            hipLaunchKernelGGL(resample_kernel(mLD, c.shuffle), dim3(gImg), dim3(256), resample_lds(mLD, c.shuffle),
                               s, nImg, mLD, mLD, cs->pD, mLD, p.wD, mLD, c.seed,
                               (uint32_t)(5000 + phase), p.anc, cs->pD, p.topD, p.cdf,
                               c.shuffle ? p.perm : nullptr, nullptr, nullptr, nullptr, 0, done);
            THX_LAUNCH_CHECK();
            THX_HIP(hipMemcpyAsync(p.tmpD, cs->d, sizeof(double) * nImg * mLD,
                                   hipMemcpyDeviceToDevice, s));
            hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, nImg, mLD, 1, p.tmpD,
                               (long)mLD, mLD, p.anc, cs->d, done);
            THX_LAUNCH_CHECK();
        }
        if (c.converge) {
            THX_RET(join());
            hipLaunchKernelGGL(k_pf_converge, dim3(gOne), dim3(256), 0, s, nImg, phase, c.minPhase,
                               phase0 + nPh - 1, p.kv, p.sv, p.bestR, p.bestT, p.done, nPD,
                               cs ? p.sdD : nullptr, cs ? p.bestD : nullptr, (int)twoD);
            THX_LAUNCH_CHECK();
            hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, nImg, p.done, p.act, p.nAct, ord);
            THX_LAUNCH_CHECK();
            if (ord) {
                hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, nImg, p.done, p.actIdx,
                                   p.nActIdx, nullptr);
                THX_LAUNCH_CHECK();
            }
            if (phase >= c.minPhase) {
                int left = 0;
                THX_HIP(hipMemcpyAsync(&left, p.nAct, sizeof(int), hipMemcpyDeviceToHost, s));
                THX_HIP(hipStreamSynchronize(s));
                if (left == 0) break;
            }
        }
    }
    THX_RET(join());     // nothing of this call stays on the side streams
    THX_RET(join2());
    if (cq != quat) {
        THX_HIP(hipMemcpyAsync(quat, cq, sizeof(double) * nImg * c.mLR * 4, hipMemcpyDeviceToDevice, s));
        THX_HIP(hipMemcpyAsync(trans, ct, sizeof(double) * nImg * c.mLT * 2, hipMemcpyDeviceToDevice, s));
    }
    if (!c.converge) {
        hipLaunchKernelGGL(k_fill_int, dim3(64), dim3(256), 0, s, nPD, (long)nImg,
                           phase0 + c.nPhase - 1);
        THX_LAUNCH_CHECK();
    }
    if (score) {
        // per-image score: the last phase's baseline (the scan's without phases)
        THX_HIP(hipMemcpyAsync(score, nPh > 0 ? p.base : p.gBase, sizeof(float) * nImg,
                               hipMemcpyDeviceToDevice, s));
    }
    return THX_OK;
}

extern "C" int thx_expectation(const thx_expect_cfg* cfg, const float* vol,
                               const double* gQuat, const double* gTrans,
                               const double* gPR, const double* gPT,
                               const float* dat, const float* ctf,
                               const float* sigRcp, const int* iCol,
                               const int* iRow, const int* pxOrder, int nOrd, int nPxl, int nImg,
                               double* quat,
                               double* trans, double* pR, double* pT,
                               float* score, int* cls, int* nPhaseOut, void* workspace,
                               size_t wsBytes, thx_stream_t stream)
{
    return expectation_impl(cfg, nullptr, vol, gQuat, gTrans, gPR, gPT, dat, ctf, sigRcp, iCol,
                            iRow, pxOrder, nOrd, nPxl, nImg, quat, trans, pR, pT, score, cls,
                            nPhaseOut, workspace, wsBytes, stream);
}

// MODE_2D (src/Optimiser.cpp's _para.mode == MODE_2D branches of
// expectationG): vol holds nK half-complex class images, rotations are the
// particle rows (cos, sin, 0, 0).
extern "C" size_t thx_expectation2d_workspace(const thx_expect_cfg* cfg, int nImg, int nPxl)
{
    if (!cfg) return 0;
    return plan(nullptr, *cfg, nImg, nPxl, nPxl, 0, true).bytes;
}

extern "C" int thx_expectation2d(const thx_expect_cfg* cfg, const float* vol, const double* gRot,
                                 const double* gTrans, const double* gPR, const double* gPT,
                                 const float* dat, const float* ctf, const float* sigRcp,
                                 const int* iCol, const int* iRow, int nPxl, int nImg, double* rot,
                                 double* trans, double* pR, double* pT, float* score, int* cls,
                                 int* nPhaseOut, void* workspace, size_t wsBytes,
                                 thx_stream_t stream)
{
    return expectation_impl(cfg, nullptr, vol, gRot, gTrans, gPR, gPT, dat, ctf, sigRcp, iCol,
                            iRow, nullptr, 0, nPxl, nImg, rot, trans, pR, pT, score, cls,
                            nPhaseOut, workspace, wsBytes, stream, true);
}

extern "C" size_t thx_expectation2d_ctf_workspace(const thx_expect_cfg* cfg,
                                                  const thx_ctf_search_cfg* cs, int nImg, int nPxl)
{
    if (!cfg || !cs || cs->mLD <= 0) return 0;
    return plan(nullptr, *cfg, nImg, nPxl, nPxl, cs->mLD, true).bytes;
}

extern "C" int thx_expectation2d_ctf(const thx_expect_cfg* cfg, const thx_ctf_search_cfg* cs,
                                     const float* vol, const float* dat, const float* sigRcp,
                                     const int* iCol, const int* iRow, int nPxl, int nImg,
                                     double* rot, double* trans, double* pR, double* pT,
                                     float* score, int* cls, int* nPhaseOut, void* workspace,
                                     size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(cs, "thx_expectation2d_ctf: null CTF-search configuration");
    return expectation_impl(cfg, cs, vol, nullptr, nullptr, nullptr, nullptr, dat, nullptr,
                            sigRcp, iCol, iRow, nullptr, 0, nPxl, nImg, rot, trans, pR, pT, score,
                            cls, nPhaseOut, workspace, wsBytes, stream, true);
}

extern "C" int thx_expectation_ctf(const thx_expect_cfg* cfg, const thx_ctf_search_cfg* cs,
                                   const float* vol, const float* dat, const float* sigRcp,
                                   const int* iCol, const int* iRow, const int* pxOrder, int nOrd,
                                   int nPxl, int nImg, double* quat, double* trans, double* pR,
                                   double* pT, float* score, int* cls, int* nPhaseOut,
                                   void* workspace, size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(cs, "thx_expectation_ctf: null CTF-search configuration");
    return expectation_impl(cfg, cs, vol, nullptr, nullptr, nullptr, nullptr, dat, nullptr,
                            sigRcp, iCol, iRow, pxOrder, nOrd, nPxl, nImg, quat, trans, pR, pT,
                            score, cls, nPhaseOut, workspace, wsBytes, stream);
}
