// optimiser.hip -- device-resident expectation driver (host orchestration in
// C++ over the device kernels), the MI355X counterpart of
// Optimiser::expectationG (src/Optimiser.cpp:1684-3403) for K = 1, 3D,
// no CTF search:
//
//   global scan (a4-a8) -> reseed every particle from the scan marginals
//   (resample nR -> mLR, nT -> mLT; src/Optimiser.cpp:1930-2131) -> nPhase
//   particle-filter phases, each: perturb (R, T) -> fused projection +
//   likelihood + marginals (a6+a7+a9) -> calVari -> resample (a10).
//
// The reference leaves the particle filter on the host and round-trips to the
// GPU once per image per phase (gpu/src/cuthunder.cu:2675-3140 with a stream
// sync at :3140); here every step runs for the whole batch on device and the
// host only enqueues kernels (nothing synchronises, so the sequence can be
// captured into a HIP graph).
//
// Simplifications of Particle (documented in DESIGN.md, row f3 of SURVEY §8):
// the rotation perturbation uses the particle's top rotation as the ACG mean
// and a diagonal ACG spread estimated from the de-meaned cloud (instead of the
// fixed-point inferACG), the rotation prior after perturbation is uniform
// (instead of 1/pdfACG), and the support is not shuffled before systematic
// resampling.  Sampling is counter-based (Philox4x32-10), so a run is
// reproducible for a given seed.
#include "common.h"

namespace {

// ------------------------------------------------------------- Philox RNG
struct Philox {
    uint4 ctr;
    uint2 key;
    THX_DEV Philox(uint64_t seed, uint32_t a, uint32_t b, uint32_t c)
    {
        key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
        ctr = make_uint4(a, b, c, 0);
    }
    THX_DEV uint4 next()
    {
        uint4 x = ctr;
        uint2 k = key;
#pragma unroll
        for (int r = 0; r < 10; r++) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * x.x;
            const uint64_t p1 = (uint64_t)0xCD9E8D57u * x.z;
            x = make_uint4((uint32_t)(p1 >> 32) ^ x.y ^ k.x, (uint32_t)p1,
                           (uint32_t)(p0 >> 32) ^ x.w ^ k.y, (uint32_t)p0);
            k.x += 0x9E3779B9u;
            k.y += 0xBB67AE85u;
        }
        ctr.w++;
        return x;
    }
    THX_DEV double uniform()   // (0, 1)
    {
        const uint4 v = next();
        const uint64_t m = ((uint64_t)v.x << 21) ^ (uint64_t)v.y;
        return ((double)(m & ((1ull << 53) - 1)) + 0.5) * (1.0 / 9007199254740992.0);
    }
    THX_DEV double2 gauss2()   // Box-Muller
    {
        const double u1 = uniform(), u2 = uniform();
        const double r = sqrt(-2.0 * log(u1));
        double s, c;
        sincos(2.0 * M_PI * u2, &s, &c);
        return make_double2(r * c, r * s);
    }
};

THX_DEV void qmul(const double* a, const double* b, double* o)
{
    // quaternion_mul (src/Geometry/Euler.cpp), Hamilton product
    const double w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    const double x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    const double y = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    const double z = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
    o[0] = w; o[1] = x; o[2] = y; o[3] = z;
}

// --------------------------------------------------------------- resample
// One wave per image: systematic resampling (src/Particle.cpp:1343-1383) of
// (w, u) -> ancestors and 1/u priors; w may be shared by all images (ldw = 0).
// u0 ~ U(0, 1/nOut) is drawn from the counter RNG.
__global__ void __launch_bounds__(256) k_pf_resample(int nImg, int nIn, int nOut,
                                                     const double* __restrict__ w, int ldw,
                                                     const float* __restrict__ u, int ldu,
                                                     uint64_t seed, uint32_t stream,
                                                     int* __restrict__ anc,
                                                     double* __restrict__ wOut,
                                                     int* __restrict__ top,
                                                     double* __restrict__ cdfWs)
{
    const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (l >= nImg) return;
    const double* wl = w + (size_t)l * ldw;
    const float* ul = u + (size_t)l * ldu;
    double* cdf = cdfWs + (size_t)l * nIn;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = lane; i < nIn; i += 64) {
        const float v = ul[i];
        if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (top && lane == 0) top[l] = bi;
    // CDF by a wave prefix scan in FP64
    double tot = 0.0;
    for (int i = lane; i < nIn; i += 64) tot += wl[i] * (double)ul[i];
    tot = wave_sum(tot);
    double carry = 0.0;
    for (int b = 0; b < nIn; b += 64) {
        const int i = b + lane;
        double v = i < nIn ? wl[i] * (double)ul[i] / tot : 0.0;
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
    double s = 0.0;
    for (int j = lane; j < nOut; j += 64) {
        const double uj = (u0 + j * 1.0 / nOut) * last;
        int lo = 0, hi = nIn - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (uj > cdf[mid]) lo = mid + 1; else hi = mid;
        }
        const float ua = ul[lo];
        anc[(size_t)l * nOut + j] = lo;
        const double x = ua > 0.f ? 1.0 / (double)ua : 0.0;
        wOut[(size_t)l * nOut + j] = x;
        s += x;
    }
    s = wave_sum(s);
    for (int j = lane; j < nOut; j += 64)
        wOut[(size_t)l * nOut + j] = s > 0.0 ? wOut[(size_t)l * nOut + j] / s : 1.0 / nOut;
}

// gather ancestors: dst[l][j][:] = src[l (or shared)][anc[l][j]][:]
__global__ void __launch_bounds__(256) k_gather(int nImg, int nOut, int width,
                                                const double* __restrict__ src, long lds,
                                                int nIn, const int* __restrict__ anc,
                                                double* __restrict__ dst)
{
    const long n = (long)nImg * nOut * width;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int c = (int)(q % width);
        const long lj = q / width;
        const int l = (int)(lj / nOut);
        const int a = anc[lj];
        dst[q] = src[(size_t)l * lds + (size_t)a * width + c];
        (void)nIn;
    }
}

// calVari + perturb + balanceWeight for one image per wave.
//   R: de-mean by the top rotation, k_j = <q_j^2> / <q_0^2> (the diagonal of
//      inferACG's A, src/Particle.cpp:1004-1098 / DirectionalStat.cpp:184-222),
//      floored at kMin; perturb r_i <- top d_i top^-1 r_i with
//      d ~ ACG(diag(1, pf^2 min(1,k1), pf^2 min(1,k2), pf^2 min(1,k3)))
//      (Particle::perturb, src/Particle.cpp:1176-1230).
//   T: s_c = sd(t_c) floored at sMin, t_i += pf * N(0, s) (src/Particle.cpp:
//      1232-1262), reCentre beyond transM (:2473-2495), pT = 1/pdf normalised
//      (balanceWeight, :2340-2375).
__global__ void __launch_bounds__(256) k_pf_perturb(int nImg, int mR, int mT,
                                                    double* __restrict__ quat,
                                                    double* __restrict__ trans,
                                                    double* __restrict__ pR,
                                                    double* __restrict__ pT,
                                                    const double* __restrict__ topQ,
                                                    double pf, double kMin, double sMin,
                                                    double transS, double transM,
                                                    uint64_t seed, uint32_t stream)
{
    const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (l >= nImg) return;
    double* Q = quat + (size_t)l * mR * 4;
    double* Tr = trans + (size_t)l * mT * 2;
    Philox rng(seed, (uint32_t)l, stream, (uint32_t)lane);

    // ---- rotation
    double top[4], topc[4];
    for (int k = 0; k < 4; k++) top[k] = topQ[4 * l + k];
    topc[0] = top[0]; topc[1] = -top[1]; topc[2] = -top[2]; topc[3] = -top[3];
    double m0 = 0, m1 = 0, m2 = 0, m3 = 0;
    for (int i = lane; i < mR; i += 64) {
        double d[4];
        qmul(topc, Q + 4 * i, d);
        m0 += d[0] * d[0]; m1 += d[1] * d[1]; m2 += d[2] * d[2]; m3 += d[3] * d[3];
    }
    m0 = wave_sum(m0); m1 = wave_sum(m1); m2 = wave_sum(m2); m3 = wave_sum(m3);
    const double k1 = fmin(1.0, fmax(kMin, m1 / m0));
    const double k2 = fmin(1.0, fmax(kMin, m2 / m0));
    const double k3 = fmin(1.0, fmax(kMin, m3 / m0));
    const double sd1 = pf * sqrt(k1), sd2 = pf * sqrt(k2), sd3 = pf * sqrt(k3);
    for (int i = lane; i < mR; i += 64) {
        const double2 g0 = rng.gauss2(), g1 = rng.gauss2();
        double d[4] = {g0.x, g0.y * sd1, g1.x * sd2, g1.y * sd3};
        const double nn = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]);
        for (int k = 0; k < 4; k++) d[k] /= nn;
        double a[4], b[4], c[4];
        qmul(topc, Q + 4 * i, a);      // conj(mean) * r
        qmul(d, a, b);                 // pert * .
        qmul(top, b, c);               // mean * .
        const double cn = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2] + c[3] * c[3]);
        for (int k = 0; k < 4; k++) Q[4 * i + k] = c[k] / cn;
        pR[(size_t)l * mR + i] = 1.0 / mR;
    }

    // ---- translation
    double sx = 0, sy = 0;
    for (int i = lane; i < mT; i += 64) { sx += Tr[2 * i]; sy += Tr[2 * i + 1]; }
    sx = wave_sum(sx) / mT; sy = wave_sum(sy) / mT;
    double vx = 0, vy = 0;
    for (int i = lane; i < mT; i += 64) {
        vx += (Tr[2 * i] - sx) * (Tr[2 * i] - sx);
        vy += (Tr[2 * i + 1] - sy) * (Tr[2 * i + 1] - sy);
    }
    vx = wave_sum(vx); vy = wave_sum(vy);
    const double s0 = fmax(sMin, mT > 1 ? sqrt(vx / (mT - 1)) : 0.0);
    const double s1 = fmax(sMin, mT > 1 ? sqrt(vy / (mT - 1)) : 0.0);
    for (int i = lane; i < mT; i += 64) {
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
    // balanceWeight(PAR_T) on the perturbed set
    sx = 0; sy = 0;
    for (int i = lane; i < mT; i += 64) { sx += Tr[2 * i]; sy += Tr[2 * i + 1]; }
    sx = wave_sum(sx) / mT; sy = wave_sum(sy) / mT;
    vx = 0; vy = 0;
    for (int i = lane; i < mT; i += 64) {
        vx += (Tr[2 * i] - sx) * (Tr[2 * i] - sx);
        vy += (Tr[2 * i + 1] - sy) * (Tr[2 * i + 1] - sy);
    }
    vx = wave_sum(vx); vy = wave_sum(vy);
    const double b0 = fmax(1e-6, mT > 1 ? sqrt(vx / (mT - 1)) : 1.0);
    const double b1 = fmax(1e-6, mT > 1 ? sqrt(vy / (mT - 1)) : 1.0);
    double tot = 0.0;
    for (int i = lane; i < mT; i += 64) {
        const double u = (Tr[2 * i] - sx) / b0, v = (Tr[2 * i + 1] - sy) / b1;
        const double p = exp(-(u * u + v * v) / 2) / (2 * M_PI * b0 * b1);
        const double x = 1.0 / fmax(p, 1e-300);
        pT[(size_t)l * mT + i] = x;
        tot += x;
    }
    tot = wave_sum(tot);
    for (int i = lane; i < mT; i += 64) pT[(size_t)l * mT + i] /= tot;
}

struct Plan {
    // carve of the driver workspace
    float* rotP; double* gMat; float* traP;
    float* gWC; float* gWR; float* gWT; float* gBase;
    void* scanWs; size_t scanWsBytes;
    int* anc; double* cdf; int* topR; int* topT;
    double* tmpQ; double* tmpT; double* topQ;
    float* wC; float* wR; float* wT; float* base; double* pC;
    void* localWs; size_t localWsBytes;
    size_t bytes;
};

Plan plan(void* base, const thx_expect_cfg& c, int nImg, int nPxl, int nVisit)
{
    thx::Carver k(base, ~size_t(0));
    Plan p;
    const int nMax = c.nR > c.nT ? c.nR : c.nT;
    p.rotP = k.take<float>((size_t)2 * c.nR * nPxl);
    p.gMat = k.take<double>((size_t)9 * c.nR);
    p.traP = k.take<float>((size_t)2 * c.nT * nPxl);
    p.gWC = k.take<float>(nImg);
    p.gWR = k.take<float>((size_t)nImg * c.nR);
    p.gWT = k.take<float>((size_t)nImg * c.nT);
    p.gBase = k.take<float>(nImg);
    p.scanWsBytes = thx_global_scan_workspace(nImg, c.nR, c.nT, nPxl, c.algo);
    p.scanWs = k.take<char>(p.scanWsBytes);
    p.anc = k.take<int>((size_t)nImg * (c.mLR > c.mLT ? c.mLR : c.mLT));
    p.cdf = k.take<double>((size_t)nImg * (nMax > c.mLR ? nMax : c.mLR));
    p.topR = k.take<int>(nImg);
    p.topT = k.take<int>(nImg);
    p.tmpQ = k.take<double>((size_t)nImg * c.mLR * 4);
    p.tmpT = k.take<double>((size_t)nImg * c.mLT * 2);
    p.topQ = k.take<double>((size_t)nImg * 4);
    p.wC = k.take<float>(nImg);
    p.wR = k.take<float>((size_t)nImg * c.mLR);
    p.wT = k.take<float>((size_t)nImg * c.mLT);
    p.base = k.take<float>(nImg);
    p.pC = k.take<double>(nImg);
    p.localWsBytes = thx_local_phase_workspace(nImg, c.mLR, c.mLT, nVisit);
    p.localWs = k.take<char>(p.localWsBytes);
    p.bytes = k.off + 256;
    return p;
}

// topQ[l] = src[l (or shared)][top[l]] -- Particle::_topR after calRank1st
__global__ void k_top_copy(int nImg, const double* __restrict__ src, long lds,
                           const int* __restrict__ top, double* __restrict__ topQ)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nImg * 4) return;
    const int l = q / 4, k = q % 4;
    topQ[q] = src[(size_t)l * lds + (size_t)top[l] * 4 + k];
}

__global__ void k_fill(double* p, long n, double v)
{
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x)
        p[q] = v;
}

}  // namespace

extern "C" size_t thx_expectation_workspace(const thx_expect_cfg* cfg, int nImg, int nPxl,
                                            int nOrd)
{
    if (!cfg) return 0;
    return plan(nullptr, *cfg, nImg, nPxl, nOrd > 0 ? nOrd : nPxl).bytes;
}

#define THX_RET(call)                  \
    do {                               \
        int st_ = (call);              \
        if (st_ != THX_OK) return st_; \
    } while (0)

extern "C" int thx_expectation(const thx_expect_cfg* cfg, const float* vol,
                               const double* gQuat, const double* gTrans,
                               const double* gPR, const double* gPT,
                               const float* dat, const float* ctf,
                               const float* sigRcp, const int* iCol,
                               const int* iRow, const int* pxOrder, int nOrd, int nPxl, int nImg,
                               double* quat,
                               double* trans, double* pR, double* pT,
                               float* score, void* workspace, size_t wsBytes,
                               thx_stream_t stream)
{
    THX_CHECK_ARG(cfg && vol && gQuat && gTrans && gPR && gPT && dat && ctf && sigRcp &&
                      iCol && iRow && quat && trans && pR && pT,
                  "thx_expectation: null argument");
    const thx_expect_cfg& c = *cfg;
    THX_CHECK_ARG(c.nR > 0 && c.nT > 0 && c.mLR > 0 && c.mLT > 0 && c.nPhase >= 0 &&
                      c.vdim == c.pf * c.idim && nImg >= 0 && nImg <= 65535 && nPxl > 0,
                  "thx_expectation: bad configuration");
    THX_CHECK_ARG(c.nR <= 65535, "thx_expectation: nR > 65535");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(!pxOrder || (nOrd > 0 && nOrd % 16 == 0),
                  "thx_expectation: nOrd must be a positive multiple of 16");
    const Plan p = plan(workspace, c, nImg, nPxl, pxOrder ? nOrd : nPxl);
    THX_CHECK_ARG(workspace && p.bytes <= wsBytes, "thx_expectation: workspace too small");
    hipStream_t s = thx::as_stream(stream);
    const unsigned gImg = thx::cdiv(nImg, 4);

    // ---- global scan (ExpectRotran + ExpectProject + ExpectGlobal3D)
    THX_RET(thx_rotmat(gQuat, c.nR, p.gMat, stream));
    THX_RET(thx_project3d(vol, c.vdim, c.pf, p.gMat, c.nR, iCol, iRow, nPxl, p.rotP, stream));
    THX_RET(thx_trans_table(gTrans, c.nT, iCol, iRow, nPxl, c.idim, p.traP, stream));
    THX_RET(thx_global_scan(p.rotP, c.nR, p.traP, c.nT, dat, ctf, sigRcp, nImg, nPxl, gPR,
                            gPT, 0, 1, p.gWC, p.gWR, p.gWT, p.gBase, c.algo, p.scanWs,
                            p.scanWsBytes, stream));

    // ---- reseed from the scan marginals (src/Optimiser.cpp:1930-2131)
    hipLaunchKernelGGL(k_pf_resample, dim3(gImg), dim3(256), 0, s, nImg, c.nR, c.mLR, gPR, 0,
                       p.gWR, c.nR, c.seed, 1000u, p.anc, pR, p.topR, p.cdf);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, nImg, c.mLR, 4, gQuat, 0L, c.nR,
                       p.anc, quat);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_top_copy, dim3(thx::cdiv(4 * nImg, 256)), dim3(256), 0, s, nImg, gQuat,
                       0L, p.topR, p.topQ);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_pf_resample, dim3(gImg), dim3(256), 0, s, nImg, c.nT, c.mLT, gPT, 0,
                       p.gWT, c.nT, c.seed, 1001u, p.anc, pT, p.topT, p.cdf);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, nImg, c.mLT, 2, gTrans, 0L, c.nT,
                       p.anc, trans);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, s, p.pC, (long)nImg, 1.0);
    THX_LAUNCH_CHECK();

    // ---- particle-filter phases (src/Optimiser.cpp:1183-1616)
    for (int phase = 1; phase <= c.nPhase; phase++) {
        const double kMin = phase == 1 ? c.kMin : 1e-8;
        const double sMin = phase == 1 ? c.sMin : 1e-6;
        hipLaunchKernelGGL(k_pf_perturb, dim3(gImg), dim3(256), 0, s, nImg, c.mLR, c.mLT, quat,
                           trans, pR, pT, p.topQ, c.perturbFactor, kMin, sMin,
                           c.transS, c.transM, c.seed, (uint32_t)(2000 + phase));
        THX_LAUNCH_CHECK();
        THX_RET(thx_local_phase(vol, 0, c.vdim, c.pf, quat, c.mLR, trans, c.mLT, p.pC, pR, pT, dat,
                                ctf, sigRcp, iCol, iRow, pxOrder, nOrd, nPxl, c.idim, nImg, p.wC, p.wR, p.wT,
                                p.base, nullptr, p.localWs, p.localWsBytes, stream));
        // resample R and T by the phase marginals; ancestors gathered in place
        hipLaunchKernelGGL(k_pf_resample, dim3(gImg), dim3(256), 0, s, nImg, c.mLR, c.mLR, pR,
                           c.mLR, p.wR, c.mLR, c.seed, (uint32_t)(3000 + phase), p.anc, pR,
                           p.topR, p.cdf);
        THX_LAUNCH_CHECK();
        THX_HIP(hipMemcpyAsync(p.tmpQ, quat, sizeof(double) * nImg * c.mLR * 4,
                               hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, nImg, c.mLR, 4, p.tmpQ,
                           (long)c.mLR * 4, c.mLR, p.anc, quat);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_top_copy, dim3(thx::cdiv(4 * nImg, 256)), dim3(256), 0, s, nImg,
                           p.tmpQ, (long)c.mLR * 4, p.topR, p.topQ);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_pf_resample, dim3(gImg), dim3(256), 0, s, nImg, c.mLT, c.mLT, pT,
                           c.mLT, p.wT, c.mLT, c.seed, (uint32_t)(4000 + phase), p.anc, pT,
                           p.topT, p.cdf);
        THX_LAUNCH_CHECK();
        THX_HIP(hipMemcpyAsync(p.tmpT, trans, sizeof(double) * nImg * c.mLT * 2,
                               hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, nImg, c.mLT, 2, p.tmpT,
                           (long)c.mLT * 2, c.mLT, p.anc, trans);
        THX_LAUNCH_CHECK();
    }
    if (score) {
        // per-image score: log of the last phase's class marginal + baseline
        THX_HIP(hipMemcpyAsync(score, c.nPhase > 0 ? p.base : p.gBase, sizeof(float) * nImg,
                               hipMemcpyDeviceToDevice, s));
    }
    return THX_OK;
}
