// symmetry.hip -- point-group symmetry (row f1 and a3 / a10 in non-C1 use).
//
// Host: the symmetry elements of a point group, Symmetry::init
// (src/Geometry/Symmetry.cpp:104-118): fillSymmetryEntry's rotation
// operations (src/Geometry/SymmetryFunctions.cpp:65-152), fillLR's powers of
// each rotation (Symmetry.cpp:146-214) and completePointGroup's closure under
// products (:232-278), with novo / SAME_MATRIX at EQUAL_ACCURACY 1e-2
// (include/Geometry/Symmetry.h:64-73, include/Macro.h:106).  Only rotation
// operations occur in the reference's groups (its reflexion / inversion
// branches are CLOG(FATAL)), so the L matrices are identity and not carried.
//
// Device:
//   k_symmetrize_ft -- SYMMETRIZE_FT (include/Geometry/Transformation.h:
//     105-194): V'(v) = V(v) + sum_i [|R_i v|^2 < r^2] V~(R_i v) over the
//     half-complex grid, V~ getByInterpolationFT's trilinear gather with the
//     Hermitian fold (interp_ft, common.h), summed element by element in
//     FP32 as ADD_FT does;
//   thx_prepare_tf -- Reconstructor::prepareTF (src/Reconstructor.cpp:
//     1056-1091): RECONSTRUCTOR_NORMALISE_T_F's 1 / T[0] (:2455-2479), then
//     symmetrizeT / symmetrizeF with r = maxRadius pf + 1 (:2676-2690);
//     the GPU twin is PrepareTF (gpu/src/cuthunder.cu:6176);
//   k_pf_symmetrise -- Particle::symmetrise (src/Particle.cpp:2445-2471) via
//     symmetryCounterpart (Symmetry.cpp:309-335): each particle becomes the
//     one of q, conj(s_i) q closest to the anchor (largest |<., anchor>|,
//     first on ties); anchor (1, 0, 0, 0) (ANCHOR_POINT_2, Particle::reset
//     :168), a given quaternion per image (the perturbation mean, perturb
//     :1234) or a uniformly drawn particle of the cloud (calVari :1028-1036).
#include <cmath>
#include <cstring>
#include <regex>
#include <string>
#include <vector>

#include "common.h"
#include "symmetry.h"

namespace {

struct M33 {
    double a[3][3];
};

M33 mat_mul(const M33& x, const M33& y)
{
    M33 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0.0;
            for (int k = 0; k < 3; k++) s += x.a[i][k] * y.a[k][j];
            r.a[i][j] = s;
        }
    return r;
}

// rotate3D(dmat33&, const dvec4&), src/Geometry/Euler.cpp:181-189
M33 rot_of_quat(const double q[4])
{
    const double A[3][3] = {{0, -q[3], q[2]}, {q[3], 0, -q[1]}, {-q[2], q[1], 0}};
    M33 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double aa = 0.0;
            for (int k = 0; k < 3; k++) aa += A[i][k] * A[k][j];
            r.a[i][j] = (i == j ? 1.0 : 0.0) + 2 * q[0] * A[i][j] + 2 * aa;
        }
    return r;
}

// quaternion(dvec4&, phi, axis) + rotate3D, Euler.cpp:102-110, 272-281
M33 rot_axis(double phi, const double axis[3])
{
    const double s = std::sin(phi / 2);
    const double q[4] = {std::cos(phi / 2), s * axis[0], s * axis[1], s * axis[2]};
    return rot_of_quat(q);
}

// quaternion(dvec4&, const dmat33&), Euler.cpp:112-123
void quat_of_rot(const M33& m, double q[4])
{
    const double (*s)[3] = m.a;
    q[0] = 0.5 * std::sqrt(std::fmax(0.0, 1 + s[0][0] + s[1][1] + s[2][2]));
    q[1] = 0.5 * std::sqrt(std::fmax(0.0, 1 + s[0][0] - s[1][1] - s[2][2]));
    q[2] = 0.5 * std::sqrt(std::fmax(0.0, 1 - s[0][0] + s[1][1] - s[2][2]));
    q[3] = 0.5 * std::sqrt(std::fmax(0.0, 1 - s[0][0] - s[1][1] + s[2][2]));
    q[1] = std::copysign(q[1], s[2][1] - s[1][2]);
    q[2] = std::copysign(q[2], s[0][2] - s[2][0]);
    q[3] = std::copysign(q[3], s[1][0] - s[0][1]);
}

bool same(const M33& x, const M33& y)
{
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            if (std::fabs(x.a[i][j] - y.a[i][j]) > 1e-2) return false;   // EQUAL_ACCURACY
    return true;
}

struct Op {
    int fold;
    double axis[3];
};

// fillSymmetryEntry, src/Geometry/SymmetryFunctions.cpp:65-152 (the point
// group from symmetryGroup's name, :13-63); false: not a known group
bool entries(const std::string& name, std::vector<Op>& e)
{
    auto cn = [&](int n) { e.push_back({n, {0.0, 0.0, 1.0}}); };
    std::smatch m;
    if (std::regex_match(name, m, std::regex("C([0-9]+)"))) {
        cn(std::stoi(m[1]));
    } else if (std::regex_match(name, m, std::regex("D([0-9]+)"))) {
        cn(std::stoi(m[1]));
        e.push_back({2, {1.0, 0.0, 0.0}});
    } else if (name == "T") {
        e.push_back({3, {0.0, 0.0, 1.0}});
        e.push_back({2, {0.0, 0.816496, 0.577350}});
    } else if (name == "O") {
        e.push_back({3, {0.5773502, 0.5773502, 0.5773502}});
        e.push_back({4, {0.0, 0.0, 1.0}});
    } else if (name == "I1") {
        e.push_back({2, {1.0, 0.0, 0.0}});
        e.push_back({5, {0.8506508, 0.0, -0.5257311}});
        e.push_back({3, {0.9341724, 0.3568221, 0.0}});
    } else if (name == "I2") {
        cn(2);
        e.push_back({5, {0.5257311, 0.0, 0.8506508}});
        e.push_back({3, {0.0, 0.3568221, 0.9341724}});
    } else if (name == "I3") {
        e.push_back({2, {-0.5257311, 0.0, 0.8506508}});
        cn(5);
        e.push_back({3, {-0.4911235, 0.3568221, 0.7946545}});
    } else if (name == "I4") {
        e.push_back({2, {0.5257311, 0.0, 0.8506508}});
        e.push_back({5, {0.8944272, 0.0, 0.4472136}});
        e.push_back({3, {0.4911235, 0.3568221, 0.7946545}});
    } else {
        return false;
    }
    for (const Op& o : e)
        if (o.fold < 1) return false;
    return true;
}

}  // namespace

extern "C" int thx_symmetry(const char* sym, int cap, double* R, double* quat, int* nSymElem)
{
    THX_CHECK_ARG(sym && nSymElem && cap >= 0 && (cap == 0 || (R && quat)),
                  "thx_symmetry: bad arguments");
    std::vector<Op> ops;
    THX_CHECK_ARG(entries(sym, ops), "thx_symmetry: unknown point group '%s'", sym);
    std::vector<M33> Rs;
    M33 I{};
    for (int i = 0; i < 3; i++) I.a[i][i] = 1.0;
    auto novo = [&](const M33& x) {
        if (same(x, I)) return false;
        for (const M33& y : Rs)
            if (same(x, y)) return false;
        return true;
    };
    // fillLR: the powers of every rotation operation; the angle is an RFLOAT
    // (FP32 in the reference's SINGLE_PRECISION build), so is angle * j
    for (const Op& o : ops) {
        const float angle = (float)(2 * M_PI / o.fold);
        for (int j = 1; j < o.fold; j++) {
            const M33 x = rot_axis((double)(angle * (float)j), o.axis);
            if (novo(x)) Rs.push_back(x);
        }
    }
    // completePointGroup: the (i, j) cells of a table that grows with every new
    // element, visited in row-major order, first unvisited cell each time
    std::vector<std::vector<char>> done(Rs.size(), std::vector<char>(Rs.size(), 0));
    for (;;) {
        int ci = -1, cj = -1;
        for (size_t i = 0; i < done.size() && ci < 0; i++)
            for (size_t j = 0; j < done.size(); j++)
                if (!done[i][j]) {
                    ci = (int)i;
                    cj = (int)j;
                    break;
                }
        if (ci < 0) break;
        done[ci][cj] = 1;
        const M33 x = mat_mul(Rs[ci], Rs[cj]);
        if (novo(x)) {
            Rs.push_back(x);
            for (auto& row : done) row.push_back(0);
            done.push_back(std::vector<char>(Rs.size(), 0));
        }
    }
    *nSymElem = (int)Rs.size();
    THX_CHECK_ARG(cap == 0 || cap >= (int)Rs.size(), "thx_symmetry: %s has %d elements, cap %d",
                  sym, (int)Rs.size(), cap);
    for (int i = 0; cap > 0 && i < (int)Rs.size(); i++) {
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) R[9 * i + 3 * a + b] = Rs[i].a[a][b];
        quat_of_rot(Rs[i], quat + 4 * i);
    }
    return THX_OK;
}

namespace {

using thx::SYM_MAX;

// trilinear gather of a real half-complex volume (T), interp_ft's taps and
// weights; the Hermitian fold leaves a real value unchanged
THX_DEV float interp_ft_real(const float* __restrict__ vol, int vdim, float x, float y, float z)
{
    if (!(x >= 0.f)) { x = -x; y = -y; z = -z; }
    const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
    const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
    const float dx = x - fx, dy = y - fy, dz = z - fz;
    const float vx[2] = {1.f - dx, dx};
    const float vy[2] = {1.f - dy, dy};
    const float vz[2] = {1.f - dz, dz};
    const int nColFT = vdim / 2 + 1;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 2; k++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const size_t row = ((size_t)wrap_idx(z0 + k, vdim) * vdim + wrap_idx(y0 + j, vdim)) * nColFT + x0;
#pragma unroll
            for (int i = 0; i < 2; i++) s += vol[row + i] * (vx[i] * vy[j] * vz[k]);
        }
    return s;
}

// One thread per half-complex voxel (i, j, k), i fastest: the rotated
// coordinate R v in FP64 (dvec3 oldCor = mat * newCor), the radius test in
// FP64, the gather at the FP32-rounded coordinate (RFLOAT arguments of
// getByInterpolationFT).  src and dst are distinct.
template <bool CPLX>
__global__ void __launch_bounds__(256) k_symmetrize_ft(const float* __restrict__ src,
                                                       float* __restrict__ dst, int vdim,
                                                       const double* __restrict__ R, int nSym,
                                                       double r2)
{
    __shared__ double sR[SYM_MAX * 9];
    for (int q = threadIdx.x; q < nSym * 9; q += blockDim.x) sR[q] = R[q];
    __syncthreads();
    const int nColFT = vdim / 2 + 1;
    const long n = (long)nColFT * vdim * vdim;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
        const int i = (int)(q % nColFT);
        const long jk = q / nColFT;
        const int jw = (int)(jk % vdim), kw = (int)(jk / vdim);
        const double x = i, y = jw < vdim / 2 ? jw : jw - vdim, z = kw < vdim / 2 ? kw : kw - vdim;
        if (CPLX) {
            const float2* s2 = reinterpret_cast<const float2*>(src);
            float2 acc = s2[q];
            for (int e = 0; e < nSym; e++) {
                const double* m = sR + 9 * e;
                const double ox = m[0] * x + m[1] * y + m[2] * z;
                const double oy = m[3] * x + m[4] * y + m[5] * z;
                const double oz = m[6] * x + m[7] * y + m[8] * z;
                if (ox * ox + oy * oy + oz * oz < r2) {
                    const float2 v = interp_ft(s2, vdim, (float)ox, (float)oy, (float)oz);
                    acc.x += v.x;
                    acc.y += v.y;
                }
            }
            reinterpret_cast<float2*>(dst)[q] = acc;
        } else {
            float acc = src[q];
            for (int e = 0; e < nSym; e++) {
                const double* m = sR + 9 * e;
                const double ox = m[0] * x + m[1] * y + m[2] * z;
                const double oy = m[3] * x + m[4] * y + m[5] * z;
                const double oz = m[6] * x + m[7] * y + m[8] * z;
                if (ox * ox + oy * oy + oz * oz < r2)
                    acc += interp_ft_real(src, vdim, (float)ox, (float)oy, (float)oz);
            }
            dst[q] = acc;
        }
    }
}

// RECONSTRUCTOR_NORMALISE_T_F: sf = 1 / T[0] (RFLOAT), F and T scaled, into
// the copies the symmetrisation reads
__global__ void __launch_bounds__(256) k_normalise_tf(const float* __restrict__ F,
                                                      const float* __restrict__ T, long n,
                                                      float* __restrict__ Fo, float* __restrict__ To)
{
    const float sf = 1.f / T[0];
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
        const float2 f = reinterpret_cast<const float2*>(F)[q];
        reinterpret_cast<float2*>(Fo)[q] = make_float2(f.x * sf, f.y * sf);
        To[q] = T[q] * sf;
    }
}

}  // namespace


namespace {

constexpr int SYM_GROUP = 8;   // lanes per image (one cloud), inside one wave

// anchorMode 0: ANCHOR_POINT_2; 1: anchor[l * 4 ..]; 2: particle draw(l) of
// the cloud itself, read before any lane of the group writes
__global__ void __launch_bounds__(256) k_pf_symmetrise(int nImg, int mR, double* __restrict__ quat,
                                                       int anchorMode,
                                                       const double* __restrict__ anchor,
                                                       const double* __restrict__ symQ, int nSym,
                                                       uint64_t seed, uint32_t stream,
                                                       const int* __restrict__ done)
{
    __shared__ double sQ[SYM_MAX * 4];
    for (int q = threadIdx.x; q < nSym * 4; q += blockDim.x) sQ[q] = symQ[q];
    __syncthreads();
    const int l = (blockIdx.x * 256 + threadIdx.x) / SYM_GROUP;
    const int lane = threadIdx.x % SYM_GROUP;
    if (l >= nImg || (done && done[l])) return;
    double* Q = quat + (size_t)l * mR * 4;
    double a[4] = {1.0, 0.0, 0.0, 0.0};
    if (anchorMode == 1) {
        for (int k = 0; k < 4; k++) a[k] = anchor[4 * l + k];
    } else if (anchorMode == 2) {
        // gsl_rng_uniform_int(engine, _nR) of calVari: one counter draw per image
        Philox rng(seed, (uint32_t)l, stream, 0u);
        const int idx = (int)(rng.uniform() * mR) % mR;
        for (int k = 0; k < 4; k++) a[k] = Q[4 * idx + k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int i = lane; i < mR; i += SYM_GROUP) thx::sym_counterpart(Q + 4 * i, a, sQ, nSym);
}

}  // namespace

namespace thx {
int pf_symmetrise_launch(int nImg, int mR, double* quat, int anchorMode, const double* anchor,
                         const double* symQ, int nSym, uint64_t seed, uint32_t stream,
                         const int* done, hipStream_t s)
{
    if (nImg == 0 || nSym == 0) return THX_OK;
    hipLaunchKernelGGL(k_pf_symmetrise, dim3(cdiv((long)nImg * SYM_GROUP, 256)), dim3(256), 0, s, nImg,
                       mR, quat, anchorMode, anchor, symQ, nSym, seed, stream, done);
    THX_LAUNCH_CHECK();
    return THX_OK;
}
}  // namespace thx

extern "C" int thx_pf_symmetrise(int nImg, int mR, double* quat, int anchorMode, const double* anchor,
                                 const double* symQuat, int nSymElem, unsigned long long seed,
                                 unsigned streamId, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && mR > 0 && nSymElem >= 0 && nSymElem <= SYM_MAX &&
                      anchorMode >= 0 && anchorMode <= 2,
                  "thx_pf_symmetrise: bad arguments");
    THX_CHECK_ARG(nImg == 0 || nSymElem == 0 || (quat && symQuat && (anchorMode != 1 || anchor)),
                  "thx_pf_symmetrise: null argument");
    return thx::pf_symmetrise_launch(nImg, mR, quat, anchorMode, anchor, symQuat, nSymElem, seed,
                                     streamId, nullptr, thx::as_stream(stream));
}

extern "C" int thx_symmetrize_ft(const float* src, float* dst, int isComplex, int vdim,
                                 const double* R, int nSymElem, double r, thx_stream_t stream)
{
    THX_CHECK_ARG(src && dst && src != dst && vdim > 0 && vdim % 2 == 0 && nSymElem >= 0 &&
                      nSymElem <= SYM_MAX && (nSymElem == 0 || R),
                  "thx_symmetrize_ft: bad arguments");
    // a voxel within r interpolates at x0 + 1 <= r + 1: still inside the
    // vdim / 2 + 1 half-complex columns only while r <= vdim / 2 - 1
    THX_CHECK_ARG(r >= 0 && r <= vdim / 2 - 1,
                  "thx_symmetrize_ft: radius %g past the half box %d (taps would leave the row)", r,
                  vdim / 2 - 1);
    hipStream_t s = thx::as_stream(stream);
    const long n = (long)(vdim / 2 + 1) * vdim * vdim;
    const unsigned grid = (unsigned)std::min<long>(thx::cdiv(n, 256), 65536L);
    if (isComplex)
        hipLaunchKernelGGL(k_symmetrize_ft<true>, dim3(grid), dim3(256), 0, s, src, dst, vdim, R,
                           nSymElem, r * r);
    else
        hipLaunchKernelGGL(k_symmetrize_ft<false>, dim3(grid), dim3(256), 0, s, src, dst, vdim, R,
                           nSymElem, r * r);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" size_t thx_prepare_tf_workspace(int vdim)
{
    if (vdim <= 0 || vdim % 2) return 0;
    return (size_t)(vdim / 2 + 1) * vdim * vdim * 3 * sizeof(float) + 512;
}

extern "C" int thx_prepare_tf(float* F, float* T, int vdim, const double* R, int nSymElem,
                              int maxRadius, int pf, void* workspace, size_t wsBytes,
                              thx_stream_t stream)
{
    THX_CHECK_ARG(F && T && vdim > 0 && vdim % 2 == 0 && pf > 0 && maxRadius >= 0 &&
                      nSymElem >= 0 && nSymElem <= SYM_MAX && (nSymElem == 0 || R),
                  "thx_prepare_tf: bad arguments");
    THX_CHECK_ARG(workspace && wsBytes >= thx_prepare_tf_workspace(vdim),
                  "thx_prepare_tf: workspace too small");
    THX_CHECK_ARG((long)maxRadius * pf + 1 <= vdim / 2 - 1,
                  "thx_prepare_tf: maxRadius * pf + 1 = %ld past the half box %d", (long)maxRadius * pf + 1,
                  vdim / 2 - 1);
    hipStream_t s = thx::as_stream(stream);
    const long n = (long)(vdim / 2 + 1) * vdim * vdim;
    thx::Carver k(workspace, wsBytes);
    float* Fc = k.take<float>(2 * (size_t)n);
    float* Tc = k.take<float>((size_t)n);
    const unsigned grid = (unsigned)std::min<long>(thx::cdiv(n, 256), 65536L);
    hipLaunchKernelGGL(k_normalise_tf, dim3(grid), dim3(256), 0, s, F, T, n, Fc, Tc);
    THX_LAUNCH_CHECK();
    const double r = (double)maxRadius * pf + 1;
    THX_RET(thx_symmetrize_ft(Tc, T, 0, vdim, R, nSymElem, r, stream));
    THX_RET(thx_symmetrize_ft(Fc, F, 1, vdim, R, nSymElem, r, stream));
    return THX_OK;
}
