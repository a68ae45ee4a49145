// reconstruct.hip -- f1: the reconstruction solve of one half-map,
// Reconstructor::reconstruct (src/Reconstructor.cpp:1129-1831; GPU twin
// reconstructG :1835, cuthunder PrepareTF / CalculateT / CalculateW /
// CalculateF, gpu/src/cuthunder.cu:6176-8826), 3D, trilinear insert kernel,
// on device with hipFFT:
//
//   MAP:      T /= FSC'(u) on shells 5 pf <= |k| < maxR pf, FSC' = the
//             half-map FSC at shell u / pf clamped to [1e-3, 1 - 1e-3]
//             (sqrt(2 FSC / (1 + FSC)) when joining halves)
//             (RECONSTRUCTOR_WIENER_FILTER_FSC, :1150-1279);
//   W = 1 inside the sphere |k| < maxR pf, 0 outside; T = max(T, 1e-25);
//   grid correction (:1356-1552): repeat C = T W -> back-transform ->
//             multiply by the MKB real-space kernel table / MKB_RL(0)
//             (convoluteC, :2595-2675) -> forward transform ->
//             W /= max(|C|, 1e-6) inside the sphere; stop when
//             max | |C| - 1 | (RECONSTRUCTOR_CHECK_C_MAX, checkC :2522-2593)
//             < 1e-2, or after >= MIN_N_ITER_BALANCE (10) iterations with two
//             in a row not below 0.95 x the previous, or at 30
//             (include/Reconstructor.h:61-69); without grid correction
//             W = 1 / max(|T|, 1e-6) (:1553-1587);
//   pad = F W inside the sphere -> back-transform (FFT::bw scales by 1/size,
//             src/FFT.cpp:204-229) -> the central N^3 box (VOL_EXTRACT_RL)
//             -> divided by TIK_RL(|r| / (pf N)) = j0(pi |r| / (pf N))^2
//             (RECONSTRUCTOR_CORRECT_CONVOLUTION_KERNEL with the trilinear
//             kernel, :1733-1818).
// Layouts: F / T / W / C half-complex [k][j][i] of box vdim = pf N (the
// Volume FT layout = hipFFT's R2C layout); real-space arrays [k][j][i] with
// the origin at index 0 and negative coordinates wrapped (Volume RL).
#include <hipfft/hipfft.h>

#include <cmath>
#include <vector>

#include <atomic>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>

#include "common.h"
#include "fft_lds.h"

#define THX_FFT(call)                                                          \
    do {                                                                       \
        hipfftResult r_ = (call);                                              \
        if (r_ != HIPFFT_SUCCESS) {                                            \
            ::thx::set_error("%s:%d %s: hipfft error %d", __FILE__, __LINE__, \
                             #call, (int)r_);                                  \
            return THX_ERR_HIP;                                                \
        }                                                                      \
    } while (0)

namespace {

constexpr int TAB_N = 100000;   // _kernelRL.init(MKB_RL_R2, 0, 1, 1e5) (src/Reconstructor.cpp:77-88)


// k of a half-complex index: i in [0, vdim/2], j, k wrapped to [-vdim/2, vdim/2)
THX_DEV void ft_coord(long q, int vdim, int& i, int& j, int& k)
{
    const int nc = vdim / 2 + 1;
    i = (int)(q % nc);
    const long r = q / nc;
    j = (int)(r % vdim);
    k = (int)(r / vdim);
    if (j >= vdim / 2) j -= vdim;
    if (k >= vdim / 2) k -= vdim;
}

#define GRID_STRIDE(q, n) \
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < (n); q += (long)gridDim.x * blockDim.x)

__global__ void k_wiener(float* __restrict__ T, int vdim, int pf, int maxR,
                         const double* __restrict__ fsc, int nFsc, int joinHalf)
{
    const long n = (long)(vdim / 2 + 1) * vdim * vdim;
    const long lo = (long)5 * pf * 5 * pf, hi = (long)maxR * pf * maxR * pf;   // WIENER_FACTOR_MIN_R 5
    GRID_STRIDE(q, n)
    {
        int i, j, k;
        ft_coord(q, vdim, i, j, k);
        const long quad = (long)i * i + (long)j * j + (long)k * k;
        if (quad < lo || quad >= hi) continue;
        const int u = (int)rintf(sqrtf((float)quad));            // AROUND(NORM_3)
        float f = (u / pf >= nFsc) ? 0.f : (float)fsc[u / pf];
        f = fmaxf(1e-3f, fminf(1.f - 1e-3f, f));                  // FSC_BASE_L / _H
        if (joinHalf) f = sqrtf(2.f * f / (1.f + f));
        T[q] = T[q] / f;
    }
}

// W = 1 inside the sphere, 0 outside; T = max(T, 1e-25)
__global__ void k_init_w(float* __restrict__ W, float* __restrict__ T, int vdim, long r2)
{
    const long n = (long)(vdim / 2 + 1) * vdim * vdim;
    GRID_STRIDE(q, n)
    {
        int i, j, k;
        ft_coord(q, vdim, i, j, k);
        W[q] = ((long)i * i + (long)j * j + (long)k * k < r2) ? 1.f : 0.f;
        T[q] = fmaxf(T[q], 1e-25f);
    }
}

// no grid correction: W = 1 / max(|T|, 1e-6) inside the sphere
__global__ void k_w_from_t(float* __restrict__ W, const float* __restrict__ T, int vdim, long r2)
{
    const long n = (long)(vdim / 2 + 1) * vdim * vdim;
    GRID_STRIDE(q, n)
    {
        int i, j, k;
        ft_coord(q, vdim, i, j, k);
        if ((long)i * i + (long)j * j + (long)k * k < r2) W[q] = 1.f / fmaxf(fabsf(T[q]), 1e-6f);
    }
}

// C = T W (T real, so C is real): the first iteration's C
__global__ void k_c_from_tw(float2* __restrict__ C, const float* __restrict__ T,
                            const float* __restrict__ W, long n)
{
    GRID_STRIDE(q, n) C[q] = make_float2(T[q] * W[q], 0.f);
}

// Per-iteration passes: a workgroup covers a slab of RB_SPLIT-th of a k-plane
// (flat over (j, i), i fastest, j by a magic-number division), so there are
// few workgroups (one atomic each) and every thread streams hundreds of
// elements.
constexpr int RB_THREADS = 512, RB_SPLIT = 4;

inline unsigned magic_u(unsigned d) { return d <= 1 ? 0u : 0xFFFFFFFFu / d + 1u; }
__device__ __forceinline__ int udiv_m(int u, int d, unsigned m)
{
    return d <= 1 ? u : (int)__umulhi((unsigned)u, m);
}

// The real-space factor of convoluteC, kernelRL(QUAD_3 / (N pf)^2) / nf
// scaled by 1/size of FFT::bw, per octant voxel (|i|, |j|, |k|), i fastest:
// it depends on |r|^2 only, so the balancing passes read it coalesced (68 MB
// at vdim 512) instead of gathering the 1e5-entry table per voxel.
__global__ void k_kernel_octant(float* __restrict__ oct, int vdim, const float* __restrict__ tab,
                                float nf, float scale)
{
    const int h1 = vdim / 2 + 1;
    const long n = (long)h1 * h1 * h1;
    const float inv = 1.f / ((float)vdim * (float)vdim);
    GRID_STRIDE(q, n)
    {
        const int a = (int)(q % h1);
        const long bc = q / h1;
        const int b = (int)(bc % h1), c = (int)(bc / h1);
        const float x = (float)(a * a + b * b + c * c) * inv;
        const int t = min(TAB_N, (int)rintf(x / 1e-5f));          // TabFunction: _tab[AROUND((x - a) / s)]
        oct[q] = scale * tab[t] / nf;
    }
}

// convoluteC in real space: c(i,j,k) * the octant factor of (|i|, |j|, |k|)
__global__ void __launch_bounds__(RB_THREADS) k_kernel_mul(float* __restrict__ c, int vdim,
                                                           const float* __restrict__ oct,
                                                           unsigned mVdim)
{
    const int k = blockIdx.y;
    const int h1 = vdim / 2 + 1;
    const int ak = k > vdim / 2 ? vdim - k : k;
    const int nPlane = vdim * vdim;
    const int q0 = (int)((long)nPlane * blockIdx.x / RB_SPLIT);
    const int q1 = (int)((long)nPlane * (blockIdx.x + 1) / RB_SPLIT);
    float* plane = c + (size_t)k * nPlane;
    const float* o = oct + (size_t)ak * h1 * h1;
    for (int q = q0 + threadIdx.x; q < q1; q += RB_THREADS) {
        const int j = udiv_m(q, vdim, mVdim), i = q - j * vdim;
        const int ai = i > vdim / 2 ? vdim - i : i, aj = j > vdim / 2 ? vdim - j : j;
        plane[q] *= o[aj * h1 + ai];
    }
}

// W /= max(|C|, 1e-6) inside the sphere; max | |C| - 1 | over the sphere;
// fused with the next iteration's C = T W (the same pass over W)
__global__ void __launch_bounds__(RB_THREADS) k_update_w(float* __restrict__ W, float2* __restrict__ C,
                                                         const float* __restrict__ T, int vdim, long r2,
                                                         unsigned mNc, unsigned* __restrict__ diffBits)
{
    const int nc = vdim / 2 + 1;
    const int k = blockIdx.y;
    const int kk = k >= vdim / 2 ? k - vdim : k;
    const int nPlane = vdim * nc;
    const int q0 = (int)((long)nPlane * blockIdx.x / RB_SPLIT);
    const int q1 = (int)((long)nPlane * (blockIdx.x + 1) / RB_SPLIT);
    const size_t base = (size_t)k * nPlane;
    float dmax = 0.f;
    for (int q = q0 + threadIdx.x; q < q1; q += RB_THREADS) {
        const int j = udiv_m(q, nc, mNc), i = q - j * nc;
        const int jj = j >= vdim / 2 ? j - vdim : j;
        const size_t e = base + q;
        float w = W[e];
        if ((long)i * i + (long)jj * jj + (long)kk * kk < r2) {
            const float2 cv = C[e];
            const float a = sqrtf(cv.x * cv.x + cv.y * cv.y);
            w = w / fmaxf(a, 1e-6f);
            W[e] = w;
            dmax = fmaxf(dmax, fabsf(a - 1.f));
        }
        C[e] = make_float2(T[e] * w, 0.f);
    }
    dmax = wave_max(dmax);
    __shared__ float sm[RB_THREADS / 64];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = dmax;
    __syncthreads();
    if (threadIdx.x == 0) {
        float m = sm[0];
        for (int w = 1; w < RB_THREADS / 64; w++) m = fmaxf(m, sm[w]);
        if (m > 0.f) atomicMax(diffBits, __float_as_uint(m));   // non-negative floats order as their bits
    }
}

// pad = F W inside the sphere, 0 outside
__global__ void k_pad(float2* __restrict__ P, const float2* __restrict__ F, const float* __restrict__ W,
                      int vdim, long r2)
{
    const long n = (long)(vdim / 2 + 1) * vdim * vdim;
    GRID_STRIDE(q, n)
    {
        int i, j, k;
        ft_coord(q, vdim, i, j, k);
        const float2 f = F[q];
        const float w = W[q];
        P[q] = ((long)i * i + (long)j * j + (long)k * k < r2) ? make_float2(f.x * w, f.y * w)
                                                              : make_float2(0.f, 0.f);
    }
}

// the central N^3 box of the back-transformed pad (VOL_EXTRACT_RL) divided by
// TIK_RL(|r| / (pf N)); both arrays origin-at-0 with wrapped negatives
__global__ void k_extract(float* __restrict__ dst, const float* __restrict__ src, int N, int vdim,
                          float scale)
{
    const long n = (long)N * N * N;
    GRID_STRIDE(q, n)
    {
        int i = (int)(q % N);
        const long r = q / N;
        int j = (int)(r % N), k = (int)(r / N);
        if (i >= N / 2) i -= N;
        if (j >= N / 2) j -= N;
        if (k >= N / 2) k -= N;
        const long s = ((long)wrap_idx(k, vdim) * vdim + wrap_idx(j, vdim)) * vdim + wrap_idx(i, vdim);
        const float rr = sqrtf((float)(i * i + j * j + k * k)) / (float)(vdim);
        const float x = (float)M_PI * rr;
        const float j0 = x == 0.f ? 1.f : sinf(x) / x;
        dst[q] = src[s] * scale / (j0 * j0);
    }
}


// ------------------------------------------------ strided passes of the 3D FFT
// hipFFT's 3D plans run the two strided axes (y, z) of a 512^3 transform at
// ~0.9 TB/s (1.25 ms per pass).  Here a workgroup takes CF_TX consecutive
// x columns (one 128-B row piece per point) of one line along y or z into
// LDS, bit-reversed, runs the radix-2 Cooley-Tukey stages there, and writes
// the columns back in place: every HBM access is a coalesced row piece.  The
// contiguous x axis stays on hipFFT (1D batched R2C / C2R), so a 3D transform
// is two of these passes and one batched 1D pass -- the decomposition of
// FFTW's / hipFFT's multi-dimensional real transforms (complex transforms
// along the full axes, the real one along the halved axis), unnormalised.
constexpr int CF_TX = 16;                // columns per tile
constexpr int CF_PITCH = CF_TX + 1;      // LDS row pitch (float2): spreads a stage's rows over banks
constexpr int CF_THREADS = 256;

template <bool INV>
__global__ void __launch_bounds__(CF_THREADS) k_col_fft(float2* __restrict__ a, int n, int logn,
                                                        long sAxis, long sOuter, int nxh,
                                                        const float2* __restrict__ tw)
{
    extern __shared__ float2 sm[];       // [n][CF_PITCH] data, then n / 2 twiddles
    float2* sTw = sm + n * CF_PITCH;
    const int x0 = blockIdx.x * CF_TX;
    const int ncol = min(CF_TX, nxh - x0);
    float2* col = a + (long)blockIdx.y * sOuter + x0;
    for (int k = threadIdx.x; k < (n >> 1); k += CF_THREADS) {
        float2 w = tw[k];                   // exp(-2 pi i k / n)
        if (INV) w.y = -w.y;
        sTw[k] = w;
    }
    // CF_THREADS / CF_TX rows per sweep; eight sweeps in flight
#pragma unroll 8
    for (int q = threadIdx.x; q < n * CF_TX; q += CF_THREADS) {
        const int p = q / CF_TX, c = q % CF_TX;
        const float2 v = c < ncol ? col[(long)p * sAxis + c] : make_float2(0.f, 0.f);
        sm[(int)(__brev((unsigned)p) >> (32 - logn)) * CF_PITCH + c] = v;
    }
    __syncthreads();
    for (int half = 1, st = n >> 1; half < n; half <<= 1, st >>= 1) {
#pragma unroll 4
        for (int q = threadIdx.x; q < (n >> 1) * CF_TX; q += CF_THREADS) {
            const int j = q / CF_TX, c = q % CF_TX;
            const int k = j & (half - 1);
            const int i0 = ((j - k) << 1) + k, i1 = i0 + half;
            const float2 w = sTw[k * st];
            const float2 u = sm[i0 * CF_PITCH + c], v = sm[i1 * CF_PITCH + c];
            const float2 t = make_float2(w.x * v.x - w.y * v.y, w.x * v.y + w.y * v.x);
            sm[i0 * CF_PITCH + c] = make_float2(u.x + t.x, u.y + t.y);
            sm[i1 * CF_PITCH + c] = make_float2(u.x - t.x, u.y - t.y);
        }
        __syncthreads();
    }
#pragma unroll 8
    for (int q = threadIdx.x; q < n * CF_TX; q += CF_THREADS) {
        const int p = q / CF_TX, c = q % CF_TX;
        if (c < ncol) col[(long)p * sAxis + c] = sm[p * CF_PITCH + c];
    }
}

// ------------------------------------------ balancing on the even half-grid
// Inside the balancing loop C = T W is real, and real + Hermitian makes it
// point-even, C(-k) = C(k); so is c = IFFT(C), c times the (even) kernel,
// and the forward transform of that.  A real point-even array is determined
// by half of it, and both transforms of the iteration run on half grids
// (N = vdim, H = N / 2 + 1):
//   frequency side: C / W / T on the half-complex grid [kz][ky][kx < H];
//   space side:     c on [nz < H][ny][nx];
//   between:        G [nz < H][ky or ny][kx < H] complex (H N H, half of a
//                   full half-complex volume).
// One iteration is four passes over G (each column / row transformed in
// LDS by one wave, wave_fft in fft_lds.h):
//   x rows   (nz, ny): Hermitian in kx -> C2R (+) -> c * kernel / N^3 -> R2C (-)
//   y columns (nz, kx): C2C (-);
//   z columns (ky, kx): Hermitian in nz (G(-nz) = conj G(nz)) -> C2R (-) =
//             the balanced C of this iteration -> W /= max(|C|, 1e-6) inside,
//             max | |C| - 1 | -> next C = T W -> R2C (+) along z;
//   y columns (nz, kx): C2C (+);
// against two full 3D transforms and two element passes over N^3 arrays.
// The kx = 0 and kx = N / 2 planes of T are replaced by their Hermitian
// average first: a C2R reads only that average of those planes (FFTW,
// hipFFT and numpy's irfftn alike), so the balanced W is unchanged.
constexpr int EV_CT = 16;          // columns per tile of the column passes
constexpr int EV_WAVES = 4;

bool even_ok(int vdim) { return vdim == 64 || vdim == 128 || vdim == 256 || vdim == 512; }

// LDS: the padded columns (rows) and the twiddle table
template <int N>
constexpr size_t even_col_lds() { return (size_t)(EV_CT * thx::fft_pitch<N>() + N) * sizeof(float2); }

template <int N>
constexpr size_t even_row_lds() { return (size_t)(EV_WAVES * thx::fft_pitch<N>() + N) * sizeof(float2); }

// the twiddle table into LDS (the stages read it at the L1-missing strides
// of k r N / (Ns R); from global memory each stage waited on L2)
template <int N>
THX_DEV const float2* even_twiddles(float2* sTw, const float2* __restrict__ tw)
{
    for (int q = threadIdx.x; q < N; q += blockDim.x) sTw[q] = tw[q];
    return sTw;
}

// T on the kx = 0 and kx = N / 2 planes := (T(k) + T(-k)) / 2
__global__ void k_sym_planes(float* __restrict__ T, int vdim)
{
    const int nc = vdim / 2 + 1;
    const long n = 2L * vdim * vdim;
    GRID_STRIDE(q, n)
    {
        const int x = q < (long)vdim * vdim ? 0 : vdim / 2;
        const long jk = q % ((long)vdim * vdim);
        const int j = (int)(jk % vdim), k = (int)(jk / vdim);
        const int pj = (vdim - j) % vdim, pk = (vdim - k) % vdim;
        const long a = ((long)k * vdim + j) * nc + x, b = ((long)pk * vdim + pj) * nc + x;
        if (a < b) {
            const float m = 0.5f * (T[a] + T[b]);
            T[a] = m;
            T[b] = m;
        }
    }
}

// blockIdx.x -> tile (-1: past the end) with runs of consecutive tiles on
// one XCD: dispatch deals workgroups round-robin over the 8 XCDs, and the
// kx-neighbouring tiles of the column passes share the 128-byte lines of
// T and W (a tile row of floats is 64 bytes), read once per XCD's L2.
THX_DEV int even_tile(int ntiles)
{
    const int per = (ntiles + 7) / 8;
    const int t = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
    return t < ntiles ? t : -1;
}

// z columns.  INIT: C = T W (W as k_init_w left it) -> R2C (+) along z.
// Otherwise first the C2R (-) along z of G's Hermitian nz-half: the balanced
// C, whose |C| updates W inside the sphere (and the max | |C| - 1 |), then the
// same as INIT.  A block: a tile of EV_CT kx columns at one ky (even_tile).
// Every global load of a thread (its G rows, then its T and W rows) is
// issued before the first LDS write, so the T / W latency hides behind the
// C2R instead of being paid once per kz.
template <int N, bool INIT>
__global__ void __launch_bounds__(64 * EV_WAVES) k_even_z(float2* __restrict__ G, float* __restrict__ W,
                                                         const float* __restrict__ T, int r2,
                                                         unsigned* __restrict__ diffBits,
                                                         const float2* __restrict__ tw)
{
    extern __shared__ float2 sm[];
    constexpr int H = N / 2 + 1, P = thx::fft_pitch<N>(), NT = (H + EV_CT - 1) / EV_CT;
    constexpr int RSTEP = 64 * EV_WAVES / EV_CT;
    constexpr int NZ = N / RSTEP, NG = (H + RSTEP - 1) / RSTEP;   // rows per thread
    float2* tile = sm;                                   // [EV_CT][P], column c rotated by c
    const float2* stw = even_twiddles<N>(sm + EV_CT * P, tw);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int t = even_tile(NT * N);
    const int kx0 = (t % NT) * EV_CT, ky = t / NT;
    const int ncol = min(EV_CT, H - kx0);
    const int c = tid % EV_CT, rr = tid / EV_CT;         // row mapping: column c, rows rr + RSTEP i
    const bool on = c < ncol;
    const int jy = ky < N / 2 ? ky : ky - N;
    const int ix = kx0 + c;
    float2* col = tile + c * P;
    float2 g[INIT ? 1 : NG];
    if (!INIT) {
#pragma unroll
        for (int i = 0; i < NG; i++) {
            const int nz = rr + i * RSTEP;
            g[i] = on && nz < H ? G[((size_t)nz * N + ky) * H + ix] : make_float2(0.f, 0.f);
        }
    }
    float w[NZ], tv[NZ];
#pragma unroll
    for (int i = 0; i < NZ; i++) {
        const size_t e = ((size_t)(rr + i * RSTEP) * N + ky) * H + ix;
        w[i] = on ? W[e] : 0.f;
        tv[i] = on ? T[e] : 0.f;
    }
    if (!INIT) {
#pragma unroll
        for (int i = 0; i < NG; i++) {
            const int nz = rr + i * RSTEP;
            if (nz < H) {
                col[thx::fft_slot<N>(nz, c)] = g[i];
                if (nz > 0 && nz < N / 2) col[thx::fft_slot<N>(N - nz, c)] = make_float2(g[i].x, -g[i].y);
            }
        }
        __syncthreads();
        for (int cc = wv; cc < ncol; cc += EV_WAVES) thx::wave_fft<N>(tile + cc * P, cc, stw, -1.f, lane);
        __syncthreads();
    }
    float dmax = 0.f;
    if (on) {
#pragma unroll
        for (int i = 0; i < NZ; i++) {
            const int kz = rr + i * RSTEP;
            const int slot = thx::fft_slot<N>(kz, c);
            float wi = w[i];
            if (!INIT) {
                const int jz = kz < N / 2 ? kz : kz - N;
                if (ix * ix + jy * jy + jz * jz < r2) {
                    const float m = fabsf(col[slot].x);
                    wi = wi / fmaxf(m, 1e-6f);
                    W[((size_t)kz * N + ky) * H + ix] = wi;
                    dmax = fmaxf(dmax, fabsf(m - 1.f));
                }
            }
            col[slot] = make_float2(tv[i] * wi, 0.f);
        }
    }
    __syncthreads();
    for (int cc = wv; cc < ncol; cc += EV_WAVES) thx::wave_fft<N>(tile + cc * P, cc, stw, 1.f, lane);
    __syncthreads();
    if (on) {
#pragma unroll
        for (int i = 0; i < NG; i++) {
            const int nz = rr + i * RSTEP;
            if (nz < H) G[((size_t)nz * N + ky) * H + ix] = col[thx::fft_slot<N>(nz, c)];
        }
    }
    if (!INIT) {
        dmax = wave_max(dmax);
        __shared__ float sMax[EV_WAVES];
        if (lane == 0) sMax[wv] = dmax;
        __syncthreads();
        if (tid == 0) {
            float m = sMax[0];
            for (int k = 1; k < EV_WAVES; k++) m = fmaxf(m, sMax[k]);
            if (m > 0.f) atomicMax(diffBits, __float_as_uint(m));
        }
    }
}

// y columns: C2C along y, sign S.  A block: a tile of EV_CT kx columns at one nz.
template <int N, int S>
__global__ void __launch_bounds__(64 * EV_WAVES) k_even_y(float2* __restrict__ G, const float2* __restrict__ tw)
{
    extern __shared__ float2 sm[];
    constexpr int H = N / 2 + 1, P = thx::fft_pitch<N>(), NT = (H + EV_CT - 1) / EV_CT;
    constexpr int RSTEP = 64 * EV_WAVES / EV_CT, NY = N / RSTEP;
    const int t = even_tile(NT * H);
    if (t < 0) return;
    float2* tile = sm;
    const float2* stw = even_twiddles<N>(sm + EV_CT * P, tw);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int kx0 = (t % NT) * EV_CT, nz = t / NT;
    const int ncol = min(EV_CT, H - kx0);
    const int c = tid % EV_CT, rr = tid / EV_CT;
    const bool on = c < ncol;
    float2* base = G + (size_t)nz * N * H + kx0 + c;
    float2* col = tile + c * P;
    float2 v[NY];
#pragma unroll
    for (int i = 0; i < NY; i++) v[i] = on ? base[(size_t)(rr + i * RSTEP) * H] : make_float2(0.f, 0.f);
#pragma unroll
    for (int i = 0; i < NY; i++) col[thx::fft_slot<N>(rr + i * RSTEP, c)] = v[i];
    __syncthreads();
    for (int cc = wv; cc < ncol; cc += EV_WAVES) thx::wave_fft<N>(tile + cc * P, cc, stw, (float)S, lane);
    __syncthreads();
    if (on) {
#pragma unroll
        for (int i = 0; i < NY; i++) base[(size_t)(rr + i * RSTEP) * H] = col[thx::fft_slot<N>(rr + i * RSTEP, c)];
    }
}

// x rows (nz < H, ny): the Hermitian kx-half -> C2R (+) -> times the kernel
// octant (1 / N^3 and 1 / nf included) -> R2C (-), in place.  One wave per
// row; the row and its octant row are loaded before the first transform.
template <int N>
__global__ void __launch_bounds__(64 * EV_WAVES) k_even_x(float2* __restrict__ G, const float* __restrict__ oct,
                                                         const float2* __restrict__ tw)
{
    extern __shared__ float2 sm[];
    constexpr int H = N / 2 + 1, P = thx::fft_pitch<N>();
    constexpr int NX = (H + 63) / 64, NO = N / 64 > 0 ? N / 64 : 1;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float2* stw = even_twiddles<N>(sm + EV_WAVES * P, tw);
    __syncthreads();
    const long row = (long)blockIdx.x * EV_WAVES + wv;
    if (row >= (long)H * N) return;
    float2* buf = sm + wv * P;
    float2* g = G + row * H;
    const int nz = (int)(row / N), ny = (int)(row % N);
    const int ay = ny <= N / 2 ? ny : N - ny;
    const float* o = oct + ((size_t)nz * H + ay) * H;
    float2 v[NX];
    float ov[NO];
#pragma unroll
    for (int i = 0; i < NX; i++) {
        const int x = lane + 64 * i;
        v[i] = x < H ? g[x] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < NO; i++) {
        const int x = lane + 64 * i;
        ov[i] = x < N ? o[x <= N / 2 ? x : N - x] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NX; i++) {
        const int x = lane + 64 * i;
        if (x < H) {
            buf[thx::fft_slot<N>(x, 0)] = v[i];
            if (x > 0 && x < N / 2) buf[thx::fft_slot<N>(N - x, 0)] = make_float2(v[i].x, -v[i].y);
        }
    }
    thx::wave_lds_sync();
    thx::wave_fft<N>(buf, 0, stw, 1.f, lane);
#pragma unroll
    for (int i = 0; i < NO; i++) {
        const int x = lane + 64 * i;
        if (x < N) {
            const int sl = thx::fft_slot<N>(x, 0);
            buf[sl] = make_float2(buf[sl].x * ov[i], 0.f);
        }
    }
    thx::wave_lds_sync();
    thx::wave_fft<N>(buf, 0, stw, -1.f, lane);
#pragma unroll
    for (int i = 0; i < NX; i++) {
        const int x = lane + 64 * i;
        if (x < H) g[x] = buf[thx::fft_slot<N>(x, 0)];
    }
}

template <int N>
int even_iteration_n(float2* G, float* W, const float* T, const float* oct, int r2, unsigned* diff,
                     const float2* tw, bool init, bool update, hipStream_t s)
{
    constexpr int H = N / 2 + 1;
    const dim3 b(64 * EV_WAVES);
    constexpr int NT = (H + EV_CT - 1) / EV_CT;
    static_assert(NT * N % 8 == 0, "k_even_z: whole runs of tiles per XCD (no early exit before its barriers)");
    const dim3 gz(NT * N), gy((NT * H + 7) / 8 * 8);
    const dim3 gx((unsigned)(((long)H * N + EV_WAVES - 1) / EV_WAVES));
    constexpr size_t lc = even_col_lds<N>(), lr = even_row_lds<N>();
    static std::atomic<unsigned> set[5];
    THX_RET(thx::set_max_lds(reinterpret_cast<const void*>(k_even_z<N, true>), (int)lc, set[0]));
    THX_RET(thx::set_max_lds(reinterpret_cast<const void*>(k_even_z<N, false>), (int)lc, set[1]));
    THX_RET(thx::set_max_lds(reinterpret_cast<const void*>(k_even_y<N, 1>), (int)lc, set[2]));
    THX_RET(thx::set_max_lds(reinterpret_cast<const void*>(k_even_y<N, -1>), (int)lc, set[3]));
    THX_RET(thx::set_max_lds(reinterpret_cast<const void*>(k_even_x<N>), (int)lr, set[4]));
    if (init) {
        hipLaunchKernelGGL((k_even_z<N, true>), gz, b, lc, s, G, W, T, r2, diff, tw);
        THX_LAUNCH_CHECK();
    }
    if (update) {
        hipLaunchKernelGGL((k_even_y<N, 1>), gy, b, lc, s, G, tw);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL((k_even_x<N>), gx, b, lr, s, G, oct, tw);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL((k_even_y<N, -1>), gy, b, lc, s, G, tw);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL((k_even_z<N, false>), gz, b, lc, s, G, W, T, r2, diff, tw);
        THX_LAUNCH_CHECK();
    }
    return THX_OK;
}

// init: G = R2C_z(T W); update: one balancing iteration (W, diff updated, G = the next C's z-transform)
int even_iteration(int vdim, float2* G, float* W, const float* T, const float* oct, long r2,
                   unsigned* diff, const float2* tw, bool init, bool update, hipStream_t s)
{
    switch (vdim) {
        case 64: return even_iteration_n<64>(G, W, T, oct, (int)r2, diff, tw, init, update, s);
        case 128: return even_iteration_n<128>(G, W, T, oct, (int)r2, diff, tw, init, update, s);
        case 256: return even_iteration_n<256>(G, W, T, oct, (int)r2, diff, tw, init, update, s);
        case 512: return even_iteration_n<512>(G, W, T, oct, (int)r2, diff, tw, init, update, s);
        default: thx::set_error("even balancing: unsupported vdim %d", vdim); return THX_ERR_ARG;
    }
}

// ---------------------------------------------------------- MKB kernel table
// MKB_RL_R2 (src/Functions/Functions.cpp, FUNCTIONS_MKB_ORDER_0):
// (2 pi)^1.5 a^3 / I0(alpha) * I_{3/2}(v) / v^1.5 (u^2 <= alpha^2) or
// J_{3/2}(v) / v^1.5, v = sqrt(|alpha^2 - u^2|), u^2 = (2 pi a)^2 r2.
double bessel_i0(double x)
{
    double s = 1.0, t = 1.0;
    for (int k = 1; k < 200; k++) {
        t *= (x * x / 4.0) / ((double)k * k);
        s += t;
        if (t < 1e-17 * s) break;
    }
    return s;
}

// I_{3/2}(v) / v^1.5 (modified = true) or J_{3/2}(v) / v^1.5
double nu15_over(double v, bool modified)
{
    if (v < 0.5) {   // series: sum (+-v^2/4)^k / (2^1.5 k! Gamma(k + 2.5))
        const double g25 = 1.329340388179137;   // Gamma(2.5)
        double term = 1.0 / (std::pow(2.0, 1.5) * g25), s = term;
        for (int k = 1; k < 30; k++) {
            term *= (modified ? 1.0 : -1.0) * (v * v / 4.0) / ((double)k * (k + 1.5));
            s += term;
        }
        return s;
    }
    const double c = std::sqrt(2.0 / (M_PI * v)) / std::pow(v, 1.5);
    return modified ? c * (std::cosh(v) - std::sinh(v) / v) : c * (std::sin(v) / v - std::cos(v));
}

double mkb_rl_r2(double r2, double a, double alpha)
{
    const double u2 = std::pow(2 * M_PI * a, 2) * r2;
    const bool in = u2 <= alpha * alpha;
    const double v = std::sqrt(in ? alpha * alpha - u2 : u2 - alpha * alpha);
    return std::pow(2 * M_PI, 1.5) * a * a * a / bessel_i0(alpha) * nu15_over(v, in);
}

struct Plans {
    hipfftHandle c2r = 0, r2c = 0, r2cN = 0;
    hipfftHandle c2rX = 0, r2cX = 0;     // 1D batched along x (the column-pass transforms)
    float2* tw = nullptr;                // vdim twiddles exp(-2 pi i k / vdim)
    bool cols = false;                   // the column-pass transforms are available
    size_t work = 0;
};

// The column-pass 3D transforms: power-of-two vdim whose LDS tile fits
bool col_fft_ok(int vdim)
{
    return vdim >= 16 && (vdim & (vdim - 1)) == 0 &&
           (size_t)vdim * (CF_PITCH + 1) * sizeof(float2) <= 160 * 1024;
}

int make_plans(Plans& p, int vdim, int N)
{
    size_t w1 = 0, w2 = 0, w3 = 0;
    THX_FFT(hipfftCreate(&p.c2r));
    THX_FFT(hipfftSetAutoAllocation(p.c2r, 0));
    THX_FFT(hipfftMakePlan3d(p.c2r, vdim, vdim, vdim, HIPFFT_C2R, &w1));
    THX_FFT(hipfftCreate(&p.r2c));
    THX_FFT(hipfftSetAutoAllocation(p.r2c, 0));
    THX_FFT(hipfftMakePlan3d(p.r2c, vdim, vdim, vdim, HIPFFT_R2C, &w2));
    THX_FFT(hipfftCreate(&p.r2cN));
    THX_FFT(hipfftSetAutoAllocation(p.r2cN, 0));
    THX_FFT(hipfftMakePlan3d(p.r2cN, N, N, N, HIPFFT_R2C, &w3));
    p.work = std::max(w1, std::max(w2, w3));
    p.cols = col_fft_ok(vdim);
    if (p.cols) {
        size_t w4 = 0, w5 = 0;
        int n[1] = {vdim}, nh[1] = {vdim / 2 + 1};
        const int batch = vdim * vdim;
        THX_FFT(hipfftCreate(&p.c2rX));
        THX_FFT(hipfftSetAutoAllocation(p.c2rX, 0));
        THX_FFT(hipfftMakePlanMany(p.c2rX, 1, n, nh, 1, vdim / 2 + 1, n, 1, vdim, HIPFFT_C2R, batch,
                                   &w4));
        THX_FFT(hipfftCreate(&p.r2cX));
        THX_FFT(hipfftSetAutoAllocation(p.r2cX, 0));
        THX_FFT(hipfftMakePlanMany(p.r2cX, 1, n, n, 1, vdim, nh, 1, vdim / 2 + 1, HIPFFT_R2C, batch,
                                   &w5));
        p.work = std::max(p.work, std::max(w4, w5));
        std::vector<float2> h(vdim);     // the column passes read k < vdim / 2, the even loop all
        for (int k = 0; k < vdim; k++) {
            const double t = -2.0 * M_PI * k / vdim;
            h[k] = make_float2((float)std::cos(t), (float)std::sin(t));
        }
        THX_HIP(hipMalloc(reinterpret_cast<void**>(&p.tw), sizeof(float2) * h.size()));
        THX_HIP(hipMemcpy(p.tw, h.data(), sizeof(float2) * h.size(), hipMemcpyHostToDevice));
    }
    return THX_OK;
}

// The 3D C2R / R2C of the balancing loop and the final pad: hipFFT's 3D
// plans (default), or (p.cols) two column passes + hipFFT's batched 1D
// transform along x.  Measured at 512^3 (profiles/r03_fft_ab.jsonl): hipFFT
// 1.48-1.49 ms per transform, the radix-2 column passes 1.64-1.81 ms, so the
// 3D plans stay (thx_fft3d's method 2 runs the column passes).
// C is overwritten either way (hipFFT's out-of-place C2R may too).
bool use_cols(const Plans& p, int method = 0)
{
    return method == 2 && p.cols;
}

int col_pass(const Plans& p, float2* C, int vdim, bool inv, bool zAxis, hipStream_t s)
{
    const int nxh = vdim / 2 + 1;
    int logn = 0;
    while ((1 << logn) < vdim) logn++;
    const dim3 g((nxh + CF_TX - 1) / CF_TX, vdim);
    const long sAxis = zAxis ? (long)vdim * nxh : nxh;
    const long sOuter = zAxis ? nxh : (long)vdim * nxh;
    const size_t lds = ((size_t)vdim * CF_PITCH + vdim / 2) * sizeof(float2);
    static std::atomic<unsigned> ldsSet[2];
    THX_RET(thx::set_max_lds(inv ? reinterpret_cast<const void*>(k_col_fft<true>)
                                 : reinterpret_cast<const void*>(k_col_fft<false>),
                             160 * 1024, ldsSet[inv ? 1 : 0]));
    if (inv)
        hipLaunchKernelGGL(k_col_fft<true>, g, dim3(CF_THREADS), lds, s, C, vdim, logn, sAxis, sOuter,
                           nxh, p.tw);
    else
        hipLaunchKernelGGL(k_col_fft<false>, g, dim3(CF_THREADS), lds, s, C, vdim, logn, sAxis, sOuter,
                           nxh, p.tw);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

int c2r3d(const Plans& p, float2* C, float* rl, int vdim, hipStream_t s, int method = 0)
{
    if (!use_cols(p, method)) {
        THX_FFT(hipfftExecC2R(p.c2r, reinterpret_cast<hipfftComplex*>(C), rl));
        return THX_OK;
    }
    int st = col_pass(p, C, vdim, true, true, s);
    if (st == THX_OK) st = col_pass(p, C, vdim, true, false, s);
    if (st != THX_OK) return st;
    THX_FFT(hipfftExecC2R(p.c2rX, reinterpret_cast<hipfftComplex*>(C), rl));
    return THX_OK;
}

int r2c3d(const Plans& p, float* rl, float2* C, int vdim, hipStream_t s, int method = 0)
{
    if (!use_cols(p, method)) {
        THX_FFT(hipfftExecR2C(p.r2c, rl, reinterpret_cast<hipfftComplex*>(C)));
        return THX_OK;
    }
    THX_FFT(hipfftExecR2C(p.r2cX, rl, reinterpret_cast<hipfftComplex*>(C)));
    int st = col_pass(p, C, vdim, false, false, s);
    if (st == THX_OK) st = col_pass(p, C, vdim, false, true, s);
    return st;
}

// Plans per (device, vdim, N, stream), made once: creating a 512^3 hipFFT
// plan costs hundreds of ms, the transforms themselves ~0.6 ms.  A plan binds
// one stream and work area, so every stream has its own; calls on one stream
// take its entry's mutex (host threads sharing a stream), calls on different
// streams -- the two hemispheres, several GPUs -- run concurrently.  The
// cache's own mutex covers only the lookup.
struct PlanEntry {
    std::mutex mu;
    Plans p;
    bool made = false;
    unsigned* bits = nullptr;   // pinned host word: the balancing loop's read-back
};

struct PlanCache {
    std::mutex mu;
    std::map<std::tuple<int, int, int, hipStream_t>, std::unique_ptr<PlanEntry>> plans;
};

PlanCache& plan_cache()
{
    static PlanCache* c = new PlanCache;    // never destroyed: no teardown ordering at exit
    return *c;
}

// the entry for (current device, vdim, N, s), its plans made; returned locked
int cached_plans(int vdim, int N, hipStream_t s, PlanEntry** out,
                 std::unique_lock<std::mutex>& lock)
{
    int dev = 0;
    THX_HIP(hipGetDevice(&dev));
    PlanCache& c = plan_cache();
    PlanEntry* e = nullptr;
    {
        std::lock_guard<std::mutex> lk(c.mu);
        auto& slot = c.plans[std::make_tuple(dev, vdim, N, s)];
        if (!slot) slot.reset(new PlanEntry);
        e = slot.get();
    }
    lock = std::unique_lock<std::mutex>(e->mu);
    if (!e->made) {
        const int st = make_plans(e->p, vdim, N);
        if (st != THX_OK) return st;
        THX_HIP(hipHostMalloc(reinterpret_cast<void**>(&e->bits), sizeof(unsigned), 0));
        e->made = true;
    }
    *out = e;
    return THX_OK;
}

// the tabulated real-space kernel per (a, alpha), computed once (1e5 Bessel
// evaluations) under its own lock
const std::vector<float>& kernel_table(float a, float alpha)
{
    static std::mutex mu;
    static std::map<std::pair<float, float>, std::vector<float>>* tabs =
        new std::map<std::pair<float, float>, std::vector<float>>;
    std::lock_guard<std::mutex> lk(mu);
    std::vector<float>& t = (*tabs)[std::make_pair(a, alpha)];
    if (t.empty()) {
        t.resize(TAB_N + 1);
        for (int q = 0; q <= TAB_N; q++) t[q] = (float)mkb_rl_r2(q * 1e-5, a, alpha);
    }
    return t;
}

}  // namespace

extern "C" size_t thx_reconstruct_workspace(int N, int pf)
{
    if (N <= 0 || pf <= 0) return 0;
    const int vdim = N * pf;
    size_t work = 0;
    {
        std::unique_lock<std::mutex> lk;
        PlanEntry* e = nullptr;
        if (cached_plans(vdim, N, nullptr, &e, lk) != THX_OK) return 0;
        work = e->p.work;
    }
    thx::Carver k(nullptr, ~size_t(0));
    const size_t dimSize = (size_t)(vdim / 2 + 1) * vdim * vdim;
    k.take<float>(dimSize);                       // W
    k.take<float2>(dimSize);                      // C / pad
    k.take<float>((size_t)vdim * vdim * vdim);    // real space
    k.take<float>(TAB_N + 1);                     // kernel table
    k.take<float>((size_t)(vdim / 2 + 1) * (vdim / 2 + 1) * (vdim / 2 + 1));   // kernel octant
    k.take<unsigned>(64);                         // diff
    k.take<char>(work);                           // hipFFT work area
    return k.off + 256;
}

extern "C" int thx_reconstruct(const float* F, float* T, int N, int pf, float a, float alpha,
                               int gridCorr, int maxRadius, int map, const double* fsc, int nFsc,
                               int joinHalf, float* dst, float* dstFT, int* nIter, float* diffOut,
                               void* workspace, size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(F && T && dst && N > 0 && N % 2 == 0 && pf > 0 && a > 0 && alpha > 0,
                  "thx_reconstruct: bad arguments");
    THX_CHECK_ARG(!map || (fsc && nFsc > 0), "thx_reconstruct: MAP needs the FSC");
    const int vdim = N * pf;
    const int maxR = maxRadius > 0 ? maxRadius : N / 2 - (int)std::ceil(a);   // Reconstructor::init
    THX_CHECK_ARG(maxR > 0 && maxR <= N / 2, "thx_reconstruct: bad maxRadius");
    const size_t need = thx_reconstruct_workspace(N, pf);
    THX_CHECK_ARG(need > 0 && workspace && wsBytes >= need, "thx_reconstruct: workspace too small");
    hipStream_t s = thx::as_stream(stream);
    std::unique_lock<std::mutex> lk;     // this stream's plans, held for the solve
    PlanEntry* pe = nullptr;
    {
        const int st = cached_plans(vdim, N, s, &pe, lk);
        if (st != THX_OK) return st;
    }
    Plans& pl = pe->p;
    const size_t work = pl.work;
    const size_t dimSize = (size_t)(vdim / 2 + 1) * vdim * vdim;
    thx::Carver k(workspace, wsBytes);
    float* W = k.take<float>(dimSize);
    float2* C = k.take<float2>(dimSize);
    float* rl = k.take<float>((size_t)vdim * vdim * vdim);
    float* tab = k.take<float>(TAB_N + 1);
    float* oct = k.take<float>((size_t)(vdim / 2 + 1) * (vdim / 2 + 1) * (vdim / 2 + 1));
    unsigned* diff = k.take<unsigned>(64);
    void* fftWork = k.take<char>(work);
    THX_FFT(hipfftSetWorkArea(pl.c2r, fftWork));
    THX_FFT(hipfftSetWorkArea(pl.r2c, fftWork));
    THX_FFT(hipfftSetStream(pl.c2r, s));
    THX_FFT(hipfftSetStream(pl.r2c, s));
    if (pl.cols) {
        THX_FFT(hipfftSetWorkArea(pl.c2rX, fftWork));
        THX_FFT(hipfftSetWorkArea(pl.r2cX, fftWork));
        THX_FFT(hipfftSetStream(pl.c2rX, s));
        THX_FFT(hipfftSetStream(pl.r2cX, s));
    }
    if (dstFT) {
        THX_FFT(hipfftSetWorkArea(pl.r2cN, fftWork));
        THX_FFT(hipfftSetStream(pl.r2cN, s));
    }
    // the tabulated real-space kernel (float, as the reference's RFLOAT table)
    const std::vector<float>& htab = kernel_table(a, alpha);
    const float nf = (float)mkb_rl_r2(0.0, a, alpha);   // MKB_RL(0, a, alpha)
    THX_HIP(hipMemcpyAsync(tab, htab.data(), sizeof(float) * (TAB_N + 1), hipMemcpyHostToDevice, s));

    const long r2 = (long)maxR * pf * maxR * pf;
    const long nFT = (long)dimSize;
    const float scaleBw = 1.f / ((float)vdim * vdim * vdim);
    const dim3 g(4096), b(256);
    if (map) {
        hipLaunchKernelGGL(k_wiener, g, b, 0, s, T, vdim, pf, maxR, fsc, nFsc, joinHalf);
        THX_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_init_w, g, b, 0, s, W, T, vdim, r2);
    THX_LAUNCH_CHECK();
    int m = 0;
    float diffC = 0.f;
    if (gridCorr) {
        float diffPrev = 3.4e38f;
        diffC = 3.4e38f;
        int nNoDec = 0;
        const dim3 gSlab(RB_SPLIT, vdim), bSlab(RB_THREADS);
        const unsigned mVdim = magic_u((unsigned)vdim), mNc = magic_u((unsigned)(vdim / 2 + 1));
        hipLaunchKernelGGL(k_kernel_octant, g, b, 0, s, oct, vdim, tab, nf, scaleBw);
        THX_LAUNCH_CHECK();
        // the even half-grid loop where its transforms exist, else two hipFFT
        // 3D transforms per iteration
        const bool even = even_ok(vdim) && pl.tw;
        if (even) {
            hipLaunchKernelGGL(k_sym_planes, g, b, 0, s, T, vdim);
            THX_LAUNCH_CHECK();
            THX_RET(even_iteration(vdim, C, W, T, oct, r2, diff, pl.tw, true, false, s));
        } else {
            hipLaunchKernelGGL(k_c_from_tw, g, b, 0, s, C, T, W, nFT);
            THX_LAUNCH_CHECK();
        }
        unsigned* bits = pe->bits;   // the entry's pinned word (no allocation per solve)
        for (m = 0; m < 30; m++) {                                // MAX_N_ITER_BALANCE
            if (even) {
                THX_HIP(hipMemsetAsync(diff, 0, sizeof(unsigned), s));
                THX_RET(even_iteration(vdim, C, W, T, oct, r2, diff, pl.tw, false, true, s));
            } else {
                THX_RET(c2r3d(pl, C, rl, vdim, s));
                hipLaunchKernelGGL(k_kernel_mul, gSlab, bSlab, 0, s, rl, vdim, oct, mVdim);
                THX_LAUNCH_CHECK();
                THX_RET(r2c3d(pl, rl, C, vdim, s));
                THX_HIP(hipMemsetAsync(diff, 0, sizeof(unsigned), s));
                // W update + the next iteration's C in one pass
                hipLaunchKernelGGL(k_update_w, gSlab, bSlab, 0, s, W, C, T, vdim, r2, mNc, diff);
                THX_LAUNCH_CHECK();
            }
            THX_HIP(hipMemcpyAsync(bits, diff, sizeof(unsigned), hipMemcpyDeviceToHost, s));
            THX_HIP(hipStreamSynchronize(s));
            diffPrev = diffC;
            diffC = __builtin_bit_cast(float, *bits);
            if (diffOut) diffOut[m] = diffC;
            if ((double)diffC > (double)diffPrev * 0.95) nNoDec += 1;   // DIFF_C_DECREASE_THRES (double)
            else nNoDec = 0;
            if ((double)diffC < 1e-2 || (m >= 10 && nNoDec == 2)) {  // DIFF_C_THRES, MIN_N_ITER, N_DIFF_C_NO_DECREASE
                m++;
                break;
            }
        }
    } else {
        hipLaunchKernelGGL(k_w_from_t, g, b, 0, s, W, T, vdim, r2);
        THX_LAUNCH_CHECK();
    }
    if (nIter) *nIter = m;
    // F W -> real space -> central box, kernel-corrected
    hipLaunchKernelGGL(k_pad, g, b, 0, s, C, reinterpret_cast<const float2*>(F), W, vdim, r2);
    THX_LAUNCH_CHECK();
    THX_RET(c2r3d(pl, C, rl, vdim, s));
    hipLaunchKernelGGL(k_extract, g, b, 0, s, dst, rl, N, vdim, scaleBw);
    THX_LAUNCH_CHECK();
    if (dstFT) {
        // the map's transform for the FSC (fft.fw(ref), src/Optimiser.cpp:7379)
        THX_FFT(hipfftExecR2C(pl.r2cN, dst, reinterpret_cast<hipfftComplex*>(dstFT)));
    }
    // the plans are shared: finish before another call rebinds their stream
    THX_HIP(hipStreamSynchronize(s));
    return THX_OK;
}

// FFT::fw / FFT::bw of a volume (src/FFT.cpp, unnormalised r2c / c2r of
// box vdim): rl [vdim^3] real, C [vdim][vdim][vdim/2+1] complex; inverse 1
// overwrites C.  method 0: the reconstruction's choice, 1: hipFFT's 3D plans,
// 2: the column passes (error if vdim is not a power of two with an LDS tile).
extern "C" size_t thx_fft3d_workspace(int vdim)
{
    if (vdim <= 0 || vdim % 2) return 0;
    std::unique_lock<std::mutex> lk;
    PlanEntry* e = nullptr;
    if (cached_plans(vdim, vdim / 2, nullptr, &e, lk) != THX_OK) return 0;
    return e->p.work + 256;
}

extern "C" int thx_fft3d(float* C, float* rl, int vdim, int inverse, int method, void* workspace,
                         size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(C && rl && vdim > 0 && vdim % 2 == 0 && method >= 0 && method <= 2,
                  "thx_fft3d: bad arguments");
    hipStream_t s = thx::as_stream(stream);
    std::unique_lock<std::mutex> lk;
    PlanEntry* pe = nullptr;
    THX_RET(cached_plans(vdim, vdim / 2, s, &pe, lk));
    Plans& pl = pe->p;
    THX_CHECK_ARG(method != 2 || pl.cols, "thx_fft3d: no column passes for this vdim");
    THX_CHECK_ARG(workspace && wsBytes >= pl.work, "thx_fft3d: workspace too small");
    for (hipfftHandle h : {pl.c2r, pl.r2c, pl.c2rX, pl.r2cX}) {
        if (!h) continue;
        THX_FFT(hipfftSetWorkArea(h, workspace));
        THX_FFT(hipfftSetStream(h, s));
    }
    if (inverse)
        THX_RET(c2r3d(pl, reinterpret_cast<float2*>(C), rl, vdim, s, method));
    else
        THX_RET(r2c3d(pl, rl, reinterpret_cast<float2*>(C), vdim, s, method));
    THX_HIP(hipStreamSynchronize(s));      // the plans are shared across calls on this stream
    return THX_OK;
}

// ------------------------------------------------------------------ MODE_2D
// The 2D branches of Reconstructor::reconstruct (src/Reconstructor.cpp:
// 1136-1589, 1669-1818; GPU twin reconstructG's ExposePT2D / ExposeWT2D /
// ExposePF2D / ExposeCorrF2D) for nK class images at once: the same MAP
// factor on rings, W = 1 in the disc |k| < maxR pf, T = max(T, 1e-25), the
// MKB balancing (convoluteC's 2D branch: kernelRL(QUAD(i, j) / (N pf)^2) /
// nf, checkC's max, the same stopping rule per class -- OPTIMISER_2D_GRID_CORR
// is on in include/Config.h:206), or W = 1 / max(|T|, 1e-6); pad = F W ->
// FFT::bw (1 / vdim^2) -> the central N^2 (IMG_EXTRACT_RL) / TIK_RL(|r| /
// (pf N)).  Layouts: F / T [nK][vdim][vdim/2+1] (Image FT, i fastest, rows
// wrapped); dst [nK][N][N] real space, origin at [0][0], negatives wrapped.
namespace {

THX_DEV void ft2_coord(long q, int vdim, int& k, int& i, int& j)
{
    const int nc = vdim / 2 + 1;
    const long per = (long)nc * vdim;
    k = (int)(q / per);
    const long r = q - (long)k * per;
    i = (int)(r % nc);
    j = (int)(r / nc);
    if (j >= vdim / 2) j -= vdim;
}

__global__ void k2_prep(float* __restrict__ T, float* __restrict__ W, int vdim, int nK, long r2,
                        int map, int pf, int maxR, const double* __restrict__ fsc, int nFsc,
                        int joinHalf)
{
    const long n = (long)nK * (vdim / 2 + 1) * vdim;
    const long lo = (long)5 * pf * 5 * pf;                 // WIENER_FACTOR_MIN_R
    GRID_STRIDE(q, n)
    {
        int k, i, j;
        ft2_coord(q, vdim, k, i, j);
        const long quad = (long)i * i + (long)j * j;
        float t = T[q];
        if (map && quad >= lo && quad < r2) {
            const int u = (int)rintf(sqrtf((float)quad));   // AROUND(NORM(i, j))
            float f = (u / pf >= nFsc) ? 0.f : (float)fsc[(size_t)k * nFsc + u / pf];
            f = fmaxf(1e-3f, fminf(1.f - 1e-3f, f));        // FSC_BASE_L / _H
            if (joinHalf) f = sqrtf(2.f * f / (1.f + f));
            t = t / f;
        }
        t = fmaxf(t, 1e-25f);
        T[q] = t;
        W[q] = quad < r2 ? 1.f : 0.f;
    }
}

__global__ void k2_w_from_t(float* __restrict__ W, const float* __restrict__ T, int vdim, int nK,
                            long r2)
{
    const long n = (long)nK * (vdim / 2 + 1) * vdim;
    GRID_STRIDE(q, n)
    {
        int k, i, j;
        ft2_coord(q, vdim, k, i, j);
        if ((long)i * i + (long)j * j < r2) W[q] = 1.f / fmaxf(fabsf(T[q]), 1e-6f);
    }
}

__global__ void k2_c_from_tw(float2* __restrict__ C, const float* __restrict__ T,
                             const float* __restrict__ W, long n)
{
    GRID_STRIDE(q, n) C[q] = make_float2(T[q] * W[q], 0.f);
}

// real space [nK][vdim][vdim]: c *= kernelRL(QUAD(i, j) / vdim^2) / nf / vdim^2
__global__ void k2_kernel_mul(float* __restrict__ c, int vdim, int nK, const float* __restrict__ tab,
                              float nf, float scale)
{
    const long n = (long)nK * vdim * vdim;
    const float inv = 1.f / ((float)vdim * (float)vdim);
    GRID_STRIDE(q, n)
    {
        const long r = q % ((long)vdim * vdim);
        int i = (int)(r % vdim), j = (int)(r / vdim);
        if (i > vdim / 2) i -= vdim;
        if (j > vdim / 2) j -= vdim;
        const float x = (float)(i * i + j * j) * inv;
        const int t = min(TAB_N, (int)rintf(x / 1e-5f));
        c[q] *= scale * tab[t] / nf;
    }
}

// W /= max(|C|, 1e-6) inside the disc for the classes still balancing; their
// max | |C| - 1 |; the next C = T W
__global__ void k2_update_w(float* __restrict__ W, float2* __restrict__ C, const float* __restrict__ T,
                            int vdim, int nK, long r2, const int* __restrict__ active,
                            unsigned* __restrict__ diffBits)
{
    const int k = blockIdx.y;
    if (!active[k]) return;
    const int nc = vdim / 2 + 1;
    const long per = (long)nc * vdim;
    float dmax = 0.f;
    for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < per; r += (long)gridDim.x * blockDim.x) {
        const long e = (long)k * per + r;
        const int i = (int)(r % nc);
        int j = (int)(r / nc);
        if (j >= vdim / 2) j -= vdim;
        float w = W[e];
        if ((long)i * i + (long)j * j < r2) {
            const float2 cv = C[e];
            const float a = sqrtf(cv.x * cv.x + cv.y * cv.y);
            w = w / fmaxf(a, 1e-6f);
            W[e] = w;
            dmax = fmaxf(dmax, fabsf(a - 1.f));
        }
        C[e] = make_float2(T[e] * w, 0.f);
    }
    dmax = wave_max(dmax);
    __shared__ float sm[4];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = dmax;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float m = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
        if (m > 0.f) atomicMax(diffBits + k, __float_as_uint(m));
    }
}

__global__ void k2_pad(float2* __restrict__ P, const float2* __restrict__ F, const float* __restrict__ W,
                       int vdim, int nK, long r2)
{
    const long n = (long)nK * (vdim / 2 + 1) * vdim;
    GRID_STRIDE(q, n)
    {
        int k, i, j;
        ft2_coord(q, vdim, k, i, j);
        const float2 f = F[q];
        const float w = W[q];
        P[q] = ((long)i * i + (long)j * j < r2) ? make_float2(f.x * w, f.y * w) : make_float2(0.f, 0.f);
    }
}

__global__ void k2_extract(float* __restrict__ dst, const float* __restrict__ src, int N, int vdim,
                           int nK, float scale)
{
    const long n = (long)nK * N * N;
    GRID_STRIDE(q, n)
    {
        const int k = (int)(q / ((long)N * N));
        const long r = q - (long)k * N * N;
        int i = (int)(r % N), j = (int)(r / N);
        if (i >= N / 2) i -= N;
        if (j >= N / 2) j -= N;
        const long s = (long)k * vdim * vdim + (long)wrap_idx(j, vdim) * vdim + wrap_idx(i, vdim);
        const float x = (float)M_PI * sqrtf((float)(i * i + j * j)) / (float)vdim;
        const float j0 = x == 0.f ? 1.f : sinf(x) / x;
        dst[q] = src[s] * scale / (j0 * j0);              // / TIK_RL
    }
}

// per-class normalisation 1 / T_k[0] (RECONSTRUCTOR_NORMALISE_T_F, MODE_2D)
__global__ void k2_normalise(float* __restrict__ F, float* __restrict__ T, int vdim, int nK)
{
    const long per = (long)(vdim / 2 + 1) * vdim;
    const int k = blockIdx.y;
    const float sf = 1.f / T[(size_t)k * per];   // element 0 is scaled last (k2_normalise_first)
    for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < per; r += (long)gridDim.x * blockDim.x) {
        const size_t e = (size_t)k * per + r;
        if (r == 0) continue;
        T[e] *= sf;
        float2* f = reinterpret_cast<float2*>(F) + e;
        *f = make_float2(f->x * sf, f->y * sf);
    }
}

__global__ void k2_normalise_first(float* __restrict__ F, float* __restrict__ T, int vdim, int nK)
{
    const long per = (long)(vdim / 2 + 1) * vdim;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nK) return;
    const size_t e = (size_t)k * per;
    const float sf = 1.f / T[e];
    T[e] *= sf;
    float2* f = reinterpret_cast<float2*>(F) + e;
    *f = make_float2(f->x * sf, f->y * sf);
}

struct Plans2 {
    hipfftHandle c2r = 0, r2c = 0;
};

int plans2d(int vdim, int nK, hipStream_t s, Plans2** out, std::unique_lock<std::mutex>& lock)
{
    static std::mutex mu;
    static std::map<std::tuple<int, int, int, hipStream_t>, std::unique_ptr<std::pair<std::mutex, Plans2>>>*
        cache = new std::map<std::tuple<int, int, int, hipStream_t>,
                             std::unique_ptr<std::pair<std::mutex, Plans2>>>;
    int dev = 0;
    THX_HIP(hipGetDevice(&dev));
    std::pair<std::mutex, Plans2>* e = nullptr;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto& slot = (*cache)[std::make_tuple(dev, vdim, nK, s)];
        if (!slot) slot.reset(new std::pair<std::mutex, Plans2>());
        e = slot.get();
    }
    lock = std::unique_lock<std::mutex>(e->first);
    Plans2& p = e->second;
    if (!p.c2r) {
        int n[2] = {vdim, vdim};
        THX_FFT(hipfftPlanMany(&p.c2r, 2, n, nullptr, 1, 0, nullptr, 1, 0, HIPFFT_C2R, nK));
        THX_FFT(hipfftPlanMany(&p.r2c, 2, n, nullptr, 1, 0, nullptr, 1, 0, HIPFFT_R2C, nK));
    }
    THX_FFT(hipfftSetStream(p.c2r, s));
    THX_FFT(hipfftSetStream(p.r2c, s));
    *out = &p;
    return THX_OK;
}

}  // namespace

extern "C" int thx_prepare_tf2d(float* F, float* T, int vdim, int nK, thx_stream_t stream)
{
    THX_CHECK_ARG(F && T && vdim > 0 && vdim % 2 == 0 && nK > 0, "thx_prepare_tf2d: bad arguments");
    hipStream_t s = thx::as_stream(stream);
    const long per = (long)(vdim / 2 + 1) * vdim;
    hipLaunchKernelGGL(k2_normalise, dim3((unsigned)std::min<long>(thx::cdiv(per, 256), 1024), nK),
                       dim3(256), 0, s, F, T, vdim, nK);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k2_normalise_first, dim3(thx::cdiv(nK, 64)), dim3(64), 0, s, F, T, vdim, nK);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" size_t thx_reconstruct2d_workspace(int N, int pf, int nK)
{
    if (N <= 0 || pf <= 0 || nK <= 0) return 0;
    const int vdim = N * pf;
    const size_t img = (size_t)(vdim / 2 + 1) * vdim * nK;
    thx::Carver k(nullptr, ~size_t(0));
    k.take<float>(img);                              // W
    k.take<float2>(img);                             // C / pad
    k.take<float>((size_t)vdim * vdim * nK);         // real space
    k.take<float>(TAB_N + 1);                        // kernel table
    k.take<unsigned>(nK);                            // diffs
    k.take<int>(nK);                                 // active classes
    return k.off + 256;
}

extern "C" int thx_reconstruct2d(const float* F, float* T, int nK, int N, int pf, float a,
                                 float alpha, int gridCorr, int maxRadius, const double* fsc,
                                 int nFsc, int joinHalf, float* dst, int* nIter, void* workspace,
                                 size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(F && T && dst && nK > 0 && N > 0 && N % 2 == 0 && pf > 0 && a > 0 && alpha > 0,
                  "thx_reconstruct2d: bad arguments");
    THX_CHECK_ARG(!fsc || nFsc > 0, "thx_reconstruct2d: fsc needs nFsc");
    const int vdim = N * pf;
    const int maxR = maxRadius > 0 ? maxRadius : N / 2 - (int)std::ceil(a);
    THX_CHECK_ARG(maxR > 0 && maxR <= N / 2, "thx_reconstruct2d: bad maxRadius");
    THX_CHECK_ARG(workspace && wsBytes >= thx_reconstruct2d_workspace(N, pf, nK),
                  "thx_reconstruct2d: workspace too small");
    hipStream_t s = thx::as_stream(stream);
    const size_t img = (size_t)(vdim / 2 + 1) * vdim * nK;
    thx::Carver k(workspace, wsBytes);
    float* W = k.take<float>(img);
    float2* C = k.take<float2>(img);
    float* rl = k.take<float>((size_t)vdim * vdim * nK);
    float* tab = k.take<float>(TAB_N + 1);
    unsigned* diff = k.take<unsigned>(nK);
    int* active = k.take<int>(nK);
    std::unique_lock<std::mutex> lk;
    Plans2* pl = nullptr;
    THX_RET(plans2d(vdim, nK, s, &pl, lk));
    const long r2 = (long)maxR * pf * maxR * pf;
    const float scaleBw = 1.f / ((float)vdim * vdim);
    const dim3 g(1024), b(256);
    hipLaunchKernelGGL(k2_prep, g, b, 0, s, T, W, vdim, nK, r2, fsc ? 1 : 0, pf, maxR, fsc, nFsc,
                       joinHalf);
    THX_LAUNCH_CHECK();
    std::vector<int> iters(nK, 0);
    if (gridCorr) {
        const std::vector<float>& htab = kernel_table(a, alpha);
        const float nf = (float)mkb_rl_r2(0.0, a, alpha);
        THX_HIP(hipMemcpyAsync(tab, htab.data(), sizeof(float) * (TAB_N + 1), hipMemcpyHostToDevice, s));
        std::vector<int> act(nK, 1), nNoDec(nK, 0);
        std::vector<float> diffC(nK, 3.4e38f), prev(nK, 3.4e38f);
        std::vector<unsigned> bits(nK);
        THX_HIP(hipMemcpyAsync(active, act.data(), sizeof(int) * nK, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k2_c_from_tw, g, b, 0, s, C, T, W, (long)img);
        THX_LAUNCH_CHECK();
        for (int m = 0; m < 30; m++) {                                  // MAX_N_ITER_BALANCE
            THX_FFT(hipfftExecC2R(pl->c2r, reinterpret_cast<hipfftComplex*>(C), rl));
            hipLaunchKernelGGL(k2_kernel_mul, g, b, 0, s, rl, vdim, nK, tab, nf, scaleBw);
            THX_LAUNCH_CHECK();
            THX_FFT(hipfftExecR2C(pl->r2c, rl, reinterpret_cast<hipfftComplex*>(C)));
            THX_HIP(hipMemsetAsync(diff, 0, sizeof(unsigned) * nK, s));
            hipLaunchKernelGGL(k2_update_w, dim3(16, nK), dim3(256), 0, s, W, C, T, vdim, nK, r2,
                               active, diff);
            THX_LAUNCH_CHECK();
            THX_HIP(hipMemcpyAsync(bits.data(), diff, sizeof(unsigned) * nK, hipMemcpyDeviceToHost, s));
            THX_HIP(hipStreamSynchronize(s));
            bool any = false;
            for (int c = 0; c < nK; c++) {
                if (!act[c]) continue;
                prev[c] = diffC[c];
                diffC[c] = __builtin_bit_cast(float, bits[c]);
                iters[c] = m + 1;
                if ((double)diffC[c] > (double)prev[c] * 0.95) nNoDec[c] += 1;   // DIFF_C_DECREASE_THRES (double)
                else nNoDec[c] = 0;
                if ((double)diffC[c] < 1e-2 || (m >= 10 && nNoDec[c] == 2)) act[c] = 0;
                any = any || act[c];
            }
            if (!any) break;
            THX_HIP(hipMemcpyAsync(active, act.data(), sizeof(int) * nK, hipMemcpyHostToDevice, s));
        }
    } else {
        hipLaunchKernelGGL(k2_w_from_t, g, b, 0, s, W, T, vdim, nK, r2);
        THX_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k2_pad, g, b, 0, s, C, reinterpret_cast<const float2*>(F), W, vdim, nK, r2);
    THX_LAUNCH_CHECK();
    THX_FFT(hipfftExecC2R(pl->c2r, reinterpret_cast<hipfftComplex*>(C), rl));
    hipLaunchKernelGGL(k2_extract, g, b, 0, s, dst, rl, N, vdim, nK, scaleBw);
    THX_LAUNCH_CHECK();
    if (nIter)
        for (int c = 0; c < nK; c++) nIter[c] = iters[c];
    THX_HIP(hipStreamSynchronize(s));      // the plans are shared across calls on this stream
    return THX_OK;
}
