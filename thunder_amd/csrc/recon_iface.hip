// recon_iface.hip -- the reconstruction / preprocessing half of the
// reference's plugin surface, gpu/interface/Interface.h:320-528, as host
// adapters over device kernels (caller owns the host arrays; each call
// allocates, copies, runs and copies back, as the cuthunder bodies do):
//
//   thx_PrepareTF            PrepareTF        (cuthunder.cu:6176)
//   thx_ExposePT / PT2D      ExposePT / 2D    (CalculateT :6647 / :6526)
//   thx_ExposeWT / WT2D      ExposeWT / 2D with the kernel table (CalculateW
//                            :7737, CalculateW2D :7015): the balancing loop
//   thx_ExposeWT_T / WT2D_T  ExposeWT / 2D without it (:8072 / :8018)
//   thx_AllocDevicePoint, thx_HostDeviceInit, thx_ExposeC, thx_ExposeForConvC,
//   thx_ExposeWC, thx_FreeDevHostPoint
//                            the split-step balancing Reconstructor::
//                            reconstructG drives with host FFTs in between
//                            (src/Reconstructor.cpp:1985-2087; cuthunder.cu:
//                            7280-7735)
//   thx_ExposePFW / PF / PF2D  CalculateFW :8496 / CalculateF :8619 / 2D :8386
//   thx_ExposeCorrF / CorrFT / CorrF2D  CorrSoftMaskF :8945 / :9074 / 2D :8827
//   thx_TranslateI / 2D      TranslateI :9319 / TranslateI2D :9235
//   thx_ReMask               reMask :9406 (thx_remask per device)
//   thx_GCTFinit             GCTF :9641 (thx_ctf_image per device)
//
// The arithmetic follows the cuthunder kernels (gpu/src/Kernel.cu) where it
// differs from the CPU Reconstructor in rounding: the kernel-table index
// rintf(((float)quad / (padSize^2)) / step), |C| by the scaled hypot of
// kernel_RecalculateW, the convolution's divide-by-size before the table
// factor, the translation phase (RFLOAT)(PI_2 * float sum).  The in-product
// solve is thx_reconstruct / thx_reconstruct2d (device-resident, fused
// passes); these adapters exist so THUNDER's Interface.cpp can forward to
// the library with src/ unchanged.
//
// Layouts: half-complex arrays [k][j][i] of (dim/2+1) x dim (x dim) with j, k
// wrapped (Volume / Image FT = hipFFT R2C), real-space arrays [k][j][i] with
// the origin at index 0 (Volume / Image RL).  2D calls are the nz = 1 case.
#include <hipfft/hipfft.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "adapter.h"

#define THX_FFT(call)                                                          \
    do {                                                                       \
        hipfftResult r_ = (call);                                              \
        if (r_ != HIPFFT_SUCCESS) {                                            \
            ::thx::set_error("%s:%d %s: hipfft error %d", __FILE__, __LINE__, \
                             #call, (int)r_);                                  \
            return THX_ERR_HIP;                                                \
        }                                                                      \
    } while (0)

using thx::DBuf;
using thx::DeviceGuard;

namespace {

constexpr double PI_2_REF = 6.28318530717959;   // PI_2 (gpu/include/acc/Constructor.cuh:35)
// double, as the reference's macros: float diffC is promoted before the compare
constexpr double DIFF_C_THRES = 1e-2, DIFF_C_DECREASE_THRES = 0.95;   // include/Reconstructor.h:65-69
constexpr int N_DIFF_C_NO_DECREASE = 2;

#define GRID_STRIDE(q, n) \
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < (n); q += (long)gridDim.x * blockDim.x)

inline unsigned grid_for(long n) { return (unsigned)std::min<long>(thx::cdiv(n, 256), 65536L); }

// (i, j, k) of half-complex index q of a (dim/2+1) x dim x nz grid
THX_DEV void hc_coord(long q, int dim, int& i, int& j, int& k)
{
    const int nc = dim / 2 + 1;
    i = (int)(q % nc);
    const long r = q / nc;
    j = (int)(r % dim);
    k = (int)(r / dim);
    if (j >= dim / 2) j -= dim;
    if (k >= dim / 2) k -= dim;
}

// |z| as kernel_RecalculateW / kernel_CheckCMAX compute it
THX_DEV float mode_of(float2 c)
{
    const float x = fabsf(c.x), y = fabsf(c.y);
    if (x < y) {
        if (x == 0.f) return y;
        const float u = x / y;
        return y * sqrtf(1.f + u * u);
    }
    if (y == 0.f) return x;
    const float u = y / x;
    return x * sqrtf(1.f + u * u);
}

// symmetrizeT's closing clamp (gpu/src/acc/Constructor.cu:547-598)
__global__ void k_clamp_t(float* __restrict__ T, long n)
{
    GRID_STRIDE(q, n) T[q] = fmaxf(T[q], 1e-25f);
}

// kernel_CalculateFSC / 2D (Kernel.cu:3538-3690): T /= FSC' on wiener <= quad
// < r, then T = max(T, 1e-25) everywhere
__global__ void k_fsc_t(float* __restrict__ T, long n, int dim, const float* __restrict__ fsc,
                        int nFsc, int joinHalf, int wiener, int r, int pf)
{
    GRID_STRIDE(q, n)
    {
        int i, j, k;
        hc_coord(q, dim, i, j, k);
        const int quad = i * i + j * j + k * k;
        float t = T[q];
        if (quad >= wiener && quad < r) {
            const int u = (int)rintf(sqrtf((float)quad));
            float f = (u / pf >= nFsc) ? 0.f : fsc[u / pf];
            f = fmaxf(1e-3f, fminf(1.f - 1e-3f, f));
            if (joinHalf) f = sqrtf(2.f * f / (1.f + f));
            t /= f;
        }
        T[q] = fmaxf(t, 1e-25f);
    }
}

// kernel_InitialW: 1 inside quad < r, 0 outside
__global__ void k_w_init(float* __restrict__ W, long n, int dim, int r)
{
    GRID_STRIDE(q, n)
    {
        int i, j, k;
        hc_coord(q, dim, i, j, k);
        W[q] = (i * i + j * j + k * k < r) ? 1.f : 0.f;
    }
}

// kernel_CalculateW: W = 1 / max(|T|, 1e-6) inside, untouched outside
__global__ void k_w_from_t(float* __restrict__ W, const float* __restrict__ T, long n, int dim, int r)
{
    GRID_STRIDE(q, n)
    {
        int i, j, k;
        hc_coord(q, dim, i, j, k);
        if (i * i + j * j + k * k < r) W[q] = 1.f / fmaxf(fabsf(T[q]), 1e-6f);
    }
}

// kernel_DeterminingC: C = (T W, 0)
__global__ void k_c_tw(float2* __restrict__ C, const float* __restrict__ T, const float* __restrict__ W,
                       long n)
{
    GRID_STRIDE(q, n) C[q] = make_float2(T[q] * W[q], 0.f);
}

// kernel_convoluteC(2D) / kernel_ConvoluteC over a dim x dim x nz real grid:
// c (/ dimSize when divSize) * kernelRL((float)|r|^2 / padSize^2) / nf
__global__ void k_conv_c(float* __restrict__ c, long n, int dim, const float* __restrict__ tab,
                         float step, int tabSize, float nf, int padSize, int divSize)
{
    const float p2 = (float)(padSize * padSize);
    GRID_STRIDE(q, n)
    {
        int i = (int)(q % dim);
        const long r = q / dim;
        int j = (int)(r % dim), k = (int)(r / dim);
        if (i >= dim / 2) i -= dim;
        if (j >= dim / 2) j -= dim;
        if (k >= dim / 2) k -= dim;
        const float x = (float)(i * i + j * j + k * k) / p2;
        int t = (int)rintf(x / step);
        t = t < 0 ? 0 : (t >= tabSize ? tabSize - 1 : t);
        float v = c[q];
        if (divSize) v = v / (float)n;
        c[q] = v * tab[t] / nf;
    }
}

// kernel_RecalculateW + kernel_CheckCMAX: W /= max(|C|, 1e-6) inside; the
// max | |C| - 1 | inside into diffBits (non-negative floats order as bits)
__global__ void __launch_bounds__(256) k_update_w(float* __restrict__ W, const float2* __restrict__ C,
                                                  long n, int dim, int r, unsigned* __restrict__ diffBits)
{
    float dmax = 0.f;
    GRID_STRIDE(q, n)
    {
        int i, j, k;
        hc_coord(q, dim, i, j, k);
        if (i * i + j * j + k * k < r) {
            const float m = mode_of(C[q]);
            W[q] /= fmaxf(m, 1e-6f);
            dmax = fmaxf(dmax, fabsf(m - 1.f));
        }
    }
    dmax = wave_max(dmax);
    __shared__ float sm[4];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = dmax;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float m = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
        if (m > 0.f) atomicMax(diffBits, __float_as_uint(m));
    }
}

// kernel_NormalizeFW(2D): the fdim grid's F W inside quad < r placed into the
// (zeroed) pdim grid, j and k re-wrapped
__global__ void k_pad_fw(float2* __restrict__ P, const float2* __restrict__ F, const float* __restrict__ W,
                         long n, int fdim, int pdim, int r)
{
    GRID_STRIDE(q, n)
    {
        int i, j, k;
        hc_coord(q, fdim, i, j, k);
        if (i * i + j * j + k * k >= r) continue;
        const int pj = j < 0 ? j + pdim : j;
        const int pk = k < 0 ? k + pdim : k;
        const float2 f = F[q];
        const float w = W[q];
        P[((size_t)pk * pdim + pj) * (pdim / 2 + 1) + i] = make_float2(f.x * w, f.y * w);
    }
}

// kernel_NormalizeP(2D): x /= size
__global__ void k_div(float* __restrict__ x, long n, float size)
{
    GRID_STRIDE(q, n) x[q] = x[q] / size;
}

// kernel_CorrectF(2D): x / table(|i|, |j|, |k|) [* nf with the MKB kernel],
// the table (dim/2+1)^nd with index folding dim - i for i >= dim / 2
__global__ void k_correct(float* __restrict__ x, long n, int dim, int nd, const float* __restrict__ tab,
                          float nf)
{
    const int h = dim / 2 + 1;
    GRID_STRIDE(q, n)
    {
        int i = (int)(q % dim);
        const long r = q / dim;
        int j = (int)(r % dim), k = nd == 3 ? (int)(r / dim) : 0;
        if (i >= dim / 2) i = dim - i;
        if (j >= dim / 2) j = dim - j;
        if (k >= dim / 2) k = dim - k;
        const float t = tab[((size_t)k * h + j) * h + i];
        x[q] = nf != 0.f ? x[q] / t * nf : x[q] / t;
    }
}

// kernel_TranslateI(2D): x exp(-i 2 pi (i ox + j oy + k oz) / dim) inside
// quad < r^2
__global__ void k_translate(float2* __restrict__ x, long n, int dim, float ox, float oy, float oz, int r)
{
    const float rc = ox / dim, rr = oy / dim, rs = oz / dim;
    GRID_STRIDE(q, n)
    {
        int i, j, k;
        hc_coord(q, dim, i, j, k);
        if (i * i + j * j + k * k >= r * r) continue;
        const float phase = (float)(PI_2_REF * (double)(i * rc + j * rr + k * rs));
        const float c = cosf(-phase), s = sinf(-phase);
        const float2 v = x[q];
        x[q] = make_float2(v.x * c - v.y * s, v.x * s + v.y * c);
    }
}

// one (Complex) CTF image per image from thx_ctf_image's real values
__global__ void k_real_to_complex(const float* __restrict__ re, float2* __restrict__ out, long n)
{
    GRID_STRIDE(q, n) out[q] = make_float2(re[q], 0.f);
}

// a 2D (nz == 1) or 3D hipFFT plan pair on the null stream
struct Fft {
    hipfftHandle c2r = 0, r2c = 0;
    ~Fft()
    {
        if (c2r) (void)hipfftDestroy(c2r);
        if (r2c) (void)hipfftDestroy(r2c);
    }
    int make(int dim, int nd, bool wantC2R, bool wantR2C)
    {
        if (nd == 3) {
            if (wantC2R) THX_FFT(hipfftPlan3d(&c2r, dim, dim, dim, HIPFFT_C2R));
            if (wantR2C) THX_FFT(hipfftPlan3d(&r2c, dim, dim, dim, HIPFFT_R2C));
        } else {
            if (wantC2R) THX_FFT(hipfftPlan2d(&c2r, dim, dim, HIPFFT_C2R));
            if (wantR2C) THX_FFT(hipfftPlan2d(&r2c, dim, dim, HIPFFT_R2C));
        }
        return THX_OK;
    }
};

inline long hc_size(int dim, int nd) { return (long)(dim / 2 + 1) * dim * (nd == 3 ? dim : 1); }
inline long rl_size(int dim, int nd) { return (long)dim * dim * (nd == 3 ? dim : 1); }

int to_dev(void* d, const void* h, size_t bytes)
{
    THX_HIP(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
    return THX_OK;
}

int to_host(void* h, const void* d, size_t bytes)
{
    THX_HIP(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
    return THX_OK;
}

int expose_pt(int gpuIdx, float* T, int maxRadius, int pf, int dim, int nd, const float* fsc,
              int nFsc, int joinHalf, int wienerF)
{
    THX_CHECK_ARG(T && (nFsc == 0 || fsc) && dim > 0 && dim % 2 == 0 && pf > 0 && nFsc >= 0,
                  "thx_ExposePT: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    const long n = hc_size(dim, nd);
    DBuf dT, dF;
    THX_DALLOC(dT, sizeof(float) * n);
    THX_DALLOC(dF, sizeof(float) * (nFsc > 0 ? nFsc : 1));
    THX_RET(to_dev(dT.p, T, sizeof(float) * n));
    if (nFsc > 0) THX_RET(to_dev(dF.p, fsc, sizeof(float) * nFsc));
    hipLaunchKernelGGL(k_fsc_t, dim3(grid_for(n)), dim3(256), 0, nullptr, dT.as<float>(), n, dim,
                       dF.as<float>(), nFsc, joinHalf, wienerF * pf * wienerF * pf,
                       maxRadius * pf * maxRadius * pf, pf);
    THX_LAUNCH_CHECK();
    return to_host(T, dT.p, sizeof(float) * n);
}

// CalculateW / CalculateW2D with the kernel table: the balancing loop on
// device, W (host) = the balanced weights; *nIter (optional) = iterations run
int expose_wt(int gpuIdx, const float* T, float* W, const float* tab, float step, int tabSize, float nf,
              int maxRadius, int pf, int dim, int nd, int maxIter, int minIter, int size, int* nIter)
{
    THX_CHECK_ARG(T && W && tab && tabSize > 0 && step > 0.f && nf != 0.f && dim > 0 && dim % 2 == 0 &&
                      pf > 0 && size > 0 && maxIter >= 0,
                  "thx_ExposeWT: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    const long n = hc_size(dim, nd), nr = rl_size(dim, nd);
    const int r = maxRadius * pf * maxRadius * pf, padSize = pf * size;
    DBuf dT, dW, dC, dR, dTab, dDiff;
    THX_DALLOC(dT, sizeof(float) * n);
    THX_DALLOC(dW, sizeof(float) * n);
    THX_DALLOC(dC, sizeof(float2) * n);
    THX_DALLOC(dR, sizeof(float) * nr);
    THX_DALLOC(dTab, sizeof(float) * tabSize);
    THX_DALLOC(dDiff, sizeof(unsigned));
    THX_RET(to_dev(dT.p, T, sizeof(float) * n));
    THX_RET(to_dev(dTab.p, tab, sizeof(float) * tabSize));
    Fft fft;
    THX_RET(fft.make(dim, nd, true, true));
    hipLaunchKernelGGL(k_w_init, dim3(grid_for(n)), dim3(256), 0, nullptr, dW.as<float>(), n, dim, r);
    THX_LAUNCH_CHECK();
    float diffC = 3.402823466e38f, diffCPrev;
    int m = 0, noDec = 0;
    for (m = 0; m < maxIter; m++) {
        hipLaunchKernelGGL(k_c_tw, dim3(grid_for(n)), dim3(256), 0, nullptr, dC.as<float2>(),
                           dT.as<float>(), dW.as<float>(), n);
        THX_LAUNCH_CHECK();
        THX_FFT(hipfftExecC2R(fft.c2r, dC.as<hipfftComplex>(), dR.as<float>()));
        hipLaunchKernelGGL(k_conv_c, dim3(grid_for(nr)), dim3(256), 0, nullptr, dR.as<float>(), nr, dim,
                           dTab.as<float>(), step, tabSize, nf, padSize, 1);
        THX_LAUNCH_CHECK();
        THX_FFT(hipfftExecR2C(fft.r2c, dR.as<float>(), dC.as<hipfftComplex>()));
        THX_HIP(hipMemset(dDiff.p, 0, sizeof(unsigned)));
        hipLaunchKernelGGL(k_update_w, dim3(std::min<unsigned>(grid_for(n), 2048u)), dim3(256), 0, nullptr,
                           dW.as<float>(), dC.as<float2>(), n, dim, r, dDiff.as<unsigned>());
        THX_LAUNCH_CHECK();
        unsigned bits = 0;
        THX_RET(to_host(&bits, dDiff.p, sizeof(unsigned)));
        diffCPrev = diffC;
        std::memcpy(&diffC, &bits, sizeof(float));
        noDec = (double)diffC > (double)diffCPrev * DIFF_C_DECREASE_THRES ? noDec + 1 : 0;
        if ((double)diffC < DIFF_C_THRES || (m >= minIter && noDec == N_DIFF_C_NO_DECREASE)) break;
    }
    if (nIter) *nIter = m < maxIter ? m + 1 : maxIter;
    return to_host(W, dW.p, sizeof(float) * n);
}

int expose_wt_t(int gpuIdx, const float* T, float* W, int maxRadius, int pf, int dim, int nd)
{
    THX_CHECK_ARG(T && W && dim > 0 && dim % 2 == 0 && pf > 0, "thx_ExposeWT_T: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    const long n = hc_size(dim, nd);
    DBuf dT, dW;
    THX_DALLOC(dT, sizeof(float) * n);
    THX_DALLOC(dW, sizeof(float) * n);
    THX_RET(to_dev(dT.p, T, sizeof(float) * n));
    THX_RET(to_dev(dW.p, W, sizeof(float) * n));
    hipLaunchKernelGGL(k_w_from_t, dim3(grid_for(n)), dim3(256), 0, nullptr, dW.as<float>(),
                       dT.as<float>(), n, dim, maxRadius * pf * maxRadius * pf);
    THX_LAUNCH_CHECK();
    return to_host(W, dW.p, sizeof(float) * n);
}

// F W padded into the pdim grid (device dP), optionally back-transformed
// into dR and divided by its size
int pad_fw(const float* F, const float* W, int maxRadius, int pf, int pdim, int fdim, int nd, DBuf& dP,
           DBuf* dR)
{
    const long nf = hc_size(fdim, nd), np = hc_size(pdim, nd), npr = rl_size(pdim, nd);
    DBuf dF, dW;
    THX_DALLOC(dF, sizeof(float2) * nf);
    THX_DALLOC(dW, sizeof(float) * nf);
    THX_DALLOC(dP, sizeof(float2) * np);
    THX_RET(to_dev(dF.p, F, sizeof(float2) * nf));
    THX_RET(to_dev(dW.p, W, sizeof(float) * nf));
    THX_HIP(hipMemset(dP.p, 0, sizeof(float2) * np));
    hipLaunchKernelGGL(k_pad_fw, dim3(grid_for(nf)), dim3(256), 0, nullptr, dP.as<float2>(),
                       dF.as<float2>(), dW.as<float>(), nf, fdim, pdim, maxRadius * pf * maxRadius * pf);
    THX_LAUNCH_CHECK();
    if (!dR) return THX_OK;
    THX_DALLOC(*dR, sizeof(float) * npr);
    Fft fft;
    THX_RET(fft.make(pdim, nd, true, false));
    THX_FFT(hipfftExecC2R(fft.c2r, dP.as<hipfftComplex>(), dR->as<float>()));
    hipLaunchKernelGGL(k_div, dim3(grid_for(npr)), dim3(256), 0, nullptr, dR->as<float>(), npr,
                       (float)npr);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

// the kernel correction of a real dim^nd array on device, then optionally
// its forward transform into dFt
int correct(DBuf& dX, const float* tab, float nf, int dim, int nd, DBuf* dFt)
{
    const long n = rl_size(dim, nd);
    const long h = dim / 2 + 1;
    const long nt = nd == 3 ? h * h * h : h * h;
    DBuf dTab;
    THX_DALLOC(dTab, sizeof(float) * nt);
    THX_RET(to_dev(dTab.p, tab, sizeof(float) * nt));
    hipLaunchKernelGGL(k_correct, dim3(grid_for(n)), dim3(256), 0, nullptr, dX.as<float>(), n, dim, nd,
                       dTab.as<float>(), nf);
    THX_LAUNCH_CHECK();
    if (!dFt) return THX_OK;
    THX_DALLOC(*dFt, sizeof(float2) * hc_size(dim, nd));
    Fft fft;
    THX_RET(fft.make(dim, nd, false, true));
    THX_FFT(hipfftExecR2C(fft.r2c, dX.as<float>(), dFt->as<hipfftComplex>()));
    return THX_OK;
}

int translate(int gpuIdx, float* img, double ox, double oy, double oz, int r, int dim, int nd)
{
    THX_CHECK_ARG(img && dim > 0 && dim % 2 == 0, "thx_TranslateI: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    const long n = hc_size(dim, nd);
    DBuf d;
    THX_DALLOC(d, sizeof(float2) * n);
    THX_RET(to_dev(d.p, img, sizeof(float2) * n));
    hipLaunchKernelGGL(k_translate, dim3(grid_for(n)), dim3(256), 0, nullptr, d.as<float2>(), n, dim,
                       (float)ox, (float)oy, (float)oz, r);
    THX_LAUNCH_CHECK();
    return to_host(img, d.p, sizeof(float2) * n);
}

// the split-step state behind the caller's void* stream[] slots: stream[0]
// holds the HIP stream every step runs on (the reference's three streams
// only overlapped its batched copies)
inline hipStream_t slot_stream(void** stream) { return static_cast<hipStream_t>(stream[0]); }

}  // namespace

// --------------------------------------------------------------- PrepareTF
extern "C" int thx_PrepareTF(int gpuIdx, float* F3D, float* T3D, const double* symMat, int nSymElem,
                             int maxRadius, int pf, int dim)
{
    THX_CHECK_ARG(F3D && T3D && dim > 0 && dim % 2 == 0 && pf > 0 && nSymElem >= 0 &&
                      (nSymElem == 0 || symMat),
                  "thx_PrepareTF: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    const long n = hc_size(dim, 3);
    const size_t ws = thx_prepare_tf_workspace(dim);
    DBuf dF, dT, dM, dWs;
    THX_DALLOC(dF, sizeof(float2) * n);
    THX_DALLOC(dT, sizeof(float) * n);
    THX_DALLOC(dM, sizeof(double) * 9 * (nSymElem > 0 ? nSymElem : 1));
    THX_DALLOC(dWs, ws);
    THX_RET(to_dev(dF.p, F3D, sizeof(float2) * n));
    THX_RET(to_dev(dT.p, T3D, sizeof(float) * n));
    // symMat as Reconstructor::prepareTFG packs it (Map<dmat33>: column-major
    // R) and Mat33::getElement reads it (row-major, gpu/src/util/Mat33.cu:
    // 30-34): each element acts as R^T = R^-1, the same group
    if (nSymElem > 0) THX_RET(to_dev(dM.p, symMat, sizeof(double) * 9 * nSymElem));
    THX_RET(thx_prepare_tf(dF.as<float>(), dT.as<float>(), dim, dM.as<double>(), nSymElem, maxRadius, pf,
                           dWs.p, ws, nullptr));
    hipLaunchKernelGGL(k_clamp_t, dim3(grid_for(n)), dim3(256), 0, nullptr, dT.as<float>(), n);
    THX_LAUNCH_CHECK();
    THX_RET(to_host(F3D, dF.p, sizeof(float2) * n));
    return to_host(T3D, dT.p, sizeof(float) * n);
}

// ----------------------------------------------------------- MAP (ExposePT)
extern "C" int thx_ExposePT(int gpuIdx, float* T3D, int maxRadius, int pf, int dim, const float* fsc,
                            int nFsc, int joinHalf, int wienerF)
{
    return expose_pt(gpuIdx, T3D, maxRadius, pf, dim, 3, fsc, nFsc, joinHalf, wienerF);
}

extern "C" int thx_ExposePT2D(int gpuIdx, float* T2D, int maxRadius, int pf, int dim, const float* fsc,
                              int nFsc, int joinHalf, int wienerF)
{
    return expose_pt(gpuIdx, T2D, maxRadius, pf, dim, 2, fsc, nFsc, joinHalf, wienerF);
}

// ------------------------------------------------------ balancing (ExposeWT)
extern "C" int thx_ExposeWT(int gpuIdx, const float* T3D, float* W3D, const float* tab, float step,
                            int tabSize, float nf, int maxRadius, int pf, int dim, int maxIter, int minIter,
                            int size, int* nIter)
{
    return expose_wt(gpuIdx, T3D, W3D, tab, step, tabSize, nf, maxRadius, pf, dim, 3, maxIter, minIter,
                     size, nIter);
}

extern "C" int thx_ExposeWT2D(int gpuIdx, const float* T2D, float* W2D, const float* tab, float step,
                              int tabSize, float nf, int maxRadius, int pf, int dim, int maxIter,
                              int minIter, int size, int* nIter)
{
    return expose_wt(gpuIdx, T2D, W2D, tab, step, tabSize, nf, maxRadius, pf, dim, 2, maxIter, minIter,
                     size, nIter);
}

extern "C" int thx_ExposeWT_T(int gpuIdx, const float* T3D, float* W3D, int maxRadius, int pf, int dim)
{
    return expose_wt_t(gpuIdx, T3D, W3D, maxRadius, pf, dim, 3);
}

extern "C" int thx_ExposeWT2D_T(int gpuIdx, const float* T2D, float* W2D, int maxRadius, int pf, int dim)
{
    return expose_wt_t(gpuIdx, T2D, W2D, maxRadius, pf, dim, 2);
}

// ------------------------------------------------- split-step balancing (3D)
extern "C" int thx_AllocDevicePoint(int gpuIdx, float** dev_C, float** dev_W, float** dev_T,
                                    float** dev_tab, float** devDiff, float** devMax, int** devCount,
                                    void** stream, int streamNum, int tabSize, int dim)
{
    THX_CHECK_ARG(dev_C && dev_W && dev_T && dev_tab && devMax && stream && streamNum >= 1 &&
                      tabSize > 0 && dim > 0 && dim % 2 == 0,
                  "thx_AllocDevicePoint: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    const long n = hc_size(dim, 3);
    *dev_C = *dev_W = *dev_T = *dev_tab = *devMax = nullptr;
    if (devDiff) *devDiff = nullptr;      // RECONSTRUCTOR_CHECK_C_AVERAGE is off (include/Config.h:101)
    if (devCount) *devCount = nullptr;
    for (int i = 0; i < streamNum; i++) stream[i] = nullptr;
    // all or nothing: the buffers are handed to the out-pointers only once
    // every allocation (and the stream) succeeded; on a failure the DBufs free
    // what was allocated and the outputs stay null
    DBuf C, W, T, tab, mx;
    // the C buffer also holds the dim^3 real-space C of ExposeForConvC
    THX_DALLOC(C, std::max(sizeof(float2) * n, sizeof(float) * rl_size(dim, 3)));
    THX_DALLOC(W, sizeof(float) * n);
    THX_DALLOC(T, sizeof(float) * n);
    THX_DALLOC(tab, sizeof(float) * tabSize);
    THX_DALLOC(mx, sizeof(unsigned));
    hipStream_t s = nullptr;
    THX_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto release = [](DBuf& b) { void* p = b.p; b.p = nullptr; return p; };
    *dev_C = static_cast<float*>(release(C));
    *dev_W = static_cast<float*>(release(W));
    *dev_T = static_cast<float*>(release(T));
    *dev_tab = static_cast<float*>(release(tab));
    *devMax = static_cast<float*>(release(mx));
    stream[0] = s;
    return THX_OK;
}

extern "C" int thx_HostDeviceInit(int gpuIdx, const float* T3D, const float* tab, float* dev_W,
                                  float* dev_T, float* dev_tab, void** stream, int streamNum, int tabSize,
                                  int maxRadius, int pf, int dim)
{
    THX_CHECK_ARG(T3D && tab && dev_W && dev_T && dev_tab && stream && stream[0] && streamNum >= 1,
                  "thx_HostDeviceInit: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    hipStream_t s = slot_stream(stream);
    const long n = hc_size(dim, 3);
    THX_HIP(hipMemcpyAsync(dev_tab, tab, sizeof(float) * tabSize, hipMemcpyHostToDevice, s));
    THX_HIP(hipMemcpyAsync(dev_T, T3D, sizeof(float) * n, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_w_init, dim3(grid_for(n)), dim3(256), 0, s, dev_W, n, dim,
                       maxRadius * pf * maxRadius * pf);
    THX_LAUNCH_CHECK();
    THX_HIP(hipStreamSynchronize(s));
    return THX_OK;
}

extern "C" int thx_ExposeC(int gpuIdx, float* C3D, float* dev_C, const float* dev_T, const float* dev_W,
                           void** stream, int streamNum, int dim)
{
    THX_CHECK_ARG(C3D && dev_C && dev_T && dev_W && stream && stream[0] && streamNum >= 1,
                  "thx_ExposeC: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    hipStream_t s = slot_stream(stream);
    const long n = hc_size(dim, 3);
    hipLaunchKernelGGL(k_c_tw, dim3(grid_for(n)), dim3(256), 0, s, reinterpret_cast<float2*>(dev_C), dev_T,
                       dev_W, n);
    THX_LAUNCH_CHECK();
    THX_HIP(hipMemcpyAsync(C3D, dev_C, sizeof(float2) * n, hipMemcpyDeviceToHost, s));
    THX_HIP(hipStreamSynchronize(s));
    return THX_OK;
}

// C3D: the caller's real-space C (dim^3, after its scaled backward FFT)
extern "C" int thx_ExposeForConvC(int gpuIdx, float* C3D, float* dev_C, const float* dev_tab,
                                  void** stream, float step, int tabSize, float nf, int streamNum,
                                  int pf, int size, int dim)
{
    THX_CHECK_ARG(C3D && dev_C && dev_tab && stream && stream[0] && streamNum >= 1 && step > 0.f &&
                      nf != 0.f && tabSize > 0,
                  "thx_ExposeForConvC: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    hipStream_t s = slot_stream(stream);
    const long nr = rl_size(dim, 3);
    THX_HIP(hipMemcpyAsync(dev_C, C3D, sizeof(float) * nr, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_conv_c, dim3(grid_for(nr)), dim3(256), 0, s, dev_C, nr, dim, dev_tab, step, tabSize,
                       nf, pf * size, 0);
    THX_LAUNCH_CHECK();
    THX_HIP(hipMemcpyAsync(C3D, dev_C, sizeof(float) * nr, hipMemcpyDeviceToHost, s));
    THX_HIP(hipStreamSynchronize(s));
    return THX_OK;
}

// C3D: the caller's forward-transformed C; *diffC = max | |C| - 1 | inside
// (RECONSTRUCTOR_CHECK_C_MAX, include/Config.h:103)
extern "C" int thx_ExposeWC(int gpuIdx, const float* C3D, float* dev_C, float* dev_W, float* devMax,
                            void** stream, float* diffC, int streamNum, int maxRadius, int pf, int dim)
{
    THX_CHECK_ARG(C3D && dev_C && dev_W && devMax && diffC && stream && stream[0] && streamNum >= 1,
                  "thx_ExposeWC: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    hipStream_t s = slot_stream(stream);
    const long n = hc_size(dim, 3);
    THX_HIP(hipMemcpyAsync(dev_C, C3D, sizeof(float2) * n, hipMemcpyHostToDevice, s));
    THX_HIP(hipMemsetAsync(devMax, 0, sizeof(unsigned), s));
    hipLaunchKernelGGL(k_update_w, dim3(std::min<unsigned>(grid_for(n), 2048u)), dim3(256), 0, s, dev_W,
                       reinterpret_cast<const float2*>(dev_C), n, dim, maxRadius * pf * maxRadius * pf,
                       reinterpret_cast<unsigned*>(devMax));
    THX_LAUNCH_CHECK();
    unsigned bits = 0;
    THX_HIP(hipMemcpyAsync(&bits, devMax, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    THX_HIP(hipStreamSynchronize(s));
    std::memcpy(diffC, &bits, sizeof(float));
    return THX_OK;
}

// volumeW (host) = the balanced W; frees what thx_AllocDevicePoint made
extern "C" int thx_FreeDevHostPoint(int gpuIdx, float** dev_C, float** dev_W, float** dev_T,
                                    float** dev_tab, float** devDiff, float** devMax, int** devCount,
                                    void** stream, float* volumeW, int streamNum, int dim)
{
    THX_CHECK_ARG(dev_C && dev_W && dev_T && dev_tab && devMax && stream && streamNum >= 1,
                  "thx_FreeDevHostPoint: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    int st = THX_OK;
    if (volumeW && *dev_W &&
        hipMemcpy(volumeW, *dev_W, sizeof(float) * hc_size(dim, 3), hipMemcpyDeviceToHost) != hipSuccess) {
        thx::set_error("thx_FreeDevHostPoint: copying W back failed");
        st = THX_ERR_HIP;
    }
    if (stream[0]) (void)hipStreamDestroy(static_cast<hipStream_t>(stream[0]));
    stream[0] = nullptr;
    for (float** p : {dev_C, dev_W, dev_T, dev_tab, devMax}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    if (devDiff) *devDiff = nullptr;
    if (devCount) *devCount = nullptr;
    return st;
}

// ---------------------------------------------------------- pad (ExposePF*)
extern "C" int thx_ExposePFW(int gpuIdx, float* padDst, const float* F3D, const float* W3D, int maxRadius,
                             int pf, int pdim, int fdim)
{
    THX_CHECK_ARG(padDst && F3D && W3D && pdim >= fdim && fdim > 0 && fdim % 2 == 0 && pdim % 2 == 0,
                  "thx_ExposePFW: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    DBuf dP;
    THX_RET(pad_fw(F3D, W3D, maxRadius, pf, pdim, fdim, 3, dP, nullptr));
    return to_host(padDst, dP.p, sizeof(float2) * hc_size(pdim, 3));
}

// padDst is scratch on the reference's side (CalculateF does not copy it back)
extern "C" int thx_ExposePF(int gpuIdx, float* padDstR, const float* F3D, const float* W3D, int maxRadius,
                            int pf, int pdim, int fdim)
{
    THX_CHECK_ARG(padDstR && F3D && W3D && pdim >= fdim && fdim > 0 && fdim % 2 == 0 && pdim % 2 == 0,
                  "thx_ExposePF: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    DBuf dP, dR;
    THX_RET(pad_fw(F3D, W3D, maxRadius, pf, pdim, fdim, 3, dP, &dR));
    return to_host(padDstR, dR.p, sizeof(float) * rl_size(pdim, 3));
}

extern "C" int thx_ExposePF2D(int gpuIdx, float* padDstR, const float* F2D, const float* W2D,
                              int maxRadius, int pf, int pdim, int fdim)
{
    THX_CHECK_ARG(padDstR && F2D && W2D && pdim >= fdim && fdim > 0 && fdim % 2 == 0 && pdim % 2 == 0,
                  "thx_ExposePF2D: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    DBuf dP, dR;
    THX_RET(pad_fw(F2D, W2D, maxRadius, pf, pdim, fdim, 2, dP, &dR));
    return to_host(padDstR, dR.p, sizeof(float) * rl_size(pdim, 2));
}

// -------------------------------------------------- correction (ExposeCorrF*)
// mkbRL: (dim/2+1)^3 (2D: ^2) table of the real-space kernel over |i|, |j|,
// |k|; nf = 0 with the trilinear kernel (dst / table), MKB_RL(0) with the MKB
// kernel (dst / table * nf) -- the two builds of kernel_CorrectF
extern "C" int thx_ExposeCorrF(int gpuIdx, float* dst, const float* mkbRL, float nf, int dim)
{
    THX_CHECK_ARG(dst && mkbRL && dim > 0 && dim % 2 == 0, "thx_ExposeCorrF: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    const long n = rl_size(dim, 3);
    DBuf dX;
    THX_DALLOC(dX, sizeof(float) * n);
    THX_RET(to_dev(dX.p, dst, sizeof(float) * n));
    THX_RET(correct(dX, mkbRL, nf, dim, 3, nullptr));
    return to_host(dst, dX.p, sizeof(float) * n);
}

// ExposeCorrF(dstN, dst): dstN corrected (on device) and forward-transformed into dst
extern "C" int thx_ExposeCorrFT(int gpuIdx, const float* dstN, float* dst, const float* mkbRL, float nf,
                                int dim)
{
    THX_CHECK_ARG(dstN && dst && mkbRL && dim > 0 && dim % 2 == 0, "thx_ExposeCorrFT: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    DBuf dX, dF;
    THX_DALLOC(dX, sizeof(float) * rl_size(dim, 3));
    THX_RET(to_dev(dX.p, dstN, sizeof(float) * rl_size(dim, 3)));
    THX_RET(correct(dX, mkbRL, nf, dim, 3, &dF));
    return to_host(dst, dF.p, sizeof(float2) * hc_size(dim, 3));
}

extern "C" int thx_ExposeCorrF2D(int gpuIdx, const float* imgDst, float* dst, const float* mkbRL, float nf,
                                 int dim)
{
    THX_CHECK_ARG(imgDst && dst && mkbRL && dim > 0 && dim % 2 == 0, "thx_ExposeCorrF2D: bad arguments");
    DeviceGuard g;
    THX_HIP(hipSetDevice(gpuIdx));
    DBuf dX, dF;
    THX_DALLOC(dX, sizeof(float) * rl_size(dim, 2));
    THX_RET(to_dev(dX.p, imgDst, sizeof(float) * rl_size(dim, 2)));
    THX_RET(correct(dX, mkbRL, nf, dim, 2, &dF));
    return to_host(dst, dF.p, sizeof(float2) * hc_size(dim, 2));
}

// ------------------------------------------------------------- TranslateI*
extern "C" int thx_TranslateI(int gpuIdx, float* ref, double ox, double oy, double oz, int r, int dim)
{
    return translate(gpuIdx, ref, ox, oy, oz, r, dim, 3);
}

extern "C" int thx_TranslateI2D(int gpuIdx, float* img, double ox, double oy, int r, int dim)
{
    return translate(gpuIdx, img, ox, oy, 0.0, r, dim, 2);
}

// ------------------------------------------------------ ReMask / GCTFinit
// img[l]: image l's half-complex transform (idim x (idim/2+1) Complex), in
// place; the images are dealt over thx_adapter_devices() as cuthunder deals
// them over its GPUs
extern "C" int thx_ReMask(float* const* img, float maskRadius, float pixelSize, float ew, int idim,
                          int imgNum)
{
    THX_CHECK_ARG(imgNum >= 0 && idim > 0 && idim % 2 == 0 && pixelSize > 0.f && ew > 0.f &&
                      (imgNum == 0 || img),
                  "thx_ReMask: bad arguments");
    if (imgNum == 0) return THX_OK;
    DeviceGuard g;
    std::vector<int> devs;
    THX_RET(thx::adapter_devices(devs));
    const float r = maskRadius / pixelSize;
    const size_t nFt = (size_t)idim * (idim / 2 + 1);
    return thx::on_devices(devs, imgNum, [&](int, int, int l0, int l1) -> int {
        const int nb = l1 - l0;
        if (nb <= 0) return THX_OK;
        DBuf dFt, dRl;
        THX_DALLOC(dFt, sizeof(float2) * nFt * nb);
        THX_DALLOC(dRl, sizeof(float) * (size_t)idim * idim * nb);
        for (int l = l0; l < l1; l++)
            THX_RET(to_dev(dFt.as<float2>() + nFt * (l - l0), img[l], sizeof(float2) * nFt));
        THX_RET(thx_remask(dFt.as<float>(), nb, idim, r, ew, dRl.as<float>(), nullptr));
        for (int l = l0; l < l1; l++)
            THX_RET(to_host(img[l], dFt.as<float2>() + nFt * (l - l0), sizeof(float2) * nFt));
        return THX_OK;
    });
}

// ctfAttr: imgNum x 7 RFLOAT (CTFAttr, include/Database.h:302-337); img[l]
// receives (CTF, 0) over its half-complex grid
extern "C" int thx_GCTFinit(float* const* img, const float* ctfAttr, float pixelSize, int idim, int imgNum)
{
    THX_CHECK_ARG(imgNum >= 0 && idim > 0 && idim % 2 == 0 && pixelSize > 0.f &&
                      (imgNum == 0 || (img && ctfAttr)),
                  "thx_GCTFinit: bad arguments");
    if (imgNum == 0) return THX_OK;
    DeviceGuard g;
    std::vector<int> devs;
    THX_RET(thx::adapter_devices(devs));
    const size_t nFt = (size_t)idim * (idim / 2 + 1);
    return thx::on_devices(devs, imgNum, [&](int, int, int l0, int l1) -> int {
        const int nb = l1 - l0;
        if (nb <= 0) return THX_OK;
        std::vector<float> a(8 * (size_t)nb);
        for (int l = l0; l < l1; l++) {
            a[8 * (size_t)(l - l0)] = pixelSize;
            for (int k = 0; k < 7; k++) a[8 * (size_t)(l - l0) + 1 + k] = ctfAttr[7 * (size_t)l + k];
        }
        DBuf dA, dRe, dC;
        THX_DALLOC(dA, sizeof(float) * a.size());
        THX_DALLOC(dRe, sizeof(float) * nFt * nb);
        THX_DALLOC(dC, sizeof(float2) * nFt * nb);
        THX_RET(to_dev(dA.p, a.data(), sizeof(float) * a.size()));
        THX_RET(thx_ctf_image(dA.as<float>(), nb, idim, dRe.as<float>(), nullptr));
        const long n = (long)(nFt * nb);
        hipLaunchKernelGGL(k_real_to_complex, dim3(grid_for(n)), dim3(256), 0, nullptr, dRe.as<float>(),
                           dC.as<float2>(), n);
        THX_LAUNCH_CHECK();
        for (int l = l0; l < l1; l++)
            THX_RET(to_host(img[l], dC.as<float2>() + nFt * (l - l0), sizeof(float2) * nFt));
        return THX_OK;
    });
}
