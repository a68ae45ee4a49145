// preprocess.hip -- f2: the per-image preprocessing of Optimiser::initImg
// (src/Optimiser.cpp:4608-5024) and the re-mask of reMaskImg / reMaskImgG
// (:6093-6190; GPU twin ReMask, gpu/interface/Interface.cpp:1296 ->
// gpu/src/cuthunder.cu:9406), plus GCTFinit's CTF images (cuthunder.cu:9641),
// on device for a whole stack.
//
// Stages (the reference's, with the compiled switches OPTIMISER_MASK_IMG and
// OPTIMISER_INIT_IMG_NORMALISE_OUT_MASK_REGION, include/Config.h:184, 190):
//   thx_img_stats   load each real-space image (as read from an MRC stack:
//                   centred, or already in the reference's corner-origin
//                   layout, ImageFile's MESH_IMAGE_INDEX read), then
//                   substractBgImg: mean / sample sd of the pixels outside
//                   the mask radius (bgMeanStddev, src/Image/ImageFunctions.
//                   cpp:607-620), x <- (x - mean) / sd; and the per-image
//                   terms of statImg (:4810-4905): bgStddev(0) outside the
//                   radius, stddev(0) over all pixels, the mean inside the
//                   radius (regionMean(img, rU, 0), src/Functions/Mask.cpp:
//                   102-127).  The caller averages them over the hemisphere
//                   (an all-reduce across ranks, as the reference's
//                   MPI_Allreduce over _hemi) into stdN.
//   thx_img_finish  maskImg (:4964-4996): keep a copy (_imgOri), soft mask
//                   with a cosine edge of EDGE_WIDTH_RL (include/Macro.h:99)
//                   to zero (zeroMask) or to Gaussian noise of sd stdN;
//                   normaliseImg (:4998-5012): both scaled by 1 / stdN;
//                   fwImg (:5014-5024): forward r2c FFT, unnormalised
//                   (FFTW's convention, src/FFT.cpp), half-complex
//                   [N][N/2+1] per image -- the layout allocPreCal gathers
//                   the pixel set from (thx_img_gather).
//   thx_remask      reMaskImg: backward FFT (scaled by 1 / N^2, as
//                   FFT::bwExecutePlan), multiply by the soft mask, forward.
// One workgroup per image for the statistics (two passes, double sums);
// hipFFT batched 2D transforms with plans cached per (device, N, batch,
// stream).
#include <hipfft/hipfft.h>

#include <cmath>
#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

#define THX_FFT(call)                                                          \
    do {                                                                       \
        hipfftResult r_ = (call);                                              \
        if (r_ != HIPFFT_SUCCESS) {                                            \
            ::thx::set_error("%s:%d %s: hipfft error %d", __FILE__, __LINE__,  \
                             #call, (int)r_);                                  \
            return THX_ERR_HIP;                                                \
        }                                                                      \
    } while (0)

namespace {

constexpr int ST_THREADS = 256;
constexpr int FFT_BATCH = 512;          // images per batched transform

// pixel (i, j) of the reference's RL grid, i, j in [-N/2, N/2), in a stored
// image: corner origin (Image::iRL, include/Image/Image.h:388-394) or
// centred as on disk (ImageFile's MESH_IMAGE_INDEX read, ImageFile.h:383)
THX_DEV size_t rl_index(int i, int j, int N, bool centred)
{
    if (centred) return (size_t)(j + N / 2) * N + (i + N / 2);
    return (size_t)(j >= 0 ? j : j + N) * N + (i >= 0 ? i : i + N);
}

template <typename T>
THX_DEV T block_sum(T v, T* sh)
{
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sh[wv] = v;
    __syncthreads();
    T s = 0;
    for (int k = 0; k < ST_THREADS / 64; k++) s += sh[k];
    return s;
}

// stats[l] = {bgMean, bgSd, bgStddev(0) after, stddev(0) after, centre mean after}
__global__ void __launch_bounds__(ST_THREADS) k_img_stats(const float* __restrict__ in, int centred,
                                                          float* __restrict__ out, int N, float r,
                                                          float* __restrict__ stats)
{
    __shared__ double sh[ST_THREADS / 64];
    const int l = blockIdx.x;
    const size_t n2 = (size_t)N * N;
    const float* src = in + (size_t)l * n2;
    float* dst = out + (size_t)l * n2;
    const double r2 = (double)r * r;
    // pass 1: background mean (QUAD(i, j) > r^2)
    double s = 0.0, c = 0.0;
    for (size_t q = threadIdx.x; q < n2; q += ST_THREADS) {
        const int j = (int)(q / N) - N / 2, i = (int)(q % N) - N / 2;
        if ((double)i * i + (double)j * j > r2) {
            s += src[rl_index(i, j, N, centred)];
            c += 1.0;
        }
    }
    s = block_sum(s, sh);
    c = block_sum(c, sh);
    const double mean = c > 0 ? s / c : 0.0;
    // pass 2: sample standard deviation about it (gsl_stats_sd_m)
    double ss = 0.0;
    for (size_t q = threadIdx.x; q < n2; q += ST_THREADS) {
        const int j = (int)(q / N) - N / 2, i = (int)(q % N) - N / 2;
        if ((double)i * i + (double)j * j > r2) {
            const double d = src[rl_index(i, j, N, centred)] - mean;
            ss += d * d;
        }
    }
    ss = block_sum(ss, sh);
    const float fm = (float)mean, fsd = (float)(c > 1 ? sqrt(ss / (c - 1)) : 1.0);
    // pass 3: x <- (x - bgMean) / bgStddev (RFLOAT arithmetic), corner-origin
    // layout out; the statImg terms of the normalised image
    double b0 = 0.0, a0 = 0.0, ci = 0.0, cn = 0.0;
    for (size_t q = threadIdx.x; q < n2; q += ST_THREADS) {
        const int j = (int)(q / N) - N / 2, i = (int)(q % N) - N / 2;
        float v = src[rl_index(i, j, N, centred)];
        v -= fm;
        v /= fsd;
        dst[rl_index(i, j, N, false)] = v;
        const double q2 = (double)i * i + (double)j * j;
        if (q2 > r2) b0 += (double)v * v;
        if (sqrt(q2) < (double)r) { ci += v; cn += 1.0; }
        a0 += (double)v * v;
    }
    b0 = block_sum(b0, sh);
    a0 = block_sum(a0, sh);
    ci = block_sum(ci, sh);
    cn = block_sum(cn, sh);
    if (threadIdx.x == 0) {
        float* st = stats + 5 * (size_t)l;
        st[0] = fm;
        st[1] = fsd;
        st[2] = (float)(c > 1 ? sqrt(b0 / (c - 1)) : 0.0);
        st[3] = (float)sqrt(a0 / (double)(n2 - 1));
        st[4] = (float)(cn > 0 ? ci / cn : 0.0);
    }
}

// softMask's weight of the image (1 - portion of background) at radius u
THX_DEV float mask_keep(float u, float r, float ew)
{
    if (u < r) return 1.f;
    if (u > r + ew) return 0.f;
    return 1.f - (0.5f - 0.5f * cosf((u - r) / ew * (float)M_PI));
}

// maskImg + normaliseImg: ori <- x / stdN; x <- softMask(x) / stdN with the
// background 0 (zeroMask) or N(0, stdN) noise per pixel (Philox; the
// reference's GSL generator is urandom-seeded)
__global__ void k_img_mask_scale(float* __restrict__ img, float* __restrict__ ori, int nImg, int N,
                                 float r, float ew, int zeroMask, float stdN, float scale,
                                 unsigned long long seed)
{
    const size_t n2 = (size_t)N * N, tot = n2 * nImg;
    for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < tot;
         q += (size_t)gridDim.x * blockDim.x) {
        const size_t p = q % n2;
        const int jj = (int)(p / N), ii = (int)(p % N);
        const int j = jj < N / 2 ? jj : jj - N, i = ii < N / 2 ? ii : ii - N;
        const float u = (float)hypot((double)i, (double)j);
        const float x = img[q];
        if (ori) ori[q] = x * scale;
        float v;
        if (zeroMask) {
            v = x * mask_keep(u, r, ew);
        } else if (u < r) {
            v = x;
        } else {
            Philox g(seed, (uint32_t)(q >> 32), (uint32_t)q, 0x6d61736bu);
            const float bg = (float)(g.gauss2().x * stdN);
            const float w = 1.f - mask_keep(u, r, ew);     // portion of background
            v = u > r + ew ? bg : bg * w + x * (1.f - w);
        }
        img[q] = v * scale;
    }
}

__global__ void k_scale_mask_rl(float* __restrict__ rl, int nImg, int N, float r, float ew,
                                float scale)
{
    const size_t n2 = (size_t)N * N, tot = n2 * nImg;
    for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < tot;
         q += (size_t)gridDim.x * blockDim.x) {
        const size_t p = q % n2;
        const int jj = (int)(p / N), ii = (int)(p % N);
        const int j = jj < N / 2 ? jj : jj - N, i = ii < N / 2 ? ii : ii - N;
        const float u = (float)hypot((double)i, (double)j);
        // bwExecutePlan's 1 / N^2, then MUL_RL by the soft mask
        rl[q] = (rl[q] * scale) * mask_keep(u, r, ew);
    }
}

// allocPreCal's gather (src/Optimiser.cpp:8043-8083): datP[l][i] = FT_l[iPxl[i]]
__global__ void k_img_gather(const float2* __restrict__ ft, int nImg, int nFT,
                             const int* __restrict__ iPxl, int nPxl, float2* __restrict__ datP)
{
    const size_t tot = (size_t)nImg * nPxl;
    for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < tot;
         q += (size_t)gridDim.x * blockDim.x) {
        const size_t l = q / nPxl, i = q % nPxl;
        datP[q] = ft[l * nFT + iPxl[i]];
    }
}

// GCTFinit: the CTF over an image's whole half-complex grid, [N][N/2+1],
// row j in [0, N) = frequency j or j - N (iFTHalf), column i in [0, N/2]
__global__ void k_ctf_image(const float* __restrict__ attr, int nImg, int N, float* __restrict__ out)
{
    const int nc = N / 2 + 1;
    const size_t per = (size_t)nc * N, tot = per * nImg;
    for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < tot;
         q += (size_t)gridDim.x * blockDim.x) {
        const size_t l = q / per, p = q % per;
        const int jj = (int)(p / nc), i = (int)(p % nc);
        const int j = jj < N / 2 ? jj : jj - N;
        const float* a = attr + 8 * l;
        out[q] = ctf_at(a, a[2], a[3], i, j, N);
    }
}

// batched 2D plans per (device, N, batch, stream): hipfftSetStream binds a
// plan to one stream, so callers on different streams never share one
struct Plan2 {
    hipfftHandle r2c = 0, c2r = 0;
};

struct PlanCache2 {
    std::mutex mu;
    std::map<std::tuple<int, int, int, hipStream_t>, Plan2> plans;
};

PlanCache2& cache2()
{
    static PlanCache2* c = new PlanCache2;
    return *c;
}

int plans2(int N, int batch, hipStream_t s, Plan2** out)
{
    int dev = 0;
    THX_HIP(hipGetDevice(&dev));
    PlanCache2& c = cache2();
    std::lock_guard<std::mutex> lk(c.mu);
    const auto key = std::make_tuple(dev, N, batch, s);
    auto it = c.plans.find(key);
    if (it == c.plans.end()) {
        Plan2 p;
        int n[2] = {N, N};
        THX_FFT(hipfftPlanMany(&p.r2c, 2, n, nullptr, 1, N * N, nullptr, 1, N * (N / 2 + 1),
                               HIPFFT_R2C, batch));
        THX_FFT(hipfftPlanMany(&p.c2r, 2, n, nullptr, 1, N * (N / 2 + 1), nullptr, 1, N * N,
                               HIPFFT_C2R, batch));
        THX_FFT(hipfftSetStream(p.r2c, s));
        THX_FFT(hipfftSetStream(p.c2r, s));
        it = c.plans.emplace(key, p).first;
    }
    *out = &it->second;
    return THX_OK;
}

// forward r2c of nImg real images [N][N] into [N][N/2+1] (unnormalised)
int fft_forward(float* rl, float2* ft, int nImg, int N, hipStream_t s)
{
    for (int l0 = 0; l0 < nImg; l0 += FFT_BATCH) {
        const int nb = nImg - l0 < FFT_BATCH ? nImg - l0 : FFT_BATCH;
        Plan2* p = nullptr;
        const int st = plans2(N, nb, s, &p);
        if (st != THX_OK) return st;
        THX_FFT(hipfftExecR2C(p->r2c, rl + (size_t)l0 * N * N,
                              reinterpret_cast<hipfftComplex*>(ft + (size_t)l0 * N * (N / 2 + 1))));
    }
    return THX_OK;
}

}  // namespace

extern "C" int thx_img_stats(const float* img, int centred, int nImg, int idim, float rMask,
                             float* out, float* stats, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && idim > 0 && idim % 2 == 0 && rMask > 0.f,
                  "thx_img_stats: bad sizes");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(img && out && stats && img != out, "thx_img_stats: null / aliased argument");
    hipLaunchKernelGGL(k_img_stats, dim3(nImg), dim3(ST_THREADS), 0, thx::as_stream(stream), img,
                       centred, out, idim, rMask, stats);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_img_finish(float* img, int nImg, int idim, float rMask, float edge, int zeroMask,
                              float stdN, unsigned long long seed, float* imgFT, float* ori,
                              float* oriFT, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && idim > 0 && idim % 2 == 0 && rMask > 0.f && edge > 0.f && stdN > 0.f,
                  "thx_img_finish: bad arguments");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(img && imgFT && (!oriFT || ori), "thx_img_finish: null argument");
    hipStream_t s = thx::as_stream(stream);
    hipLaunchKernelGGL(k_img_mask_scale, dim3(2048), dim3(256), 0, s, img, ori, nImg, idim, rMask,
                       edge, zeroMask, stdN, 1.f / stdN, seed);
    THX_LAUNCH_CHECK();
    const int st = fft_forward(img, reinterpret_cast<float2*>(imgFT), nImg, idim, s);
    if (st != THX_OK) return st;
    if (oriFT) return fft_forward(ori, reinterpret_cast<float2*>(oriFT), nImg, idim, s);
    return THX_OK;
}

extern "C" int thx_remask(float* imgFT, int nImg, int idim, float rMask, float edge, float* rl,
                          thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && idim > 0 && idim % 2 == 0 && rMask > 0.f && edge > 0.f,
                  "thx_remask: bad arguments");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(imgFT && rl, "thx_remask: null argument");
    hipStream_t s = thx::as_stream(stream);
    const int N = idim;
    for (int l0 = 0; l0 < nImg; l0 += FFT_BATCH) {
        const int nb = nImg - l0 < FFT_BATCH ? nImg - l0 : FFT_BATCH;
        Plan2* p = nullptr;
        const int st = plans2(N, nb, s, &p);
        if (st != THX_OK) return st;
        float2* ft = reinterpret_cast<float2*>(imgFT) + (size_t)l0 * N * (N / 2 + 1);
        float* r = rl + (size_t)l0 * N * N;
        THX_FFT(hipfftExecC2R(p->c2r, reinterpret_cast<hipfftComplex*>(ft), r));
        hipLaunchKernelGGL(k_scale_mask_rl, dim3(2048), dim3(256), 0, s, r, nb, N, rMask, edge,
                           1.f / ((float)N * N));
        THX_LAUNCH_CHECK();
        THX_FFT(hipfftExecR2C(p->r2c, r, reinterpret_cast<hipfftComplex*>(ft)));
    }
    return THX_OK;
}

extern "C" int thx_img_gather(const float* imgFT, int nImg, int idim, const int* iPxl, int nPxl,
                              float* datP, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && idim > 0 && nPxl >= 0, "thx_img_gather: bad sizes");
    if (nImg == 0 || nPxl == 0) return THX_OK;
    THX_CHECK_ARG(imgFT && iPxl && datP, "thx_img_gather: null argument");
    hipLaunchKernelGGL(k_img_gather, dim3(2048), dim3(256), 0, thx::as_stream(stream),
                       reinterpret_cast<const float2*>(imgFT), nImg, (idim / 2 + 1) * idim, iPxl,
                       nPxl, reinterpret_cast<float2*>(datP));
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_ctf_image(const float* attr, int nImg, int idim, float* ctf,
                             thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && idim > 0 && idim % 2 == 0, "thx_ctf_image: bad sizes");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(attr && ctf, "thx_ctf_image: null argument");
    hipLaunchKernelGGL(k_ctf_image, dim3(2048), dim3(256), 0, thx::as_stream(stream), attr, nImg,
                       idim, ctf);
    THX_LAUNCH_CHECK();
    return THX_OK;
}
