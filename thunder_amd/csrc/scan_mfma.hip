// scan_mfma.hip -- a7 + a8, algo 1: the global scan as an FP32 MFMA product.
//
// The likelihood of kernel_logDataVS / logDataVSPrior (gpu/src/Kernel.cu:
// 947-1004; src/Optimiser.cpp:9187-9213) expands, with |traP| = 1, into
//   dvp[l][r][t] = A_l + B[l][r] + X[l][(r,t)]
//   A_l        = sum_i s_li |d_li|^2
//   B[l][r]    = sum_i s_li c_li^2 |P_ri|^2
//   X[l][(r,t)] = sum_i (-2 s_li c_li d_li) . (T_ti P_ri)      (real dot of
//                 the complex pair (re, im) -> 2 K-steps per pixel)
// X is a real GEMM with M = images, N = (rotation, translation) pairs,
// K = 2 nPxl; its B operand Z = T (.) P is generated in registers from LDS
// tiles of traP and rotP, so the 2 GB pair matrix never exists.  It runs on
// v_mfma_f32_32x32x2_f32: exact FP32 products, FP32 accumulation (the same
// arithmetic class as the reference's FP32 sums), 4 flops per
// (image, rotation, translation, pixel) instead of 15 on the VALU.
//
// Workgroup = 8 waves = 2 image halves x 4 rotations; each wave owns a
// 32-image x NT_PAD-translation tile of ONE rotation (NF = NT_PAD/32
// accumulators of 32x32).  Epilogue: bias, per-(image, rotation) max and
// wR marginal, then a block-local merge of the 4 rotations into a
// (max, wT[NT_PAD]) partial per image; a combine kernel folds the partials
// of all rotation blocks with exp(m_b - base) rescaling -- the same result as
// the CPU online baseline (src/Optimiser.cpp:834-894) evaluated at its final
// baseline.
#include "common.h"
#include "scan_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int KC = 16;        // pixels per LDS stage
constexpr int IMG_TILE = 64;  // images per workgroup
constexpr int ROT_TILE = 4;   // rotations per workgroup (one per wave column)
constexpr int THREADS = 512;

inline int pad_to(int v, int m) { return (v + m - 1) / m * m; }

struct Dims {
    int nImg, nR, nT, nPxl;
    int nImgPad, nPxlPad, nTPad, nRB;
};

Dims dims(int nImg, int nR, int nT, int nPxl)
{
    Dims d;
    d.nImg = nImg; d.nR = nR; d.nT = nT; d.nPxl = nPxl;
    d.nImgPad = pad_to(nImg, IMG_TILE);
    d.nPxlPad = pad_to(nPxl, KC);
    d.nTPad = pad_to(nT, 32);
    d.nRB = (nR + ROT_TILE - 1) / ROT_TILE;
    return d;
}

struct WS {
    float* Ahat;    // [nPxlPad][2][nImgPad]   -2 s c d (re plane, im plane)
    float* Bhat;    // [nPxlPad][nImgPad]      s c^2
    float* Aconst;  // [nImgPad]               sum s |d|^2
    float2* Tt;     // [nPxlPad][nTPad]        traP transposed, zero padded
    float2* wRp;    // [nImg][nR]              (max_t dvp, sum_t e^(dvp-max) pT)
    float* pM;      // [nRB][nImgPad]          block max
    float* pWT;     // [nRB][nImgPad][nTPad]   block wT relative to pM
    float* pTf;     // [nTPad]                 pT as float, 0 in padding
    size_t bytes;
};

WS carve(void* base, const Dims& d)
{
    thx::Carver c(base, ~size_t(0));
    WS w;
    w.Ahat = c.take<float>((size_t)d.nPxlPad * 2 * d.nImgPad);
    w.Bhat = c.take<float>((size_t)d.nPxlPad * d.nImgPad);
    w.Aconst = c.take<float>(d.nImgPad);
    w.Tt = c.take<float2>((size_t)d.nPxlPad * d.nTPad);
    w.wRp = c.take<float2>((size_t)d.nImg * d.nR);
    w.pM = c.take<float>((size_t)d.nRB * d.nImgPad);
    w.pWT = c.take<float>((size_t)d.nRB * d.nImgPad * d.nTPad);
    w.pTf = c.take<float>(d.nTPad);
    w.bytes = c.off + 256;
    return w;
}

// ---------------------------------------------------------------- prep ---
// Pixel-major, zero-padded operands.  One thread per (pixel, image), image
// fastest so the writes are coalesced.
__global__ void __launch_bounds__(256) k_prep_images(const float2* __restrict__ dat,
                                                     const float* __restrict__ ctf,
                                                     const float* __restrict__ sig,
                                                     int nImg, int nPxl, int nImgPad,
                                                     int nPxlPad,
                                                     float* __restrict__ Ahat,
                                                     float* __restrict__ Bhat)
{
    const long n = (long)nPxlPad * nImgPad;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int l = (int)(q % nImgPad), i = (int)(q / nImgPad);
        float ar = 0.f, ai = 0.f, b = 0.f;
        if (l < nImg && i < nPxl) {
            const size_t s = (size_t)l * nPxl + i;
            const float2 d = dat[s];
            const float c = ctf[s], sg = sig[s];
            const float k = -2.f * sg * c;
            ar = k * d.x;
            ai = k * d.y;
            b = sg * c * c;
        }
        Ahat[((size_t)i * 2 + 0) * nImgPad + l] = ar;
        Ahat[((size_t)i * 2 + 1) * nImgPad + l] = ai;
        Bhat[(size_t)i * nImgPad + l] = b;
    }
}

__global__ void __launch_bounds__(256) k_prep_aconst(const float2* __restrict__ dat,
                                                     const float* __restrict__ sig,
                                                     int nImg, int nPxl, int nImgPad,
                                                     float* __restrict__ Aconst)
{
    // one wave per image
    const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (l >= nImgPad) return;
    float a = 0.f;
    if (l < nImg)
        for (int i = lane; i < nPxl; i += 64) {
            const float2 d = dat[(size_t)l * nPxl + i];
            a += sig[(size_t)l * nPxl + i] * (d.x * d.x + d.y * d.y);
        }
    a = wave_sum(a);
    if (lane == 0) Aconst[l] = a;
}

__global__ void __launch_bounds__(256) k_prep_trans(const float2* __restrict__ traP,
                                                    const double* __restrict__ pT,
                                                    int nT, int nPxl, int nTPad,
                                                    int nPxlPad,
                                                    float2* __restrict__ Tt,
                                                    float* __restrict__ pTf)
{
    const long n = (long)nPxlPad * nTPad;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int t = (int)(q % nTPad), i = (int)(q / nTPad);
        float2 v = make_float2(0.f, 0.f);
        if (t < nT && i < nPxl) v = traP[(size_t)t * nPxl + i];
        Tt[q] = v;
        if (i == 0) pTf[t] = t < nT ? (float)pT[t] : 0.f;
    }
}

// ---------------------------------------------------------------- main ---
template <int NF>
struct Smem {
    static constexpr int NTP = NF * 32;
    // staging: T [KC][NTP] float2 | A [KC][2][64] | B [KC][64] | P [ROT_TILE][KC] float2
    static constexpr int T_F = KC * NTP * 2;
    static constexpr int P_F = ROT_TILE * KC * 2;
    static constexpr int A_F = KC * 2 * IMG_TILE;
    static constexpr int B_F = KC * IMG_TILE;
    static constexpr int STAGE_F = T_F + P_F + A_F + B_F;
    // epilogue: bias[8][32] | rmax[2][4][32] | wT[32][NTP]
    static constexpr int EPI_F = 8 * 32 + 2 * 4 * 32 + 2 * 32 * NTP;   // sWT: u64
    static constexpr int TOTAL_F = STAGE_F > EPI_F ? STAGE_F : EPI_F;
    static constexpr int T4 = T_F / 4, A4 = A_F / 4, B4 = B_F / 4;
    static constexpr int G4 = T4 + A4 + B4;          // float4 loads per stage
    static constexpr int G4_PER_THREAD = (G4 + THREADS - 1) / THREADS;
};

template <int NF>
__global__ void __launch_bounds__(THREADS) k_scan_mfma(const float* __restrict__ Ahat,
                                                       const float* __restrict__ Bhat,
                                                       const float* __restrict__ Aconst,
                                                       const float2* __restrict__ Tt,
                                                       const float2* __restrict__ rotP,
                                                       const float* __restrict__ pTf,
                                                       const double* __restrict__ pR,
                                                       int nImg, int nR, int nT, int nPxl,
                                                       int nImgPad, int nPxlPad,
                                                       float2* __restrict__ wRp,
                                                       float* __restrict__ pM,
                                                       float* __restrict__ pWT)
{
    using S = Smem<NF>;
    constexpr int NTP = S::NTP;
    __shared__ __attribute__((aligned(16))) float lds[S::TOTAL_F];
    float* sT = lds;                 // T | A | B contiguous: one float4 image
    float* sA = sT + S::T_F;
    float* sB = sA + S::A_F;
    float* sP = sB + S::B_F;

    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    const int q = w & 3, h = w >> 2;    // rotation column, image half
    const int n = lane & 31, kk = lane >> 5;
    const int l0 = blockIdx.x * IMG_TILE;
    const int rb = blockIdx.y;
    const int r = rb * ROT_TILE + q;
    const bool rValid = r < nR;

    f32x16 acc[NF];
#pragma unroll
    for (int f = 0; f < NF; f++)
#pragma unroll
        for (int j = 0; j < 16; j++) acc[f][j] = 0.f;
    float bsum = 0.f;

    // register-staged prefetch of one KC chunk (T, A, B as float4; P as float2)
    float4 g[S::G4_PER_THREAD];
    float2 gp = make_float2(0.f, 0.f);
    auto load_chunk = [&](int i0) {
#pragma unroll
        for (int u = 0; u < S::G4_PER_THREAD; u++) {
            const int x = tid + u * THREADS;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (x < S::T4) {
                v = reinterpret_cast<const float4*>(Tt + (size_t)i0 * NTP)[x];
            } else if (x < S::T4 + S::A4) {
                const int y = x - S::T4;               // [kc][k][16 float4]
                const int kc = y / 32, k2 = (y / 16) & 1, c4 = y & 15;
                v = reinterpret_cast<const float4*>(
                    Ahat + ((size_t)(i0 + kc) * 2 + k2) * nImgPad + l0)[c4];
            } else if (x < S::G4) {
                const int y = x - S::T4 - S::A4;       // [kc][16 float4]
                const int kc = y / 16, c4 = y & 15;
                v = reinterpret_cast<const float4*>(
                    Bhat + (size_t)(i0 + kc) * nImgPad + l0)[c4];
            }
            g[u] = v;
        }
        if (tid < ROT_TILE * KC) {
            const int qq = tid / KC, kc = tid % KC;
            const int rr = rb * ROT_TILE + qq, i = i0 + kc;
            gp = (rr < nR && i < nPxl) ? rotP[(size_t)rr * nPxl + i]
                                       : make_float2(0.f, 0.f);
        }
    };
    auto store_chunk = [&]() {
#pragma unroll
        for (int u = 0; u < S::G4_PER_THREAD; u++) {
            const int x = tid + u * THREADS;
            if (x < S::G4) reinterpret_cast<float4*>(sT)[x] = g[u];
        }
        if (tid < ROT_TILE * KC) reinterpret_cast<float2*>(sP)[tid] = gp;
    };

    load_chunk(0);
    for (int i0 = 0; i0 < nPxlPad; i0 += KC) {
        __syncthreads();               // previous chunk fully consumed
        store_chunk();
        __syncthreads();
        if (i0 + KC < nPxlPad) load_chunk(i0 + KC);
#pragma unroll 4
        for (int kc = 0; kc < KC; kc++) {
            const float a = sA[(kc * 2 + kk) * IMG_TILE + h * 32 + n];
            const float2 p = reinterpret_cast<const float2*>(sP)[q * KC + kc];
            if (kk == 0) bsum += sB[kc * IMG_TILE + h * 32 + n] * (p.x * p.x + p.y * p.y);
            // Z = T * P; lane half kk = 0 takes Re, kk = 1 takes Im.
            const float u = kk ? p.y : p.x;
            const float v = kk ? p.x : -p.y;
#pragma unroll
            for (int f = 0; f < NF; f++) {
                const float2 tv = reinterpret_cast<const float2*>(sT)[kc * NTP + f * 32 + n];
                const float z = tv.x * u + tv.y * v;
                acc[f] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, z, acc[f], 0, 0, 0);
            }
        }
    }
    __syncthreads();

    // ------------------------------------------------------------ epilogue
    float* sBias = lds;                  // [8 waves][32]
    float* sMax = sBias + 8 * 32;        // [2][4][32]
    // [32][NTP] 2^56 fixed point (the 4 rotations' terms lie in [0, 1])
    unsigned long long* sWT = reinterpret_cast<unsigned long long*>(sMax + 2 * 4 * 32);
    if (kk == 0) sBias[w * 32 + n] = bsum;
    __syncthreads();

    float pTv[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) pTv[f] = pTf[f * 32 + n];
    const float pRr = rValid ? (float)pR[r] : 0.f;

    float rmax[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int m = (j & 3) + 8 * (j >> 2) + 4 * kk;
        const int l = l0 + h * 32 + m;
        const float b = Aconst[l] + sBias[w * 32 + m];
        float mx = -INFINITY;
#pragma unroll
        for (int f = 0; f < NF; f++) {
            const float d = acc[f][j] + b;
            acc[f][j] = d;
            if (f * 32 + n < nT) mx = fmaxf(mx, d);
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        if (!rValid) mx = -INFINITY;
        rmax[j] = mx;
        float sR = 0.f;
#pragma unroll
        for (int f = 0; f < NF; f++) {
            const float e = (f * 32 + n < nT && rValid) ? __expf(acc[f][j] - mx) : 0.f;
            acc[f][j] = e;
            sR += e * pTv[f];
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) sR += __shfl_xor(sR, o, 64);
        if (n == 0) {
            sMax[(h * 4 + q) * 32 + m] = mx;
            if (rValid && l < nImg) wRp[(size_t)l * nR + r] = make_float2(mx, sR);
        }
    }
    __syncthreads();

    // merge the 4 rotations of this block, one image half at a time
    for (int hh = 0; hh < 2; hh++) {
        for (int x = tid; x < 32 * NTP; x += THREADS) sWT[x] = 0ull;
        __syncthreads();
        if (h == hh) {
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const int m = (j & 3) + 8 * (j >> 2) + 4 * kk;
                const float M = fmaxf(fmaxf(sMax[(h * 4 + 0) * 32 + m], sMax[(h * 4 + 1) * 32 + m]),
                                      fmaxf(sMax[(h * 4 + 2) * 32 + m], sMax[(h * 4 + 3) * 32 + m]));
                const float sc = rValid ? __expf(rmax[j] - M) * pRr : 0.f;
#pragma unroll
                for (int f = 0; f < NF; f++)
                    atomicAdd(&sWT[m * NTP + f * 32 + n], fx56(acc[f][j] * sc));
            }
        }
        __syncthreads();
        for (int x = tid; x < 32 * NTP; x += THREADS) {
            const int m = x / NTP, t = x % NTP;
            const int l = l0 + hh * 32 + m;
            pWT[((size_t)rb * nImgPad + l) * NTP + t] = unfx56(sWT[x]);
            if (t == 0) {
                const float M = fmaxf(fmaxf(sMax[(hh * 4 + 0) * 32 + m], sMax[(hh * 4 + 1) * 32 + m]),
                                      fmaxf(sMax[(hh * 4 + 2) * 32 + m], sMax[(hh * 4 + 3) * 32 + m]));
                pM[(size_t)rb * nImgPad + l] = M;
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------- combine ---
__global__ void __launch_bounds__(256) k_scan_combine(const float2* __restrict__ wRp,
                                                      const float* __restrict__ pM,
                                                      const float* __restrict__ pWT,
                                                      const double* __restrict__ pR,
                                                      int nR, int nT, int nTPad,
                                                      int nRB, int nImgPad, int kIdx,
                                                      int nK, float* __restrict__ wC,
                                                      float* __restrict__ wR,
                                                      float* __restrict__ wT,
                                                      float* __restrict__ baseL)
{
    extern __shared__ float sScale[];   // [nRB]
    __shared__ float sm[4];
    __shared__ double sd[4];
    const int l = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float m = -INFINITY;
    for (int b = threadIdx.x; b < nRB; b += blockDim.x) m = fmaxf(m, pM[(size_t)b * nImgPad + l]);
    m = wave_max(m);
    if (lane == 0) sm[wv] = m;
    __syncthreads();
    m = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    const float base = merge_baseline(l, m, kIdx, nK, nR, nT, wC, wR, wT, baseL);
    for (int b = threadIdx.x; b < nRB; b += blockDim.x)
        sScale[b] = expf(pM[(size_t)b * nImgPad + l] - base);
    __syncthreads();
    float* wTl = wT + ((size_t)l * nK + kIdx) * nT;
    for (int t = threadIdx.x; t < nT; t += blockDim.x) {
        double a = 0.0;
        for (int b = 0; b < nRB; b++)
            a += (double)(sScale[b] * pWT[((size_t)b * nImgPad + l) * nTPad + t]);
        wTl[t] = (float)a;
    }
    float* wRl = wR + ((size_t)l * nK + kIdx) * nR;
    double c = 0.0;
    for (int r = threadIdx.x; r < nR; r += blockDim.x) {
        const float2 v = wRp[(size_t)l * nR + r];
        const float x = expf(v.x - base) * v.y;
        wRl[r] = x;
        c += (double)x * pR[r];
    }
    c = wave_sum(c);
    if (lane == 0) sd[wv] = c;
    __syncthreads();
    if (threadIdx.x == 0) wC[(size_t)l * nK + kIdx] = (float)(sd[0] + sd[1] + sd[2] + sd[3]);
}

template <int NF>
int launch_main(const WS& ws, const Dims& d, const float* rotP, const double* pR,
                hipStream_t s)
{
    dim3 grid(d.nImgPad / IMG_TILE, d.nRB);
    hipLaunchKernelGGL(k_scan_mfma<NF>, grid, dim3(THREADS), 0, s, ws.Ahat,
                       ws.Bhat, ws.Aconst, ws.Tt,
                       reinterpret_cast<const float2*>(rotP), ws.pTf, pR,
                       d.nImg, d.nR, d.nT, d.nPxl, d.nImgPad, d.nPxlPad, ws.wRp,
                       ws.pM, ws.pWT);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

}  // namespace

namespace thx {

size_t scan_mfma_workspace(int nImg, int nR, int nT, int nPxl)
{
    return carve(nullptr, dims(nImg, nR, nT, nPxl)).bytes;
}

int scan_mfma(const float* rotP, int nR, const float* traP, int nT,
              const float* dat, const float* ctf, const float* sigRcp,
              int nImg, int nPxl, const double* pR, const double* pT, int kIdx,
              int nK, float* wC, float* wR, float* wT, float* baseL,
              void* workspace, size_t wsBytes, hipStream_t s)
{
    const Dims d = dims(nImg, nR, nT, nPxl);
    THX_CHECK_ARG(d.nTPad <= 256, "thx_global_scan(algo=1): nT=%d > 256", nT);
    THX_CHECK_ARG(d.nImgPad / IMG_TILE <= 0x7fffffff && d.nRB <= 65535,
                  "thx_global_scan(algo=1): grid too large");
    const WS ws = carve(workspace, d);
    THX_CHECK_ARG(ws.bytes <= wsBytes, "thx_global_scan(algo=1): workspace too small");
    const float2* dat2 = reinterpret_cast<const float2*>(dat);
    hipLaunchKernelGGL(k_prep_images, dim3(2048), dim3(256), 0, s, dat2, ctf,
                       sigRcp, nImg, nPxl, d.nImgPad, d.nPxlPad, ws.Ahat, ws.Bhat);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_prep_aconst, dim3(thx::cdiv(d.nImgPad, 4)), dim3(256), 0,
                       s, dat2, sigRcp, nImg, nPxl, d.nImgPad, ws.Aconst);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_prep_trans, dim3(512), dim3(256), 0, s,
                       reinterpret_cast<const float2*>(traP), pT, nT, nPxl,
                       d.nTPad, d.nPxlPad, ws.Tt, ws.pTf);
    THX_LAUNCH_CHECK();
    int st;
    switch (d.nTPad / 32) {
        case 1: st = launch_main<1>(ws, d, rotP, pR, s); break;
        case 2: st = launch_main<2>(ws, d, rotP, pR, s); break;
        case 3: st = launch_main<3>(ws, d, rotP, pR, s); break;
        case 4: st = launch_main<4>(ws, d, rotP, pR, s); break;
        case 5: st = launch_main<5>(ws, d, rotP, pR, s); break;
        case 6: st = launch_main<6>(ws, d, rotP, pR, s); break;
        case 7: st = launch_main<7>(ws, d, rotP, pR, s); break;
        default: st = launch_main<8>(ws, d, rotP, pR, s); break;
    }
    if (st != THX_OK) return st;
    hipLaunchKernelGGL(k_scan_combine, dim3(nImg), dim3(256),
                       sizeof(float) * d.nRB, s, ws.wRp, ws.pM, ws.pWT, pR, nR,
                       nT, d.nTPad, d.nRB, d.nImgPad, kIdx, nK, wC, wR, wT, baseL);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

}  // namespace thx
