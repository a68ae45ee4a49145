// scan_bf16x3.hip -- a7 + a8, algo 2: the global scan's cross term on the
// bf16 matrix cores with a three-product split (bf16x3).
//
// Same expansion as algo 1 (scan_mfma.hip):
//   dvp[l][r][t] = A_l + B[l][r] + sum_i a_li . z_rti,  a = -2 s c d,
//   z = T_t (.) P_r,  A_l = sum s|d|^2,  B[l][r] = sum s c^2 |P|^2 (FP32).
// Each FP32 operand is split as x = x_hi + x_lo with x_hi = bf16(x) and
// x_lo = bf16(x - x_hi), and the dot product is accumulated in FP32 as
//   a_hi z_hi + a_hi z_lo + a_lo z_hi
// on v_mfma_f32_32x32x16_bf16 (K = 16 = 8 pixels per instruction).  The
// dropped a_lo z_lo term and the 16-bit split leave a relative error of
// ~2^-16 per product; summed over K = 2 nPxl terms of random sign this is
// ~1e-7 of |dvp| -- the same order as the reference's own sequential FP32
// sum (tests/test_gpu_parity.py holds it to the same 1e-5 bar as algo 1).
// Three bf16 MFMAs cost 96 cycles per 8 pixels against 512 for eight FP32
// 32x32x2 MFMAs, so the matrix work drops ~5x.
//
// Workgroup = 4 waves = 4 rotations x 64 images; each wave holds 2 image
// fragments x NF translation fragments (2 NF accumulators of 32x32).
#include "common.h"
#include "scan_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int KC = 16;          // pixels per LDS stage (2 MFMA k-steps)
constexpr int IMG_TILE = 64;
constexpr int ROT_TILE = 4;
constexpr int THREADS = 256;
constexpr int AROW = KC * 2 + 8;   // bf16 per image row in LDS (80 B, bank spread)

inline int pad_to(int v, int m) { return (v + m - 1) / m * m; }

struct Dims {
    int nImg, nR, nT, nPxl, nImgPad, nPxlPad, nTPad, nRB, nCk;
};

Dims dims(int nImg, int nR, int nT, int nPxl)
{
    Dims d;
    d.nImg = nImg; d.nR = nR; d.nT = nT; d.nPxl = nPxl;
    d.nImgPad = pad_to(nImg, IMG_TILE);
    d.nPxlPad = pad_to(nPxl, KC);
    d.nTPad = pad_to(nT, 32);
    d.nRB = (nR + ROT_TILE - 1) / ROT_TILE;
    d.nCk = d.nPxlPad / KC;
    return d;
}

struct WS {
    __bf16* Ahi;    // [nCk][nImgPad][KC*2]
    __bf16* Alo;    // [nCk][nImgPad][KC*2]
    float* Bhat;    // [nPxlPad][nImgPad]
    float* Aconst;  // [nImgPad]
    float2* Tt;     // [nPxlPad][nTPad]
    float2* wRp;    // [nImg][nR]
    float* pM;      // [nRB][nImgPad]
    float* pWT;     // [nRB][nImgPad][nTPad]
    float* pTf;     // [nTPad]
    size_t bytes;
};

WS carve(void* base, const Dims& d)
{
    thx::Carver c(base, ~size_t(0));
    WS w;
    w.Ahi = c.take<__bf16>((size_t)d.nPxlPad * d.nImgPad * 2);
    w.Alo = c.take<__bf16>((size_t)d.nPxlPad * d.nImgPad * 2);
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

THX_DEV void split_bf16(float x, __bf16& hi, __bf16& lo)
{
    hi = (__bf16)x;
    lo = (__bf16)(x - (float)hi);
}

__global__ void __launch_bounds__(256) k_prep_bf(const float2* __restrict__ dat,
                                                 const float* __restrict__ ctf,
                                                 const float* __restrict__ sig, int nImg,
                                                 int nPxl, int nImgPad, int nPxlPad,
                                                 __bf16* __restrict__ Ahi,
                                                 __bf16* __restrict__ Alo,
                                                 float* __restrict__ Bhat)
{
    // thread per (image, pixel) with pixel fastest: the bf16 writes of one
    // image row are contiguous
    const long n = (long)nImgPad * nPxlPad;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int i = (int)(q % nPxlPad), l = (int)(q / nPxlPad);
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
        const size_t o = (((size_t)(i / KC) * nImgPad + l) * KC + (i % KC)) * 2;
        __bf16 h, lo;
        split_bf16(ar, h, lo); Ahi[o] = h; Alo[o] = lo;
        split_bf16(ai, h, lo); Ahi[o + 1] = h; Alo[o + 1] = lo;
        Bhat[(size_t)i * nImgPad + l] = b;
    }
}

__global__ void __launch_bounds__(256) k_prep_aconst_bf(const float2* __restrict__ dat,
                                                        const float* __restrict__ sig,
                                                        int nImg, int nPxl, int nImgPad,
                                                        float* __restrict__ Aconst)
{
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

__global__ void __launch_bounds__(256) k_prep_trans_bf(const float2* __restrict__ traP,
                                                       const double* __restrict__ pT, int nT,
                                                       int nPxl, int nTPad, int nPxlPad,
                                                       float2* __restrict__ Tt,
                                                       float* __restrict__ pTf)
{
    const long n = (long)nPxlPad * nTPad;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int t = (int)(q % nTPad), i = (int)(q / nTPad);
        Tt[q] = (t < nT && i < nPxl) ? traP[(size_t)t * nPxl + i] : make_float2(0.f, 0.f);
        if (i == 0) pTf[t] = t < nT ? (float)pT[t] : 0.f;
    }
}

template <int NF>
struct Smem {
    static constexpr int NTP = NF * 32;
    static constexpr int T_F = KC * NTP * 2;               // floats
    static constexpr int A_H = IMG_TILE * AROW;            // bf16 per part
    static constexpr int B_F = KC * IMG_TILE;
    static constexpr int P_F = ROT_TILE * KC * 2;
    static constexpr int STAGE_B = T_F * 4 + 2 * A_H * 2 + B_F * 4 + P_F * 4;
    static constexpr int EPI_B = (4 * 64 + 2 * 4 * 32 + 32 * NTP) * 4;
    static constexpr int TOTAL_B = STAGE_B > EPI_B ? STAGE_B : EPI_B;
};

template <int NF>
__global__ void __launch_bounds__(THREADS, NF <= 5 ? 2 : 1) k_scan_bf16x3(const __bf16* __restrict__ Ahi,
                                                            const __bf16* __restrict__ Alo,
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
    __shared__ __attribute__((aligned(16))) char lds[S::TOTAL_B];
    float2* sT = reinterpret_cast<float2*>(lds);                              // [KC][NTP]
    __bf16* sAh = reinterpret_cast<__bf16*>(lds + S::T_F * 4);                 // [64][AROW]
    __bf16* sAl = sAh + S::A_H;
    float* sB = reinterpret_cast<float*>(sAl + S::A_H);                        // [KC][64]
    float2* sP = reinterpret_cast<float2*>(sB + S::B_F);                       // [4][KC]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = lane & 31, h = lane >> 5;
    const int l0 = blockIdx.x * IMG_TILE;
    const int rb = blockIdx.y;
    const int r = rb * ROT_TILE + w;
    const bool rValid = r < nR;

    f32x16 acc[2][NF];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int f = 0; f < NF; f++)
#pragma unroll
            for (int j = 0; j < 16; j++) acc[a][f][j] = 0.f;
    float bsum = 0.f;

    for (int ck = 0; ck * KC < nPxlPad; ck++) {
        const int i0 = ck * KC;
        // ---- stage T, A (hi, lo), B, P
        {
            const float4* gT = reinterpret_cast<const float4*>(Tt + (size_t)i0 * NTP);
            float4* dT = reinterpret_cast<float4*>(sT);
            for (int x = tid; x < S::T_F / 4; x += THREADS) dT[x] = gT[x];
            const float4* gAh = reinterpret_cast<const float4*>(Ahi + ((size_t)ck * nImgPad + l0) * KC * 2);
            const float4* gAl = reinterpret_cast<const float4*>(Alo + ((size_t)ck * nImgPad + l0) * KC * 2);
            // 64 rows x 4 float4 (KC*2 bf16 = 64 B)
            {
                const int row = tid >> 2, qd = tid & 3;
                *reinterpret_cast<float4*>(sAh + row * AROW + qd * 8) = gAh[tid];
                *reinterpret_cast<float4*>(sAl + row * AROW + qd * 8) = gAl[tid];
            }
            {
                const int kc = tid >> 4, c4 = tid & 15;
                reinterpret_cast<float4*>(sB)[tid] =
                    reinterpret_cast<const float4*>(Bhat + (size_t)(i0 + kc) * nImgPad + l0)[c4];
            }
            if (tid < ROT_TILE * KC) {
                const int qq = tid / KC, kc = tid % KC;
                const int rr = rb * ROT_TILE + qq, i = i0 + kc;
                sP[tid] = (rr < nR && i < nPxl) ? rotP[(size_t)rr * nPxl + i] : make_float2(0.f, 0.f);
            }
        }
        __syncthreads();
        // bias: lane = image of the 64-image tile
#pragma unroll
        for (int kc = 0; kc < KC; kc++) {
            const float2 p = sP[w * KC + kc];
            bsum += sB[kc * IMG_TILE + lane] * (p.x * p.x + p.y * p.y);
        }
#pragma unroll
        for (int s = 0; s < KC / 8; s++) {
            bf16x8 ah[2], al[2];
#pragma unroll
            for (int a = 0; a < 2; a++) {
                ah[a] = *reinterpret_cast<const bf16x8*>(sAh + (a * 32 + n) * AROW + 16 * s + 8 * h);
                al[a] = *reinterpret_cast<const bf16x8*>(sAl + (a * 32 + n) * AROW + 16 * s + 8 * h);
            }
            float2 pv[4];
#pragma unroll
            for (int qd = 0; qd < 4; qd++) pv[qd] = sP[w * KC + 8 * s + 4 * h + qd];
#pragma unroll
            for (int f = 0; f < NF; f++) {
                bf16x8 bh, bl;
#pragma unroll
                for (int qd = 0; qd < 4; qd++) {
                    const float2 tv = sT[(8 * s + 4 * h + qd) * NTP + f * 32 + n];
                    const float zr = tv.x * pv[qd].x - tv.y * pv[qd].y;
                    const float zi = tv.x * pv[qd].y + tv.y * pv[qd].x;
                    __bf16 x0, x1;
                    split_bf16(zr, x0, x1); bh[2 * qd] = x0; bl[2 * qd] = x1;
                    split_bf16(zi, x0, x1); bh[2 * qd + 1] = x0; bl[2 * qd + 1] = x1;
                }
#pragma unroll
                for (int a = 0; a < 2; a++) {
                    acc[a][f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh, acc[a][f], 0, 0, 0);
                    acc[a][f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl, acc[a][f], 0, 0, 0);
                    acc[a][f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh, acc[a][f], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }

    // ------------------------------------------------------------ epilogue
    float* sBias = reinterpret_cast<float*>(lds);        // [4 waves][64]
    float* sMax = sBias + 4 * 64;                        // [2 halves][4][32]
    float* sWT = sMax + 2 * 4 * 32;                      // [32][NTP]
    sBias[w * 64 + lane] = bsum;
    __syncthreads();

    float pTv[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) pTv[f] = pTf[f * 32 + n];
    const float pRr = rValid ? (float)pR[r] : 0.f;

#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int m = (j & 3) + 8 * (j >> 2) + 4 * h;
            const int row = a * 32 + m;
            const int l = l0 + row;
            const float b = Aconst[l] + sBias[w * 64 + row];
            float mx = -INFINITY;
#pragma unroll
            for (int f = 0; f < NF; f++) {
                const float d = acc[a][f][j] + b;
                acc[a][f][j] = d;
                if (f * 32 + n < nT) mx = fmaxf(mx, d);
            }
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
            if (!rValid) mx = -INFINITY;
            float sR = 0.f;
#pragma unroll
            for (int f = 0; f < NF; f++) {
                const float e = (f * 32 + n < nT && rValid) ? expf(acc[a][f][j] - mx) : 0.f;
                acc[a][f][j] = e;
                sR += e * pTv[f];
            }
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) sR += __shfl_xor(sR, o, 64);
            if (n == 0) {
                sMax[(a * 4 + w) * 32 + m] = mx;
                if (rValid && l < nImg) wRp[(size_t)l * nR + r] = make_float2(mx, sR);
            }
        }
    __syncthreads();

#pragma unroll
    for (int a = 0; a < 2; a++) {
        for (int x = tid; x < 32 * NTP; x += THREADS) sWT[x] = 0.f;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int m = (j & 3) + 8 * (j >> 2) + 4 * h;
            const float M = fmaxf(fmaxf(sMax[(a * 4 + 0) * 32 + m], sMax[(a * 4 + 1) * 32 + m]),
                                  fmaxf(sMax[(a * 4 + 2) * 32 + m], sMax[(a * 4 + 3) * 32 + m]));
            const float sc = rValid ? expf(sMax[(a * 4 + w) * 32 + m] - M) * pRr : 0.f;
#pragma unroll
            for (int f = 0; f < NF; f++) atomicAdd(&sWT[m * NTP + f * 32 + n], acc[a][f][j] * sc);
        }
        __syncthreads();
        for (int x = tid; x < 32 * NTP; x += THREADS) {
            const int m = x / NTP, t = x % NTP;
            const int l = l0 + a * 32 + m;
            pWT[((size_t)rb * nImgPad + l) * NTP + t] = sWT[x];
            if (t == 0) {
                const float M = fmaxf(fmaxf(sMax[(a * 4 + 0) * 32 + m], sMax[(a * 4 + 1) * 32 + m]),
                                      fmaxf(sMax[(a * 4 + 2) * 32 + m], sMax[(a * 4 + 3) * 32 + m]));
                pM[(size_t)rb * nImgPad + l] = M;
            }
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) k_scan_combine_bf(const float2* __restrict__ wRp,
                                                         const float* __restrict__ pM,
                                                         const float* __restrict__ pWT,
                                                         const double* __restrict__ pR, int nR,
                                                         int nT, int nTPad, int nRB, int nImgPad,
                                                         int kIdx, int nK, float* __restrict__ wC,
                                                         float* __restrict__ wR,
                                                         float* __restrict__ wT,
                                                         float* __restrict__ baseL)
{
    extern __shared__ float sScale[];
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
int launch_main(const WS& ws, const Dims& d, const float* rotP, const double* pR, hipStream_t s)
{
    dim3 grid(d.nImgPad / IMG_TILE, d.nRB);
    hipLaunchKernelGGL(k_scan_bf16x3<NF>, grid, dim3(THREADS), 0, s, ws.Ahi, ws.Alo, ws.Bhat,
                       ws.Aconst, ws.Tt, reinterpret_cast<const float2*>(rotP), ws.pTf, pR,
                       d.nImg, d.nR, d.nT, d.nPxl, d.nImgPad, d.nPxlPad, ws.wRp, ws.pM, ws.pWT);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

}  // namespace

namespace thx {

size_t scan_bf16x3_workspace(int nImg, int nR, int nT, int nPxl)
{
    return carve(nullptr, dims(nImg, nR, nT, nPxl)).bytes;
}

int scan_bf16x3(const float* rotP, int nR, const float* traP, int nT, const float* dat,
                const float* ctf, const float* sigRcp, int nImg, int nPxl, const double* pR,
                const double* pT, int kIdx, int nK, float* wC, float* wR, float* wT,
                float* baseL, void* workspace, size_t wsBytes, hipStream_t s)
{
    const Dims d = dims(nImg, nR, nT, nPxl);
    THX_CHECK_ARG(d.nTPad <= 256, "thx_global_scan(algo=2): nT=%d > 256", nT);
    THX_CHECK_ARG(d.nRB <= 65535, "thx_global_scan(algo=2): grid too large");
    const WS ws = carve(workspace, d);
    THX_CHECK_ARG(ws.bytes <= wsBytes, "thx_global_scan(algo=2): workspace too small");
    const float2* dat2 = reinterpret_cast<const float2*>(dat);
    hipLaunchKernelGGL(k_prep_bf, dim3(2048), dim3(256), 0, s, dat2, ctf, sigRcp, nImg, nPxl,
                       d.nImgPad, d.nPxlPad, ws.Ahi, ws.Alo, ws.Bhat);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_prep_aconst_bf, dim3(thx::cdiv(d.nImgPad, 4)), dim3(256), 0, s, dat2,
                       sigRcp, nImg, nPxl, d.nImgPad, ws.Aconst);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_prep_trans_bf, dim3(512), dim3(256), 0, s,
                       reinterpret_cast<const float2*>(traP), pT, nT, nPxl, d.nTPad, d.nPxlPad,
                       ws.Tt, ws.pTf);
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
    hipLaunchKernelGGL(k_scan_combine_bf, dim3(nImg), dim3(256), sizeof(float) * d.nRB, s,
                       ws.wRp, ws.pM, ws.pWT, pR, nR, nT, d.nTPad, d.nRB, d.nImgPad, kIdx, nK,
                       wC, wR, wT, baseL);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

}  // namespace thx
