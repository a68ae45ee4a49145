// scan_bf16x3.hip -- a7 + a8, algo 2: the global scan's cross term on the
// bf16 matrix cores with a three-product split (bf16x3).
//
// Same expansion as algo 1 (scan_mfma.hip): with |T| = 1
//   dvp[l][r][t] = A_l + B[l][r] + X[l][r][t],  A_l = sum s|d|^2,
//   B[l][r] = sum s c^2 |P_r|^2 (FP32),
//   X = sum_i Re(a conj(T P)) = sum_i Re(w_lri conj(T_ti)),  w = a conj(P_r),
//   a = -2 s c d.
// Regrouped this way, for one rotation X is a GEMM whose B operand is the
// translation table T -- the same for every rotation and image, split ONCE
// into bf16 hi/lo planes in the prep -- and whose A operand w = a conj(P_r)
// is formed per (image tile, rotation) in registers and split there.  Each
// generated A fragment is reused across all NF translation fragments, and
// each T fragment read from LDS feeds both image fragments of the wave.
// FP32 operands x = x_hi + x_lo (x_hi = bf16(x), x_lo = bf16(x - x_hi)) are
// multiplied as w_hi T_hi + w_hi T_lo + w_lo T_hi with FP32 accumulation on
// v_mfma_f32_32x32x16_bf16 (K = 16 = 8 pixels per instruction).  The
// dropped lo*lo term and the 16-bit split leave ~2^-16 relative error per
// product; summed over K = 2 nPxl terms of random sign that is ~1e-7 of
// |dvp|, the order of the reference's own sequential FP32 sum
// (tests/test_gpu_parity.py holds it to the same bar as algo 1).
//
// Workgroup = 8 waves = 8 rotations x 64 images; each wave owns a
// 64-image x NT_PAD-translation tile of ONE rotation (2 x NF accumulators
// of 32x32).  Epilogue: per-(image, rotation) max + wR marginal, then a
// block-local merge of the 8 rotations into a (max, wT[NT_PAD]) partial per
// image; k_scan_combine_bf folds the partials of all rotation blocks.
#include "common.h"
#include "scan_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int KC = 16;            // pixels per LDS stage (2 MFMA k-steps)
constexpr int IMG_TILE = 64;
constexpr int ROT_TILE = 8;
constexpr int THREADS = 512;
constexpr int TROW = KC * 2 + 8;  // bf16 per translation row of the T tile (80 B)
constexpr int APITCH = KC + 1;    // float2 per image row of the a tile (odd: conflict-free b64)
constexpr int BPITCH = KC + 1;    // float per image row of the b tile

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
    float2* Ac;     // [nCk][nImgPad][KC]   a = -2 s c d
    float* Bc;      // [nCk][nImgPad][KC]   b = s c^2
    float* Aconst;  // [nImgPad]
    __bf16* Thi;    // [nCk][nTPad][KC*2]   T split, (re, im) interleaved
    __bf16* Tlo;
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
    w.Ac = c.take<float2>((size_t)d.nPxlPad * d.nImgPad);
    w.Bc = c.take<float>((size_t)d.nPxlPad * d.nImgPad);
    w.Aconst = c.take<float>(d.nImgPad);
    w.Thi = c.take<__bf16>((size_t)d.nPxlPad * d.nTPad * 2);
    w.Tlo = c.take<__bf16>((size_t)d.nPxlPad * d.nTPad * 2);
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

// a, b in pixel-chunked image rows; pixel fastest so writes are contiguous
__global__ void __launch_bounds__(256) k_prep_img(const float2* __restrict__ dat,
                                                  const float* __restrict__ ctf,
                                                  const float* __restrict__ sig, int nImg,
                                                  int nPxl, int nImgPad, int nPxlPad,
                                                  float2* __restrict__ Ac,
                                                  float* __restrict__ Bc)
{
    const long n = (long)nImgPad * nPxlPad;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int i = (int)(q % nPxlPad), l = (int)(q / nPxlPad);
        float2 a = make_float2(0.f, 0.f);
        float b = 0.f;
        if (l < nImg && i < nPxl) {
            const size_t s = (size_t)l * nPxl + i;
            const float2 d = dat[s];
            const float c = ctf[s], sg = sig[s];
            const float k = -2.f * sg * c;
            a = make_float2(k * d.x, k * d.y);
            b = sg * c * c;
        }
        const size_t o = ((size_t)(i / KC) * nImgPad + l) * KC + (i % KC);
        Ac[o] = a;
        Bc[o] = b;
    }
}

__global__ void __launch_bounds__(256) k_prep_aconst2(const float2* __restrict__ dat,
                                                      const float* __restrict__ sig, int nImg,
                                                      int nPxl, int nImgPad,
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

__global__ void __launch_bounds__(256) k_prep_tsplit(const float2* __restrict__ traP,
                                                     const double* __restrict__ pT, int nT,
                                                     int nPxl, int nTPad, int nPxlPad,
                                                     __bf16* __restrict__ Thi,
                                                     __bf16* __restrict__ Tlo,
                                                     float* __restrict__ pTf)
{
    const long n = (long)nTPad * nPxlPad;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int i = (int)(q % nPxlPad), t = (int)(q / nPxlPad);
        const float2 v = (t < nT && i < nPxl) ? traP[(size_t)t * nPxl + i] : make_float2(0.f, 0.f);
        const size_t o = (((size_t)(i / KC) * nTPad + t) * KC + (i % KC)) * 2;
        __bf16 h, lo;
        split_bf16(v.x, h, lo); Thi[o] = h; Tlo[o] = lo;
        split_bf16(v.y, h, lo); Thi[o + 1] = h; Tlo[o + 1] = lo;
        if (i == 0) pTf[t] = t < nT ? (float)pT[t] : 0.f;
    }
}

template <int NF>
struct Smem {
    static constexpr int NTP = NF * 32;
    static constexpr int T_H = NTP * TROW;                 // bf16 per hi / lo plane
    static constexpr int A_F2 = IMG_TILE * APITCH;         // float2
    static constexpr int B_F = IMG_TILE * BPITCH;          // float
    static constexpr int P_F2 = ROT_TILE * KC;             // float2
    static constexpr int STAGE_B = 2 * T_H * 2 + A_F2 * 8 + B_F * 4 + P_F2 * 8;
    static constexpr int EPI_B = (ROT_TILE * 64 + ROT_TILE * 64 + 32 * NTP) * 4;
    static constexpr int TOTAL_B = STAGE_B > EPI_B ? STAGE_B : EPI_B;
    static constexpr int T16 = NTP * KC * 2 * 2 / 16;      // 16-B pieces per plane
};

template <int NF>
__global__ void __launch_bounds__(THREADS) k_scan_bf16x3(const float2* __restrict__ Ac,
                                                         const float* __restrict__ Bc,
                                                         const float* __restrict__ Aconst,
                                                         const __bf16* __restrict__ Thi,
                                                         const __bf16* __restrict__ Tlo,
                                                         const float2* __restrict__ rotP,
                                                         const float* __restrict__ pTf,
                                                         const double* __restrict__ pR,
                                                         int nImg, int nR, int nT, int nPxl,
                                                         int nImgPad, int nPxlPad, int nTPad,
                                                         float2* __restrict__ wRp,
                                                         float* __restrict__ pM,
                                                         float* __restrict__ pWT)
{
    using S = Smem<NF>;
    constexpr int NTP = S::NTP;
    __shared__ __attribute__((aligned(16))) char lds[S::TOTAL_B];
    __bf16* sTh = reinterpret_cast<__bf16*>(lds);                   // [NTP][TROW]
    __bf16* sTl = sTh + S::T_H;
    float2* sA = reinterpret_cast<float2*>(sTl + S::T_H);           // [64][APITCH]
    float* sB = reinterpret_cast<float*>(sA + S::A_F2);             // [64][BPITCH]
    float2* sP = reinterpret_cast<float2*>(sB + S::B_F);            // [8][KC]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = lane & 31, h = lane >> 5;
    const int l0 = blockIdx.x * IMG_TILE;
    const int rb = blockIdx.y;
    const int r = rb * ROT_TILE + w;        // this wave's rotation
    const bool rValid = r < nR;

    f32x16 acc[2][NF];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int f = 0; f < NF; f++)
#pragma unroll
            for (int j = 0; j < 16; j++) acc[a][f][j] = 0.f;
    float bsum = 0.f;                         // bias of image `lane`, rotation r

    // register-staged prefetch of one pixel chunk (global -> regs during the
    // previous chunk's MFMAs, regs -> LDS after the barrier)
    constexpr int TPER = (S::T16 + THREADS - 1) / THREADS;
    float4 gTh[TPER], gTl[TPER], gA;
    float4 gB = make_float4(0.f, 0.f, 0.f, 0.f);
    float2 gP = make_float2(0.f, 0.f);
    auto load_chunk = [&](int ck) {
        const float4* gh = reinterpret_cast<const float4*>(Thi + (size_t)ck * nTPad * KC * 2);
        const float4* gl = reinterpret_cast<const float4*>(Tlo + (size_t)ck * nTPad * KC * 2);
#pragma unroll
        for (int u = 0; u < TPER; u++) {
            const int x = tid + u * THREADS;
            if (x < S::T16) { gTh[u] = gh[x]; gTl[u] = gl[x]; }
        }
        gA = reinterpret_cast<const float4*>(Ac + ((size_t)ck * nImgPad + l0) * KC)[tid];
        if (tid < IMG_TILE * KC / 4)
            gB = reinterpret_cast<const float4*>(Bc + ((size_t)ck * nImgPad + l0) * KC)[tid];
        if (tid < ROT_TILE * KC) {
            const int qq = tid / KC, kc = tid % KC;
            const int rr = rb * ROT_TILE + qq, i = ck * KC + kc;
            gP = (rr < nR && i < nPxl) ? rotP[(size_t)rr * nPxl + i] : make_float2(0.f, 0.f);
        }
    };
    auto store_chunk = [&]() {
#pragma unroll
        for (int u = 0; u < TPER; u++) {
            const int x = tid + u * THREADS;
            if (x < S::T16) {                      // KC/4 pieces of 16 B per row
                const int row = x / (KC / 4), qd = x % (KC / 4);
                *reinterpret_cast<float4*>(sTh + row * TROW + qd * 8) = gTh[u];
                *reinterpret_cast<float4*>(sTl + row * TROW + qd * 8) = gTl[u];
            }
        }
        {                                          // 2 float2 of image row tid / (KC/2)
            const int row = tid / (KC / 2), c2 = (tid % (KC / 2)) * 2;
            sA[row * APITCH + c2] = make_float2(gA.x, gA.y);
            sA[row * APITCH + c2 + 1] = make_float2(gA.z, gA.w);
        }
        if (tid < IMG_TILE * KC / 4) {
            const int row = tid / (KC / 4), c4 = (tid % (KC / 4)) * 4;
            sB[row * BPITCH + c4] = gB.x; sB[row * BPITCH + c4 + 1] = gB.y;
            sB[row * BPITCH + c4 + 2] = gB.z; sB[row * BPITCH + c4 + 3] = gB.w;
        }
        if (tid < ROT_TILE * KC) sP[tid] = gP;
    };

    load_chunk(0);
    for (int ck = 0; ck * KC < nPxlPad; ck++) {
        __syncthreads();                   // previous chunk consumed
        store_chunk();
        __syncthreads();
        if ((ck + 1) * KC < nPxlPad) load_chunk(ck + 1);
#pragma unroll
        for (int kc = 0; kc < KC; kc++) {
            const float2 p = sP[w * KC + kc];
            bsum += sB[lane * BPITCH + kc] * (p.x * p.x + p.y * p.y);
        }
#pragma unroll
        for (int s = 0; s < KC / 8; s++) {
            // A fragments: w = a conj(P_r) for images a*32 + n, pixels 8s+4h+{0..3}
            bf16x8 wh[2], wl[2];
#pragma unroll
            for (int qd = 0; qd < 4; qd++) {
                const int px = 8 * s + 4 * h + qd;
                const float2 p = sP[w * KC + px];
#pragma unroll
                for (int a = 0; a < 2; a++) {
                    const float2 av = sA[(a * 32 + n) * APITCH + px];
                    const float wr = av.x * p.x + av.y * p.y;
                    const float wi = av.y * p.x - av.x * p.y;
                    __bf16 x0, x1;
                    split_bf16(wr, x0, x1); wh[a][2 * qd] = x0; wl[a][2 * qd] = x1;
                    split_bf16(wi, x0, x1); wh[a][2 * qd + 1] = x0; wl[a][2 * qd + 1] = x1;
                }
            }
#pragma unroll
            for (int f = 0; f < NF; f++) {
                const int row = (f * 32 + n) * TROW + 16 * s + 8 * h;
                const bf16x8 th = *reinterpret_cast<const bf16x8*>(sTh + row);
                const bf16x8 tl = *reinterpret_cast<const bf16x8*>(sTl + row);
#pragma unroll
                for (int a = 0; a < 2; a++) {
                    acc[a][f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[a], th, acc[a][f], 0, 0, 0);
                    acc[a][f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[a], tl, acc[a][f], 0, 0, 0);
                    acc[a][f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl[a], th, acc[a][f], 0, 0, 0);
                }
            }
        }
    }
    __syncthreads();

    // ------------------------------------------------------------ epilogue
    float* sBias = reinterpret_cast<float*>(lds);      // [8 waves][64]
    float* sMax = sBias + ROT_TILE * 64;               // [8 waves][64 rows]
    float* sWT = sMax + ROT_TILE * 64;                 // [32][NTP]
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
            const int row = a * 32 + (j & 3) + 8 * (j >> 2) + 4 * h;
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
                sMax[w * 64 + row] = mx;
                if (rValid && l < nImg) wRp[(size_t)l * nR + r] = make_float2(mx, sR);
            }
        }
    __syncthreads();

#pragma unroll
    for (int a = 0; a < 2; a++) {          // merge the 8 rotations, 32 image rows at a time
        for (int x = tid; x < 32 * NTP; x += THREADS) sWT[x] = 0.f;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int m = (j & 3) + 8 * (j >> 2) + 4 * h;
            const int row = a * 32 + m;
            float M = sMax[row];
#pragma unroll
            for (int k = 1; k < ROT_TILE; k++) M = fmaxf(M, sMax[k * 64 + row]);
            const float sc = rValid ? expf(sMax[w * 64 + row] - M) * pRr : 0.f;
#pragma unroll
            for (int f = 0; f < NF; f++) atomicAdd(&sWT[m * NTP + f * 32 + n], acc[a][f][j] * sc);
        }
        __syncthreads();
        for (int x = tid; x < 32 * NTP; x += THREADS) {
            const int m = x / NTP, t = x % NTP;
            const int row = a * 32 + m;
            const int l = l0 + row;
            pWT[((size_t)rb * nImgPad + l) * NTP + t] = sWT[x];
            if (t == 0) {
                float M = sMax[row];
#pragma unroll
                for (int k = 1; k < ROT_TILE; k++) M = fmaxf(M, sMax[k * 64 + row]);
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
    hipLaunchKernelGGL(k_scan_bf16x3<NF>, grid, dim3(THREADS), 0, s, ws.Ac, ws.Bc, ws.Aconst,
                       ws.Thi, ws.Tlo, reinterpret_cast<const float2*>(rotP), ws.pTf, pR,
                       d.nImg, d.nR, d.nT, d.nPxl, d.nImgPad, d.nPxlPad, d.nTPad, ws.wRp, ws.pM,
                       ws.pWT);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

}  // namespace

namespace thx {

int scan_mfma(const float* rotP, int nR, const float* traP, int nT, const float* dat,
              const float* ctf, const float* sigRcp, int nImg, int nPxl, const double* pR,
              const double* pT, int kIdx, int nK, float* wC, float* wR, float* wT,
              float* baseL, void* workspace, size_t wsBytes, hipStream_t stream);
size_t scan_mfma_workspace(int nImg, int nR, int nT, int nPxl);

size_t scan_bf16x3_workspace(int nImg, int nR, int nT, int nPxl)
{
    const Dims d = dims(nImg, nR, nT, nPxl);
    if (d.nTPad > 160) return scan_mfma_workspace(nImg, nR, nT, nPxl);
    return carve(nullptr, d).bytes;
}

int scan_bf16x3(const float* rotP, int nR, const float* traP, int nT, const float* dat,
                const float* ctf, const float* sigRcp, int nImg, int nPxl, const double* pR,
                const double* pT, int kIdx, int nK, float* wC, float* wR, float* wT,
                float* baseL, void* workspace, size_t wsBytes, hipStream_t s)
{
    const Dims d = dims(nImg, nR, nT, nPxl);
    if (d.nTPad > 160)   // 2 x NF accumulators no longer fit one wave: FP32 MFMA path
        return scan_mfma(rotP, nR, traP, nT, dat, ctf, sigRcp, nImg, nPxl, pR, pT, kIdx, nK,
                         wC, wR, wT, baseL, workspace, wsBytes, s);
    THX_CHECK_ARG(d.nRB <= 65535, "thx_global_scan(algo=2): grid too large");
    const WS ws = carve(workspace, d);
    THX_CHECK_ARG(ws.bytes <= wsBytes, "thx_global_scan(algo=2): workspace too small");
    const float2* dat2 = reinterpret_cast<const float2*>(dat);
    hipLaunchKernelGGL(k_prep_img, dim3(2048), dim3(256), 0, s, dat2, ctf, sigRcp, nImg, nPxl,
                       d.nImgPad, d.nPxlPad, ws.Ac, ws.Bc);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_prep_aconst2, dim3(thx::cdiv(d.nImgPad, 4)), dim3(256), 0, s, dat2,
                       sigRcp, nImg, nPxl, d.nImgPad, ws.Aconst);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_prep_tsplit, dim3(512), dim3(256), 0, s,
                       reinterpret_cast<const float2*>(traP), pT, nT, nPxl, d.nTPad, d.nPxlPad,
                       ws.Thi, ws.Tlo, ws.pTf);
    THX_LAUNCH_CHECK();
    int st;
    switch (d.nTPad / 32) {
        case 1: st = launch_main<1>(ws, d, rotP, pR, s); break;
        case 2: st = launch_main<2>(ws, d, rotP, pR, s); break;
        case 3: st = launch_main<3>(ws, d, rotP, pR, s); break;
        case 4: st = launch_main<4>(ws, d, rotP, pR, s); break;
        default: st = launch_main<5>(ws, d, rotP, pR, s); break;
    }
    if (st != THX_OK) return st;
    hipLaunchKernelGGL(k_scan_combine_bf, dim3(nImg), dim3(256), sizeof(float) * d.nRB, s,
                       ws.wRp, ws.pM, ws.pWT, pR, nR, nT, d.nTPad, d.nRB, d.nImgPad, kIdx, nK,
                       wC, wR, wT, baseL);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

}  // namespace thx
