// scan_split.hip -- a7 + a8 on 16-bit matrix cores: the global scan's cross
// term with FP32 operands split into 16-bit pieces.
//   algo 4 (BF16X6, the product path): every FP32 operand split EXACTLY into
//                    three bf16 (x = hi + mid + lo: 8 + 8 + 8 significant
//                    bits, |mid| <= 2^-8 |x|, |lo| <= 2^-16 |x|), six products
//                    (hh, hm, mh, hl, mm, lh); of the three dropped, ml and lm
//                    are <= 2^-24 |w||T| each (ll <= 2^-32), about 2^-23
//                    together: comparable to the FP32 rounding of one product
//                    (2^-24); FP32 accumulation;
//   algo 2 (BF16X3): bf16 hi/lo of both operands, three products
//                    (hi hi + hi lo + lo hi), ~2^-16 relative per product;
//
// Same expansion as algo 1 (scan_mfma.hip): with |T| = 1
//   dvp[l][r][t] = A_l + B[l][r] + X[l][r][t],  A_l = sum s|d|^2,
//   B[l][r] = sum s c^2 |P_r|^2 (FP32, its own small GEMM: k_scan_bias),
//   X = sum_i Re(a conj(T P)) = sum_i Re(w_lri conj(T_ti)),  w = a conj(P_r),
//   a = -2 s c d.
// For one rotation X is a GEMM whose B operand is the translation table T --
// the same for every rotation and image, split ONCE in the prep -- and whose A
// operand w = a conj(P_r) is formed per (image tile, rotation) in registers
// and split there.  Each generated A fragment is reused across all NF
// translation fragments, and each T fragment read from LDS feeds both image
// fragments of the wave.
//
// Workgroup = 8 waves = 8 rotations x 64 images; each wave owns a
// 64-image x NT_PAD-translation tile of ONE rotation (2 x NF accumulators
// of 32x32).  Per 16-pixel chunk a wave reads its a / P operands with four
// ds_read_b128 and the T fragments with NF (fp16) or 2 NF (bf16) more.
// Epilogue: per-(image, rotation) max + wR marginal, then a block-local merge
// of the 8 rotations into a (max, wT[NT_PAD]) partial per image;
// k_scan_combine_bf folds the partials of all rotation blocks.
#include "common.h"
#include "scan_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum Mode { BF16X3 = 0, BF16X6 = 2 };
typedef __bf16 H;
typedef bf16x8 HV;

// planes of the translation table staged per chunk
template <int MODE> constexpr int nplane() { return MODE == BF16X6 ? 3 : 2; }

// Cancellation guard of the expanded form dvp = (A + B) + X: where
// |A| + |B| + |X| > SCAN_GUARD |dvp| (signal-dominated samples near the true
// pose) the expansion loses log2 of that ratio in bits to cancellation, so
// those samples are recomputed in the reference's direct form.
constexpr float SCAN_GUARD = 4.f;
constexpr int GCAP = 32;   // guard list entries per wave and round

constexpr int KC = 16;            // pixels per LDS stage (KC / 8 MFMA k-steps)
static_assert(KC % 16 == 0, "whole float4 rows per thread in the stagers");
constexpr int IMG_TILE = 64;
constexpr int ROT_TILE = 8;       // rotations per workgroup, one per wave
constexpr int THREADS = 64 * ROT_TILE;
constexpr int NWAVE = ROT_TILE;
constexpr int TROW = KC * 2 + 8;  // 16-bit elements per translation row of the T tile (80 B)
constexpr int APITCH = KC + 2;    // float2 per image row of the a tile (144 B: aligned, conflict-free b128)

inline int pad_to(int v, int m) { return (v + m - 1) / m * m; }

struct Dims {
    int nImg, nR, nT, nPxl, nImgPad, nPxlPad, nTPad, nRB, nCk, nRBias;
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
    d.nRBias = pad_to(nR, 64);
    return d;
}

struct WS {
    float2* Ac;     // [nCk][nImgPad][APITCH]  a = -2 s c d, LDS image
    float* Bc;      // [nCk][nImgPad][KC]   b = s c^2
    float* Aconst;  // [nImgPad]
    float* bias;    // [nImgPad][nRBias]  B[l][r]
    uint16_t* Thi;  // [nCk][nTPad][TROW]   T split, (re, im) interleaved, LDS image
    uint16_t* Tlo;  //   second plane (lo of bf16x3, mid of bf16x6)
    uint16_t* Tl2;  //   third plane (lo of bf16x6)
    float2* Pc;     // [nCk][nRB * ROT_TILE][KC]  projections, chunk-major
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
    w.Ac = c.take<float2>((size_t)d.nCk * d.nImgPad * APITCH);
    w.Bc = c.take<float>((size_t)d.nPxlPad * d.nImgPad);
    w.Aconst = c.take<float>(d.nImgPad);
    w.bias = c.take<float>((size_t)d.nImgPad * d.nRBias);
    w.Thi = c.take<uint16_t>((size_t)d.nCk * d.nTPad * TROW);
    w.Tlo = c.take<uint16_t>((size_t)d.nCk * d.nTPad * TROW);
    w.Tl2 = c.take<uint16_t>((size_t)d.nCk * d.nTPad * TROW);
    w.Pc = c.take<float2>((size_t)d.nCk * d.nRB * ROT_TILE * KC);
    w.wRp = c.take<float2>((size_t)d.nImg * d.nR);
    w.pM = c.take<float>((size_t)d.nRB * d.nImgPad);
    w.pWT = c.take<float>((size_t)d.nRB * d.nImgPad * d.nTPad);
    w.pTf = c.take<float>(d.nTPad);
    w.bytes = c.off + 256;
    return w;
}

template <typename H>
THX_DEV void split16(float x, H& hi, H& lo)
{
    hi = (H)x;
    lo = (H)(x - (float)hi);
}

// x = hi + mid + lo exactly: hi takes the top 8 significant bits, the
// residual x - hi (exact in FP32) keeps at most 16, mid the next 8, and the
// residual after mid (again exact) at most 8, which lo holds exactly.
THX_DEV void split3(float x, __bf16& hi, __bf16& mid, __bf16& lo)
{
    hi = (__bf16)x;
    const float r = x - (float)hi;
    mid = (__bf16)r;
    lo = (__bf16)(r - (float)mid);
}

// split3 of a (re, im) pair, each level one packed round (v_cvt_pk_bf16_f32),
// two unpacking bit operations and one packed subtraction: the same three
// planes as split3 on each component, (re, im) interleaved per plane
typedef float f2v __attribute__((ext_vector_type(2)));
THX_DEV void split3x2(f2v x, uint32_t& hi, uint32_t& mid, uint32_t& lo)
{
    auto pk = [](float a, float b) { return __builtin_bit_cast(uint32_t, bf16x2{(__bf16)a, (__bf16)b}); };
    auto unpk = [](uint32_t v) { return f2v{__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)}; };
    // (the empty asm keeps each packed level opaque: left visible, the
    // compiler re-derives its low half by a second v_cvt_pk_bf16_f32)
    hi = pk(x.x, x.y);
    asm volatile("" : "+v"(hi));
    const f2v r = x - unpk(hi);
    mid = pk(r.x, r.y);
    asm volatile("" : "+v"(mid));
    const f2v r2 = r - unpk(mid);
    lo = pk(r2.x, r2.y);
}

// Per image: A_l = sum s|d|^2
__global__ void __launch_bounds__(256) k_prep_aconst(const float2* __restrict__ dat,
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
            const size_t s = (size_t)l * nPxl + i;
            const float2 d = dat[s];
            a += sig[s] * (d.x * d.x + d.y * d.y);
        }
    a = wave_sum(a);
    if (lane == 0) Aconst[l] = a;
}

// a, b in pixel-chunked image rows; pixel fastest so writes are contiguous
__global__ void __launch_bounds__(256) k_prep_img(const float2* __restrict__ dat,
                                                  const float* __restrict__ ctf,
                                                  const float* __restrict__ sig,
                                                  int nImg,
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
        Ac[((size_t)(i / KC) * nImgPad + l) * APITCH + (i % KC)] = a;
        Bc[((size_t)(i / KC) * nImgPad + l) * KC + (i % KC)] = b;
    }
}

// P rows regrouped chunk-major so one rotation block's chunk is contiguous
// (KC / 16 KiB; zero past nR / nPxl)
__global__ void __launch_bounds__(256) k_prep_pchunk(const float2* __restrict__ rotP, int nR,
                                                     int nPxl, int nRRows, int nPxlPad,
                                                     float2* __restrict__ Pc)
{
    const long n = (long)nRRows * nPxlPad;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int i = (int)(q % nPxlPad), r = (int)(q / nPxlPad);
        Pc[((size_t)(i / KC) * nRRows + r) * KC + (i % KC)] =
            (r < nR && i < nPxl) ? rotP[(size_t)r * nPxl + i] : make_float2(0.f, 0.f);
    }
}

template <int MODE>
__global__ void __launch_bounds__(256) k_prep_tsplit(const float2* __restrict__ traP,
                                                     const double* __restrict__ pT, int nT,
                                                     int nPxl, int nTPad, int nPxlPad,
                                                     uint16_t* __restrict__ Thi,
                                                     uint16_t* __restrict__ Tlo,
                                                     uint16_t* __restrict__ Tl2,
                                                     float* __restrict__ pTf)
{
    const long n = (long)nTPad * nPxlPad;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int i = (int)(q % nPxlPad), t = (int)(q / nPxlPad);
        const float2 v = (t < nT && i < nPxl) ? traP[(size_t)t * nPxl + i] : make_float2(0.f, 0.f);
        const size_t o = ((size_t)(i / KC) * nTPad + t) * TROW + (i % KC) * 2;
        H h, lo;
        if constexpr (MODE == BF16X6) {
            H m;
            split3(v.x, h, m, lo);
            Thi[o] = __builtin_bit_cast(uint16_t, h);
            Tlo[o] = __builtin_bit_cast(uint16_t, m);
            Tl2[o] = __builtin_bit_cast(uint16_t, lo);
            split3(v.y, h, m, lo);
            Thi[o + 1] = __builtin_bit_cast(uint16_t, h);
            Tlo[o + 1] = __builtin_bit_cast(uint16_t, m);
            Tl2[o + 1] = __builtin_bit_cast(uint16_t, lo);
        } else {
            split16(v.x, h, lo);
            Thi[o] = __builtin_bit_cast(uint16_t, h);
            Tlo[o] = __builtin_bit_cast(uint16_t, lo);
            split16(v.y, h, lo);
            Thi[o + 1] = __builtin_bit_cast(uint16_t, h);
            Tlo[o + 1] = __builtin_bit_cast(uint16_t, lo);
        }
        if (i == 0) pTf[t] = t < nT ? (float)pT[t] : 0.f;
    }
}

// B[l][r] = sum_i b_li |P_ri|^2 as an FP32 GEMM on v_mfma_f32_32x32x2_f32:
// workgroup = 64 images x 64 rotations, 4 waves of 32 x 32, 16-pixel chunks.
__global__ void __launch_bounds__(256) k_scan_bias(const float* __restrict__ Bc,
                                                   const float2* __restrict__ rotP, int nR,
                                                   int nPxl, int nImgPad, int nCk, int nRBias,
                                                   float* __restrict__ bias)
{
    __shared__ float sA[64][KC + 1];
    __shared__ float sB[64][KC + 1];
    const int l0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wi = w & 1, wr = w >> 1, n = lane & 31, h = lane >> 5;
    f32x16 acc;
#pragma unroll
    for (int j = 0; j < 16; j++) acc[j] = 0.f;
    for (int ck = 0; ck < nCk; ck++) {
#pragma unroll
        for (int v = 0; v < KC / 16; v++) {
            const int x = tid + v * 256;
            const float4 a = reinterpret_cast<const float4*>(Bc + ((size_t)ck * nImgPad + l0) * KC)[x];
            const int row = x / (KC / 4), c4 = (x % (KC / 4)) * 4;
            sA[row][c4] = a.x; sA[row][c4 + 1] = a.y; sA[row][c4 + 2] = a.z; sA[row][c4 + 3] = a.w;
        }
#pragma unroll
        for (int u = 0; u < KC / 4; u++) {
            const int x = tid + u * 256, rr = x / KC, kc = x % KC;
            const int r = r0 + rr, i = ck * KC + kc;
            float p2 = 0.f;
            if (r < nR && i < nPxl) {
                const float2 p = rotP[(size_t)r * nPxl + i];
                p2 = p.x * p.x + p.y * p.y;
            }
            sB[rr][kc] = p2;
        }
        __syncthreads();
#pragma unroll
        for (int k2 = 0; k2 < KC / 2; k2++)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sA[32 * wi + n][2 * k2 + h],
                                                       sB[32 * wr + n][2 * k2 + h], acc, 0, 0, 0);
        __syncthreads();
    }
    // C layout: col = n (rotation), row = (j & 3) + 8 (j >> 2) + 4 h (image)
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int row = (j & 3) + 8 * (j >> 2) + 4 * h;
        bias[(size_t)(l0 + 32 * wi + row) * nRBias + r0 + 32 * wr + n] = acc[j];
    }
}

// max / sum over the 32 lanes sharing lane >> 5 (the translation columns of
// one accumulator row): DPP inside each row of 16 lanes, then the row pairs
// (0, 1) and (2, 3) through v_permlane16_swap -- no ds_bpermute round trips
// through the LDS pipe (the shuffles were 320 of them per wave, each waited
// on).  Lane n == 0's sum is the one stored.
template <bool MAX>
THX_DEV float half_reduce(float v)
{
    auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xb1, 0xf, 0xf, false)));
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4e, 0xf, 0xf, false)));
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false)));
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false)));
    const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return op(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
}

// LDS stages of the chunk pipeline: chunk ck + STAGES - 1 is copied while
// chunk ck is multiplied, so each copy has STAGES - 1 chunks to land
constexpr int SCAN_STAGES = 2;

template <int N>
THX_DEV void wait_vm()
{
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int MODE, int NF>
struct Smem {
    static constexpr int NTP = NF * 32;
    static constexpr int NPLANE = nplane<MODE>();
    static constexpr int T_H = NTP * TROW;                 // 16-bit elements per plane
    static constexpr int A_F2 = IMG_TILE * APITCH;         // float2
    static constexpr int P_F2 = ROT_TILE * KC;             // float2
    // one stage = [T planes | a tile] (the global LDS images, copied by LDS-DMA
    // in 16-B pieces, each part rounded up to whole 1-KiB wave instructions so
    // every instruction reads one part) + the P rows; two stages
    static constexpr int T_PC = T_H * 2 / 16;              // 16-B pieces per plane
    static constexpr int A_PC = A_F2 * 8 / 16;
    static constexpr int TQ = (T_PC + 63) / 64;            // wave instructions per plane
    static constexpr int AQ = (A_PC + 63) / 64;
    static constexpr int P_PC = P_F2 * 8 / 16;             // 16-B pieces of the P rows
    static constexpr int PQ = (P_PC + 63) / 64;
    static constexpr int NQ = NPLANE * TQ + AQ + PQ;
    static constexpr int TL_OFF = TQ * 1024;               // bytes: second / third plane, a tile, P rows
    static constexpr int TL2_OFF = 2 * TQ * 1024;
    static constexpr int A_OFF = NPLANE * TQ * 1024;
    static constexpr int P_OFF = (NPLANE * TQ + AQ) * 1024;
    static constexpr int STAGE_B = NQ * 1024;
    static constexpr int EPI_B = (ROT_TILE * 64 * 3 + 64 + ROT_TILE * 8 * NTP + ROT_TILE * GCAP) * 4;
    static constexpr int TOTAL_B = SCAN_STAGES * STAGE_B > EPI_B ? SCAN_STAGES * STAGE_B : EPI_B;
};

// 16 bytes global -> LDS without registers: lane L's piece lands at
// ldsBase + 16 L (ldsBase wave-uniform)
THX_DEV void dma16(const void* g, void* ldsBase)
{
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)g,
        (__attribute__((address_space(3))) void*)ldsBase, 16, 0, 0);
}

// The reference's direct form of one sample (logDataVSPrior_m_huabin,
// src/Optimiser.cpp:9187-9213, with the T P product of :756-826 first):
// per pixel ctf (T P), d minus it, |.|^2 times sigRcp, in FP32 without
// contraction; the pixels strided over the wave's lanes, then a wave sum.
// Used by the cancellation guard for the few samples it flags.
THX_DEV float direct_dvp(const float2* __restrict__ dat,
                                                      const float* __restrict__ ctf,
                                                      const float* __restrict__ sig,
                                                      const float2* __restrict__ traP,
                                                      const float2* __restrict__ rotP,
                                                      int nPxl, int l, int r, int t)
{
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const float2* D = dat + (size_t)l * nPxl;
    const float* C = ctf + (size_t)l * nPxl;
    const float* S = sig + (size_t)l * nPxl;
    const float2* Tt = traP + (size_t)t * nPxl;
    const float2* Pr = rotP + (size_t)r * nPxl;
    float acc = 0.f;
    for (int i = lane; i < nPxl; i += 64) {
        const float2 tp = Tt[i], p = Pr[i], d = D[i];
        const float c = C[i], sg = S[i];
        const float pr = tp.x * p.x - tp.y * p.y;
        const float pi = tp.x * p.y + tp.y * p.x;
        const float er = d.x - c * pr;
        const float ei = d.y - c * pi;
        acc += (er * er + ei * ei) * sg;
    }
    return wave_sum(acc);
}

struct Guard {
    const float2* dat;
    const float* ctf;
    const float* sig;
    const float2* traP;
    const float2* rotP;
    float kmax;       // <= 0: off
    float* dvpOut;    // optional [nImg][nR][nT] dump of the final dvp
};

// The cancellation guard over one wave's tile acc[NA][NF] (per accumulator
// 32 rows x 32 translation columns, row = 32 a + (j & 3) + 8 (j >> 2) + 4 h;
// values already dvp = X + (A + B)).  A sample is flagged when
// |A| + |B| + |X| > kmax |dvp|.  Flagged samples are recomputed by the whole
// wave (direct_dvp) in rounds of at most GCAP into a per-wave LDS list, then
// every flagged lane picks its value up by its rank -- the accumulator
// registers are only ever indexed at compile time.  sABr / sBiasr: |A| + |B|
// and A + B per row; lr(row) = (image, rotation) of a row, x < 0 = no sample.
template <int NA, int NF, typename LR>
THX_DEV void guard_tile(f32x16 (&acc)[NA][NF], const Guard& gd, const float* sABr,
                        const float* sBiasr, float* sVal, LR lr, int nT, int nPxl)
{
    static_assert(NA * 16 <= 32, "one bit per (a, j) in a 32-bit word");
    const int lane = threadIdx.x & 63, n = lane & 31, h = lane >> 5;
    unsigned fw[NF];              // bit q = a * 16 + j of translation fragment f
#pragma unroll
    for (int f = 0; f < NF; f++) fw[f] = 0;
#pragma unroll
    for (int a = 0; a < NA; a++)
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int row = a * 32 + (j & 3) + 8 * (j >> 2) + 4 * h;
            const float b = sBiasr[row], ab = sABr[row];
            const bool ok = lr(row).x >= 0;
#pragma unroll
            for (int f = 0; f < NF; f++) {
                const float d = acc[a][f][j];
                const float x = d - b;   // X up to one rounding: the flag is a ratio test
                if (ok && f * 32 + n < nT && ab + fabsf(x) > gd.kmax * fabsf(d))
                    fw[f] |= 1u << (a * 16 + j);
            }
        }
    unsigned any = 0;
#pragma unroll
    for (int f = 0; f < NF; f++) any |= fw[f];
    while (__ballot(any != 0)) {
        unsigned pw[NF];          // the entries of this round
#pragma unroll
        for (int f = 0; f < NF; f++) pw[f] = 0;
        int cnt = 0;
        for (int q = 0; q < NA * 16 && cnt < GCAP; q++) {
#pragma unroll
            for (int f = 0; f < NF; f++) {
                uint64_t m = __ballot((fw[f] >> q) & 1u);
                while (m && cnt < GCAP) {
                    const int L = __builtin_ctzll(m);
                    const int j = q & 15;
                    const int2 sm = lr((q >> 4) * 32 + (j & 3) + 8 * (j >> 2) + 4 * (L >> 5));
                    const float v = direct_dvp(gd.dat, gd.ctf, gd.sig, gd.traP, gd.rotP, nPxl, sm.x,
                                               sm.y, f * 32 + (L & 31));
                    if (lane == 0) sVal[cnt] = v;
                    if (lane == L) {
                        fw[f] &= ~(1u << q);
                        pw[f] |= 1u << q;
                    }
                    cnt++;
                    m &= m - 1;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // entries were appended in (q, f, lane) order: a lane's slot is the
        // count of earlier (q, f) groups plus the processed lanes below it
        int base = 0;
#pragma unroll
        for (int a = 0; a < NA; a++)
#pragma unroll
            for (int j = 0; j < 16; j++)
#pragma unroll
                for (int f = 0; f < NF; f++) {
                    const bool mine = (pw[f] >> (a * 16 + j)) & 1u;
                    const uint64_t m = __ballot(mine);
                    if (m) {
                        if (mine)
                            acc[a][f][j] = sVal[base + __builtin_amdgcn_mbcnt_hi(
                                (unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0))];
                        base += __builtin_popcountll(m);
                    }
                }
        __builtin_amdgcn_wave_barrier();
        any = 0;
#pragma unroll
        for (int f = 0; f < NF; f++) any |= fw[f];
    }
}

template <int MODE, int NF>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(2))) k_scan_split(const float2* __restrict__ Ac,
                                                        const float* __restrict__ Aconst,
                                                        const float* __restrict__ bias,
                                                        const uint16_t* __restrict__ Thi,
                                                        const uint16_t* __restrict__ Tlo,
                                                        const uint16_t* __restrict__ Tl2,
                                                        const float2* __restrict__ Pc,
                                                        const float* __restrict__ pTf,
                                                        const double* __restrict__ pR,
                                                        int nImg, int nR, int nT, int nPxl,
                                                        int nImgPad, int nPxlPad, int nTPad,
                                                        int nRBias, int nIT,
                                                        float2* __restrict__ wRp,
                                                        float* __restrict__ pM,
                                                        float* __restrict__ pWT, Guard gd)
{
    using S = Smem<MODE, NF>;
    constexpr int NTP = S::NTP;
    extern __shared__ __attribute__((aligned(16))) char lds[];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = lane & 31, h = lane >> 5;
    // XCD-aware order: workgroup b runs on XCD b % 8, and every XCD walks its
    // own contiguous range of (image tile, rotation block) pairs, image-major,
    // so the 64-image a tile of a tile stays in that XCD's L2 for all its
    // rotation blocks (the translation table is shared by all)
    const int nB = nIT * ((nR + ROT_TILE - 1) / ROT_TILE);
    const int per = (nB + 7) / 8;
    const int pq = (blockIdx.x % 8) * per + blockIdx.x / 8;
    if (pq >= nB) return;
    const int nRBk = (nR + ROT_TILE - 1) / ROT_TILE;
    const int l0 = (pq / nRBk) * IMG_TILE;
    const int rb = pq % nRBk;
    const int r = rb * ROT_TILE + w;        // this wave's rotation
    const bool rValid = r < nR;

    f32x16 acc[2][NF];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int f = 0; f < NF; f++)
#pragma unroll
            for (int j = 0; j < 16; j++) acc[a][f][j] = 0.f;

    // Two stages.  Chunk ck+1's T planes and a tile are copied by LDS-DMA into
    // the other stage while chunk ck is multiplied, and its P rows ride in one
    // register; the barrier closing chunk ck retires both.
    // A wave's LDS-DMA instructions q = u NWAVE + w are fixed for the whole
    // launch: their sources (part, first byte, per-chunk stride), LDS slots
    // and lane counts are worked out once, in scalar registers (w through
    // readfirstlane), so a chunk's copies cost one scalar multiply-add and no
    // VALU each.  (Selected per chunk from the wave index they took ~10 VALU
    // per copy, ~65 per wave and chunk: VALU issue adds to the MFMA time on
    // gfx950, tools/probes/coexec.hip.)
    constexpr int QS = (S::NQ + NWAVE - 1) / NWAVE;
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const char* dmaG[QS];
    size_t dmaStride[QS];
    int dmaN[QS];               // lanes that copy (0: no instruction)
    {
        const size_t tStride = (size_t)nTPad * TROW * 2;
#pragma unroll
        for (int u = 0; u < QS; u++) {
            const int q = u * NWAVE + wu;
            const char* g = nullptr;
            size_t st = 0;
            int pc = 0, lim = 0;
            if (q < S::TQ) {
                g = reinterpret_cast<const char*>(Thi); st = tStride; pc = q * 64; lim = S::T_PC;
            } else if (S::NPLANE >= 2 && q < 2 * S::TQ) {
                g = reinterpret_cast<const char*>(Tlo); st = tStride; pc = (q - S::TQ) * 64; lim = S::T_PC;
            } else if (S::NPLANE >= 3 && q < 3 * S::TQ) {
                g = reinterpret_cast<const char*>(Tl2); st = tStride; pc = (q - 2 * S::TQ) * 64; lim = S::T_PC;
            } else if (q < S::NQ - S::PQ) {
                g = reinterpret_cast<const char*>(Ac + (size_t)l0 * APITCH);
                st = (size_t)nImgPad * APITCH * sizeof(float2);
                pc = (q - S::NPLANE * S::TQ) * 64; lim = S::A_PC;
            } else if (q < S::NQ) {
                g = reinterpret_cast<const char*>(Pc + (size_t)rb * ROT_TILE * KC);
                st = (size_t)nRBk * ROT_TILE * KC * sizeof(float2);
                pc = (q - (S::NQ - S::PQ)) * 64; lim = S::P_PC;
            }
            dmaG[u] = g + (size_t)pc * 16;
            dmaStride[u] = st;
            dmaN[u] = q < S::NQ ? min(64, lim - pc) : 0;
        }
    }
    const unsigned laneB = (unsigned)lane * 16u;
    auto issue_chunk = [&](int ck, char* stage) {
#pragma unroll
        for (int u = 0; u < QS; u++)
            if (lane < dmaN[u])
                dma16(dmaG[u] + (size_t)ck * dmaStride[u] + laneB, stage + (u * NWAVE + wu) * 1024);
    };
    auto stage_at = [&](int ck) { return lds + (ck % SCAN_STAGES) * S::STAGE_B; };
    const int nCk = nPxlPad / KC;
    // LDS-DMA instructions this wave issues per chunk (issue_chunk's q = u NWAVE + w)
    constexpr int QLO = S::NQ / NWAVE, QREM = S::NQ % NWAVE;
    const bool qHi = w < QREM;
    // wait until at most the copies of the newest `ahead` chunks are in flight
    auto wait_ahead = [&](int ahead) {
        if (SCAN_STAGES == 3 && ahead == 1) {
            if (qHi) wait_vm<QLO + 1>(); else wait_vm<QLO>();
        } else {
            wait_vm<0>();
        }
    };
#pragma unroll
    for (int k = 0; k < SCAN_STAGES - 1; k++)
        if (k < nCk) issue_chunk(k, stage_at(k));
    wait_ahead(nCk > 1 && SCAN_STAGES == 3 ? 1 : 0);
    __syncthreads();
    for (int ck = 0; ck < nCk; ck++) {
        // the stage chunk ck + STAGES - 1 lands in was last read in chunk ck - 1
        const bool more = ck + SCAN_STAGES - 1 < nCk;
        if (more) issue_chunk(ck + SCAN_STAGES - 1, stage_at(ck + SCAN_STAGES - 1));
        const char* stage = stage_at(ck);
        const uint16_t* sTh = reinterpret_cast<const uint16_t*>(stage);
        const uint16_t* sTl = reinterpret_cast<const uint16_t*>(stage + S::TL_OFF);
        const float2* sA = reinterpret_cast<const float2*>(stage + S::A_OFF);
        const float2* sP = reinterpret_cast<const float2*>(stage + S::P_OFF);
#pragma unroll
        for (int s = 0; s < KC / 8; s++) {
            // A fragments: w = a conj(P_r) for images a*32 + n, pixels 8s+4h+{0..3}
            const int px0 = 8 * s + 4 * h;
            const f32x4v p01 = *reinterpret_cast<const f32x4v*>(sP + w * KC + px0);
            const f32x4v p23 = *reinterpret_cast<const f32x4v*>(sP + w * KC + px0 + 2);
            const float pr[4] = {p01.x, p01.z, p23.x, p23.z};
            const float pi[4] = {p01.y, p01.w, p23.y, p23.w};
            // w fragments of image half a (hi, lo split in registers)
            auto make_w = [&](int a, HV& wh, HV& wl) {
                const float2* rowA = sA + (a * 32 + n) * APITCH + px0;
                const f32x4v a01 = *reinterpret_cast<const f32x4v*>(rowA);
                const f32x4v a23 = *reinterpret_cast<const f32x4v*>(rowA + 2);
                const float ar[4] = {a01.x, a01.z, a23.x, a23.z};
                const float ai[4] = {a01.y, a01.w, a23.y, a23.w};
#pragma unroll
                for (int qd = 0; qd < 4; qd++) {
                    const float wr = ar[qd] * pr[qd] + ai[qd] * pi[qd];
                    const float wi = ai[qd] * pr[qd] - ar[qd] * pi[qd];
                    H x0, x1;
                    split16(wr, x0, x1); wh[2 * qd] = x0; wl[2 * qd] = x1;
                    split16(wi, x0, x1); wh[2 * qd + 1] = x0; wl[2 * qd + 1] = x1;
                }
            };
            if constexpr (MODE == BF16X6) {
                // both image halves' w in three pieces (24 VGPRs), then per
                // translation fragment the three T planes feed 2 x 6 products
                // (smallest first into the running FP32 sum)
                const uint16_t* sT2 = reinterpret_cast<const uint16_t*>(stage + S::TL2_OFF);
                auto make_w3 = [&](int a, HV (&wq)[3]) {
                    const float2* rowA = sA + (a * 32 + n) * APITCH + px0;
                    const f32x4v a01 = *reinterpret_cast<const f32x4v*>(rowA);
                    const f32x4v a23 = *reinterpret_cast<const f32x4v*>(rowA + 2);
                    const f2v av[4] = {f2v{a01.x, a01.y}, f2v{a01.z, a01.w}, f2v{a23.x, a23.y},
                                       f2v{a23.z, a23.w}};   // (re, im) of a, one pixel each
                    u32x4 hq, mq, lq;
#pragma unroll
                    for (int qd = 0; qd < 4; qd++) {
                        // w = a conj(P) in two packed operations: (ar pr, ai pr), then
                        // (ai pi + ar pr, -ar pi + ai pr) -- the swap, the broadcast
                        // and the sign are operand modifiers of v_pk_fma_f32 (the
                        // component-wise form compiled to three, half their
                        // products unused)
                        const f2v t = av[qd] * (f2v)pr[qd];
                        const f2v w = __builtin_elementwise_fma(f2v{av[qd].y, av[qd].x},
                                                                f2v{pi[qd], -pi[qd]}, t);
                        uint32_t x0, x1, x2;
                        split3x2(w, x0, x1, x2);
                        hq[qd] = x0; mq[qd] = x1; lq[qd] = x2;
                    }
                    wq[0] = __builtin_bit_cast(HV, hq);
                    wq[1] = __builtin_bit_cast(HV, mq);
                    wq[2] = __builtin_bit_cast(HV, lq);
                };
                auto mma6 = [&](f32x16& c, const HV (&wq)[3], const HV& th, const HV& tm, const HV& tl) {
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wq[2], th, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wq[1], tm, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wq[0], tl, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wq[1], th, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wq[0], tm, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wq[0], th, c, 0, 0, 0);
                };
                HV wp[2][3];
                make_w3(0, wp[0]);
                make_w3(1, wp[1]);
#pragma unroll
                for (int f = 0; f < NF; f++) {
                    const int row = (f * 32 + n) * TROW + 16 * s + 8 * h;
                    const HV th = *reinterpret_cast<const HV*>(sTh + row);
                    const HV tm = *reinterpret_cast<const HV*>(sTl + row);
                    const HV tl = *reinterpret_cast<const HV*>(sT2 + row);
#pragma unroll
                    for (int a = 0; a < 2; a++) mma6(acc[a][f], wp[a], th, tm, tl);
                }
            } else if constexpr (MODE == BF16X3) {
                // one image half at a time (register budget of the three products)
#pragma unroll
                for (int a = 0; a < 2; a++) {
                    HV wh, wl;
                    make_w(a, wh, wl);
#pragma unroll
                    for (int f = 0; f < NF; f++) {
                        const int row = (f * 32 + n) * TROW + 16 * s + 8 * h;
                        const HV th = *reinterpret_cast<const HV*>(sTh + row);
                        const HV tl = *reinterpret_cast<const HV*>(sTl + row);
                        acc[a][f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, th, acc[a][f], 0, 0, 0);
                        acc[a][f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, tl, acc[a][f], 0, 0, 0);
                        acc[a][f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, th, acc[a][f], 0, 0, 0);
                    }
                }
            }
        }
        // chunk ck + 1 must have landed; the newer copy may stay in flight
        wait_ahead(more && SCAN_STAGES == 3 ? 1 : 0);
        __syncthreads();
    }

    // ------------------------------------------------------------ epilogue
    float* sBias = reinterpret_cast<float*>(lds);      // [8 waves][64]  A_l + B[l][r]
    float* sMax = sBias + ROT_TILE * 64;               // [8 waves][64 rows]
    float* sRowM = sMax + ROT_TILE * 64;               // [64]           max over the tile's rotations
    float* sAB = sRowM + 64;                           // [8 waves][64]  |A_l| + |B[l][r]|
    float* sT = sAB + ROT_TILE * 64;                   // [8 waves][8 rows][NTP] scaled terms
    float* sGVal = sT + ROT_TILE * 8 * NTP;            // [8 waves][GCAP] guard list
    {
        const float A = Aconst[l0 + lane], B = rValid ? bias[(size_t)(l0 + lane) * nRBias + r] : 0.f;
        sBias[w * 64 + lane] = A + B;
        sAB[w * 64 + lane] = fabsf(A) + fabsf(B);
    }
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
            const float b = sBias[w * 64 + row];
#pragma unroll
            for (int f = 0; f < NF; f++) acc[a][f][j] += b;
        }
    if (gd.kmax > 0.f)
        guard_tile<2, NF>(acc, gd, sAB + w * 64, sBias + w * 64, sGVal + w * GCAP,
                          [&](int row) { return make_int2(rValid && l0 + row < nImg ? l0 + row : -1, r); },
                          nT, nPxl);
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int row = a * 32 + (j & 3) + 8 * (j >> 2) + 4 * h;
            const int l = l0 + row;
            if (gd.dvpOut && rValid && l < nImg) {
#pragma unroll
                for (int f = 0; f < NF; f++)
                    if (f * 32 + n < nT) gd.dvpOut[((size_t)l * nR + r) * nT + f * 32 + n] = acc[a][f][j];
            }
            float mx = -INFINITY;
#pragma unroll
            for (int f = 0; f < NF; f++)
                if (f * 32 + n < nT) mx = fmaxf(mx, acc[a][f][j]);
            mx = half_reduce<true>(mx);
            if (!rValid) mx = -INFINITY;
            float sR = 0.f;
#pragma unroll
            for (int f = 0; f < NF; f++) {
                const float e = (f * 32 + n < nT && rValid) ? __expf(acc[a][f][j] - mx) : 0.f;
                acc[a][f][j] = e;
                sR += e * pTv[f];
            }
            sR = half_reduce<false>(sR);
            if (n == 0) {
                sMax[w * 64 + row] = mx;
                if (rValid && l < nImg) wRp[(size_t)l * nR + r] = make_float2(mx, sR);
            }
        }
    __syncthreads();
    if (tid < 64) {
        float M = sMax[tid];
#pragma unroll
        for (int k = 1; k < ROT_TILE; k++) M = fmaxf(M, sMax[k * 64 + tid]);
        sRowM[tid] = M;
        pM[(size_t)rb * nImgPad + l0 + tid] = M;
    }
    __syncthreads();
    // the t-marginal partial of the tile, 8 image rows at a time: every wave
    // stages its rotation's scaled terms, then each (row, t) sums the 8
    // rotations in wave order (deterministic, no atomics)
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int g = 0; g < 4; g++) {
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const int j = 4 * g + jj, mm = jj + 4 * h;    // row 8 g + mm of half a
                const int row = a * 32 + 8 * g + mm;
                const float sc = rValid ? __expf(sMax[w * 64 + row] - sRowM[row]) * pRr : 0.f;
#pragma unroll
                for (int f = 0; f < NF; f++) sT[(w * 8 + mm) * NTP + f * 32 + n] = acc[a][f][j] * sc;
            }
            __syncthreads();
            for (int x = tid; x < 8 * NTP; x += THREADS) {
                const int mm = x / NTP, t = x % NTP;
                float sum = 0.f;
#pragma unroll
                for (int k = 0; k < ROT_TILE; k++) sum += sT[(k * 8 + mm) * NTP + t];
                pWT[((size_t)rb * nImgPad + l0 + a * 32 + 8 * g + mm) * NTP + t] = sum;
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

template <int MODE, int NF>
int launch_main(const WS& ws, const Dims& d, const double* pR, const Guard& gd, hipStream_t s)
{
    const int nIT = d.nImgPad / IMG_TILE;
    dim3 grid((unsigned)(8 * thx::cdiv(nIT * d.nRB, 8)));
    constexpr int lds = Smem<MODE, NF>::TOTAL_B;
    static_assert(lds <= 160 * 1024, "scan stages exceed the LDS");
    static std::atomic<unsigned> ldsSet{0};
    const int st = thx::set_max_lds(reinterpret_cast<const void*>(k_scan_split<MODE, NF>), lds, ldsSet);
    if (st != THX_OK) return st;
    hipLaunchKernelGGL((k_scan_split<MODE, NF>), grid, dim3(THREADS), lds, s, ws.Ac, ws.Aconst,
                       ws.bias, ws.Thi, ws.Tlo, ws.Tl2, ws.Pc,
                       ws.pTf, pR, d.nImg, d.nR, d.nT, d.nPxl, d.nImgPad, d.nPxlPad, d.nTPad,
                       d.nRBias, nIT, ws.wRp, ws.pM, ws.pWT, gd);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

template <int MODE>
int scan_split(const float* rotP, int nR, const float* traP, int nT, const float* dat,
               const float* ctf, const float* sigRcp, int nImg, int nPxl, const double* pR,
               const double* pT, int kIdx, int nK, float* wC, float* wR, float* wT,
               float* baseL, float guard, float* dvpOut, void* workspace, size_t wsBytes,
               hipStream_t s)
{
    const Dims d = dims(nImg, nR, nT, nPxl);
    THX_CHECK_ARG(d.nRB <= 65535 && d.nRBias / 64 <= 65535, "thx_global_scan: grid too large");
    const WS ws = carve(workspace, d);
    THX_CHECK_ARG(ws.bytes <= wsBytes, "thx_global_scan: workspace too small");
    const float2* dat2 = reinterpret_cast<const float2*>(dat);
    const float2* rot2 = reinterpret_cast<const float2*>(rotP);
    hipLaunchKernelGGL(k_prep_aconst, dim3(thx::cdiv(d.nImgPad, 4)), dim3(256), 0, s, dat2, sigRcp,
                       nImg, nPxl, d.nImgPad, ws.Aconst);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_prep_img, dim3(2048), dim3(256), 0, s, dat2, ctf, sigRcp, nImg,
                       nPxl, d.nImgPad, d.nPxlPad, ws.Ac, ws.Bc);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_prep_pchunk, dim3(2048), dim3(256), 0, s, rot2, nR, nPxl,
                       d.nRB * ROT_TILE, d.nPxlPad, ws.Pc);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_prep_tsplit<MODE>, dim3(512), dim3(256), 0, s,
                       reinterpret_cast<const float2*>(traP), pT, nT, nPxl, d.nTPad, d.nPxlPad,
                       ws.Thi, ws.Tlo, ws.Tl2, ws.pTf);
    THX_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_scan_bias, dim3(d.nImgPad / 64, d.nRBias / 64), dim3(256), 0, s, ws.Bc,
                       rot2, nR, nPxl, d.nImgPad, d.nCk, d.nRBias, ws.bias);
    THX_LAUNCH_CHECK();
    const Guard gd{dat2, ctf, sigRcp, reinterpret_cast<const float2*>(traP), rot2, guard, dvpOut};
    int st;
    switch (d.nTPad / 32) {
        case 1: st = launch_main<MODE, 1>(ws, d, pR, gd, s); break;
        case 2: st = launch_main<MODE, 2>(ws, d, pR, gd, s); break;
        case 3: st = launch_main<MODE, 3>(ws, d, pR, gd, s); break;
        case 4: st = launch_main<MODE, 4>(ws, d, pR, gd, s); break;
        default: st = launch_main<MODE, 5>(ws, d, pR, gd, s); break;
    }
    if (st != THX_OK) return st;
    hipLaunchKernelGGL(k_scan_combine_bf, dim3(nImg), dim3(256), sizeof(float) * d.nRB, s,
                       ws.wRp, ws.pM, ws.pWT, pR, nR, nT, d.nTPad, d.nRB, d.nImgPad, kIdx, nK,
                       wC, wR, wT, baseL);
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

// nT > 160: 2 x NF accumulators no longer fit one wave -- FP32 MFMA path (algo 1)
size_t scan_split_workspace(int nImg, int nR, int nT, int nPxl)
{
    const Dims d = dims(nImg, nR, nT, nPxl);
    if (d.nTPad > 160) return scan_mfma_workspace(nImg, nR, nT, nPxl);
    return carve(nullptr, d).bytes;
}

float scan_guard_default() { return SCAN_GUARD; }

// algo 2 (bf16x3), 4 (bf16x6); guard = the cancellation ratio
// above which a sample is recomputed directly (0 = off); dvpOut (optional)
// receives every sample's final dvp
int scan_split_algo(int algo, const float* rotP, int nR, const float* traP, int nT,
                    const float* dat, const float* ctf, const float* sigRcp, int nImg, int nPxl,
                    const double* pR, const double* pT, int kIdx, int nK, float* wC, float* wR,
                    float* wT, float* baseL, float guard, float* dvpOut, void* workspace,
                    size_t wsBytes, hipStream_t s)
{
    if (pad_to(nT, 32) > 160) {
        THX_CHECK_ARG(dvpOut == nullptr,
                      "thx_global_scan_dvp: nT = %d > 160 runs the FP32-MFMA scan, which keeps no dvp", nT);
        return scan_mfma(rotP, nR, traP, nT, dat, ctf, sigRcp, nImg, nPxl, pR, pT, kIdx, nK,
                         wC, wR, wT, baseL, workspace, wsBytes, s);
    }
    if (algo == 2)
        return scan_split<BF16X3>(rotP, nR, traP, nT, dat, ctf, sigRcp, nImg, nPxl, pR, pT, kIdx,
                                  nK, wC, wR, wT, baseL, guard, dvpOut, workspace, wsBytes, s);
    return scan_split<BF16X6>(rotP, nR, traP, nT, dat, ctf, sigRcp, nImg, nPxl, pR, pT, kIdx, nK,
                              wC, wR, wT, baseL, guard, dvpOut, workspace, wsBytes, s);
}

}  // namespace thx
