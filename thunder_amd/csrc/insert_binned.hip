// insert_binned.hip -- a12 as a binned deposition: the weighted trilinear
// back-projection of Reconstructor::insertP (src/Reconstructor.cpp:782-863,
// Volume::addFT src/Image/Volume.cpp:340-375; GPU twin cuthunder::InsertFT,
// gpu/src/cuthunder.cu:5570-5826) reorganised so that every half-map voxel is
// summed in LDS by one owner and reaches HBM once per owner.
//
// Memory-side float atomics run at ~1.3 TB/s only for 256 contiguous bytes per
// wave-instruction and ~17x slower for scattered lanes (MI355X_MICROARCH.md,
// global float atomics); the per-(image, patch) LDS boxes of
// k_insert_patches still flush ~45 GB per 6250-image hemisphere launch at the
// bench's clouds and re-run their samples per z-chunk when the posterior is
// wide.  Here:
//   1. k_bin_groups   per image: samples with bitwise-identical quaternions
//      (resampled particles are copies of their ancestors; 46 of 100 distinct
//      at the bench's median) form one group -- the taps depend only on the
//      rotation, so a group deposits sum_m src_m once.  Also insertDir /
//      counter (src/Reconstructor.cpp:407-422).
//   2. k_bin_pass<false>  per (image, 2048 visiting slots): folded cell
//      corner of every (group, pixel) -> tile of 16^3 corners, per-workgroup
//      LDS histogram, one global add per (workgroup, tile).
//   3. k_bin_scan     tile offsets and deposit chunks (<= BIN_E entries each).
//   4. k_bin_pass<true>   the same workgroups: reserve each tile's range
//      once, then write the entries (folded x, y, z; value sum over the
//      group's members; ctf^2 w |group|) with wave-aggregated slots.
//   5. k_bin_deposit  per chunk: the tile's 17^3 voxels (corners + the +1 tap
//      halo) in LDS as 64-bit fixed point, 8 taps x 3 ds_add_u64 per entry,
//      then one row-contiguous global float add per non-zero voxel component.
// LDS float atomics are the wrong tool on gfx950: ds_add_f32 retires one
// wave-instruction per ~193 CU cycles whatever the address pattern, while
// ds_add_u64 takes 7-12 (tools/probes/lds_atomic.hip,
// profiles/r02_lds_atomic.jsonl).  The fixed point is exact: k_bin_pass<true>
// records the batch's largest |value|, and the deposit scales by 2^e with
// |value * weight * 2^e| < 2^47, so <= 2^15 entries of a chunk sum without
// overflow and the tap products (the float products of the float path) are
// rounded once, at 2^-48 of the largest value of their own kind: F (re, im)
// and T carry separate maxima and exponents, so T far below the data's scale
// (data >> ctf^2, pixels near CTF zeros) keeps its own 2^-48 relative grid;
// the tile sums are exact and independent of order.  Non-finite values take a float-atomic path so NaN /
// Inf propagate as in the reference.
// Entries live in the caller's workspace; images are processed in batches
// so the entry buffer stays bounded (thx_insert3d_binned_workspace).
// The F / T values and coordinates are those of k_insert3d (same FP64
// rotation, FP32 phase / value formulas); only the FP32 summation order
// differs.
#include <climits>

#include "common.h"

namespace {

constexpr int BT = 16;                    // tile edge in cell corners
constexpr int BH = BT + 1;                // + the taps' +1 halo
constexpr int BVOX = BH * BH * BH;        // 4913 voxels
constexpr int BIN_E = 32768;              // entries per deposit chunk
constexpr int BIN_MAXM = 1024;            // samples per image the grouping handles
constexpr int BIN_KCH = 2048;             // visiting slots per binning workgroup
constexpr int BIN_MAX_TILES = 16384;      // LDS histogram (64 KB)
constexpr long BIN_ENT_CAP = 1L << 28;    // entries per batch (6 GiB)
constexpr int G_THREADS = 128, C_THREADS = 256, D_THREADS = 1024;
constexpr size_t DEP_LDS = 3 * BVOX * sizeof(unsigned long long);   // 118 KB: one workgroup per CU

struct Entry {                            // 24 B: folded coordinate + values
    float x, y, z, vr, vi, tv;
};

struct TileGrid {
    int R;                                // |coordinate| <= R - 1, corners in [-R, R - 1]
    int ntx, nty, ntz;
    THX_DEV int tile(int x0, int y0, int z0) const
    {
        if (x0 < 0 || x0 >= ntx * BT) return -1;
        const int ty = (y0 + R) / BT, tz = (z0 + R) / BT;
        if (y0 + R < 0 || z0 + R < 0 || ty >= nty || tz >= ntz) return -1;
        return (tz * nty + ty) * ntx + x0 / BT;
    }
};

TileGrid make_grid(int pf, int rMax)
{
    TileGrid g;
    g.R = pf * rMax + 2;
    g.ntx = (g.R + BT - 1) / BT;
    g.nty = g.ntz = (2 * g.R + BT - 1) / BT;
    return g;
}

// folded cell corner of R (iCol pf, iRow pf, 0) (Volume::addFT's conjHalf)
THX_DEV void folded(const double* __restrict__ m, int ic, int ir, int pf, float& x, float& y,
                    float& z, bool& conj)
{
    const double X = (double)(ic * pf), Y = (double)(ir * pf);
    x = (float)(m[0] * X + m[3] * Y);
    y = (float)(m[1] * X + m[4] * Y);
    z = (float)(m[2] * X + m[5] * Y);
    conj = !(x >= 0.f);
    if (conj) { x = -x; y = -y; z = -z; }
}

// 1. groups of identical rotations, their matrices and members' shifts;
// insertDir(-R (t - off, 0)) and the counter once per image.
__global__ void __launch_bounds__(G_THREADS) k_bin_groups(const double* __restrict__ quat,
                                                          const double* __restrict__ trans,
                                                          const double* __restrict__ offS,
                                                          const int* __restrict__ nCnt, int mReco,
                                                          int l0, int idim, int* __restrict__ nG,
                                                          int* __restrict__ gStart,
                                                          double* __restrict__ gMat,
                                                          float2* __restrict__ mShift,
                                                          double* __restrict__ O,
                                                          int* __restrict__ counter,
                                                          const double* __restrict__ dS,
                                                          double* __restrict__ mDef)
{
    __shared__ int sLead[BIN_MAXM];
    __shared__ int sGid[BIN_MAXM];
    __shared__ double sO[G_THREADS / 64][3];
    const int b = blockIdx.x, l = l0 + b, tid = threadIdx.x;
    const int nM = nCnt ? max(0, min(nCnt[l], mReco)) : mReco;
    const double* Q = quat + (size_t)l * mReco * 4;
    for (int m = tid; m < nM; m += G_THREADS) {
        const double q0 = Q[4 * m], q1 = Q[4 * m + 1], q2 = Q[4 * m + 2], q3 = Q[4 * m + 3];
        int lead = m;
        for (int j = 0; j < m; j++)
            if (Q[4 * j] == q0 && Q[4 * j + 1] == q1 && Q[4 * j + 2] == q2 && Q[4 * j + 3] == q3) {
                lead = j;
                break;
            }
        sLead[m] = lead;
    }
    __syncthreads();
    for (int m = tid; m < nM; m += G_THREADS) {
        if (sLead[m] != m) continue;
        int g = 0;
        for (int j = 0; j < m; j++) g += sLead[j] == j;
        sGid[m] = g;
    }
    __syncthreads();
    int* gs = gStart + (size_t)b * (mReco + 1);
    double* gm = gMat + (size_t)b * mReco * 6;
    float2* ms = mShift + (size_t)b * mReco;
    const double offx = offS[2 * l], offy = offS[2 * l + 1];
    double o0 = 0.0, o1 = 0.0, o2 = 0.0;
    for (int m = tid; m < nM; m += G_THREADS) {
        const int lead = sLead[m];
        // members of lower groups = samples whose leader index is below ours
        int start = 0, pos = 0;
        for (int k = 0; k < nM; k++) {
            start += sLead[k] < lead;
            pos += (k < m) & (sLead[k] == lead);
        }
        const size_t sIdx = (size_t)l * mReco + m;
        double q[4] = {Q[4 * m], Q[4 * m + 1], Q[4 * m + 2], Q[4 * m + 3]};
        double R[9];
        quat_to_mat(q, R);
        const double dx = trans[2 * sIdx] - offx, dy = trans[2 * sIdx + 1] - offy;
        ms[start + pos] = make_float2((float)(-dx) / idim, (float)(-dy) / idim);
        if (dS) mDef[(size_t)b * mReco + start + pos] = dS[sIdx];
        if (lead == m) {
            const int g = sGid[m];
            gs[g] = start;
            for (int k = 0; k < 6; k++) gm[6 * g + k] = R[k];
        }
        o0 -= R[0] * dx + R[3] * dy;
        o1 -= R[1] * dx + R[4] * dy;
        o2 -= R[2] * dx + R[5] * dy;
    }
    o0 = wave_sum(o0); o1 = wave_sum(o1); o2 = wave_sum(o2);
    if ((tid & 63) == 0) { sO[tid >> 6][0] = o0; sO[tid >> 6][1] = o1; sO[tid >> 6][2] = o2; }
    __syncthreads();
    if (tid == 0) {
        int ng = 0;
        for (int m = 0; m < nM; m++) ng += sLead[m] == m;
        nG[b] = ng;
        gs[ng] = nM;
        if (nM > 0) {
            double a0 = 0.0, a1 = 0.0, a2 = 0.0;
            for (int k = 0; k < G_THREADS / 64; k++) { a0 += sO[k][0]; a1 += sO[k][1]; a2 += sO[k][2]; }
            atomicAdd(O + 0, a0);
            atomicAdd(O + 1, a1);
            atomicAdd(O + 2, a2);
            atomicAdd(counter, nM);
        }
    }
}

// wave-aggregated add of 1 per lane into sh[t] (lanes with t < 0 skip);
// returns this lane's slot (old value + rank among the lanes of its tile)
template <bool RET>
THX_DEV int wave_add(int* sh, int t)
{
    const int lane = threadIdx.x & 63;
    unsigned long long act = __ballot(t >= 0);
    int slot = -1;
    while (act) {
        const int first = __ffsll((long long)act) - 1;
        const int t0 = __shfl(t, first, 64);
        const unsigned long long same = __ballot(t == t0);
        int base = 0;
        if (lane == first) base = atomicAdd(&sh[t0], __popcll(same));
        if (RET) {
            base = __shfl(base, first, 64);
            if (t == t0) slot = base + __popcll(same & ((1ull << lane) - 1ull));
        }
        act &= ~same;
    }
    return slot;
}

// 2. / 4. per image: entries (group g, visiting slot k)
template <bool FILL>
__global__ void __launch_bounds__(C_THREADS) k_bin_pass(TileGrid G, int vdim, int pf, int mReco,
                                                        int l0, const int* __restrict__ nG,
                                                        const int* __restrict__ gStart,
                                                        const double* __restrict__ gMat,
                                                        const float2* __restrict__ mShift,
                                                        const int* __restrict__ iCol,
                                                        const int* __restrict__ iRow,
                                                        const int* __restrict__ order, int nOrd,
                                                        int nPxl, const float2* __restrict__ dat,
                                                        const float* __restrict__ ctf,
                                                        const float* __restrict__ w,
                                                        int* __restrict__ count,
                                                        int* __restrict__ cursor,
                                                        Entry* __restrict__ ent,
                                                        unsigned* __restrict__ vmaxBits,   // [F, T]
                                                        float2* __restrict__ F,
                                                        float* __restrict__ T,
                                                        const float* __restrict__ attr,
                                                        const double* __restrict__ mDef,
                                                        int idim)
{
    extern __shared__ int sHist[];
    const int b = blockIdx.x, l = l0 + b, tid = threadIdx.x;
    const int nt = G.ntx * G.nty * G.ntz;
    const int ng = nG[b];
    const int* gs = gStart + (size_t)b * (mReco + 1);
    const double* gm = gMat + (size_t)b * mReco * 6;
    for (int t = tid; t < nt; t += C_THREADS) sHist[t] = 0;
    __syncthreads();
    // this workgroup's visiting slots [k0, k0 + nK) of every group
    const int k0 = blockIdx.y * BIN_KCH, nK = min(BIN_KCH, nOrd - k0);
    const long nE = (long)ng * nK;
    // the histogram of this image's entries over the tiles
    for (long e0 = 0; e0 < nE; e0 += C_THREADS) {      // uniform trip count (wave ballots)
        const long e = e0 + tid;
        int t = -1;
        if (e < nE) {
            const int g = (int)(e / nK), k = k0 + (int)(e - (long)g * nK);
            const int p = order[k];
            if (p >= 0) {
                double m[6];
                for (int q = 0; q < 6; q++) m[q] = gm[6 * g + q];
                float x, y, z;
                bool cj;
                folded(m, iCol[p], iRow[p], pf, x, y, z, cj);
                t = G.tile((int)floorf(x), (int)floorf(y), (int)floorf(z));
            }
        }
        wave_add<false>(sHist, t);
    }
    __syncthreads();
    if (!FILL) {
        for (int t = tid; t < nt; t += C_THREADS)
            if (sHist[t]) atomicAdd(count + t, sHist[t]);
        return;
    }
    // reserve this image's range of every tile once
    for (int t = tid; t < nt; t += C_THREADS)
        if (sHist[t]) sHist[t] = atomicAdd(cursor + t, sHist[t]);
    __syncthreads();
    const float2* D = dat + (size_t)l * nPxl;
    const float* C = attr ? nullptr : ctf + (size_t)l * nPxl;
    const float* A = attr ? attr + 8 * (size_t)l : nullptr;
    const double* md = mDef + (size_t)b * mReco;
    const float2* ms = mShift + (size_t)b * mReco;
    const float wl = w[l];
    float vmaxF = 0.f, vmaxT = 0.f;
    for (long e0 = 0; e0 < nE; e0 += C_THREADS) {
        const long e = e0 + tid;
        int t = -1;
        Entry en;
        bool live = false;
        if (e < nE) {
            const int g = (int)(e / nK), k = k0 + (int)(e - (long)g * nK);
            const int p = order[k];
            if (p >= 0) {
                live = true;
                double m[6];
                for (int q = 0; q < 6; q++) m[q] = gm[6 * g + q];
                const int ic = iCol[p], ir = iRow[p];
                bool cj;
                folded(m, ic, ir, pf, en.x, en.y, en.z, cj);
                const float2 d = D[p];
                float vr = 0.f, vi = 0.f;
                const int s0 = gs[g], s1 = gs[g + 1];
                if (!A) {
                    const float c = C[p];
                    for (int s = s0; s < s1; s++) {
                        const float2 sh = ms[s];
                        const float2 src = cmul(d, phase_shift(ic, ir, sh.x, sh.y));
                        vr += (src.x * c) * wl;
                        vi += (src.y * c) * wl;
                    }
                    en.tv = ((float)((double)c * c) * wl) * (float)(s1 - s0);
                } else {
                    // CTF search: each member's CTF at its own defocus factor,
                    // CTF(dU d, dV d) (src/Optimiser.cpp:7101-7120)
                    float tv = 0.f;
                    for (int s = s0; s < s1; s++) {
                        const float2 sh = ms[s];
                        const float c = ctf_at(A, (float)(A[2] * md[s]), (float)(A[3] * md[s]), ic,
                                               ir, idim);
                        const float2 src = cmul(d, phase_shift(ic, ir, sh.x, sh.y));
                        vr += (src.x * c) * wl;
                        vi += (src.y * c) * wl;
                        tv += (float)((double)c * c) * wl;
                    }
                    en.tv = tv;
                }
                en.vr = vr;
                en.vi = cj ? -vi : vi;
                vmaxF = fmaxf(vmaxF, fmaxf(fabsf(en.vr), fabsf(en.vi)));
                vmaxT = fmaxf(vmaxT, fabsf(en.tv));
                if (!(fabsf(en.vr) + fabsf(en.vi) + fabsf(en.tv) <= 3.4e38f)) vmaxF = INFINITY;
                t = G.tile((int)floorf(en.x), (int)floorf(en.y), (int)floorf(en.z));
            }
        }
        const int slot = wave_add<true>(sHist, t);
        if (t >= 0) {
            ent[slot] = en;
        } else if (live) {
            // outside the tile grid (a pixel beyond rMax): straight to HBM
            scatter_ft(F, T, vdim, en.x, en.y, en.z, en.vr, en.vi, en.tv);
        }
    }
    // the batch's largest |F| and |T| (non-negative float bits order like uints)
    vmaxF = wave_max(vmaxF);
    vmaxT = wave_max(vmaxT);
    if ((tid & 63) == 0 && vmaxF > 0.f) atomicMax(vmaxBits, __float_as_uint(vmaxF));
    if ((tid & 63) == 0 && vmaxT > 0.f) atomicMax(vmaxBits + 1, __float_as_uint(vmaxT));
}

// 3. tile offsets, cursors and deposit chunks (one workgroup)
__global__ void __launch_bounds__(1024) k_bin_scan(const int* __restrict__ count, int nt,
                                                   int* __restrict__ cursor,
                                                   int4* __restrict__ chunks, int maxChunks,
                                                   int* __restrict__ ctl)
{
    __shared__ long sA[1024];
    __shared__ int sB[1024];
    __shared__ long carryE;
    __shared__ int carryC;
    const int tid = threadIdx.x;
    if (tid == 0) { carryE = 0; carryC = 0; }
    __syncthreads();
    for (int t0 = 0; t0 < nt; t0 += 1024) {
        const int t = t0 + tid;
        const int c = t < nt ? count[t] : 0;
        const int nch = (c + BIN_E - 1) / BIN_E;
        sA[tid] = c;
        sB[tid] = nch;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {        // inclusive Hillis-Steele scans
            const long a = tid >= o ? sA[tid - o] : 0;
            const int bb = tid >= o ? sB[tid - o] : 0;
            __syncthreads();
            sA[tid] += a;
            sB[tid] += bb;
            __syncthreads();
        }
        const long off = carryE + sA[tid] - c;
        const int cb = carryC + sB[tid] - nch;
        if (t < nt) {
            cursor[t] = (int)off;
            for (int k = 0; k < nch && cb + k < maxChunks; k++)
                chunks[cb + k] = make_int4(t, (int)(off + (long)k * BIN_E), min(BIN_E, c - k * BIN_E), 0);
        }
        __syncthreads();
        if (tid == 1023) { carryE += sA[1023]; carryC += sB[1023]; }
        __syncthreads();
    }
    if (tid == 0) { ctl[0] = min(carryC, maxChunks); ctl[1] = (int)carryE; ctl[2] = 0; ctl[3] = 0; }
}

// 5. one chunk of one tile: 64-bit fixed-point LDS accumulation, row-contiguous flush
__global__ void __launch_bounds__(D_THREADS) k_bin_deposit(TileGrid G, int vdim,
                                                           const int4* __restrict__ chunks,
                                                           const int* __restrict__ ctl,
                                                           const Entry* __restrict__ ent,
                                                           float* __restrict__ F,
                                                           float* __restrict__ T)
{
    extern __shared__ unsigned long long sQ[];      // [voxel][re, im, T]
    const int c = blockIdx.x, tid = threadIdx.x;
    if (c >= ctl[0]) return;
    const int4 ch = chunks[c];
    const int t = ch.x;
    const int tx = t % G.ntx, ty = (t / G.ntx) % G.nty, tz = t / (G.ntx * G.nty);
    const int ox = tx * BT, oy = ty * BT - G.R, oz = tz * BT - G.R;
    const int nColFT = vdim / 2 + 1;
    const float vmaxF = __uint_as_float((unsigned)ctl[2]);
    const float vmaxT = __uint_as_float((unsigned)ctl[3]);
    if (!(vmaxF <= 3.4e38f) || !(vmaxT <= 3.4e38f)) {
        // non-finite values: float atomics straight to HBM (NaN / Inf propagate)
        for (int i = tid; i < ch.z; i += D_THREADS) {
            const Entry e = ent[(size_t)ch.y + i];
            scatter_ft(reinterpret_cast<float2*>(F), T, vdim, e.x, e.y, e.z, e.vr, e.vi, e.tv);
        }
        return;
    }
    // 2^e with vmax * 2^e < 2^47 (frexp: vmax = m 2^k, m in [0.5, 1)), one
    // exponent for F (re, im) and one for T
    int kF = 0, kT = 0;
    if (vmaxF > 0.f) frexpf(vmaxF, &kF);
    if (vmaxT > 0.f) frexpf(vmaxT, &kT);
    const int exF = 47 - kF, exT = 47 - kT;
    for (int v = tid; v < 3 * BVOX; v += D_THREADS) sQ[v] = 0ull;
    __syncthreads();
    for (int i = tid; i < ch.z; i += D_THREADS) {
        const Entry e = ent[(size_t)ch.y + i];
        const float fx = floorf(e.x), fy = floorf(e.y), fz = floorf(e.z);
        const int lx = (int)fx - ox, ly = (int)fy - oy, lz = (int)fz - oz;
        const float dx = e.x - fx, dy = e.y - fy, dz = e.z - fz;
        const float wx[2] = {1.f - dx, dx}, wy[2] = {1.f - dy, dy}, wz[2] = {1.f - dz, dz};
        const int a = (lz * BH + ly) * BH + lx;
#pragma unroll
        for (int kz = 0; kz < 2; kz++)
#pragma unroll
            for (int jy = 0; jy < 2; jy++)
#pragma unroll
                for (int ix = 0; ix < 2; ix++) {
                    const float wt = wx[ix] * wy[jy] * wz[kz];
                    const int v = 3 * (a + (kz * BH + jy) * BH + ix);
                    // the float products of the float path, scaled exactly, rounded once
                    atomicAdd(&sQ[v], (unsigned long long)__float2ll_rn(ldexpf(e.vr * wt, exF)));
                    atomicAdd(&sQ[v + 1], (unsigned long long)__float2ll_rn(ldexpf(e.vi * wt, exF)));
                    atomicAdd(&sQ[v + 2], (unsigned long long)__float2ll_rn(ldexpf(e.tv * wt, exT)));
                }
    }
    __syncthreads();
    // flush: one (z, y) row per wave pass; lanes 0..33 the row's F floats,
    // lanes 34..50 its T floats
    const int lane = tid & 63, wv = tid >> 6;
    for (int row = wv; row < BH * BH; row += D_THREADS / 64) {
        const int z = row / BH, y = row - z * BH;
        long long q = 0;
        int xi = -1;
        if (lane < 2 * BH) { xi = lane >> 1; q = (long long)sQ[3 * (row * BH + xi) + (lane & 1)]; }
        else if (lane < 3 * BH) { xi = lane - 2 * BH; q = (long long)sQ[3 * (row * BH + xi) + 2]; }
        if (xi < 0 || q == 0 || ox + xi >= nColFT) continue;
        const float v = (float)ldexp((double)q, lane < 2 * BH ? -exF : -exT);
        const int gy = wrap_idx(oy + y, vdim), gz = wrap_idx(oz + z, vdim);
        const size_t g = ((size_t)gz * vdim + gy) * nColFT + ox + xi;
        if (lane < 2 * BH) atomicAdd(F + 2 * g + (lane & 1), v);
        else atomicAdd(T + g, v);
    }
}

struct BinPlan {
    TileGrid G;
    int nt, nB, maxChunks;
    long cap;
};

BinPlan plan(int nImg, int mReco, int nOrd, int pf, int rMax)
{
    BinPlan P;
    P.G = make_grid(pf, rMax);
    P.nt = P.G.ntx * P.G.nty * P.G.ntz;
    const long perImg = (long)mReco * nOrd;
    long nB = perImg > 0 ? BIN_ENT_CAP / perImg : nImg;
    nB = nB < 1 ? 1 : (nB > nImg ? nImg : nB);
    P.nB = (int)nB;
    P.cap = nB * perImg;
    P.maxChunks = (int)(P.nt + P.cap / BIN_E + 1);
    return P;
}

size_t carve(thx::Carver& cv, const BinPlan& P, int mReco, int** nG, int** gStart, double** gMat,
             float2** mShift, double** mDef, int** count, int** cursor, int4** chunks, int** ctl,
             Entry** ent)
{
    *nG = cv.take<int>(P.nB);
    *gStart = cv.take<int>((size_t)P.nB * (mReco + 1));
    *gMat = cv.take<double>((size_t)P.nB * mReco * 6);
    *mShift = cv.take<float2>((size_t)P.nB * mReco);
    *mDef = cv.take<double>((size_t)P.nB * mReco);
    *count = cv.take<int>(P.nt);
    *cursor = cv.take<int>(P.nt);
    *chunks = cv.take<int4>(P.maxChunks);
    *ctl = cv.take<int>(4);
    *ent = cv.take<Entry>(P.cap);
    return cv.off + 256;
}

}  // namespace

extern "C" size_t thx_insert3d_binned_workspace(int nImg, int mReco, int nOrd, int pf, int rMax)
{
    if (nImg <= 0 || mReco <= 0 || nOrd <= 0 || pf <= 0 || rMax <= 0) return 256;
    const BinPlan P = plan(nImg, mReco, nOrd, pf, rMax);
    thx::Carver cv(nullptr, 0);
    int *a, *b, *c, *d, *e;
    double *gm, *md;
    float2* ms;
    int4* ch;
    Entry* en;
    return carve(cv, P, mReco, &a, &b, &gm, &ms, &md, &c, &d, &ch, &e, &en);
}

// attr / nD (CTF search, both or neither): sample (l, m) inserts with the CTF
// of image l's attributes at defocus factor nD[l][m]; ctf is then unused.
static int insert_binned_impl(float* F, float* T, double* O, int* counter, int vdim, int pf,
                              const float* dat, const float* ctf, const float* attr,
                              const double* nD, const double* quat, const double* trans,
                              const double* offS, const float* w, const int* nC, int nImg,
                              int mReco, const int* iCol, const int* iRow, const int* pxOrder,
                              int nOrd, int nPxl, int idim, int rMax, void* workspace,
                              size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0 && pf > 0 && nImg >= 0 && mReco >= 0 && nPxl >= 0 &&
                      idim > 0 && rMax > 0,
                  "thx_insert3d_binned: bad sizes");
    THX_CHECK_ARG(mReco <= BIN_MAXM, "thx_insert3d_binned: mReco above %d (use thx_insert3d_tiled)",
                  BIN_MAXM);
    THX_CHECK_ARG(pf * rMax + 2 <= vdim / 2 - 1,
                  "thx_insert3d_binned: rMax * pf reaches the volume edge");
    if (nImg == 0 || mReco == 0 || nPxl == 0) return THX_OK;
    THX_CHECK_ARG(pxOrder && nOrd > 0, "thx_insert3d_binned: pxOrder required");
    const BinPlan P = plan(nImg, mReco, nOrd, pf, rMax);
    THX_CHECK_ARG(P.nt <= BIN_MAX_TILES,
                  "thx_insert3d_binned: %d tiles exceed the %d-tile histogram (use thx_insert3d_tiled)",
                  P.nt, BIN_MAX_TILES);
    THX_CHECK_ARG(F && T && O && counter && dat && (ctf || attr) && quat && trans && offS && w &&
                      iCol && iRow && workspace && (!ctf || !attr) && !attr == !nD,
                  "thx_insert3d_binned: null argument");
    thx::Carver cv(workspace, wsBytes);
    int *nG, *gStart, *count, *cursor, *ctl;
    double *gMat, *mDef;
    float2* mShift;
    int4* chunks;
    Entry* ent;
    carve(cv, P, mReco, &nG, &gStart, &gMat, &mShift, &mDef, &count, &cursor, &chunks, &ctl, &ent);
    THX_CHECK_ARG(cv.ok() && wsBytes >= cv.off, "thx_insert3d_binned: workspace too small");
    hipStream_t s = thx::as_stream(stream);
    const size_t hist = (size_t)P.nt * sizeof(int);
    static std::atomic<unsigned> ldsSet[3];
    int st = thx::set_max_lds(reinterpret_cast<const void*>(k_bin_deposit), (int)DEP_LDS, ldsSet[0]);
    if (st == THX_OK)
        st = thx::set_max_lds(reinterpret_cast<const void*>(k_bin_pass<false>), BIN_MAX_TILES * 4,
                              ldsSet[1]);
    if (st == THX_OK)
        st = thx::set_max_lds(reinterpret_cast<const void*>(k_bin_pass<true>), BIN_MAX_TILES * 4,
                              ldsSet[2]);
    if (st != THX_OK) return st;
    for (int l0 = 0; l0 < nImg; l0 += P.nB) {
        const int nb = nImg - l0 < P.nB ? nImg - l0 : P.nB;
        THX_HIP(hipMemsetAsync(count, 0, hist, s));
        hipLaunchKernelGGL(k_bin_groups, dim3(nb), dim3(G_THREADS), 0, s, quat, trans, offS, nC,
                           mReco, l0, idim, nG, gStart, gMat, mShift, O, counter, nD, mDef);
        THX_LAUNCH_CHECK();
        const dim3 pg(nb, (nOrd + BIN_KCH - 1) / BIN_KCH);
        hipLaunchKernelGGL(k_bin_pass<false>, pg, dim3(C_THREADS), hist, s, P.G, vdim, pf,
                           mReco, l0, nG, gStart, gMat, mShift, iCol, iRow, pxOrder, nOrd, nPxl,
                           reinterpret_cast<const float2*>(dat), ctf, w, count, cursor, ent,
                           reinterpret_cast<unsigned*>(ctl + 2), reinterpret_cast<float2*>(F), T,
                           attr, mDef, idim);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_bin_scan, dim3(1), dim3(1024), 0, s, count, P.nt, cursor, chunks,
                           P.maxChunks, ctl);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_bin_pass<true>, pg, dim3(C_THREADS), hist, s, P.G, vdim, pf,
                           mReco, l0, nG, gStart, gMat, mShift, iCol, iRow, pxOrder, nOrd, nPxl,
                           reinterpret_cast<const float2*>(dat), ctf, w, count, cursor, ent,
                           reinterpret_cast<unsigned*>(ctl + 2), reinterpret_cast<float2*>(F), T,
                           attr, mDef, idim);
        THX_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_bin_deposit, dim3(P.maxChunks), dim3(D_THREADS), DEP_LDS, s, P.G, vdim,
                           chunks, ctl, ent, F, T);
        THX_LAUNCH_CHECK();
    }
    return THX_OK;
}

extern "C" int thx_insert3d_binned(float* F, float* T, double* O, int* counter, int vdim, int pf,
                                   const float* dat, const float* ctf, const double* quat,
                                   const double* trans, const double* offS, const float* w,
                                   const int* nC, int nImg, int mReco, const int* iCol,
                                   const int* iRow, const int* pxOrder, int nOrd, int nPxl,
                                   int idim, int rMax, void* workspace, size_t wsBytes,
                                   thx_stream_t stream)
{
    return insert_binned_impl(F, T, O, counter, vdim, pf, dat, ctf, nullptr, nullptr, quat, trans,
                              offS, w, nC, nImg, mReco, iCol, iRow, pxOrder, nOrd, nPxl, idim,
                              rMax, workspace, wsBytes, stream);
}

extern "C" int thx_insert3d_binned_d(float* F, float* T, double* O, int* counter, int vdim,
                                     int pf, const float* dat, const float* attr,
                                     const double* nD, const double* quat, const double* trans,
                                     const double* offS, const float* w, const int* nC, int nImg,
                                     int mReco, const int* iCol, const int* iRow,
                                     const int* pxOrder, int nOrd, int nPxl, int idim, int rMax,
                                     void* workspace, size_t wsBytes, thx_stream_t stream)
{
    return insert_binned_impl(F, T, O, counter, vdim, pf, dat, nullptr, attr, nD, quat, trans,
                              offS, w, nC, nImg, mReco, iCol, iRow, pxOrder, nOrd, nPxl, idim,
                              rMax, workspace, wsBytes, stream);
}
