// local.hip -- a6 + a7 + a9: one particle-filter phase for a batch of images,
// each image with its own rotation / translation samples.
//
// The reference runs this per image with a host round trip per phase
// (ExpectLocalRTD -> ExpectLocalPreI3D -> ExpectLocalM ->
// cudaStreamSynchronize, gpu/src/cuthunder.cu:2675-3140) or, on the CPU, as
// the FOR_EACH_R / FOR_EACH_T loop of src/Optimiser.cpp:1205-1402.  Here one
// launch covers the whole batch, one workgroup per (image, 128 rotations).
//
// Per pixel i and translation t the likelihood term expands, with |T| = 1, to
//   s|d - c T P|^2 = s|d|^2 + P.re U_t + P.im V_t + b |P|^2
//   U_t = Re(Y) T.re + Im(Y) T.im,  V_t = Im(Y) T.re - Re(Y) T.im,
//   Y = -2 s c d,  b = s c^2,
// so dvp[r][t] = A_l + B_r + sum_i [P.re, P.im]_ri . [U, V]_it with the
// per-rotation bias B_r = sum_i b_i |P_ri|^2: a K = 2 nPxl product of a
// (rotation x 2 nPxl) projection tile and a (2 nPxl x translation) image tile,
// reduced on v_mfma_f32_16x16x4_f32 (two pixels per MFMA).
//
// The projection tile is the expensive part: 8 trilinear taps per
// (rotation, pixel).  A particle cloud is a few degrees wide, so the 128
// rotated copies of a compact 16-pixel patch (thx_pixel_tile_order) land in a
// small neighbourhood of the projectee.  k_patch_boxes bounds that
// neighbourhood exactly for every (image, rotation tile, patch): the
// per-rotation hull of the patch corners, split into the part with x >= 0 and
// the Hermitian-folded part with x < 0 (two boxes of one shape).
// k_local_fused streams the patches through a two-barrier software pipeline:
// while it gathers patch c from LDS the voxels of patch c+1 are in flight from
// L2/HBM into registers.  A patch whose neighbourhood exceeds the LDS box is
// gathered straight from `vol`.  Both routes sum the same taps with the same
// weights in the same order as interp_ft.
//
// Thread mapping (8 waves): wave w owns rotations 16w .. 16w+15, lane l works
// on rotation 16w + (l & 15) -- its rotation matrix lives in registers for the
// whole launch -- and on pixel 4s + (l >> 4) of step s of a patch.  After a
// step the (re, im) of the four pixels are regrouped across lane rows with
// v_permlane16_swap into the A operands of two 16x16x4 MFMAs (k = re, im of
// two pixels), so the projection tile never goes through LDS.  The y-pair
// form (LAYOUT_YPAIR2, the bench's route) maps lanes differently: two lanes
// per sample, and each tap load covers 8 rotations x the 4 pixels of a step
// (pair_step), regrouped into the same A operands with ds_bpermute.
#include <climits>

#include <cmath>

#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "patch.h"

namespace {

constexpr int THREADS = 512;
constexpr int NWAVE = THREADS / 64;
constexpr int RT = 16 * NWAVE;   // rotations per workgroup (one 16-row M-tile per wave)
constexpr int TT = 16;           // translations per workgroup (one N-tile)
constexpr int KC = thx::PATCH_KC;          // pixels per stage: one patch of the tile order
constexpr int BOX_CAP = 8192;               // LDS voxels (64 KiB) for a patch neighbourhood
constexpr int NIT = BOX_CAP / 4 / THREADS;   // 32-B box items in flight per thread
// the big-box variant (one workgroup per CU, 128 KiB of box): the
// neighbourhoods of a 1-3 degree cloud at full resolution of a large box
// (box 512: radius ~508 voxels) exceed 64 KiB
constexpr int BOX_CAP_BIG = thx::PATCH_BOX_CAP;
static_assert(BOX_CAP_BIG == 2 * BOX_CAP, "records carry offsets for the big boxes");
constexpr int REC = thx::PATCH_REC;         // ints per patch record
static_assert(RT == thx::PATCH_RT, "one record tile per workgroup");
static_assert(KC * TT <= THREADS, "one (pixel, translation) of the image tile per thread");
static_assert(BOX_CAP % (4 * THREADS) == 0, "whole prefetch rounds");
static_assert(KC == 16, "four steps of four pixels");

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(8)));

// Cell-expanded projectee (thx_volume_cells): the 8 taps of the trilinear
// cell with base (x0, y0, z0) are 64 contiguous bytes, so one gather is one
// aligned 64-B segment instead of four 16-B pieces on four rows.
THX_DEV float2 interp_cells(const float4* __restrict__ cells, int vdim, float x,
                            float y, float z)
{
    const bool conj = !(x >= 0.f);
    if (conj) { x = -x; y = -y; z = -z; }
    const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
    const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
    const float dx = x - fx, dy = y - fy, dz = z - fz;
    const int nColFT = vdim / 2 + 1;
    const size_t c = (((size_t)wrap_idx(z0, vdim) * vdim + wrap_idx(y0, vdim)) * nColFT + x0) * 4;
    const float4 q0 = cells[c], q1 = cells[c + 1], q2 = cells[c + 2], q3 = cells[c + 3];
    const float ax = 1.f - dx, ay = 1.f - dy, az = 1.f - dz;
    float w, re = 0.f, im = 0.f;
    w = ax * ay * az; re += q0.x * w; im += q0.y * w;
    w = dx * ay * az; re += q0.z * w; im += q0.w * w;
    w = ax * dy * az; re += q1.x * w; im += q1.y * w;
    w = dx * dy * az; re += q1.z * w; im += q1.w * w;
    w = ax * ay * dz; re += q2.x * w; im += q2.y * w;
    w = dx * ay * dz; re += q2.z * w; im += q2.w * w;
    w = ax * dy * dz; re += q3.x * w; im += q3.y * w;
    w = dx * dy * dz; re += q3.z * w; im += q3.w * w;
    return make_float2(re, conj ? -im : im);
}

// Quad-cooperative gather from the cell-expanded projectee: lane j (0..3) of
// the quad that evaluates one sample reads the 16-B piece j of its 64-B cell
// -- taps (dz, dy) = (j >> 1, j & 1), dx = 0, 1 -- so one wave instruction
// covers 16 samples with 16 segment accesses (the L1 merges a quad's pieces:
// tools/probes/l2_roof.hip coop64), against 64 row-piece accesses for 16
// samples in the half-complex layout.  Returns the piece's weighted part of
// interp_ft's sum (same weights; the quad sum is a tree).
THX_DEV float2 interp_cell_piece(const float4* __restrict__ cells, int vdim, float x, float y,
                                 float z, int j)
{
    const bool conj = !(x >= 0.f);
    if (conj) { x = -x; y = -y; z = -z; }
    const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
    const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
    const float dx = x - fx, dy = y - fy, dz = z - fz;
    const int nColFT = vdim / 2 + 1;
    const size_t c = (((size_t)wrap_idx(z0, vdim) * vdim + wrap_idx(y0, vdim)) * nColFT + x0) * 4 + j;
    const float4 q = cells[c];
    const float wy = (j & 1) ? dy : 1.f - dy, wz = (j >> 1) ? dz : 1.f - dz;
    const float w0 = (1.f - dx) * wy * wz, w1 = dx * wy * wz;
    const float re = q.x * w0 + q.z * w1, im = q.y * w0 + q.w * w1;
    return make_float2(re, conj ? -im : im);
}

// The quad pieces from a sample's precomputed cell (folded base x0, y0, z0,
// fractions, conj): the quad's lanes compute the coordinates of four
// different samples once and share them (coop_step), instead of each lane
// repeating all four samples' FP64 rotation -- the same values either way.
struct Cell {
    int x0, y0, z0;
    float dx, dy, dz;
    bool conj;
};
THX_DEV Cell cell_of(float x, float y, float z)
{
    Cell c;
    c.conj = !(x >= 0.f);
    if (c.conj) { x = -x; y = -y; z = -z; }
    const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
    c.x0 = (int)fx; c.y0 = (int)fy; c.z0 = (int)fz;
    c.dx = x - fx; c.dy = y - fy; c.dz = z - fz;
    return c;
}
THX_DEV float2 cell_piece(const float4* __restrict__ cells, int vdim, const Cell& c, int j)
{
    const int nColFT = vdim / 2 + 1;
    const size_t e = (((size_t)wrap_idx(c.z0, vdim) * vdim + wrap_idx(c.y0, vdim)) * nColFT + c.x0) * 4 + j;
    const float4 q = cells[e];
    const float wy = (j & 1) ? c.dy : 1.f - c.dy, wz = (j >> 1) ? c.dz : 1.f - c.dz;
    const float w0 = (1.f - c.dx) * wy * wz, w1 = c.dx * wy * wz;
    const float re = q.x * w0 + q.z * w1, im = q.y * w0 + q.w * w1;
    return make_float2(re, c.conj ? -im : im);
}
// lane p's value of a quad, to all four lanes (DPP quad_perm [p, p, p, p])
template <int P>
THX_DEV int quad_bcast(int v)
{
    return __builtin_amdgcn_mov_dpp(v, P | (P << 2) | (P << 4) | (P << 6), 0xf, 0xf, true);
}
template <int P>
THX_DEV Cell quad_bcast_cell(const Cell& c)
{
    Cell o;
    o.x0 = quad_bcast<P>(c.x0);
    o.y0 = quad_bcast<P>(c.y0);
    o.z0 = quad_bcast<P>(c.z0);
    o.dx = __int_as_float(quad_bcast<P>(__float_as_int(c.dx)));
    o.dy = __int_as_float(quad_bcast<P>(__float_as_int(c.dy)));
    o.dz = __int_as_float(quad_bcast<P>(__float_as_int(c.dz)));
    o.conj = quad_bcast<P>((int)c.conj) != 0;
    return o;
}

// Pair form of the y-pair gather (LAYOUT_YPAIR2): lane j of a pair reads
// element x0 + j of slices z0 and z0 + 1 (two 16-B loads); the pair's two
// lanes meet on the same 32-B pieces, so a sample costs two accesses.
// A pair-form sample as its rotating lane hands it to the pair: the two
// slices' element offsets (32-bit: the y-pair copy has < 2^31 elements up to
// vdim 1024) and the fractions, the Hermitian fold in dx's sign bit -- five
// DPP broadcasts and one address computation per sample instead of seven
// broadcasts and 64-bit index arithmetic in both lanes.
struct PCell {
    unsigned e0, e1;
    float dx, dy, dz;
};
// index of element (x, y, z) of the whole y-pair copy (thx_volume_ypair),
// nc = vdim / 2 + 1
// The whole y-pair copy has its slices z, z+1 (z even) interleaved element
// by element as in the ball: for even z0 a sample's four 16-B elements are
// one contiguous 64-B piece (full resolution, box 256: 14.0 -> 12.1 ms at 1.5
// deg, 18.4 -> 16.0 at 2 deg, 27.5 -> 23.0 at 3, profiles/r04_fullres_wzil_ab.jsonl)
// (24-bit multiplies, mad24: every factor is below 2^24 and every result
// below 2^32 up to vdim 1024)
THX_DEV unsigned ypair_elem(unsigned z, unsigned y, unsigned x, unsigned vdim, unsigned nc)
{
    return mad24(mad24(z >> 1, vdim, y), nc, x) * 2u + (z & 1u);
}
// In the compact ball slices z and z + 1 (z + R even) are interleaved element
// by element, so for such z0 a sample's four 16-B elements (x0, x0 + 1 of
// both slices) are one contiguous 64-B piece
// ballR > 0: the copy is the compact ball of thx::volume_ypair_ball --
// elements (x, y, z), 0 <= x < ballR + 2, -ballR <= y, z < ballR + 2, no
// wrap (every tap of the pixel ring lies inside)
THX_DEV unsigned ypair_ball_elem(int z, int y, int x, int ballR)
{
    const unsigned Y = 2u * ballR + 2u, X = (unsigned)ballR + 2u;
    const unsigned zc = (unsigned)(z + ballR), yc = (unsigned)(y + ballR);
    return mad24(mad24(zc >> 1, Y, yc), X, (unsigned)x) * 2u + (zc & 1u);
}
THX_DEV PCell pcell_of(float x, float y, float z, int vdim, int ballR = 0)
{
    const bool conj = !(x >= 0.f);
    if (conj) { x = -x; y = -y; z = -z; }
    const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
    const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
    const unsigned nc = (unsigned)(vdim / 2 + 1);
    const unsigned yw = (unsigned)wrap_idx(y0, vdim);
    PCell c;
    if (ballR > 0) {
        // slice z0 + 1: the other element of the interleaved pair when z0 + R
        // is even, else the first element of the next pair of slices
        c.e0 = ypair_ball_elem(z0, y0, x0, ballR);
        const unsigned X2Y = 2u * ((unsigned)ballR + 2u) * (2u * ballR + 2u);   // (uniform)
        c.e1 = c.e0 + (((unsigned)(z0 + ballR) & 1u) ? X2Y - 1u : 1u);
    } else {
        c.e0 = ypair_elem((unsigned)wrap_idx(z0, vdim), yw, (unsigned)x0, (unsigned)vdim, nc);
        c.e1 = ypair_elem((unsigned)wrap_idx(z0 + 1, vdim), yw, (unsigned)x0, (unsigned)vdim, nc);
    }
    c.dx = __uint_as_float(__float_as_uint(x - fx) | (conj ? 0x80000000u : 0u));
    c.dy = y - fy;
    c.dz = z - fz;
    return c;
}
// lane j of the pair: element x0 + j of slices z0 and z0 + 1
// (xs: the element stride of x -- 2 in the z-interleaved ball, else 1);
// the loads apart from the interpolation, so a step issues all its loads
// before the first one is waited on
struct PTaps { float4 q0, q1; };
THX_DEV PTaps ypair_pcell_load(const float4* __restrict__ yp, const PCell& c, int j, unsigned xs)
{
    const unsigned dj = xs * (unsigned)j;   // element x0 + j
    return PTaps{yp[c.e0 + dj], yp[c.e1 + dj]};
}
THX_DEV float2 ypair_pcell_lerp(const PTaps& t, const PCell& c, int j)
{
    const float4 q0 = t.q0, q1 = t.q1;
    const bool conj = (__float_as_uint(c.dx) >> 31) != 0;
    const float dx = fabsf(c.dx);
    const float wx = j ? dx : 1.f - dx;
    const float wa = wx * (1.f - c.dz), wb = wx * c.dz;
    const float w00 = wa * (1.f - c.dy), w01 = wa * c.dy, w10 = wb * (1.f - c.dy), w11 = wb * c.dy;
    // (re, im) pairs of the four taps as packed operands (v_pk_fma_f32 with
    // the weight broadcast), in the order of the scalar sum
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v r = f2v{q0.x, q0.y} * w00 + f2v{q0.z, q0.w} * w01 + f2v{q1.x, q1.y} * w10 +
                  f2v{q1.z, q1.w} * w11;
    return make_float2(r.x, conj ? -r.y : r.y);
}
// the pair's other lane's value (DPP quad_perm [1, 0, 3, 2])
THX_DEV float pair_swap(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xb1, 0xf, 0xf, true));
}
// lane IT of each pair, to both lanes (quad_perm [IT, IT, 2 + IT, 2 + IT])
template <int IT>
THX_DEV int pair_bcast(int v)
{
    return __builtin_amdgcn_mov_dpp(v, IT | (IT << 2) | ((2 + IT) << 4) | ((2 + IT) << 6), 0xf, 0xf,
                                    true);
}
template <int IT>
THX_DEV PCell pair_bcast_pcell(const PCell& c)
{
    PCell o;
    o.e0 = (unsigned)pair_bcast<IT>((int)c.e0);
    o.e1 = (unsigned)pair_bcast<IT>((int)c.e1);
    o.dx = __int_as_float(pair_bcast<IT>(__float_as_int(c.dx)));
    o.dy = __int_as_float(pair_bcast<IT>(__float_as_int(c.dy)));
    o.dz = __int_as_float(pair_bcast<IT>(__float_as_int(c.dz)));
    return o;
}
// sum over the lanes of each quad (DPP quad permutations), every lane gets it
THX_DEV float quad_sum(float v)
{
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xb1, 0xf, 0xf, true));
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4e, 0xf, 0xf, true));
    return v;
}

// Projectee layouts of the phase: the half-complex volume (0), its
// cell-expanded copy (1, quad-cooperative gathers, no LDS boxes) and its
// y-pair copy (2, thx_volume_ypair: element (x, y, z) holds v(x, y, z) and
// v(x, y + 1, z), so a trilinear cell is two 32-B pieces, gathered by lane
// pairs -- ypair_pcell_load / ypair_pcell_lerp).
enum { LAYOUT_FT = 0, LAYOUT_CELLS = 1, LAYOUT_YPAIR2 = 2 };
// layouts gathered quad-cooperatively (no LDS boxes, no patch records)
constexpr bool coop_layout(int l) { return l == LAYOUT_CELLS; }

// Patch record (k_patch_boxes -> k_local_fused): layout in patch.h.
struct Rec {
    int v[REC];
    THX_DEV bool staged() const { return v[10] <= BOX_CAP; }
};

THX_DEV Rec load_rec(const int* __restrict__ p)
{
    Rec r;
    const int4* q = reinterpret_cast<const int4*>(p);
#pragma unroll
    for (int k = 0; k < REC / 4; k++) {
        const int4 a = q[k];
        r.v[4 * k] = a.x; r.v[4 * k + 1] = a.y; r.v[4 * k + 2] = a.z; r.v[4 * k + 3] = a.w;
    }
    return r;
}

// Wave-wide integer min / max: 4 DPP steps inside each row of 16, then the
// four row results through readlane.  |v| < 2^30.
THX_DEV int wave_min_i(int v)
{
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0xb1, 0xf, 0xf, false));   // quad_perm 1032
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x4e, 0xf, 0xf, false));   // quad_perm 2301
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x124, 0xf, 0xf, false));  // row_ror 4
    v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x128, 0xf, 0xf, false));  // row_ror 8
    return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
               min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

THX_DEV int wave_max_i(int v) { return -wave_min_i(-v); }

// Exact u / d for u * d < 2^32 with m = magic(d) (round-up reciprocal).
THX_DEV unsigned magic(unsigned d) { return d <= 1 ? 0u : 0xFFFFFFFFu / d + 1u; }
THX_DEV int udiv(int u, int d, unsigned m) { return d <= 1 ? u : (int)__umulhi((unsigned)u, m); }

constexpr int BIG = 1 << 29;

// The patch record from the folded-box bounds e (side 0 lo xyz, hi xyz; side 1).
THX_DEV int store_rec(const int (&e)[12], int ic0, int ir0, int vdim, int* __restrict__ out)
{
    const int nColFT = vdim / 2 + 1, half = vdim / 2;
    int o[REC] = {0};
    int lo[2][3], n[2][3];
    bool any[2];
    for (int s = 0; s < 2; s++) {
        // clamp into the half volume (rows / slices wrap once at most)
        lo[s][0] = max(e[6 * s], 0) & ~3;   // whole 4-voxel items (32 B, a brick row)
        lo[s][1] = max(e[6 * s + 1], -half);
        lo[s][2] = max(e[6 * s + 2], -half);
        n[s][0] = min(e[6 * s + 3], nColFT - 1) - lo[s][0] + 1;
        n[s][1] = min(e[6 * s + 4], half) - lo[s][1] + 1;
        n[s][2] = min(e[6 * s + 5], half) - lo[s][2] + 1;
        any[s] = n[s][0] > 0 && n[s][1] > 0 && n[s][2] > 0;
    }
    int nx = 4, ny = 1, nz = 1;
    for (int s = 0; s < 2; s++)
        if (any[s]) {
            nx = max(nx, (n[s][0] + 3) & ~3);   // rows padded to 4 voxels (32 B)
            ny = max(ny, n[s][1]);
            nz = max(nz, n[s][2]);
        }
    // LDS bank spread: the 16 lanes of a ds_read2_b64 group read 8-B voxels
    // whose index mod 16 picks the bank pair; a row pitch of 4 x odd and a
    // slice pitch = 2 mod 16 keep the neighbouring rows / slices that the 16
    // rotations of one pixel touch on different banks
    if ((nx / 4) % 2 == 0) nx += 4;
    long sp = (long)nx * ny;
    sp += ((2 - sp % 16) + 16) % 16;
    const long nv = sp * nz;
    const long nv0 = any[0] ? nv : 0, nv1 = any[1] ? nv : 0;
    const long ni = (long)(nx / 4) * ny * nz;
    for (int s = 0; s < 3; s++) { o[s] = lo[0][s]; o[3 + s] = lo[1][s]; }
    o[6] = nx;
    o[7] = (int)min(sp, (long)BIG);
    o[8] = ny;
    o[9] = (int)min(nv0, (long)BIG);
    o[10] = (int)min(nv0 + nv1, (long)BIG);
    o[11] = (int)min(any[0] ? ni : 0, (long)BIG);
    o[12] = (int)min((any[0] ? ni : 0) + (any[1] ? ni : 0), (long)BIG);
    o[13] = (int)magic((unsigned)nx / 4);
    o[14] = (int)magic((unsigned)ny);
    if (nv0 + nv1 <= BOX_CAP_BIG) {
        o[15] = -(lo[0][2] * o[7] + lo[0][1] * nx + lo[0][0]);
        o[16] = o[9] - (lo[1][2] * o[7] + lo[1][1] * nx + lo[1][0]);
    }
    o[17] = ic0;
    o[18] = ir0;
    int4* dst = reinterpret_cast<int4*>(out);
    for (int k = 0; k < REC / 4; k++)
        dst[k] = make_int4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
    return o[10];
}

// Route of a phase (FT layout, 64 KiB boxes): a sample of the images' patch
// records is counted first (route[0] patches whose box fits, route[1]
// patches); below STAGE_MIN_PCT per cent staged, the phase gathers every
// patch from L2 with the box-less kernel (6 waves per SIMD instead of 4, no
// records), otherwise records are built for all images and the staged kernel
// runs.  Both kernels are launched; the one not chosen exits at entry, so the
// choice needs no host round trip.
constexpr int STAGE_MIN_PCT = 50;
constexpr int ROUTE_SAMPLE = 64;   // every 64th image's records are counted (16: 41 us per
                                   // phase at 12 500 images, 64: the same routes)

// Third route (round 3): when the caller supplies a y-pair copy (route[2] =
// 1), every phase whose boxes do not pay gathers from it with the pair form
// (LAYOUT_YPAIR2: two lanes per sample, the 32-B pieces of slices z0 and
// z0 + 1), two accesses per sample where the half-complex rows take four;
// faster than the box-less half-complex kernel in all ten bench phases
// (profiles/r03_pair_ab.jsonl), so with a y-pair copy the box-less
// half-complex kernel is not launched at all.
// route[0]: sampled patches whose box fits, route[1]: sampled patches,
// route[2]: a y-pair copy exists.
constexpr int ROUTE_STAGED = 0, ROUTE_NOBOX = 1, ROUTE_YPAIR = 2;
THX_DEV bool route_nostage(const int* __restrict__ route)
{
    return (long)route[0] * 100 < (long)STAGE_MIN_PCT * route[1];
}
THX_DEV int route_pick(const int* __restrict__ route)
{
    if (!route_nostage(route)) return ROUTE_STAGED;
    return route[2] == 1 ? ROUTE_YPAIR : ROUTE_NOBOX;
}
// the route's choice to the caller (thx_local_phase_routed, the driver's
// phaseRoute)
__global__ void k_route_out(const int* __restrict__ route, int* __restrict__ out)
{
    if (threadIdx.x == 0) *out = route_pick(route);
}


// 3D Morton code of three 10-bit coordinates.
THX_DEV unsigned morton3(unsigned x, unsigned y, unsigned z)
{
    auto spread = [](unsigned v) {
        v &= 0x3ffu;
        v = (v | (v << 16)) & 0x030000ffu;
        v = (v | (v << 8)) & 0x0300f00fu;
        v = (v | (v << 4)) & 0x030c30c3u;
        v = (v | (v << 2)) & 0x09249249u;
        return v;
    };
    return spread(x) | (spread(y) << 1) | (spread(z) << 2);
}

// Lane slot -> rotation of the tile.  A particle cloud arrives in resampling
// order (copies of one ancestor adjacent, ancestors in no spatial order), so
// the 16 rotations a wave gathers for one pixel can land anywhere in the
// cloud.  Ranking the tile's rotations by the Morton code of their vector
// part relative to the tile's first rotation (10 bits per axis, 0.22 deg)
// gives each wave a compact group of rotations: its 16 lanes then read
// neighbouring voxels (shared cache lines on the L2 gathers, spread banks on
// the LDS taps).  Per-rotation arithmetic is unchanged, only which lane does
// it; rows past nRl keep key ~0u and sort last.
THX_DEV void rotation_slots(const double* __restrict__ q4, int nRl, int tid,
                            unsigned* __restrict__ sKey, int* __restrict__ sPerm)
{
    if (tid < RT) {
        unsigned key = ~0u;
        if (tid < nRl) {
            const double a0 = q4[0], a1 = -q4[1], a2 = -q4[2], a3 = -q4[3];   // conj(q_0)
            const double* b = q4 + 4 * tid;
            double w = a0 * b[0] - a1 * b[1] - a2 * b[2] - a3 * b[3];
            double x = a0 * b[1] + a1 * b[0] + a2 * b[3] - a3 * b[2];
            double y = a0 * b[2] - a1 * b[3] + a2 * b[0] + a3 * b[1];
            double z = a0 * b[3] + a1 * b[2] - a2 * b[1] + a3 * b[0];
            if (w < 0.0) { x = -x; y = -y; z = -z; }
            auto qz = [](double v) { return (unsigned)min(1023.0, max(0.0, (v + 1.0) * 512.0)); };
            key = morton3(qz(x), qz(y), qz(z)) ;
        } else if (tid < nRl) {
            key = (unsigned)tid;
        }
        sKey[tid] = key;
    }
    __syncthreads();
    if (tid < RT) {
        const unsigned k = sKey[tid];
        int rank = 0;
        for (int j = 0; j < RT; j++) {
            const unsigned kj = sKey[j];
            rank += (kj < k) || (kj == k && j < tid);
        }
        sPerm[rank] = tid;
    }
    __syncthreads();
}

// Slot -> rotation of the tile (rotation_slots' sPerm): slots past nRl (the
// tile's padding rows, never stored) take their wave group's first rotation,
// so the 16 rotations a wave gathers for stay one compact group; a group of
// padding only takes the tile's first.
THX_DEV int slot_rotation(const int* __restrict__ sPerm, int slot, int nRl)
{
    const int rp = sPerm[slot];
    if (rp < nRl) return rp;
    const int g0 = sPerm[slot & ~15];
    return g0 < nRl ? g0 : 0;
}

// One workgroup per (image, rotation tile), one lane per patch, the tile's
// rotation slots (rotation_slots: the Morton-ranked order k_local_fused's
// waves take them in) split over the 4 waves: the LDS boxes that hold every
// tap of the patch's samples under the tile's rotations.  The matrices sit
// in LDS and are read as broadcasts; per rotation and axis the extremes of
// the rotated patch rectangle are its corners picked by the signs of the two
// matrix entries.  The waves' partial bounds meet in LDS.
constexpr int PB_WAVES = 4;
constexpr int PB_SLOTS = RT / PB_WAVES;   // 32 slots per wave

__global__ void __launch_bounds__(64 * PB_WAVES) k_patch_boxes(const double* __restrict__ quat,
                                                               int nR,
                                                               const int* __restrict__ iCol,
                                                               const int* __restrict__ iRow,
                                                               const int* __restrict__ order,
                                                               int nVisit, int pf, int vdim,
                                                               int* __restrict__ rec,
                                                               const int* __restrict__ act,
                                                               const int* __restrict__ nAct,
                                                               int* __restrict__ route = nullptr,
                                                               int routeMode = 0)
{
    __shared__ float sM[RT][6];
    __shared__ int sE[PB_WAVES][12][64];
    __shared__ unsigned sKey[RT];
    __shared__ int sPerm[RT];
    // routeMode 1: count the records of every ROUTE_SAMPLE-th image into
    // route; 2: build all records unless the count chose the box-less kernel
    if (routeMode == 2 && route_pick(route) != ROUTE_STAGED) return;
    const int nC = (nVisit + KC - 1) / KC, nRT = (nR + RT - 1) / RT;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ry = blockIdx.x % nRT;
    int l = (blockIdx.x / nRT) * (routeMode == 1 ? ROUTE_SAMPLE : 1);
    if (act) {                     // active-image list: slots past the count exit
        if (l >= *nAct) return;
        l = act[l];
    }
    int nFit = 0, nAll = 0;
    const int nRl = min(RT, nR - ry * RT);
    const double* Q = quat + ((size_t)l * nR + ry * RT) * 4;
    rotation_slots(Q, nRl, threadIdx.x, sKey, sPerm);
    for (int k = threadIdx.x; k < RT; k += 64 * PB_WAVES) {
        const int r = slot_rotation(sPerm, k, nRl);
        double q[4], m[9];
        for (int a = 0; a < 4; a++) q[a] = Q[(size_t)r * 4 + a];
        quat_to_mat(q, m);
        for (int a = 0; a < 6; a++) sM[k][a] = (float)m[a];
    }
    __syncthreads();
    const int rBeg = wv * PB_SLOTS, rEnd = rBeg + PB_SLOTS;
    // every rotated point lies in the corner hull; the bounds are FP32
    // (|error| < 1e-4 voxel against the FP64-then-rounded sample coordinates),
    // widened by EPS before the floor; a cell spans floor(c) .. floor(c) + 1.
    // The extremes are tracked in FP32 and floored once: floor and the clamp
    // at 0 are monotone, so this equals flooring every rotation's bound.
    constexpr float EPS = 1e-3f;
    for (int c0 = 0; c0 < nC; c0 += 64) {
        const int c = c0 + lane;
        int cLo = BIG, cHi = -BIG, rLo = BIG, rHi = -BIG, ic0 = 0, ir0 = 0;
        int pk[KC], pc[KC], pr[KC];
#pragma unroll
        for (int k = 0; k < KC; k++) pk[k] = patch_pixel(order, nVisit, c * KC + k);
#pragma unroll
        for (int k = KC - 1; k >= 0; k--) {
            pc[k] = iCol[max(pk[k], 0)];    // loads in flight together
            pr[k] = iRow[max(pk[k], 0)];
            if (pk[k] >= 0) {
                cLo = min(cLo, pc[k]); cHi = max(cHi, pc[k]);
                rLo = min(rLo, pr[k]); rHi = max(rHi, pr[k]);
                ic0 = pc[k]; ir0 = pr[k];   // ends on the patch's first pixel
            }
        }
        int e[12];
#pragma unroll
        for (int k = 0; k < 12; k++) e[k] = (k % 6) < 3 ? BIG : -BIG;
        if (cLo <= cHi) {
            const float X0 = (float)(cLo * pf), X1 = (float)(cHi * pf);
            const float Y0 = (float)(rLo * pf), Y1 = (float)(rHi * pf);
            float f[12];
#pragma unroll
            for (int k = 0; k < 12; k++) f[k] = (k % 6) < 3 ? INFINITY : -INFINITY;
            for (int r = rBeg; r < rEnd; r++) {
                const float* m = sM[r];
                float mn[3], mx[3];
#pragma unroll
                for (int a = 0; a < 3; a++) {
                    const float u = m[a], v = m[a + 3];
                    mn[a] = u * (u >= 0 ? X0 : X1) + v * (v >= 0 ? Y0 : Y1);
                    mx[a] = u * (u >= 0 ? X1 : X0) + v * (v >= 0 ? Y1 : Y0);
                }
                if (mx[0] >= -EPS)
#pragma unroll
                    for (int a = 0; a < 3; a++) {
                        f[a] = fminf(f[a], mn[a]);
                        f[3 + a] = fmaxf(f[3 + a], mx[a]);
                    }
                if (mn[0] < EPS)
#pragma unroll
                    for (int a = 0; a < 3; a++) {
                        f[6 + a] = fminf(f[6 + a], -mx[a]);
                        f[9 + a] = fmaxf(f[9 + a], -mn[a]);
                    }
            }
            if (f[0] != INFINITY) {
                e[0] = (int)floorf(fmaxf(f[0] - EPS, 0.f));
                e[1] = (int)floorf(f[1] - EPS);
                e[2] = (int)floorf(f[2] - EPS);
                e[3] = (int)floorf(f[3] + EPS) + 1;
                e[4] = (int)floorf(f[4] + EPS) + 1;
                e[5] = (int)floorf(f[5] + EPS) + 1;
            }
            if (f[6] != INFINITY) {
                e[6] = (int)floorf(fmaxf(f[6] - EPS, 0.f));
                e[7] = (int)floorf(f[7] - EPS);
                e[8] = (int)floorf(f[8] - EPS);
                e[9] = (int)floorf(f[9] + EPS) + 1;
                e[10] = (int)floorf(f[10] + EPS) + 1;
                e[11] = (int)floorf(f[11] + EPS) + 1;
            }
        }
#pragma unroll
        for (int k = 0; k < 12; k++) sE[wv][k][lane] = e[k];
        __syncthreads();
        if (wv == 0 && c < nC) {
            for (int w = 1; w < PB_WAVES; w++)
#pragma unroll
                for (int k = 0; k < 12; k++)
                    e[k] = (k % 6) < 3 ? min(e[k], sE[w][k][lane]) : max(e[k], sE[w][k][lane]);
            const int nv = store_rec(e, ic0, ir0, vdim, rec + (((size_t)l * nRT + ry) * nC + c) * REC);
            nFit += nv <= BOX_CAP;
            nAll += 1;
        }
        __syncthreads();
    }
    if (routeMode == 1 && wv == 0) {
        nFit = wave_sum(nFit);
        nAll = wave_sum(nAll);
        if (lane == 0) {
            atomicAdd(&route[0], nFit);
            atomicAdd(&route[1], nAll);
        }
    }
}

// Pixel of the image tile a staging thread owns: (iCol, iRow), data.
struct Pix {
    int p, ic, ir;
    float2 d;
    float c, s;
};

THX_DEV Pix load_pix(int p, const int* __restrict__ iCol, const int* __restrict__ iRow,
                     const float2* __restrict__ D, const float* __restrict__ C,
                     const float* __restrict__ S)
{
    Pix x{p, 0, 0, make_float2(0.f, 0.f), 0.f, 0.f};
    if (p >= 0) {
        x.ic = iCol[p];
        x.ir = iRow[p];
        x.d = D[p];
        x.c = C[p];
        x.s = S[p];
    }
    return x;
}

// The items (4 consecutive voxels of a box row, 32 B) of a staged patch this
// thread moves: item it = tid + j THREADS, LDS voxel dst[j].
template <int LAYOUT, int NI = NIT, int CAP = BOX_CAP>
THX_DEV void fetch_box(f32x4 (&pre)[NI][2], int (&dst)[NI], const Rec& b,
                       const float2* __restrict__ vol, int vdim, int tid)
{
    if (coop_layout(LAYOUT) || !(b.v[10] <= CAP)) return;   // cells / y-pairs: never staged
    const int nColFT = vdim / 2 + 1;
    const int nq = b.v[6] >> 2, ny = b.v[8];
#pragma unroll
    for (int j = 0; j < NI; j++) {
        const int it = tid + j * THREADS;
        if (it < b.v[12]) {
            const bool s1 = it >= b.v[11];
            const int u = s1 ? it - b.v[11] : it;
            const int row = udiv(u, nq, (unsigned)b.v[13]);
            const int xq = u - row * nq;
            const int z = udiv(row, ny, (unsigned)b.v[14]);
            const int y = row - z * ny;
            dst[j] = (s1 ? b.v[9] : 0) + z * b.v[7] + y * b.v[6] + 4 * xq;
            const int gx = (s1 ? b.v[3] : b.v[0]) + 4 * xq;
            const int gy = wrap_idx((s1 ? b.v[4] : b.v[1]) + y, vdim);
            const int gz = wrap_idx((s1 ? b.v[5] : b.v[2]) + z, vdim);
            const unsigned g = ((unsigned)gz * vdim + gy) * nColFT + gx;
            if (LAYOUT == LAYOUT_FT && gx + 3 < nColFT) {
                const f32x4u* p = reinterpret_cast<const f32x4u*>(vol + g);
                const f32x4u lo = p[0], hi = p[1];
                pre[j][0] = f32x4{lo.x, lo.y, lo.z, lo.w};
                pre[j][1] = f32x4{hi.x, hi.y, hi.z, hi.w};
                continue;
            }
            float2 e[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                e[k] = make_float2(0.f, 0.f);
                if (gx + k < nColFT) {
                    if (LAYOUT == LAYOUT_CELLS) {
                        const float4 q = reinterpret_cast<const float4*>(vol)[(size_t)(g + k) * 4];
                        e[k] = make_float2(q.x, q.y);
                    } else {
                        e[k] = vol[g + k];
                    }
                }
            }
            pre[j][0] = f32x4{e[0].x, e[0].y, e[1].x, e[1].y};
            pre[j][1] = f32x4{e[2].x, e[2].y, e[3].x, e[3].y};
        }
    }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));


// Trilinear gather of getByInterpolationFT (the taps and weights of
// interp_ft, common.h) from the staged boxes, on packed FP32: the weights are
// vx (vy vz) and (re, im) accumulates with v_pk_fma_f32 -- fused, so it can
// differ from interp_ft in the last bits.
THX_DEV float2 interp_box(const float2* __restrict__ box, int nx, int sp, int off0, int off1,
                          float x, float y, float z)
{
    const bool conj = !(x >= 0.f);
    if (conj) { x = -x; y = -y; z = -z; }
    const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
    const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
    const float dx = x - fx, dy = y - fy, dz = z - fz;
    const f32x2 vx = {1.f - dx, dx};
    const float vy0 = 1.f - dy, vz0 = 1.f - dz;
    // |coordinates| < 2^23: 24-bit multiplies (full rate) for the LDS index
    const int a = __mul24(z0, sp) + __mul24(y0, nx) + x0 + (conj ? off1 : off0);
    const f32x2* bx = reinterpret_cast<const f32x2*>(box);
    const f32x2 a0 = bx[a], a1 = bx[a + 1];
    const f32x2 b0 = bx[a + nx], b1 = bx[a + nx + 1];
    const f32x2 c0 = bx[a + sp], c1 = bx[a + sp + 1];
    const f32x2 d0 = bx[a + sp + nx], d1 = bx[a + sp + nx + 1];
    const f32x2 w00 = vx * (vy0 * vz0), w10 = vx * (dy * vz0);
    const f32x2 w01 = vx * (vy0 * dz), w11 = vx * (dy * dz);
    f32x2 s = a0 * w00.x;
    s = __builtin_elementwise_fma(a1, (f32x2)w00.y, s);
    s = __builtin_elementwise_fma(b0, (f32x2)w10.x, s);
    s = __builtin_elementwise_fma(b1, (f32x2)w10.y, s);
    s = __builtin_elementwise_fma(c0, (f32x2)w01.x, s);
    s = __builtin_elementwise_fma(c1, (f32x2)w01.y, s);
    s = __builtin_elementwise_fma(d0, (f32x2)w11.x, s);
    s = __builtin_elementwise_fma(d1, (f32x2)w11.y, s);
    return make_float2(s.x, conj ? -s.y : s.y);
}


// CS (CTF search, SEARCH_TYPE_CTF): the columns are the nT x nD (t, d) pairs
// of kernel_logDataVSLC (gpu/src/Kernel.cu:889-939), column j = t nD + d; the
// image tile takes its CTF from ctfD[l][d] (thx_ctf_search) per column, and
// the bias sum_i s c_d^2 |P|^2 now depends on the column, so it runs on the
// MFMA as well: A = (re^2, im^2) regrouped like (re, im), B = (b_j, b_j).
// A CS workgroup covers NCT column tiles of 16 (up to 96 (t, d) columns), so
// the projection -- the expensive part -- is gathered once for all of them;
// each step then issues 4 NCT MFMAs against NCT accumulators.
// the big-box kernel from a pixel ring of BIGBOX_MIN_R projectee voxels on
// (C5 full resolution; profiles/r02_local_bigbox_ab.jsonl)
constexpr double BIGBOX_MIN_R = 300;
// box-less and y-pair kernels: 6 waves per SIMD (4 / 5 / 8 measured slower,
// profiles/r03_nobox_waves_ab.jsonl, r04_pair_waves_ball_ab.jsonl)
constexpr int NOBOX_WAVES = 6;
template <int LAYOUT, bool CS = false, int NCT = 1, bool BIGBOX = false, bool STAGE = true>
// non-CS: two workgroups per CU (LDS-bound), 4 waves per SIMD, 128 VGPRs;
// CS: the NCT accumulators and CTF prefetches need the 256-VGPR budget;
// BIGBOX: 128 KiB of box, one workgroup per CU, twice the prefetch registers;
// no LDS box (cell layout, or STAGE = false): no box prefetch registers, so
// 6 waves per SIMD (three workgroups per CU) for the L2 gathers
__global__ void __launch_bounds__(THREADS)
__attribute__((amdgpu_waves_per_eu((CS || BIGBOX) ? 2 : (coop_layout(LAYOUT) || LAYOUT == LAYOUT_YPAIR2 || !STAGE) ? NOBOX_WAVES : 4)))
k_local_fused(const float2* __restrict__ vol,
                                                            int vdim, int pf,
                                                            const double* __restrict__ quat,
                                                            int nR,
                                                            const double* __restrict__ trans,
                                                            int nT,
                                                            const float2* __restrict__ dat,
                                                            const float* __restrict__ ctf,
                                                            const float* __restrict__ sig,
                                                            const int* __restrict__ iCol,
                                                            const int* __restrict__ iRow,
                                                            const int* __restrict__ order,
                                                            int nVisit, int nPxl, int idim,
                                                            const int* __restrict__ rec,
                                                            float* __restrict__ dvp,
                                                            const int* __restrict__ act,
                                                            const int* __restrict__ nAct,
                                                            const int* __restrict__ cls,
                                                            long volStride, int nD = 1,
                                                            const double* __restrict__ pC = nullptr,
                                                            const double* __restrict__ pR = nullptr,
                                                            const double* __restrict__ pT = nullptr,
                                                            float* __restrict__ wC = nullptr,
                                                            float* __restrict__ wR = nullptr,
                                                            float* __restrict__ wT = nullptr,
                                                            float* __restrict__ baseL = nullptr,
                                                            const int* __restrict__ route = nullptr,
                                                            int ballR = 0)
{
    // routed phases launch the staged and the box-less kernel; one exits
    if (route && route_pick(route) != (LAYOUT == LAYOUT_YPAIR2 ? ROUTE_YPAIR
                                       : STAGE ? ROUTE_STAGED : ROUTE_NOBOX)) return;
    int l = blockIdx.x;
    if (act) {
        if (l >= *nAct) return;
        l = act[l];
    }
    // classification: image l projects its own class's volume
    if (cls) vol += (size_t)cls[l] * volStride;
    static_assert(CS || NCT == 1, "column tiles per workgroup: CTF search only");
    constexpr int BOXC = BIGBOX ? BOX_CAP_BIG : BOX_CAP;
    constexpr int NITC = BOXC / 4 / THREADS;
    // the cell layout gathers every sample quad-cooperatively: no LDS box, no
    // patch records (padding entries sample pixel (0, 0)), so a CU holds as
    // many workgroups as the VGPRs allow
    constexpr bool COOP = coop_layout(LAYOUT);
    // STAGE = false: every patch gathered from L2 (no box, no records)
    // the pair form of the y-pair gather (two lanes per sample)
    constexpr bool PAIR = LAYOUT == LAYOUT_YPAIR2;
    constexpr bool NOBOX = COOP || PAIR || !STAGE;
    auto staged = [](const Rec& r) { return !NOBOX && r.v[10] <= BOXC; };
    constexpr int NC = NCT * TT;   // columns per workgroup
    // box-less kernels stage PP patches' image tiles per barrier pair (fewer
    // barriers, 4 PP independent steps between them); CS keeps one.  PP 2:
    // full-res cells -2.5 %, the bench's phases unchanged; PP 4 needs two
    // image-tile elements per thread and spills (profiles/r03_nobox_pp_ab.jsonl)
    constexpr int PP = (coop_layout(LAYOUT) || PAIR || !STAGE) && !CS ? 2 : 1;
    constexpr int PKC = PP * KC;                        // pixels per iteration
    constexpr int NE = (PKC * TT + THREADS - 1) / THREADS;   // image-tile elements per thread
    const int r0 = blockIdx.y * RT, t0 = blockIdx.z * NC;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nRl = min(RT, nR - r0);
    __shared__ __attribute__((aligned(16))) float2 sBox[NOBOX ? 8 : BOXC];
    __shared__ __attribute__((aligned(16))) float sB[PKC * 2 * NC];  // [px][U, V][t]
    // (iCol pf, iRow pf): small integers, exact in FP32 and widened exactly to
    // FP64 by the FP64 rotations
    // (kept in FP64: the rotations read them as doubles, no per-step widening)
    __shared__ __attribute__((aligned(16))) double2 sXY[PKC];
    __shared__ float sBq[CS ? KC * NC : PKC];                        // b = s c^2 ([px][col] for CS)
    __shared__ int sValid[PKC];                                      // 0: padding entry
    __shared__ float sTr[NC][2];
    __shared__ float sRed[NWAVE];
    __shared__ float sBias[RT];
    __shared__ unsigned sKey[RT];
    __shared__ int sPerm[RT];   // lane slot -> rotation of the tile

    rotation_slots(quat + ((size_t)l * nR + r0) * 4, nRl, tid, sKey, sPerm);
    // this lane's rotation (rows past nR reuse the tile's first rotation, so
    // their taps stay inside the staged box; those rows are never stored)
    const int rl = wv * 16 + (lane & 15);
    double m[6];
    {
        // COOP: lane 4 r + j works on rotation slot 16 wv + r (its quad's sample)
        // PAIR: lane 2 k + j works on rotation slot 16 wv + (k & 15)
        // PAIR: lane 2 k + j (k = r8 + 8 p) works on rotation slot 16 wv + r8 + 8 j
        const int pairSlot = wv * 16 + ((lane >> 1) & 7) + 8 * (lane & 1);
        const int r = r0 + slot_rotation(sPerm, COOP ? wv * 16 + (lane >> 2)
                                                : PAIR ? pairSlot : rl, nRl);
        double q[4], mm[9];
        for (int k = 0; k < 4; k++) q[k] = quat[((size_t)l * nR + r) * 4 + k];
        quat_to_mat(q, mm);
        for (int k = 0; k < 6; k++) m[k] = mm[k];
    }

    // columns: translations, or (t, d) pairs for CS (nT counts the columns)
    if (tid < NC) {
        const int t = CS ? (t0 + tid) / nD : t0 + tid;
        float tx = 0.f, ty = 0.f;
        if (t0 + tid < nT) {
            const size_t ti = (size_t)l * (CS ? nT / nD : nT) + t;   // translation rows
            tx = (float)trans[ti * 2];
            ty = (float)trans[ti * 2 + 1];
        }
        sTr[tid][0] = tx / idim;   // rCol of translate(), ImageFunctions.cpp:243
        sTr[tid][1] = ty / idim;
    }

    const float2* D = dat + (size_t)l * nPxl;
    const int bpx = tid / TT, bt = tid % TT;
    // CS: a staging thread's columns bt + 16 ct have fixed defocus samples, so
    // their CTF rows are fixed (row of column tile 0 here, the rest in cRow)
    const float* C = ctf + ((size_t)l * nD + (CS ? (t0 + bt) % nD : 0)) * nPxl;
    int cRow[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ct++) cRow[ct] = CS ? (l * nD + (t0 + ct * TT + bt) % nD) : 0;
    float cc[NCT];      // CS: the CTF of this thread's (next) pixel per column tile
    auto load_cc = [&](int p) {
        if (CS)
#pragma unroll
            for (int ct = 0; ct < NCT; ct++) cc[ct] = p >= 0 ? ctf[(size_t)cRow[ct] * nPxl + p] : 0.f;
    };
    const float* S = sig + (size_t)l * nPxl;
    const int nC = (nVisit + KC - 1) / KC;
    const int* R = rec + ((size_t)l * gridDim.y + blockIdx.y) * nC * REC;
    f32x4 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ct++) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bias = 0.f, aConst = 0.f;
    float biasHi = 0.f;     // PAIR: the bias of rotation r8 + 8 (bias: r8)
    // image-tile elements tid + j THREADS (< PKC TT): pixel bpx + j THREADS / TT
    // of the iteration's PKC, column bt
    constexpr int PSTEP = THREADS / TT;
    auto stager = [&](int j) { return tid + j * THREADS < PKC * TT; };
    const int g = lane >> 4;       // pixel slot of this lane in a step
    const int kk = lane >> 4, tc = lane & 15;   // B-operand row / column

    // pipeline prologue: patches 0 .. PP-1 data + box, the next PP's order
    // entries + record
    Pix px[NE];
    int pNext[NE];
#pragma unroll
    for (int j = 0; j < NE; j++) {
        px[j] = load_pix(stager(j) ? patch_pixel(order, nVisit, bpx + j * PSTEP) : -1, iCol, iRow, D, C, S);
        pNext[j] = stager(j) ? patch_pixel(order, nVisit, PKC + bpx + j * PSTEP) : -1;
    }
    load_cc(px[0].p);
    Rec rc = NOBOX ? Rec{} : load_rec(R);
    Rec rn = NOBOX || nC <= 1 ? rc : load_rec(R + REC);
    f32x4 pre[NITC][2];
    int dst[NITC];
    if (!NOBOX) fetch_box<LAYOUT, NITC, BOXC>(pre, dst, rc, vol, vdim, tid);

    __syncthreads();
    for (int c = 0; c < nC; c += PP) {
        // ---- stage patch c: box voxels, image tile B[px][U, V][t], b, (iCol, iRow) pf
        if (staged(rc)) {
            f32x4* box4 = reinterpret_cast<f32x4*>(sBox);
#pragma unroll
            for (int j = 0; j < NITC; j++) {
                const int it = tid + j * THREADS;
                if (it < rc.v[12]) {
                    box4[dst[j] / 2] = pre[j][0];
                    box4[dst[j] / 2 + 1] = pre[j][1];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < NE; j++) {
            if (!stager(j)) continue;
            const Pix& x = px[j];
            const int q = bpx + j * PSTEP;      // pixel of the iteration
            const bool ok = x.p >= 0;
#pragma unroll
            for (int ct = 0; ct < NCT; ct++) {
                const int col = ct * TT + bt;
                const float cv = CS ? cc[ct] : x.c;
                float U = 0.f, V = 0.f;
                if (ok && t0 + col < nT) {
                    const float k2 = -2.f * x.s * cv;
                    const float yr = k2 * x.d.x, yi = k2 * x.d.y;
                    const float2 T = phase_shift(x.ic, x.ir, sTr[col][0], sTr[col][1]);
                    U = yr * T.x + yi * T.y;
                    V = yi * T.x - yr * T.y;
                }
                sB[(q * 2) * NC + col] = U;
                sB[(q * 2 + 1) * NC + col] = V;
                if (CS) sBq[q * NC + col] = ok && t0 + col < nT ? x.s * cv * cv : 0.f;
            }
            if (bt == 0) {
                if (ok) aConst += x.s * (x.d.x * x.d.x + x.d.y * x.d.y);
                if (!CS) sBq[q] = ok ? x.s * x.c * x.c : 0.f;
                sValid[q] = ok;
                // padding entries sample the patch's first pixel (inside the box)
                const int ic = ok ? x.ic : NOBOX ? 0 : rc.v[17], ir = ok ? x.ir : NOBOX ? 0 : rc.v[18];
                sXY[q] = make_double2((double)(ic * pf), (double)(ir * pf));
            }
        }
        __syncthreads();
        // ---- prefetch patches c + PP .. (in flight during the gathers below)
        Rec r2 = rn;
        if (c + PP < nC) {
#pragma unroll
            for (int j = 0; j < NE; j++) {
                if (!stager(j)) continue;
                px[j] = load_pix(pNext[j], iCol, iRow, D, C, S);
                if (j == 0) load_cc(pNext[0]);
                pNext[j] = patch_pixel(order, nVisit, (c + 2 * PP) * KC + bpx + j * PSTEP);
            }
            if (!NOBOX) fetch_box<LAYOUT, NITC, BOXC>(pre, dst, rn, vol, vdim, tid);
            if (!NOBOX && c + 2 < nC) r2 = load_rec(R + (size_t)(c + 2) * REC);
        }
        // ---- projection samples: this lane's rotation x pixels 4s + g
        // one step: the sample's bias term, then (re, im) of pixels 4s, 4s+2 and
        // 4s+1, 4s+3 regrouped into two MFMA A operands against [U, V]
        auto reduce_step = [&](int s, float2 P) {
            if (!CS) bias += sBq[4 * s + g] * (P.x * P.x + P.y * P.y);
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(P.x),
                                                             __float_as_uint(P.y), false, false);
            const int q0 = 4 * s + (kk < 2 ? 0 : 2), q1 = q0 + 1;
#pragma unroll
            for (int ct = 0; ct < NCT; ct++) {
                const float b0 = sB[(q0 * 2 + (kk & 1)) * NC + ct * TT + tc];
                const float b1 = sB[(q1 * 2 + (kk & 1)) * NC + ct * TT + tc];
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(sw[0]), b0, acc[ct],
                                                               0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(sw[1]), b1, acc[ct],
                                                               0, 0, 0);
            }
            if (CS) {
                const auto sq = __builtin_amdgcn_permlane16_swap(
                    __float_as_uint(P.x * P.x), __float_as_uint(P.y * P.y), false, false);
#pragma unroll
                for (int ct = 0; ct < NCT; ct++) {
                    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        __uint_as_float(sq[0]), sBq[q0 * NC + ct * TT + tc], acc[ct], 0, 0, 0);
                    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        __uint_as_float(sq[1]), sBq[q1 * NC + ct * TT + tc], acc[ct], 0, 0, 0);
                }
            }
        };
        // a step whose four pixels are all padding adds exactly zero (U = V = b
        // = 0): skipped, wave-uniformly
        auto pad_step = [&](int s) {
            return !(sValid[4 * s] | sValid[4 * s + 1] | sValid[4 * s + 2] | sValid[4 * s + 3]);
        };
        // COOP step: quad r of the wave evaluates rotation 16 wv + r at the four
        // pixels 4s + p, one cooperative cell read each, summed over the quad;
        // the (re, im) of pixels (4s, 4s+2) and (4s+1, 4s+3) then reach the
        // MFMA A layout (row r = lane & 15, k = lane >> 4) by ds_bpermute from
        // lane 4 r + k of the quad layout
        auto coop_step = [&](int s) {
            const int j = lane & 3;
            // lane j of the quad rotates pixel 4s + j; the four cells are then
            // shared across the quad (quad_bcast_cell)
            Cell mine;
            {
                const double2 xy = sXY[4 * s + j];
                mine = cell_of((float)(m[0] * xy.x + m[3] * xy.y), (float)(m[1] * xy.x + m[4] * xy.y),
                               (float)(m[2] * xy.x + m[5] * xy.y));
            }
            float2 P[4];
#pragma unroll
            for (int p = 0; p < 4; p++) {
                const Cell c = p == 0 ? quad_bcast_cell<0>(mine) : p == 1 ? quad_bcast_cell<1>(mine)
                             : p == 2 ? quad_bcast_cell<2>(mine) : quad_bcast_cell<3>(mine);
                const float2 v = cell_piece(reinterpret_cast<const float4*>(vol), vdim, c, j);
                P[p] = make_float2(quad_sum(v.x), quad_sum(v.y));
            }
            if (!CS)
#pragma unroll
                for (int p = 0; p < 4; p++) bias += sBq[4 * s + p] * (P[p].x * P[p].x + P[p].y * P[p].y);
            const int k = lane & 3;
            const int src = (4 * (lane & 15) + (lane >> 4)) * 4;     // byte address of the source lane
            const float v1 = k == 0 ? P[0].x : k == 1 ? P[0].y : k == 2 ? P[2].x : P[2].y;
            const float v2 = k == 0 ? P[1].x : k == 1 ? P[1].y : k == 2 ? P[3].x : P[3].y;
            const float a1 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v1)));
            const float a2 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v2)));
            const int q0 = 4 * s + (kk < 2 ? 0 : 2), q1 = q0 + 1;
#pragma unroll
            for (int ct = 0; ct < NCT; ct++) {
                const float b0 = sB[(q0 * 2 + (kk & 1)) * NC + ct * TT + tc];
                const float b1 = sB[(q1 * 2 + (kk & 1)) * NC + ct * TT + tc];
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2, b1, acc[ct], 0, 0, 0);
            }
            if (CS) {
                const float u1 = k == 0 ? P[0].x * P[0].x : k == 1 ? P[0].y * P[0].y
                               : k == 2 ? P[2].x * P[2].x : P[2].y * P[2].y;
                const float u2 = k == 0 ? P[1].x * P[1].x : k == 1 ? P[1].y * P[1].y
                               : k == 2 ? P[3].x * P[3].x : P[3].y * P[3].y;
                const float c1 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(u1)));
                const float c2 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(u2)));
#pragma unroll
                for (int ct = 0; ct < NCT; ct++) {
                    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(c1, sBq[q0 * NC + ct * TT + tc],
                                                                   acc[ct], 0, 0, 0);
                    acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(c2, sBq[q1 * NC + ct * TT + tc],
                                                                   acc[ct], 0, 0, 0);
                }
            }
        };
        // PAIR step: pair (r, h) = lanes 2 (16 h + r) + j evaluates rotation 16 wv +
        // r at pixels 4s + h (it 0) and 4s + h + 2 (it 1); lane j rotates the
        // it = j sample and the pair shares the cells.  MFMA A rows: (pixels
        // 4s, 4s + 2) from the h = 0 pairs, (4s + 1, 4s + 3) from the h = 1 pairs.
        constexpr unsigned yxs = 2u;   // x stride of the copy's elements (slices interleaved)
        // PAIR step, 8 rotations x 4 pixels per load: pair (r8, p) = lanes 2 (r8 + 8 p) + j
        // evaluates pixel 4s + p for rotations 16 wv + r8 (it 0) and 16 wv + r8 + 8
        // (it 1); lane j rotates the it = j sample and the pair shares the cells, so
        // one load instruction covers 8 rotations of a 4-pixel patch row (the
        // patch's neighbouring pixels share lines where a wide cloud's rotations
        // do not).  MFMA A rows: rotation rho's (pixels 4s, 4s + 2) from pairs
        // (rho & 7, 0 / 2), (4s + 1, 4s + 3) from (rho & 7, 1 / 3), it = rho >> 3.
        auto pair_step = [&](int s) {
            const int j = lane & 1, p = lane >> 4;
            PCell mine;
            {
                const double2 xy = sXY[4 * s + p];
                mine = pcell_of((float)(m[0] * xy.x + m[3] * xy.y), (float)(m[1] * xy.x + m[4] * xy.y),
                                (float)(m[2] * xy.x + m[5] * xy.y), vdim, ballR);
            }
            const PCell pc0 = pair_bcast_pcell<0>(mine), pc1 = pair_bcast_pcell<1>(mine);
            const float4* yp = reinterpret_cast<const float4*>(vol);
            const PTaps t0 = ypair_pcell_load(yp, pc0, j, yxs), t1 = ypair_pcell_load(yp, pc1, j, yxs);
            __builtin_amdgcn_sched_barrier(0);
            float2 P[2];
#pragma unroll
            for (int it = 0; it < 2; it++) {
                const float2 v = ypair_pcell_lerp(it == 0 ? t0 : t1, it == 0 ? pc0 : pc1, j);
                P[it] = make_float2(v.x + pair_swap(v.x), v.y + pair_swap(v.y));
            }
            if (!CS) {
                const float bq = sBq[4 * s + p];
                bias += bq * (P[0].x * P[0].x + P[0].y * P[0].y);
                biasHi += bq * (P[1].x * P[1].x + P[1].y * P[1].y);
            }
            const float c0 = j ? P[0].y : P[0].x, c1 = j ? P[1].y : P[1].x;
            const int rho = lane & 15;
            const int sa = ((kk & 1) + 2 * (rho & 7) + 16 * (kk < 2 ? 0 : 2)) * 4;
            const float t10 = __int_as_float(__builtin_amdgcn_ds_bpermute(sa, __float_as_int(c0)));
            const float t11 = __int_as_float(__builtin_amdgcn_ds_bpermute(sa, __float_as_int(c1)));
            const float t20 = __int_as_float(__builtin_amdgcn_ds_bpermute(sa + 64, __float_as_int(c0)));
            const float t21 = __int_as_float(__builtin_amdgcn_ds_bpermute(sa + 64, __float_as_int(c1)));
            const float a1 = rho < 8 ? t10 : t11, a2 = rho < 8 ? t20 : t21;
            const int q0 = 4 * s + (kk < 2 ? 0 : 2), q1 = q0 + 1;
#pragma unroll
            for (int ct = 0; ct < NCT; ct++) {
                const float b0 = sB[(q0 * 2 + (kk & 1)) * NC + ct * TT + tc];
                const float b1 = sB[(q1 * 2 + (kk & 1)) * NC + ct * TT + tc];
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2, b1, acc[ct], 0, 0, 0);
            }
        };
        if (PAIR) {
            // every step of the iteration, no padding branch (a padding step
            // adds exactly zero: U = V = b = 0; 90.1k vs 87.5k images/s with
            // the per-step branch, profiles/r04_pair_pipe_ab.jsonl), two steps
            // per unrolled body: with the packed cells a full unroll hoists
            // more loads than 80 VGPRs hold (62 spills); unrolled twice: phases
            // 8.67 vs 9.26 ms for the round-3 cells, full unroll with FP32
            // rotations 8.71, with buffer-descriptor loads 8.66, full unroll at
            // 8 waves 8.98 (profiles/r04_pair_ab.jsonl)
#pragma unroll 2
            for (int s = 0; s < 4 * PP; s++) pair_step(s);
        } else if (COOP) {
// all four steps unrolled: 16 cell reads in flight per wave (C5 +3-4 %,
// full-res 1.5-3 deg 2-5 % over 2; profiles/r03_coop_unroll_ab.jsonl)
#pragma unroll 4
            for (int s = 0; s < 4 * PP; s++) {
                if (pad_step(s)) continue;
                coop_step(s);
            }
        } else if (staged(rc)) {
            const int nx = rc.v[6], sp = rc.v[7], off0 = rc.v[15], off1 = rc.v[16];
#pragma unroll
            for (int s = 0; s < 4 * PP; s++) {
                if (pad_step(s)) continue;
                const double2 xy = sXY[4 * s + g];
                const float x = (float)(m[0] * xy.x + m[3] * xy.y);
                const float y = (float)(m[1] * xy.x + m[4] * xy.y);
                const float z = (float)(m[2] * xy.x + m[5] * xy.y);
                reduce_step(s, interp_box(sBox, nx, sp, off0, off1, x, y, z));
            }
        } else {
#pragma unroll 2
            for (int s = 0; s < 4 * PP; s++) {
                if (pad_step(s)) continue;
                const double2 xy = sXY[4 * s + g];
                const float x = (float)(m[0] * xy.x + m[3] * xy.y);
                const float y = (float)(m[1] * xy.x + m[4] * xy.y);
                const float z = (float)(m[2] * xy.x + m[5] * xy.y);
                reduce_step(s, interp_ft(vol, vdim, x, y, z));
            }
        }
        rc = rn;
        rn = r2;
        __syncthreads();
    }
    // A_l = sum_i s |d|^2 (staging threads with bt == 0 accumulated it)
    aConst = wave_sum(aConst);
    if (lane == 0) sRed[wv] = aConst;
    // B_r: the four pixel slots of a rotation are lanes l, l + 16, l + 32, l + 48
    // (COOP: every lane of quad r holds rotation r's whole sum)
    if (PAIR) {
        // rotation rho's pixels are split over the pairs (rho & 7, p = 0..3),
        // its sum in bias (rho < 8) or biasHi
        bias += __shfl_xor(bias, 16, 64);
        bias += __shfl_xor(bias, 32, 64);
        biasHi += __shfl_xor(biasHi, 16, 64);
        biasHi += __shfl_xor(biasHi, 32, 64);
        const float lo = __shfl(bias, 2 * (lane & 7), 64), hi = __shfl(biasHi, 2 * (lane & 7), 64);
        bias = (lane & 8) ? hi : lo;
    } else if (COOP) {
        bias = __shfl(bias, 4 * (lane & 15), 64);
    } else {
        bias += __shfl_xor(bias, 16, 64);
        bias += __shfl_xor(bias, 32, 64);
    }
    if (lane < 16) sBias[rl] = CS ? 0.f : bias;
    __syncthreads();
    float Al = 0.f;
    for (int k = 0; k < NWAVE; k++) Al += sRed[k];
    if (!CS && wR) {
        // one workgroup holds the image's whole (r, t) table (nR <= 128, nT <=
        // 16): the per-image normalisation of k_local_weights
        // (src/Optimiser.cpp:1383-1402) in the epilogue, no dvp round trip
        __shared__ float sMax[NWAVE];
        __shared__ double sWT[NWAVE][TT];
        __shared__ double sWC[NWAVE];
        const int t = tc;
        const bool tv = t < nT;
        float v[4];
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int rr = wv * 16 + 4 * kk + j;
            v[j] = Al + sBias[rr] + acc[0][j];
            if (tv && rr < nRl) {
                mx = fmaxf(mx, v[j]);
                if (dvp) dvp[((size_t)l * nR + r0 + sPerm[rr]) * nT + t] = v[j];
            }
        }
        mx = wave_max(mx);
        if (lane == 0) sMax[wv] = mx;
        __syncthreads();
        float base = sMax[0];
        for (int w = 1; w < NWAVE; w++) base = fmaxf(base, sMax[w]);
        const double c = pC[l];
        const double ptl = tv ? pT[(size_t)l * nT + t] : 0.0;
        double colT = 0.0, cw = 0.0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int rr = wv * 16 + 4 * kk + j;
            const bool ok = tv && rr < nRl;
            const int r = r0 + sPerm[rr < nRl ? rr : 0];
            const double pr = pR[(size_t)l * nR + r];
            const double e = ok ? (double)expf(v[j] - base) : 0.0;
            double rs = e * ptl;          // the row's sum over its 16 translation lanes
            rs += __shfl_xor(rs, 1, 64);
            rs += __shfl_xor(rs, 2, 64);
            rs += __shfl_xor(rs, 4, 64);
            rs += __shfl_xor(rs, 8, 64);
            if (tc == 0 && rr < nRl) wR[(size_t)l * nR + r] = (float)(rs * c);
            if (rr < nRl) cw += rs * pr;
            colT += e * pr;
        }
        colT += __shfl_xor(colT, 16, 64);
        colT += __shfl_xor(colT, 32, 64);
        cw += __shfl_xor(cw, 16, 64);
        cw += __shfl_xor(cw, 32, 64);
        if (lane < TT) sWT[wv][lane] = colT;
        if (lane == 0) sWC[wv] = cw;
        __syncthreads();
        if (tid < nT) {
            double a = 0.0;
            for (int w = 0; w < NWAVE; w++) a += sWT[w][tid];
            wT[(size_t)l * nT + tid] = (float)(a * c);
        }
        if (tid == 0) {
            double a = 0.0;
            for (int w = 0; w < NWAVE; w++) a += sWC[w];
            wC[l] = (float)a;
            baseL[l] = base;
        }
        return;
    }
    // C layout of 16x16x4: col = lane & 15 (translation), row = 4 (lane >> 4) + j
#pragma unroll
    for (int ct = 0; ct < NCT; ct++) {
        const int t = t0 + ct * TT + tc;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int rr = wv * 16 + 4 * kk + j;
            if (t < nT && rr < nRl)
                dvp[((size_t)l * nR + r0 + sPerm[rr]) * nT + t] = Al + sBias[rr] + acc[ct][j];
        }
    }
}

// Per-image normalisation of src/Optimiser.cpp:1383-1402 (nC = nD = 1,
// wD = 1) evaluated at the final baseline: s = exp(dvp - max),
// wC += s pR pT, wR[r] += s pC pT, wT[t] += s pC pR.
__global__ void __launch_bounds__(256) k_local_weights(const float* __restrict__ dvp,
                                                       int nR, int nT,
                                                       const double* __restrict__ pC,
                                                       const double* __restrict__ pR,
                                                       const double* __restrict__ pT,
                                                       float* __restrict__ wC,
                                                       float* __restrict__ wR,
                                                       float* __restrict__ wT,
                                                       float* __restrict__ baseL,
                                                       const int* __restrict__ act,
                                                       const int* __restrict__ nAct)
{
    int l = blockIdx.x;
    if (act) {
        if (l >= *nAct) return;
        l = act[l];
    }
    const float* Dl = dvp + (size_t)l * nR * nT;
    const double* pRl = pR + (size_t)l * nR;
    const double* pTl = pT + (size_t)l * nT;
    const double c = pC[l];
    __shared__ float sm[4];
    __shared__ double sd[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float m = -INFINITY;
    for (int q = threadIdx.x; q < nR * nT; q += blockDim.x) m = fmaxf(m, Dl[q]);
    m = wave_max(m);
    if (lane == 0) sm[wv] = m;
    __syncthreads();
    const float base = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    double cacc = 0.0;
    for (int r = threadIdx.x; r < nR; r += blockDim.x) {
        double a = 0.0;
        for (int t = 0; t < nT; t++) a += (double)expf(Dl[r * nT + t] - base) * pTl[t];
        wR[(size_t)l * nR + r] = (float)(a * c);
        cacc += a * pRl[r];
    }
    __shared__ double sT[256];
    if (nT <= 64) {
        // wT: groups of nT threads stride over the rotations (a handful of
        // translations would leave 247 of 256 threads idle on a 125-long
        // serial chain), partial sums in a fixed order through LDS
        const int G = 256 / nT, t = threadIdx.x % nT, gq = threadIdx.x / nT;
        double a = 0.0;
        if (gq < G)
            for (int r = gq; r < nR; r += G) a += (double)expf(Dl[r * nT + t] - base) * pRl[r];
        sT[threadIdx.x] = a;
        __syncthreads();
        if (threadIdx.x < nT) {
            double w = 0.0;
            for (int k = 0; k < G; k++) w += sT[k * nT + threadIdx.x];
            wT[(size_t)l * nT + threadIdx.x] = (float)(w * c);
        }
    } else {
        for (int t = threadIdx.x; t < nT; t += blockDim.x) {
            double a = 0.0;
            for (int r = 0; r < nR; r++) a += (double)expf(Dl[r * nT + t] - base) * pRl[r];
            wT[(size_t)l * nT + t] = (float)(a * c);
        }
    }
    cacc = wave_sum(cacc);
    if (lane == 0) sd[wv] = cacc;
    __syncthreads();
    if (threadIdx.x == 0) {
        wC[l] = (float)(sd[0] + sd[1] + sd[2] + sd[3]);
        baseL[l] = base;
    }
}

// CTF search: the normalisation of src/Optimiser.cpp:1383-1402 with the
// defocus axis (nC = 1): over dvp[r][t][d], s = exp(dvp - max),
// wC = sum s pR pT pD, wR[r] = pC sum_{t,d} s pT pD, wT[t] = pC sum_{r,d} s pR pD,
// wD[d] = pC sum_{r,t} s pR pT.  a[t][d] = sum_r s pR goes through LDS.
constexpr int LOCAL_D_MAXCOL = 1024;
__global__ void __launch_bounds__(256) k_local_weights_d(const float* __restrict__ dvp, int nR,
                                                         int nT, int nD,
                                                         const double* __restrict__ pC,
                                                         const double* __restrict__ pR,
                                                         const double* __restrict__ pT,
                                                         const double* __restrict__ pD,
                                                         float* __restrict__ wC,
                                                         float* __restrict__ wR,
                                                         float* __restrict__ wT,
                                                         float* __restrict__ wD,
                                                         float* __restrict__ baseL,
                                                         const int* __restrict__ act,
                                                         const int* __restrict__ nAct)
{
    int l = blockIdx.x;
    if (act) {
        if (l >= *nAct) return;
        l = act[l];
    }
    const int nCol = nT * nD;
    const float* Dl = dvp + (size_t)l * nR * nCol;
    const double* pRl = pR + (size_t)l * nR;
    const double* pTl = pT + (size_t)l * nT;
    const double* pDl = pD + (size_t)l * nD;
    const double c = pC[l];
    __shared__ float sm[4];
    __shared__ double sA[LOCAL_D_MAXCOL];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float m = -INFINITY;
    for (int q = threadIdx.x; q < nR * nCol; q += blockDim.x) m = fmaxf(m, Dl[q]);
    m = wave_max(m);
    if (lane == 0) sm[wv] = m;
    __syncthreads();
    const float base = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    for (int r = threadIdx.x; r < nR; r += blockDim.x) {
        double a = 0.0;
        for (int t = 0; t < nT; t++)
            for (int d = 0; d < nD; d++)
                a += (double)expf(Dl[(size_t)r * nCol + t * nD + d] - base) * (pTl[t] * pDl[d]);
        wR[(size_t)l * nR + r] = (float)(a * c);
    }
    for (int q = threadIdx.x; q < nCol; q += blockDim.x) {
        double a = 0.0;
        for (int r = 0; r < nR; r++) a += (double)expf(Dl[(size_t)r * nCol + q] - base) * pRl[r];
        sA[q] = a;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < nT; t += blockDim.x) {
        double a = 0.0;
        for (int d = 0; d < nD; d++) a += sA[t * nD + d] * pDl[d];
        wT[(size_t)l * nT + t] = (float)(a * c);
    }
    for (int d = threadIdx.x; d < nD; d += blockDim.x) {
        double a = 0.0;
        for (int t = 0; t < nT; t++) a += sA[t * nD + d] * pTl[t];
        wD[(size_t)l * nD + d] = (float)(a * c);
    }
    if (threadIdx.x == 0) {
        double a = 0.0;
        for (int q = 0; q < nCol; q++) a += sA[q] * (pTl[q / nD] * pDl[q % nD]);
        wC[l] = (float)a;
        baseL[l] = base;
    }
}

// One thread per cell: the 8 taps (dz, dy, dx) of base voxel (i, j, k), rows
// and slices wrapped like iFTHalf, i + 1 past the half-plane edge -> 0.
__global__ void __launch_bounds__(256) k_volume_cells(const float2* __restrict__ vol,
                                                      int vdim, float2* __restrict__ cells)
{
    const int nColFT = vdim / 2 + 1;
    const long n = (long)nColFT * vdim * vdim;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int i = (int)(q % nColFT);
        const long jk = q / nColFT;
        const int j = (int)(jk % vdim), k = (int)(jk / vdim);
        const int j1 = j + 1 == vdim ? 0 : j + 1, k1 = k + 1 == vdim ? 0 : k + 1;
        float2 v[8];
        const int zz[2] = {k, k1}, yy[2] = {j, j1};
#pragma unroll
        for (int dz = 0; dz < 2; dz++)
#pragma unroll
            for (int dy = 0; dy < 2; dy++)
#pragma unroll
                for (int dx = 0; dx < 2; dx++) {
                    const int x = i + dx;
                    v[dz * 4 + dy * 2 + dx] =
                        x < nColFT ? vol[((size_t)zz[dz] * vdim + yy[dy]) * nColFT + x]
                                   : make_float2(0.f, 0.f);
                }
        float4* o = reinterpret_cast<float4*>(cells + 8 * (size_t)q);
#pragma unroll
        for (int u = 0; u < 4; u++) o[u] = make_float4(v[2 * u].x, v[2 * u].y, v[2 * u + 1].x, v[2 * u + 1].y);
    }
}

// One thread per element of the y-pair copy: (v(x, y, z), v(x, y + 1, z)),
// rows wrapped like iFTHalf.
__global__ void __launch_bounds__(256) k_volume_ypair(const float2* __restrict__ vol, int vdim,
                                                      float4* __restrict__ yp)
{
    const int nColFT = vdim / 2 + 1;
    const long n = (long)nColFT * vdim * vdim;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int i = (int)(q % nColFT);
        const long jk = q / nColFT;
        const int j = (int)(jk % vdim), k = (int)(jk / vdim);
        const int j1 = j + 1 == vdim ? 0 : j + 1;
        const float2 a = vol[q], b = vol[((size_t)k * vdim + j1) * nColFT + i];
        yp[ypair_elem((unsigned)k, (unsigned)j, (unsigned)i, (unsigned)vdim, (unsigned)nColFT)] =
            make_float4(a.x, a.y, b.x, b.y);
    }
}

// the compact ball of the y-pair copy (ypair_ball_elem): elements
// (x, y, z), 0 <= x < R + 2, -R <= y, z < R + 2, from the half-complex
// volume with its wrap
__global__ void __launch_bounds__(256) k_volume_ypair_ball(const float2* __restrict__ vol, int vdim,
                                                           int R, float4* __restrict__ yp)
{
    const int nColFT = vdim / 2 + 1;
    const int X = R + 2, Y = 2 * R + 2;
    const long n = (long)X * Y * Y;
    for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n;
         q += (long)gridDim.x * blockDim.x) {
        const int x = (int)(q % X);
        const long yz = q / X;
        const int y = (int)(yz % Y) - R, z = (int)(yz / Y) - R;
        const int zw = wrap_idx(z, vdim), yw = wrap_idx(y, vdim), yw1 = wrap_idx(y + 1, vdim);
        const float2 a = x < nColFT ? vol[((size_t)zw * vdim + yw) * nColFT + x] : make_float2(0.f, 0.f);
        const float2 b = x < nColFT ? vol[((size_t)zw * vdim + yw1) * nColFT + x] : make_float2(0.f, 0.f);
        yp[ypair_ball_elem(z, y, x, R)] = make_float4(a.x, a.y, b.x, b.y);
    }
}

size_t dvp_bytes(int nImg, int nR, int nT) { return (size_t)nImg * nR * nT * sizeof(float); }

size_t rec_bytes(int nImg, int nR, int nVisit)
{
    return (size_t)nImg * thx::cdiv(nR, RT) * thx::cdiv(nVisit, KC) * REC * sizeof(int);
}

}  // namespace

namespace thx {

size_t patch_rec_bytes(int nImg, int nR, int nVisit) { return rec_bytes(nImg, nR, nVisit); }

// the per-image normalisation of a materialised dvp (also the 2D phase's)
int launch_local_weights(const float* dvp, int nR, int nT, const double* pC, const double* pR,
                         const double* pT, float* wC, float* wR, float* wT, float* baseL, int nImg,
                         hipStream_t s, const int* act, const int* nAct)
{
    hipLaunchKernelGGL(k_local_weights, dim3(nImg), dim3(256), 0, s, dvp, nR, nT, pC, pR, pT, wC,
                       wR, wT, baseL, act, nAct);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

int launch_local_weights_d(const float* dvp, int nR, int nT, int nD, const double* pC,
                           const double* pR, const double* pT, const double* pD, float* wC,
                           float* wR, float* wT, float* wD, float* baseL, int nImg, hipStream_t s,
                           const int* act, const int* nAct)
{
    hipLaunchKernelGGL(k_local_weights_d, dim3(nImg), dim3(256), 0, s, dvp, nR, nT, nD, pC, pR,
                       pT, pD, wC, wR, wT, wD, baseL, act, nAct);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

int launch_patch_boxes(const double* quat, int nR, const int* iCol, const int* iRow,
                       const int* order, int nVisit, int pf, int vdim, int nImg, int* rec,
                       hipStream_t s)
{
    hipLaunchKernelGGL(k_patch_boxes, dim3((unsigned)nImg * cdiv(nR, RT)), dim3(64 * PB_WAVES), 0,
                       s, quat, nR, iCol, iRow, order, nVisit, pf, vdim, rec, nullptr, nullptr);
    THX_LAUNCH_CHECK();
    return THX_OK;
}

size_t ypair_ball_elems(int R);

}  // namespace thx

extern "C" int thx_volume_cells(const float* vol, int vdim, float* cells,
                                thx_stream_t stream)
{
    THX_CHECK_ARG(vdim > 0 && vdim % 2 == 0, "thx_volume_cells: bad vdim");
    hipLaunchKernelGGL(k_volume_cells, dim3(4096), dim3(256), 0, thx::as_stream(stream),
                       reinterpret_cast<const float2*>(vol), vdim,
                       reinterpret_cast<float2*>(cells));
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_volume_ypair(const float* vol, int vdim, float* ypair, thx_stream_t stream)
{
    THX_CHECK_ARG(vol && ypair && vdim > 0 && vdim % 2 == 0, "thx_volume_ypair: bad arguments");
    hipLaunchKernelGGL(k_volume_ypair, dim3(4096), dim3(256), 0, thx::as_stream(stream),
                       reinterpret_cast<const float2*>(vol), vdim, reinterpret_cast<float4*>(ypair));
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" size_t thx_local_phase_workspace(int nImg, int nR, int nT, int nVisit)
{
    return dvp_bytes(nImg, nR, nT) + rec_bytes(nImg, nR, nVisit) + 256 + 768;
}

// nD = 0: the phase without CTF search; nD >= 1: CTF search over nD defocus
// samples (ctf = ctfD[nImg][nD][nPxl], priors pD[nImg][nD], marginal wD).
static int local_phase_impl(const thx_local_sel* sel, hipEvent_t evBeg, hipEvent_t evEnd,
                            const float* vol, int volLayout, int vdim,
                            int pf, const double* quat, int nR, const double* trans, int nT,
                            const double* pC, const double* pR, const double* pT, const float* dat,
                            const float* ctf, const float* sigRcp, const int* iCol, const int* iRow,
                            const int* pxOrder, int nOrd, int nPxl, int idim, int nImg, float* wC,
                            float* wR, float* wT, float* baseL, float* dvp, void* workspace,
                            size_t wsBytes, thx_stream_t stream, int nD = 0,
                            const double* pD = nullptr, float* wD = nullptr,
                            const float* ypair = nullptr, int* routeOut = nullptr,
                            const int* const* routeSample = nullptr, int ypairR = 0)
{
    THX_CHECK_ARG(nR > 0 && nT > 0 && nPxl > 0 && nImg >= 0 && vdim > 0 && pf > 0 && nD >= 0,
                  "thx_local_phase: bad sizes");
    THX_CHECK_ARG(!nD || (pD && wD && (long)nT * nD <= LOCAL_D_MAXCOL),
                  "thx_local_phase_d: needs pD, wD and nT * nD <= 1024");
    const int nCol = nD ? nT * nD : nT;
    THX_CHECK_ARG(volLayout >= 0 && volLayout <= 2, "thx_local_phase: volLayout must be 0 .. 2");
    THX_CHECK_ARG(volLayout != LAYOUT_YPAIR2 || !nD, "thx_local_phase_d: no y-pair layout with CTF search");
    THX_CHECK_ARG((long)nImg * ((nR + RT - 1) / RT) <= 0x7fffffff && (nR + RT - 1) / RT <= 65535 &&
                      (nCol + TT - 1) / TT <= 65535,
                  "thx_local_phase: grid too large");
    THX_CHECK_ARG(!pxOrder || (nOrd > 0 && nOrd % KC == 0),
                  "thx_local_phase: nOrd must be a positive multiple of 16 (thx_pixel_tile_order)");
    const int* act = sel ? sel->active : nullptr;
    const int* nAct = sel ? sel->nActive : nullptr;
    const int* cls = sel ? sel->cls : nullptr;
    THX_CHECK_ARG(!act == !nAct, "thx_local_phase_sel: active and nActive go together");
    THX_CHECK_ARG(!cls || (sel->volStride > 0), "thx_local_phase_sel: cls needs a volStride");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(!ypair || (volLayout == LAYOUT_FT && pxOrder && !nD),
                  "thx_local_phase_routed: a y-pair copy goes with the half-complex layout and pxOrder");
    const int nVisit = pxOrder ? nOrd : nPxl;
    THX_CHECK_ARG(workspace && wsBytes >= thx_local_phase_workspace(nImg, nR, nCol, nVisit),
                  "thx_local_phase: workspace too small");
    thx::Carver ws(workspace, wsBytes);
    float* d = dvp ? dvp : ws.take<float>((size_t)nImg * nR * nCol);
    int* rec = ws.take<int>(rec_bytes(nImg, nR, nVisit) / sizeof(int));
    int* route = ws.take<int>(64);
    hipStream_t s = thx::as_stream(stream);
    // big LDS boxes for large full-resolution pixel sets: the ring's outer
    // radius in projectee voxels, pf sqrt(2 nPxl / pi), past BIGBOX_MIN_R
    const bool big = pf * std::sqrt(2.0 * nPxl / M_PI) >= BIGBOX_MIN_R;
    // the staged / box-less (or y-pair) route of a half-complex phase, chosen
    // on the device from a sample of the patch records (route_pick)
    const bool routed = volLayout == LAYOUT_FT && !nD && !big;
    const unsigned nRT = thx::cdiv(nR, RT);
    if (routed) {
        THX_HIP(hipMemsetAsync(route, 0, 2 * sizeof(int), s));
        THX_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(route + 2), ypair ? 1 : 0, 1, s));
        // the route's sample: every ROUTE_SAMPLE-th entry of the active list,
        // or of the list the caller names (routeSample = {list, count}, both
        // null = every image in index order), so that a reordered active list
        // does not change the sample and with it the kernel
        const int* sAct = routeSample ? routeSample[0] : act;
        const int* sNAct = routeSample ? routeSample[1] : nAct;
        hipLaunchKernelGGL(k_patch_boxes, dim3((unsigned)thx::cdiv(nImg, ROUTE_SAMPLE) * nRT),
                           dim3(64 * PB_WAVES), 0, s, quat, nR, iCol, iRow, pxOrder, nVisit, pf, vdim,
                           rec, sAct, sNAct, route, 1);
        THX_LAUNCH_CHECK();
        if (routeOut) {
            hipLaunchKernelGGL(k_route_out, dim3(1), dim3(64), 0, s, route, routeOut);
            THX_LAUNCH_CHECK();
        }
        hipLaunchKernelGGL(k_patch_boxes, dim3((unsigned)nImg * nRT), dim3(64 * PB_WAVES), 0, s, quat,
                           nR, iCol, iRow, pxOrder, nVisit, pf, vdim, rec, act, nAct, route, 2);
        THX_LAUNCH_CHECK();
    } else if (!coop_layout(volLayout) && volLayout != LAYOUT_YPAIR2) {   // no boxes for these
        if (routeOut) THX_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(routeOut), -1, 1, s));
        hipLaunchKernelGGL(k_patch_boxes, dim3((unsigned)nImg * nRT), dim3(64 * PB_WAVES), 0, s, quat,
                           nR, iCol, iRow, pxOrder, nVisit, pf, vdim, rec, act, nAct, nullptr, 0);
        THX_LAUNCH_CHECK();
    }
    dim3 grid(nImg, thx::cdiv(nR, RT), thx::cdiv(nCol, TT));
    const long vs = cls ? (long)sel->volStride : 0L;
    if (evBeg) THX_HIP(hipEventRecord(evBeg, s));
    if (nD) {
        // all (t, d) columns of a workgroup in NCT tiles (one gather of the
        // projection), up to 96 per workgroup
        const int need = (int)thx::cdiv(nCol, TT);
        const int nct = need <= 1 ? 1 : need <= 2 ? 2 : need <= 4 ? 4 : 6;
        auto pick = [&](auto c1, auto c2, auto c4, auto c6) {
            return nct == 1 ? c1 : nct == 2 ? c2 : nct == 4 ? c4 : c6;
        };
        auto kern = volLayout == LAYOUT_CELLS
                        ? pick(k_local_fused<LAYOUT_CELLS, true, 1>, k_local_fused<LAYOUT_CELLS, true, 2>,
                               k_local_fused<LAYOUT_CELLS, true, 4>, k_local_fused<LAYOUT_CELLS, true, 6>)
                        : pick(k_local_fused<LAYOUT_FT, true, 1>, k_local_fused<LAYOUT_FT, true, 2>,
                               k_local_fused<LAYOUT_FT, true, 4>, k_local_fused<LAYOUT_FT, true, 6>);
        grid.z = thx::cdiv(nCol, TT * nct);
        hipLaunchKernelGGL(kern, grid, dim3(THREADS), 0, s, reinterpret_cast<const float2*>(vol),
                           vdim, pf, quat, nR, trans, nCol, reinterpret_cast<const float2*>(dat),
                           ctf, sigRcp, iCol, iRow, pxOrder, nVisit, nPxl, idim, rec, d, act, nAct,
                           cls, vs, nD, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                           nullptr, 0);
        THX_LAUNCH_CHECK();
        if (evEnd) THX_HIP(hipEventRecord(evEnd, s));
        hipLaunchKernelGGL(k_local_weights_d, dim3(nImg), dim3(256), 0, s, d, nR, nT, nD, pC, pR,
                           pT, pD, wC, wR, wT, wD, baseL, act, nAct);
        THX_LAUNCH_CHECK();
        return THX_OK;
    }
    auto kern =
        volLayout == LAYOUT_YPAIR2 ? k_local_fused<LAYOUT_YPAIR2>
        : volLayout == LAYOUT_CELLS
            ? (big ? k_local_fused<LAYOUT_CELLS, false, 1, true> : k_local_fused<LAYOUT_CELLS>)
            : (big ? k_local_fused<LAYOUT_FT, false, 1, true> : k_local_fused<LAYOUT_FT>);
    // one workgroup per image (nR <= 128, nT <= 16, the phases' 125 x 9):
    // the normalisation runs in the kernel's epilogue and dvp is only written
    // when the caller asks for it
    const bool fuse = grid.y == 1 && grid.z == 1;
    auto launch = [&](auto k, const int* rt) {
        hipLaunchKernelGGL(k, grid, dim3(THREADS), 0, s, reinterpret_cast<const float2*>(vol), vdim,
                           pf, quat, nR, trans, nT, reinterpret_cast<const float2*>(dat), ctf, sigRcp,
                           iCol, iRow, pxOrder, nVisit, nPxl, idim, rec, fuse ? dvp : d, act, nAct,
                           cls, vs, 1, pC, pR, pT, fuse ? wC : nullptr, fuse ? wR : nullptr,
                           fuse ? wT : nullptr, fuse ? baseL : nullptr, rt, 0);
    };
    if (routed) {
        // two launches, the staged kernel and (with a y-pair copy) the pair-form
        // y-pair kernel or (without) the box-less half-complex one; the kernel
        // the route did not pick exits at entry
        launch(k_local_fused<LAYOUT_FT, false, 1, false, true>, route);
        if (ypair) {
            hipLaunchKernelGGL(k_local_fused<LAYOUT_YPAIR2>, grid, dim3(THREADS), 0, s,
                               reinterpret_cast<const float2*>(ypair), vdim, pf, quat, nR, trans, nT,
                               reinterpret_cast<const float2*>(dat), ctf, sigRcp, iCol, iRow, pxOrder,
                               nVisit, nPxl, idim, rec, fuse ? dvp : d, act, nAct, cls,
                               cls ? (ypairR > 0 ? 2L * (long)thx::ypair_ball_elems(ypairR) : 2 * vs) : 0L, 1,
                               pC, pR, pT, fuse ? wC : nullptr, fuse ? wR : nullptr,
                               fuse ? wT : nullptr, fuse ? baseL : nullptr, route, ypairR);
        } else {
            launch(k_local_fused<LAYOUT_FT, false, 1, false, false>, route);
        }
    } else {
        launch(kern, nullptr);
    }
    THX_LAUNCH_CHECK();
    if (evEnd) THX_HIP(hipEventRecord(evEnd, s));
    if (!fuse) {
        hipLaunchKernelGGL(k_local_weights, dim3(nImg), dim3(256), 0, s, d, nR, nT, pC, pR, pT, wC,
                           wR, wT, baseL, act, nAct);
        THX_LAUNCH_CHECK();
    }
    return THX_OK;
}

extern "C" int thx_local_phase(const float* vol, int volLayout, int vdim, int pf,
                               const double* quat, int nR, const double* trans,
                               int nT, const double* pC, const double* pR,
                               const double* pT, const float* dat,
                               const float* ctf, const float* sigRcp,
                               const int* iCol, const int* iRow, const int* pxOrder,
                               int nOrd, int nPxl, int idim, int nImg, float* wC, float* wR,
                               float* wT, float* baseL, float* dvp,
                               void* workspace, size_t wsBytes,
                               thx_stream_t stream)
{
    return local_phase_impl(nullptr, nullptr, nullptr, vol, volLayout, vdim, pf, quat, nR, trans,
                            nT, pC, pR, pT,
                            dat, ctf, sigRcp, iCol, iRow, pxOrder, nOrd, nPxl, idim, nImg, wC, wR,
                            wT, baseL, dvp, workspace, wsBytes, stream);
}

extern "C" int thx_local_phase_sel(const thx_local_sel* sel, const float* vol, int volLayout,
                                   int vdim, int pf, const double* quat, int nR,
                                   const double* trans, int nT, const double* pC,
                                   const double* pR, const double* pT, const float* dat,
                                   const float* ctf, const float* sigRcp, const int* iCol,
                                   const int* iRow, const int* pxOrder, int nOrd, int nPxl,
                                   int idim, int nImg, float* wC, float* wR, float* wT,
                                   float* baseL, float* dvp, void* workspace, size_t wsBytes,
                                   thx_stream_t stream)
{
    return local_phase_impl(sel, nullptr, nullptr, vol, volLayout, vdim, pf, quat, nR, trans, nT,
                            pC, pR, pT, dat, ctf, sigRcp, iCol, iRow, pxOrder, nOrd, nPxl, idim,
                            nImg, wC, wR, wT, baseL, dvp, workspace, wsBytes, stream);
}

extern "C" int thx_local_phase_d(const thx_local_sel* sel, const float* vol, int volLayout,
                                 int vdim, int pf, const double* quat, int nR,
                                 const double* trans, int nT, int nD, const double* pC,
                                 const double* pR, const double* pT, const double* pD,
                                 const float* dat, const float* ctfD, const float* sigRcp,
                                 const int* iCol, const int* iRow, const int* pxOrder, int nOrd,
                                 int nPxl, int idim, int nImg, float* wC, float* wR, float* wT,
                                 float* wD, float* baseL, float* dvp, void* workspace,
                                 size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(nD > 0, "thx_local_phase_d: nD must be positive");
    return local_phase_impl(sel, nullptr, nullptr, vol, volLayout, vdim, pf, quat, nR, trans, nT,
                            pC, pR, pT, dat, ctfD, sigRcp, iCol, iRow, pxOrder, nOrd, nPxl, idim,
                            nImg, wC, wR, wT, baseL, dvp, workspace, wsBytes, stream, nD, pD, wD);
}

extern "C" int thx_local_phase_routed(const thx_local_sel* sel, const float* vol,
                                      const float* ypair, int vdim, int pf, const double* quat,
                                      int nR, const double* trans, int nT, const double* pC,
                                      const double* pR, const double* pT, const float* dat,
                                      const float* ctf, const float* sigRcp, const int* iCol,
                                      const int* iRow, const int* pxOrder, int nOrd, int nPxl,
                                      int idim, int nImg, float* wC, float* wR, float* wT,
                                      float* baseL, float* dvp, int* route, void* workspace,
                                      size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(pxOrder, "thx_local_phase_routed: needs pxOrder (thx_pixel_tile_order)");
    return local_phase_impl(sel, nullptr, nullptr, vol, LAYOUT_FT, vdim, pf, quat, nR, trans, nT,
                            pC, pR, pT, dat, ctf, sigRcp, iCol, iRow, pxOrder, nOrd, nPxl, idim,
                            nImg, wC, wR, wT, baseL, dvp, workspace, wsBytes, stream, 0, nullptr,
                            nullptr, ypair, route);
}

// max iCol^2 + iRow^2 over the pixel set (one workgroup)
__global__ void __launch_bounds__(256) k_ring_r2(const int* __restrict__ iCol,
                                                 const int* __restrict__ iRow, int nPxl,
                                                 int* __restrict__ out)
{
    __shared__ int sm[4];
    int m = 0;
    for (int i = threadIdx.x; i < nPxl; i += 256) m = max(m, iCol[i] * iCol[i] + iRow[i] * iRow[i]);
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) *out = max(max(sm[0], sm[1]), max(sm[2], sm[3]));
}

extern "C" size_t thx_ypair_ball_elems(int R)
{
    return R > 0 ? (size_t)(R + 2) * (2 * R + 2) * (2 * R + 2) : 0;
}

extern "C" int thx_volume_ypair_ball(const float* vol, int vdim, int R, float* ball,
                                     thx_stream_t stream)
{
    THX_CHECK_ARG(vol && ball && vdim > 0 && vdim % 2 == 0 && R > 0 && R + 2 <= vdim / 2 + 1,
                  "thx_volume_ypair_ball: bad arguments (R = %d, vdim = %d)", R, vdim);
    hipLaunchKernelGGL(k_volume_ypair_ball, dim3(2048), dim3(256), 0, thx::as_stream(stream),
                       reinterpret_cast<const float2*>(vol), vdim, R, reinterpret_cast<float4*>(ball));
    THX_LAUNCH_CHECK();
    return THX_OK;
}

extern "C" int thx_local_phase_routed_ball(const thx_local_sel* sel, const float* vol,
                                           const float* ball, int ballR, int vdim, int pf,
                                           const double* quat, int nR, const double* trans, int nT,
                                           const double* pC, const double* pR, const double* pT,
                                           const float* dat, const float* ctf, const float* sigRcp,
                                           const int* iCol, const int* iRow, const int* pxOrder,
                                           int nOrd, int nPxl, int idim, int nImg, float* wC,
                                           float* wR, float* wT, float* baseL, float* dvp,
                                           int* route, void* workspace, size_t wsBytes,
                                           thx_stream_t stream)
{
    THX_CHECK_ARG(pxOrder && ball && ballR > 0 && ballR + 2 <= vdim / 2 + 1 && nPxl > 0 && iCol && iRow,
                  "thx_local_phase_routed_ball: bad arguments");
    // every tap must fall inside the ball: pf r_max + 2 <= R, checked on the
    // pixel set itself (one read-back)
    hipStream_t s = thx::as_stream(stream);
    thx::Carver c(workspace, wsBytes);
    int* r2d = c.take<int>(1);
    THX_CHECK_ARG(c.ok(), "thx_local_phase_routed_ball: workspace too small");
    hipLaunchKernelGGL(k_ring_r2, dim3(1), dim3(256), 0, s, iCol, iRow, nPxl, r2d);
    THX_LAUNCH_CHECK();
    int r2 = 0;
    THX_HIP(hipMemcpyAsync(&r2, r2d, sizeof(int), hipMemcpyDeviceToHost, s));
    THX_HIP(hipStreamSynchronize(s));
    THX_CHECK_ARG(pf * std::sqrt((double)r2) + 2 <= ballR,
                  "thx_local_phase_routed_ball: the pixel ring (pf r_max = %g) needs ballR >= %d",
                  pf * std::sqrt((double)r2), (int)std::ceil(pf * std::sqrt((double)r2)) + 2);
    return local_phase_impl(sel, nullptr, nullptr, vol, LAYOUT_FT, vdim, pf, quat, nR, trans, nT,
                            pC, pR, pT, dat, ctf, sigRcp, iCol, iRow, pxOrder, nOrd, nPxl, idim,
                            nImg, wC, wR, wT, baseL, dvp, workspace, wsBytes, stream, 0, nullptr,
                            nullptr, ball, route, nullptr, ballR);
}

namespace thx {
// float4 elements of the compact y-pair ball of radius R
size_t ypair_ball_elems(int R) { return (size_t)(R + 2) * (2 * R + 2) * (2 * R + 2); }

int volume_ypair_ball(const float* vol, int vdim, int R, float* ypair, hipStream_t s)
{
    THX_CHECK_ARG(vol && ypair && vdim > 0 && vdim % 2 == 0 && R > 0 && R + 2 <= vdim / 2 + 1,
                  "volume_ypair_ball: bad arguments");
    hipLaunchKernelGGL(k_volume_ypair_ball, dim3(2048), dim3(256), 0, s,
                       reinterpret_cast<const float2*>(vol), vdim, R, reinterpret_cast<float4*>(ypair));
    THX_LAUNCH_CHECK();
    return THX_OK;
}

int local_phase_timed(const thx_local_sel* sel, hipEvent_t evBeg, hipEvent_t evEnd,
                      const float* vol, int volLayout, int vdim, int pf, const double* quat, int nR,
                      const double* trans, int nT, const double* pC, const double* pR,
                      const double* pT, const float* dat, const float* ctf, const float* sigRcp,
                      const int* iCol, const int* iRow, const int* pxOrder, int nOrd, int nPxl,
                      int idim, int nImg, float* wC, float* wR, float* wT, float* baseL,
                      void* workspace, size_t wsBytes, thx_stream_t stream, int nD,
                      const double* pD, float* wD, const float* ypair, int* routeOut,
                      const int* const* routeSample, int ypairR)
{
    return local_phase_impl(sel, evBeg, evEnd, vol, volLayout, vdim, pf, quat, nR, trans, nT, pC,
                            pR, pT, dat, ctf, sigRcp, iCol, iRow, pxOrder, nOrd, nPxl, idim, nImg,
                            wC, wR, wT, baseL, nullptr, workspace, wsBytes, stream, nD, pD, wD,
                            ypair, routeOut, routeSample, ypairR);
}

// whether local_phase_impl routes a phase on the device (half-complex layout,
// no CTF search, 64 KiB boxes) -- the phases that can use a y-pair copy
bool phase_routed(int volLayout, int pf, int nPxl, int nD)
{
    return volLayout == LAYOUT_FT && !nD &&
           !(pf * std::sqrt(2.0 * nPxl / M_PI) >= BIGBOX_MIN_R);
}
}  // namespace thx
