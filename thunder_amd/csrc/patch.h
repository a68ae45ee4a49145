// patch.h -- patch neighbourhoods shared by the local phase (local.hip) and
// the insert (insert.hip).  Pixels are visited in 16-pixel patches
// (thx_pixel_tile_order); for every (image, tile of PATCH_RT rotations,
// patch) k_patch_boxes writes a PATCH_REC-int record bounding the voxels the
// 8 trilinear taps of all the patch's samples can touch, in folded (x >= 0)
// coordinates, as two boxes of one shape (side 0: samples with x >= 0,
// side 1: Hermitian-folded ones), laid out [z][y][x] with bank-spread pitches:
//   [0..2] side-0 origin (x, y, z; rows / slices signed, unwrapped)
//   [3..5] side-1 origin  [6] row pitch nx  [7] slice pitch sp  [8] ny
//   [9] side-0 voxels (= offset of side 1)  [10] total voxels
//   [11] side-0 items (4 voxels = 32 B of a row)  [12] total items
//   [13] magic(nx / 4)  [14] magic(ny)  (udiv)
//   [15] / [16] index of voxel (0, 0, 0) for side 0 / 1 (may be negative),
//   set when [10] <= PATCH_BOX_CAP
//   [17], [18] (iCol, iRow) of the patch's first pixel (stand-in for padding)
#pragma once
#include "common.h"

namespace thx {

constexpr int PATCH_KC = 16;        // pixels per patch
constexpr int PATCH_RT = 128;       // rotations per record tile
constexpr int PATCH_REC = 20;       // ints per record
constexpr int PATCH_BOX_CAP = 16384; // largest box the records carry LDS offsets for

size_t patch_rec_bytes(int nImg, int nR, int nVisit);
// records for quat [nImg][nR][4] (device), one per (image, rotation tile, patch)
int launch_patch_boxes(const double* quat, int nR, const int* iCol, const int* iRow,
                       const int* order, int nVisit, int pf, int vdim, int nImg, int* rec,
                       hipStream_t s);

}  // namespace thx

THX_DEV int patch_pixel(const int* __restrict__ order, int nVisit, int k)
{
    return k < nVisit ? (order ? order[k] : k) : -1;
}
