// order.hip -- the local phases' image order: images sorted by the central
// slice their particle cloud projects through.
//
// The y-pair projectee a phase gathers from is a half ball of radius
// rU pf + 1 voxels (box 256, rU 24: ~3.9 MB), a little more than one XCD's
// 4 MB L2 with the image tiles next to it.  A workgroup touches only the
// slab around the central slice of its image's cloud (the plane through the
// origin with normal R e_z, a few degrees thick).  In batch order the
// orientations are random, every L2 sees the whole ball at once and the
// gathers miss to the fabric; with the images ordered along a space-filling
// curve of the slice normal, the workgroups in flight at one time (a few per
// cent of a 12 500-image batch) share a normal cone of ~15-20 degrees, whose
// slab is about a third of the ball.  Only which workgroup handles which
// image changes: every image's arithmetic is the same.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"

namespace {

// index of (x, y) on the Hilbert curve through the 2^16 x 2^16 grid (its
// runs of consecutive indices are connected, where a Morton order's jump)
THX_DEV unsigned curve16(unsigned x, unsigned y)
{
    constexpr unsigned N = 1u << 16;
    unsigned d = 0;
    for (unsigned s = N / 2; s > 0; s >>= 1) {
        const unsigned rx = (x & s) ? 1u : 0u, ry = (y & s) ? 1u : 0u;
        d += s * s * ((3u * rx) ^ ry);
        if (ry == 0) {
            if (rx == 1) { x = N - 1 - x; y = N - 1 - y; }
            const unsigned t = x; x = y; y = t;
        }
    }
    return d;
}

// key of image l: the slice normal n = R(q) e_z of the cloud's first
// particle (column 2 of quat_to_mat's column-major R), n and -n being one
// plane (n_z >= 0), octahedral map onto [-1, 1]^2, 16-bit cells, their
// Hilbert index
__global__ void __launch_bounds__(256) k_view_key(int nImg, int mLR, const double* __restrict__ quat,
                                                  unsigned* __restrict__ key, int* __restrict__ idx)
{
    const int l = blockIdx.x * 256 + threadIdx.x;
    if (l >= nImg) return;
    double m[9];
    quat_to_mat(quat + (size_t)l * mLR * 4, m);
    double nx = m[6], ny = m[7], nz = m[8];
    if (nz < 0.0) { nx = -nx; ny = -ny; nz = -nz; }
    const double s = fabs(nx) + fabs(ny) + nz;
    const double u = s > 0.0 ? nx / s : 0.0, v = s > 0.0 ? ny / s : 0.0;
    auto q16 = [](double t) { return (unsigned)fmin(65535.0, fmax(0.0, (t + 1.0) * 32768.0)); };
    key[l] = curve16(q16(u), q16(v));
    idx[l] = l;
}

}  // namespace

namespace thx {

// device bytes view_order needs beyond its 2 x nImg keys and indices
size_t view_order_tmp_bytes(int nImg)
{
    size_t b = 0;
    if (nImg <= 0) return 0;
    if (rocprim::radix_sort_pairs(nullptr, b, (unsigned*)nullptr, (unsigned*)nullptr, (int*)nullptr,
                                  (int*)nullptr, (size_t)nImg, 0, 32) != hipSuccess)
        return 0;
    return b;
}

// ord[0 .. nImg): the images sorted (stably) by k_view_key; keys / keysOut /
// idx scratch of nImg each, tmp of view_order_tmp_bytes(nImg)
int view_order(int nImg, int mLR, const double* quat, unsigned* keys, unsigned* keysOut, int* idx,
               int* ord, void* tmp, size_t tmpBytes, hipStream_t s)
{
    if (nImg <= 0) return THX_OK;
    hipLaunchKernelGGL(k_view_key, dim3(cdiv(nImg, 256)), dim3(256), 0, s, nImg, mLR, quat, keys, idx);
    THX_LAUNCH_CHECK();
    size_t b = tmpBytes;
    if (rocprim::radix_sort_pairs(tmp, b, keys, keysOut, idx, ord, (size_t)nImg, 0, 32, s) != hipSuccess) {
        set_error("view_order: radix sort failed");
        return THX_ERR_HIP;
    }
    return THX_OK;
}

}  // namespace thx

// bytes of one 4-byte-per-image scratch array, 256-aligned
static size_t ord_slot(int nImg) { return ((size_t)nImg * 4 + 255) / 256 * 256; }

extern "C" size_t thx_view_order_workspace(int nImg)
{
    if (nImg <= 0) return 0;
    return 3 * ord_slot(nImg) + thx::view_order_tmp_bytes(nImg);
}

extern "C" int thx_view_order(int nImg, int mLR, const double* quat, int* ord, void* workspace,
                              size_t wsBytes, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && mLR > 0, "thx_view_order: bad sizes");
    if (nImg == 0) return THX_OK;
    THX_CHECK_ARG(quat && ord && workspace, "thx_view_order: null argument");
    THX_CHECK_ARG(wsBytes >= thx_view_order_workspace(nImg), "thx_view_order: workspace too small");
    char* w = static_cast<char*>(workspace);
    const size_t a = ord_slot(nImg);
    unsigned* keys = reinterpret_cast<unsigned*>(w);
    unsigned* keysOut = reinterpret_cast<unsigned*>(w + a);
    int* idx = reinterpret_cast<int*>(w + 2 * a);
    return thx::view_order(nImg, mLR, quat, keys, keysOut, idx, ord, w + 3 * a,
                           thx::view_order_tmp_bytes(nImg), thx::as_stream(stream));
}
