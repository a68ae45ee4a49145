// common.h -- shared helpers for the gfx950 kernels and the C-ABI glue.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/thunder_amd.h"

namespace thx {

// Thread-local last-error text behind thx_last_error().
void set_error(const char* fmt, ...);

// Error convention: every exported entry point returns a THX_* status; the
// reference's exit(1) on any CUDA error (gpu/config/Device.cuh.in:27-58) is
// replaced by a status code + message the caller can act on.
#define THX_CHECK_ARG(cond, ...)                \
    do {                                        \
        if (!(cond)) {                          \
            ::thx::set_error(__VA_ARGS__);      \
            return THX_ERR_ARG;                 \
        }                                       \
    } while (0)

#define THX_HIP(call)                                                          \
    do {                                                                       \
        hipError_t e_ = (call);                                                \
        if (e_ != hipSuccess) {                                                \
            ::thx::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call,        \
                             hipGetErrorString(e_));                           \
            return THX_ERR_HIP;                                                \
        }                                                                      \
    } while (0)

#define THX_LAUNCH_CHECK() THX_HIP(hipGetLastError())

// propagate a THX_* status
#define THX_RET(call)                  \
    do {                               \
        int st_ = (call);              \
        if (st_ != THX_OK) return st_; \
    } while (0)

// Raise a kernel's dynamic-LDS limit once per device (the attribute is per
// device; a host may drive several GPUs from one process).  `done` is the
// kernel's own device bit mask.
inline int set_max_lds(const void* fn, int bytes, std::atomic<unsigned>& done)
{
    int dev = 0;
    THX_HIP(hipGetDevice(&dev));
    const unsigned bit = dev < 32 ? 1u << dev : 0u;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return THX_OK;
    THX_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    done.fetch_or(bit, std::memory_order_release);
    return THX_OK;
}

// the devices the host adapters use and getAviDevice reports (interface.hip)
int adapter_devices(std::vector<int>& devs);

// the device an RCCL communicator was created on (halfmap.hip)
int comm_device(void* comm, int* dev);

// the RCCL half-map all-reduce with oDim doubles of O per class (halfmap.hip)
int halfmap_allreduce_impl(void* comm, float* F, float* T, double* O, int oDim, int* counter,
                           long long dimSize, int nK, hipStream_t s);

inline hipStream_t as_stream(thx_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

// Workspace carving: 256-B aligned sub-buffers of a caller-provided device
// allocation (no hipMalloc inside launch functions, so callers may capture
// them into a HIP graph).
struct Carver {
    char* base;
    size_t cap;
    size_t off = 0;
    Carver(void* b, size_t c) : base(static_cast<char*>(b)), cap(c) {}
    template <typename T>
    T* take(size_t n) {
        off = (off + 255) & ~size_t(255);
        T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
        off += n * sizeof(T);
        return p;
    }
    bool ok() const { return off <= cap; }
};

}  // namespace thx

// ---------------------------------------------------------------- device ---
#define THX_DEV __device__ __forceinline__

// Negative row / slice indices wrap by +vdim: Volume::iFTHalf
// (include/Image/Volume.h:567-575).
THX_DEV int wrap_idx(int v, int n) { return v >= 0 ? v : v + n; }

// a * b + c on the full-rate 24-bit multiplier (v_mad_u32_u24) for index
// arithmetic whose factors are below 2^24 and whose result fits 32 bits.
// Written out because the compiler folds __umul24 + add into the 64-bit
// v_mad_u64_u32 (or a v_mul_lo_u32), both quarter rate, and in the local
// phases VALU issue is what the late phases are bound by.
THX_DEV unsigned mad24(unsigned a, unsigned b, unsigned c)
{
    unsigned r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

THX_DEV float2 cmul(float2 a, float2 b)
{
    // operator* of include/Complex.h:195-203
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

template <typename T>
THX_DEV T wave_sum(T v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

THX_DEV float wave_max(float v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Trilinear Fourier-space gather of Volume::getByInterpolationFT
// (src/Image/Volume.cpp:314-338): Hermitian fold when x < 0 (conjHalf,
// include/Image/Volume.h:135-147), floor + 8 weights
// (WG_TRI_INTERP_LINEAR, include/Functions/Interpolation.h:187-200), taps
// summed in box order k, j, i (getFTHalf, src/Image/Volume.cpp:491-563).
THX_DEV float2 interp_ft(const float2* __restrict__ vol, int vdim, float x,
                         float y, float z)
{
    const bool conj = !(x >= 0.f);
    if (conj) { x = -x; y = -y; z = -z; }
    const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
    const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
    const float dx = x - fx, dy = y - fy, dz = z - fz;
    const float vx[2] = {1.f - dx, dx};
    const float vy[2] = {1.f - dy, dy};
    const float vz[2] = {1.f - dz, dz};
    const int nColFT = vdim / 2 + 1;
    const int ya = wrap_idx(y0, vdim), yb = wrap_idx(y0 + 1, vdim);
    const int za = wrap_idx(z0, vdim), zb = wrap_idx(z0 + 1, vdim);
    const size_t r00 = ((size_t)za * vdim + ya) * nColFT + x0;
    const size_t r01 = ((size_t)za * vdim + yb) * nColFT + x0;
    const size_t r10 = ((size_t)zb * vdim + ya) * nColFT + x0;
    const size_t r11 = ((size_t)zb * vdim + yb) * nColFT + x0;
    const float2 a0 = vol[r00], a1 = vol[r00 + 1];
    const float2 b0 = vol[r01], b1 = vol[r01 + 1];
    const float2 c0 = vol[r10], c1 = vol[r10 + 1];
    const float2 d0 = vol[r11], d1 = vol[r11 + 1];
    float re = 0.f, im = 0.f;
    float w;
    w = vx[0] * vy[0] * vz[0]; re += a0.x * w; im += a0.y * w;
    w = vx[1] * vy[0] * vz[0]; re += a1.x * w; im += a1.y * w;
    w = vx[0] * vy[1] * vz[0]; re += b0.x * w; im += b0.y * w;
    w = vx[1] * vy[1] * vz[0]; re += b1.x * w; im += b1.y * w;
    w = vx[0] * vy[0] * vz[1]; re += c0.x * w; im += c0.y * w;
    w = vx[1] * vy[0] * vz[1]; re += c1.x * w; im += c1.y * w;
    w = vx[0] * vy[1] * vz[1]; re += d0.x * w; im += d0.y * w;
    w = vx[1] * vy[1] * vz[1]; re += d1.x * w; im += d1.y * w;
    return make_float2(re, conj ? -im : im);
}

// Rotated Fourier coordinate of Projector::project (src/Projector.cpp:
// 365-368): FP64 R * (iCol*pf, iRow*pf, 0), then cast to FP32.
THX_DEV void rot_coord(const double* m, int ic, int ir, int pf, float& x,
                       float& y, float& z)
{
    const double nx = (double)(ic * pf), ny = (double)(ir * pf);
    x = (float)(m[0] * nx + m[3] * ny);
    y = (float)(m[1] * nx + m[4] * ny);
    z = (float)(m[2] * nx + m[5] * ny);
}

// Translation phase exp(-2*pi*i*(iCol*tx + iRow*ty)/N) of translate()
// (src/Image/ImageFunctions.cpp:233-252).  The phase is formed in FP32 like
// the reference; the hardware sin/cos take revolutions, so the 2*pi product
// never has to be rounded.
THX_DEV float2 phase_shift(int ic, int ir, float rCol, float rRow)
{
    const float rev = -(ic * rCol + ir * rRow);
    const float f = rev - rintf(rev);
    return make_float2(__builtin_amdgcn_cosf(f), __builtin_amdgcn_sinf(f));
}

// CTF(RFLOAT*, ...) (src/CTF.cpp:113-151) at pixel (ic, ir) of an idim box
// for attr a = {pixelSize, voltage, dU, dV, theta, Cs, ampContrast,
// phaseShift} with the defocus pair (dU, dV) given separately (the CTF
// search inserts with (dU d, dV d), src/Optimiser.cpp:7105-7119); the
// per-image constants are formed as there (FP64 wavelength, then RFLOAT).
THX_DEV float ctf_at(const float* a, float dU, float dV, int ic, int ir, int idim)
{
    const float pixelSize = a[0], voltage = a[1], theta = a[4], Cs = a[5];
    const float ampC = a[6], phaseShift = a[7];
    const float lambda =
        (float)(12.2643247 / sqrt((double)voltage * (1 + (double)voltage * 0.978466e-6)));
    const float w1 = sqrtf(1.f - (float)((double)ampC * ampC));
    const float K1 = (float)(M_PI * lambda);
    const float K2 = (float)(M_PI_2 * Cs * (float)((double)lambda * lambda * lambda));
    const float fa = ic / (pixelSize * idim);
    const float fb = ir / (pixelSize * idim);
    const float u = (float)hypot((double)fa, (double)fb);
    const float angle = (float)(atan2((double)ir, (double)ic) - theta);
    const float defocus = -(dU + dV + (dU - dV) * cosf(2.f * angle)) / 2.f;
    const float u2 = (float)((double)u * u);
    const float u4 = (float)((double)u * u * u * u);
    const float ki = K1 * defocus * u2 + K2 * u4 - phaseShift;
    return -w1 * sinf(ki) + ampC * cosf(ki);
}

// The CTF-search CTF of one pixel (kernel_CalCTFL, gpu/src/Kernel.cu:481-515;
// src/Optimiser.cpp:1258-1270): ki = K1 defocusP d f^2 + K2 f^4 - phaseShift,
// -sqrt(1 - conT^2) sin(ki) + conT cos(ki).
THX_DEV float ctf_search_at(float k1, float dfo, double d, float f, float k2, float ps,
                            float conT)
{
    const float w1 = sqrtf(1.f - (float)((double)conT * conT));
    const double f2 = (double)f * f;
    const float ki = (float)((double)(k1 * dfo) * d * f2 + k2 * (f2 * f2) - ps);
    return -w1 * sinf(ki) + conT * cosf(ki);
}

// rotate3D, src/Geometry/Euler.cpp:181-189: R = I + 2 q0 A + 2 A A with
// A = [[0,-q3,q2],[q3,0,-q1],[-q2,q1,0]], stored column-major.
THX_DEV void quat_to_mat(const double* q, double* m)
{
    const double A[3][3] = {{0, -q[3], q[2]}, {q[3], 0, -q[1]}, {-q[2], q[1], 0}};
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) {
            double aa = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) aa += (2 * A[r][k]) * A[k][c];
            m[c * 3 + r] = (r == c ? 1.0 : 0.0) + (2 * q[0]) * A[r][c] + aa;
        }
}

// Trilinear scatter of Volume::addFT (src/Image/Volume.cpp:340-375):
// Hermitian fold conjugates the complex value, 8 taps in box order, FP32
// device-scope atomics (global_atomic_add_f32) on F (re, im) and T.
THX_DEV void scatter_ft(float2* __restrict__ F, float* __restrict__ T, int vdim,
                        float x, float y, float z, float vr, float vi, float tv)
{
    if (!(x >= 0.f)) { x = -x; y = -y; z = -z; vi = -vi; }
    const float fx = floorf(x), fy = floorf(y), fz = floorf(z);
    const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
    const float dx = x - fx, dy = y - fy, dz = z - fz;
    const float vx[2] = {1.f - dx, dx};
    const float vy[2] = {1.f - dy, dy};
    const float vz[2] = {1.f - dz, dz};
    const int nColFT = vdim / 2 + 1;
#pragma unroll
    for (int k = 0; k < 2; k++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const size_t row = ((size_t)wrap_idx(z0 + k, vdim) * vdim +
                                wrap_idx(y0 + j, vdim)) * nColFT + x0;
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const float w = vx[i] * vy[j] * vz[k];
                float* f = reinterpret_cast<float*>(F + row + i);
                atomicAdd(f, vr * w);
                atomicAdd(f + 1, vi * w);
                atomicAdd(T + row + i, tv * w);
            }
        }
}

// Philox-4x32-10 counter RNG (reproducible per (seed, counter); the reference
// draws from an urandom-seeded GSL mt19937, src/Functions/Random.cpp:51-73)
struct Philox {
    uint4 ctr;
    uint2 key;
    THX_DEV Philox(uint64_t seed, uint32_t a, uint32_t b, uint32_t c)
    {
        key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
        ctr = make_uint4(a, b, c, 0);
    }
    THX_DEV uint4 next()
    {
        uint4 x = ctr;
        uint2 k = key;
#pragma unroll
        for (int r = 0; r < 10; r++) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * x.x;
            const uint64_t p1 = (uint64_t)0xCD9E8D57u * x.z;
            x = make_uint4((uint32_t)(p1 >> 32) ^ x.y ^ k.x, (uint32_t)p1,
                           (uint32_t)(p0 >> 32) ^ x.w ^ k.y, (uint32_t)p0);
            k.x += 0x9E3779B9u;
            k.y += 0xBB67AE85u;
        }
        ctr.w++;
        return x;
    }
    THX_DEV double uniform()   // (0, 1)
    {
        const uint4 v = next();
        const uint64_t m = ((uint64_t)v.x << 21) ^ (uint64_t)v.y;
        return ((double)(m & ((1ull << 53) - 1)) + 0.5) * (1.0 / 9007199254740992.0);
    }
    THX_DEV double2 gauss2()   // Box-Muller
    {
        const double u1 = uniform(), u2 = uniform();
        const double r = sqrt(-2.0 * log(u1));
        double s, c;
        sincos(2.0 * M_PI * u2, &s, &c);
        return make_double2(r * c, r * s);
    }
};

// 2^56 fixed point for LDS sums of a few values in [0, 8): ds_add_u64 retires
// a wave-instruction in 7-12 CU cycles where ds_add_f32 takes ~193 on gfx950
// (tools/probes/lds_atomic.hip); the integer sum is exact and order-free.
THX_DEV unsigned long long fx56(float v)
{
    return (unsigned long long)__float2ll_rn(ldexpf(v, 56));
}
THX_DEV float unfx56(unsigned long long q) { return (float)ldexp((double)(long long)q, -56); }
