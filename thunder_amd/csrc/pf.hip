// pf.hip -- a10: particle-filter resampling on device, for all images of a
// batch at once (the reference does it per image on the host between GPU
// round trips, src/Optimiser.cpp:1403-1480 -> Particle::resample).
#include "common.h"

constexpr int RESAMPLE_MAX_IN = 8192;

// One wave per image.  The weighted CDF is built by lane 0 in the exact
// sequential FP64 order of the CPU restatement (w*u, running sum, divide,
// running cumsum, divide by the last element: src/Particle.cpp:1347-1356), so
// ancestors agree bit for bit; the nOut systematic points u_j = u0 + j/nOut
// are then placed in parallel by binary search for the first i with
// u_j <= cdf[i] -- the index at which the reference's
// `while (uj > cdf[i]) i++` walk stops (src/Particle.cpp:1360-1377).
__global__ void __launch_bounds__(64) k_resample(int nIn, const double* __restrict__ w,
                                                 const float* __restrict__ u, int nOut,
                                                 const double* __restrict__ u0,
                                                 int* __restrict__ ancestor,
                                                 double* __restrict__ wOut,
                                                 int* __restrict__ iMax)
{
    extern __shared__ double cdf[];
    const int l = blockIdx.x;
    const int lane = threadIdx.x;
    const double* wl = w + (size_t)l * nIn;
    const float* ul = u + (size_t)l * nIn;

    // iMax (src/Particle.cpp:1880-1891): first index of the maximum of u
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = lane; i < nIn; i += 64) {
        const float v = ul[i];
        if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) iMax[l] = bi;

    for (int i = lane; i < nIn; i += 64) cdf[i] = wl[i] * (double)ul[i];
    __syncthreads();
    if (lane == 0) {
        double sum = 0.0;
        for (int i = 0; i < nIn; i++) sum += cdf[i];
        double acc = 0.0;
        for (int i = 0; i < nIn; i++) { acc += cdf[i] / sum; cdf[i] = acc; }
        const double last = cdf[nIn - 1];
        for (int i = 0; i < nIn; i++) cdf[i] /= last;
    }
    __syncthreads();

    double s = 0.0;
    const double ul0 = u0[l];
    for (int j = lane; j < nOut; j += 64) {
        const double uj = ul0 + j * 1.0 / nOut;
        int lo = 0, hi = nIn - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (uj > cdf[mid]) lo = mid + 1; else hi = mid;
        }
        ancestor[(size_t)l * nOut + j] = lo;
        const double x = 1.0 / (double)ul[lo];   // PARTICLE_PRIOR_ONE
        wOut[(size_t)l * nOut + j] = x;
    }
    __syncthreads();
    if (lane == 0) {                               // normW, sequential sum
        for (int j = 0; j < nOut; j++) s += wOut[(size_t)l * nOut + j];
        cdf[0] = s;
    }
    __syncthreads();
    s = cdf[0];
    for (int j = lane; j < nOut; j += 64) wOut[(size_t)l * nOut + j] /= s;
}

extern "C" int thx_resample(int nImg, int nIn, const double* w, const float* u,
                            int nOut, const double* u0, int* ancestor,
                            double* wOut, int* iMax, thx_stream_t stream)
{
    THX_CHECK_ARG(nImg >= 0 && nIn > 0 && nOut > 0, "thx_resample: bad sizes");
    THX_CHECK_ARG(nIn <= RESAMPLE_MAX_IN, "thx_resample: nIn=%d > %d", nIn,
                  RESAMPLE_MAX_IN);
    if (nImg == 0) return THX_OK;
    hipLaunchKernelGGL(k_resample, dim3(nImg), dim3(64),
                       sizeof(double) * (size_t)nIn, thx::as_stream(stream), nIn,
                       w, u, nOut, u0, ancestor, wOut, iMax);
    THX_LAUNCH_CHECK();
    return THX_OK;
}
