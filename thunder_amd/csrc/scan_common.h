// scan_common.h -- class-merge step shared by the global-scan variants.
#pragma once
#include "common.h"

// Called by every thread of the block owning image l, with m = the max dvp of
// class kIdx.  kIdx == 0 starts a fresh accumulation (other classes zeroed, as
// the host arrays of src/Optimiser.cpp:1788-1790 are); kIdx > 0 raises the
// running baseline and rescales the classes already accumulated by
// exp(old - new), the step of kernel_setBaseLine (gpu/src/Kernel.cu:1096-1128)
// and of the CPU loop (src/Optimiser.cpp:842-872).  Returns the baseline the
// caller must use for class kIdx.
THX_DEV float merge_baseline(int l, float m, int kIdx, int nK, int nR, int nT,
                             float* __restrict__ wC, float* __restrict__ wR,
                             float* __restrict__ wT, float* __restrict__ baseL)
{
    const float old = baseL[l];
    __syncthreads();
    float base;
    if (kIdx == 0) {
        base = m;
        for (int k = 1; k < nK; k++) {
            if (threadIdx.x == 0) wC[(size_t)l * nK + k] = 0.f;
            for (int r = threadIdx.x; r < nR; r += blockDim.x)
                wR[((size_t)l * nK + k) * nR + r] = 0.f;
            for (int t = threadIdx.x; t < nT; t += blockDim.x)
                wT[((size_t)l * nK + k) * nT + t] = 0.f;
        }
    } else {
        base = (old != old) ? m : fmaxf(old, m);
        if (base > old) {
            const float nf = expf(old - base);
            for (int k = 0; k < nK; k++) {
                if (k == kIdx) continue;
                if (threadIdx.x == 0) wC[(size_t)l * nK + k] *= nf;
                for (int r = threadIdx.x; r < nR; r += blockDim.x)
                    wR[((size_t)l * nK + k) * nR + r] *= nf;
                for (int t = threadIdx.x; t < nT; t += blockDim.x)
                    wT[((size_t)l * nK + k) * nT + t] *= nf;
            }
        }
    }
    if (threadIdx.x == 0) baseL[l] = base;
    return base;
}
