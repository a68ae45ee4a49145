// timing.hip -- HIP event pairs for in-process kernel timing (thx_expect_cfg
// phaseEvents): the caller allocates n pairs, the driver records them on its
// launch stream around every phase's k_local_fused, and the elapsed times
// come back as milliseconds per pair.  No reference counterpart (its
// gettimeofday timers are commented out, src/Optimiser.cpp:1782-1786).
#include <vector>

#include "common.h"

extern "C" int thx_event_pairs_create(int n, void** events)
{
    THX_CHECK_ARG(n > 0 && events, "thx_event_pairs_create: bad arguments");
    hipEvent_t* ev = new hipEvent_t[2 * (size_t)n]();
    for (int i = 0; i < 2 * n; i++) {
        if (hipEventCreate(&ev[i]) != hipSuccess) {
            for (int j = 0; j < i; j++) (void)hipEventDestroy(ev[j]);
            delete[] ev;
            thx::set_error("thx_event_pairs_create: hipEventCreate failed");
            return THX_ERR_HIP;
        }
    }
    *events = ev;
    return THX_OK;
}

// ms[i] = time between begin and end of pair i (synchronises on the end events);
// a pair whose events were never recorded gives -1
extern "C" int thx_event_pairs_elapsed(void* events, int n, float* ms)
{
    THX_CHECK_ARG(events && ms && n > 0, "thx_event_pairs_elapsed: bad arguments");
    hipEvent_t* ev = static_cast<hipEvent_t*>(events);
    for (int i = 0; i < n; i++) {
        float t = -1.f;
        if (hipEventSynchronize(ev[2 * i + 1]) == hipSuccess &&
            hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]) != hipSuccess)
            t = -1.f;
        ms[i] = t;
    }
    (void)hipGetLastError();   // unrecorded events leave an error behind
    return THX_OK;
}

extern "C" int thx_event_pairs_destroy(void* events, int n)
{
    if (!events) return THX_OK;
    hipEvent_t* ev = static_cast<hipEvent_t*>(events);
    for (int i = 0; i < 2 * n; i++) (void)hipEventDestroy(ev[i]);
    delete[] ev;
    return THX_OK;
}
