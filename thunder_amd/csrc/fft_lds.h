// fft_lds.h -- one wave's complex FFT of a power-of-two length N (16 .. 512)
// held in LDS: mixed-radix Stockham autosort stages (radix 8 while 8 divides
// the remaining length, then one radix-4 or radix-2 stage), ping-ponging
// between the column buffer and a scratch buffer of the wave, unnormalised,
// sign s = -1 (forward, e^{-2 pi i k n / N}) or +1 (inverse).  Each lane takes
// the N / R butterflies j = lane, lane + 64, ...: it reads R values a distance
// N / R apart, applies the twiddles W_{Ns R}^{(j mod Ns) r} (the table holds
// e^{-2 pi i q / N}, q < N), runs the R-point DFT in registers and writes the
// outputs Ns apart from (j / Ns) Ns R + j mod Ns.
// A column buffer may be rotated: element i of the column lives at
// base[(i + off) & (N - 1)] (the load / store tiles of the column passes use
// off = column index so that a row of columns spreads over the LDS banks).
#pragma once
#include "common.h"

namespace thx {

THX_DEV float2 cmulf(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }

// s i z
THX_DEV float2 mul_si(float2 z, float s) { return make_float2(-s * z.y, s * z.x); }

template <int R>
THX_DEV void dft_small(float2* v, float s)
{
    if constexpr (R == 2) {
        const float2 a = v[0], b = v[1];
        v[0] = make_float2(a.x + b.x, a.y + b.y);
        v[1] = make_float2(a.x - b.x, a.y - b.y);
    } else if constexpr (R == 4) {
        const float2 e0 = make_float2(v[0].x + v[2].x, v[0].y + v[2].y);
        const float2 e1 = make_float2(v[0].x - v[2].x, v[0].y - v[2].y);
        const float2 o0 = make_float2(v[1].x + v[3].x, v[1].y + v[3].y);
        const float2 o1 = mul_si(make_float2(v[1].x - v[3].x, v[1].y - v[3].y), s);
        v[0] = make_float2(e0.x + o0.x, e0.y + o0.y);
        v[2] = make_float2(e0.x - o0.x, e0.y - o0.y);
        v[1] = make_float2(e1.x + o1.x, e1.y + o1.y);
        v[3] = make_float2(e1.x - o1.x, e1.y - o1.y);
    } else {
        static_assert(R == 8, "radix 2, 4 or 8");
        float2 e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
        dft_small<4>(e, s);
        dft_small<4>(o, s);
        constexpr float c = 0.70710678118654752f;
        // w^k o[k], w = e^{s 2 pi i / 8}
        const float2 t0 = o[0];
        const float2 t1 = make_float2(c * (o[1].x - s * o[1].y), c * (o[1].y + s * o[1].x));
        const float2 t2 = mul_si(o[2], s);
        const float2 t3 = make_float2(c * (-o[3].x - s * o[3].y), c * (s * o[3].x - o[3].y));
        v[0] = make_float2(e[0].x + t0.x, e[0].y + t0.y);
        v[4] = make_float2(e[0].x - t0.x, e[0].y - t0.y);
        v[1] = make_float2(e[1].x + t1.x, e[1].y + t1.y);
        v[5] = make_float2(e[1].x - t1.x, e[1].y - t1.y);
        v[2] = make_float2(e[2].x + t2.x, e[2].y + t2.y);
        v[6] = make_float2(e[2].x - t2.x, e[2].y - t2.y);
        v[3] = make_float2(e[3].x + t3.x, e[3].y + t3.y);
        v[7] = make_float2(e[3].x - t3.x, e[3].y - t3.y);
    }
}

// LDS visibility between the lanes of one wave
THX_DEV void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int N, int NS>
THX_DEV void fft_stages(float2* a, int aOff, float2* b, int bOff, const float2* __restrict__ tw, float s,
                        int lane, float2** out, int* outOff)
{
    if constexpr (NS >= N) {
        *out = a;
        *outOff = aOff;
    } else {
        constexpr int REM = N / NS;
        constexpr int R = REM % 8 == 0 ? 8 : REM;
        constexpr int M = N / R;            // butterflies per stage
        constexpr int TS = N / (NS * R);    // twiddle index step
        constexpr int MASK = N - 1;
        for (int j = lane; j < M; j += 64) {
            float2 v[R];
#pragma unroll
            for (int r = 0; r < R; r++) v[r] = a[(j + r * M + aOff) & MASK];
            const int k = j % NS;
            if (NS > 1) {
#pragma unroll
                for (int r = 1; r < R; r++) {
                    const float2 w = tw[(k * r * TS) & MASK];
                    v[r] = cmulf(v[r], make_float2(w.x, -s * w.y));
                }
            }
            dft_small<R>(v, s);
            const int d = (j / NS) * NS * R + k;
#pragma unroll
            for (int r = 0; r < R; r++) b[(d + r * NS + bOff) & MASK] = v[r];
        }
        wave_lds_sync();
        fft_stages<N, NS * R>(b, bOff, a, aOff, tw, s, lane, out, outOff);
    }
}

// In place on the column (col, colOff): the result is copied back from the
// scratch when the stage count is odd.  tw: e^{-2 pi i q / N}, q < N.
template <int N>
THX_DEV void wave_fft(float2* col, int colOff, float2* scratch, const float2* __restrict__ tw, float s,
                      int lane)
{
    float2* res;
    int resOff;
    fft_stages<N, 1>(col, colOff, scratch, 0, tw, s, lane, &res, &resOff);
    if (res != col) {
        for (int i = lane; i < N; i += 64) col[(i + colOff) & (N - 1)] = scratch[i];
        wave_lds_sync();
    }
}

}  // namespace thx
