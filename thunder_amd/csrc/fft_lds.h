// fft_lds.h -- one wave's complex FFT of a power-of-two length N (16 .. 512)
// held in LDS: mixed-radix Stockham autosort stages (radix 8 while 8 divides
// the remaining length, then one radix-4 or radix-2 stage), unnormalised,
// sign s = -1 (forward, e^{-2 pi i k n / N}) or +1 (inverse).  A stage has
// N / R <= 64 butterflies: lane j reads R values N / R apart, applies the
// twiddles W_{Ns R}^{(j mod Ns) r} (the table holds e^{-2 pi i q / N},
// q < N), runs the R-point DFT in registers and writes the outputs Ns apart
// from (j / Ns) Ns R + j mod Ns.  Every lane holds all its inputs in
// registers before any lane writes (one butterfly per lane, the wave in
// lockstep), so the stages run in place in one buffer.
// Layout of a column: element i lives at slot q = (i + off) mod N (off: the
// column's rotation -- the load / store tiles of the column passes rotate
// column c by c so a row of columns spreads over the banks), stored at
// q + q / 8: one pad slot every 8 elements, which turns the stride-8 and
// stride-64-group writes of the first two radix-8 stages from 8-way bank
// conflicts into the 2-way minimum of 8-byte accesses.
#pragma once
#include "common.h"

namespace thx {

// LDS slots a padded column of N elements occupies
template <int N>
constexpr int fft_pitch() { return N + N / 8; }

template <int N>
THX_DEV int fft_slot(int i, int off)
{
    const int q = (i + off) & (N - 1);
    return q + (q >> 3);
}

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
THX_DEV void fft_stages(float2* a, int off, const float2* __restrict__ tw, float s, int lane)
{
    if constexpr (NS < N) {
        constexpr int REM = N / NS;
        constexpr int R = REM % 8 == 0 ? 8 : REM;
        constexpr int M = N / R;            // butterflies per stage (<= 64)
        constexpr int TS = N / (NS * R);    // twiddle index step
        static_assert(M <= 64, "one butterfly per lane");
        if (lane < M) {
            const int j = lane;
            float2 v[R];
#pragma unroll
            for (int r = 0; r < R; r++) v[r] = a[fft_slot<N>(j + r * M, off)];
            const int k = j % NS;
            if (NS > 1) {
#pragma unroll
                for (int r = 1; r < R; r++) {
                    const float2 w = tw[(k * r * TS) & (N - 1)];
                    v[r] = cmulf(v[r], make_float2(w.x, -s * w.y));
                }
            }
            dft_small<R>(v, s);
            const int d = (j / NS) * NS * R + k;
            // every lane's reads of this stage precede its writes, in lockstep
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < R; r++) a[fft_slot<N>(d + r * NS, off)] = v[r];
        }
        wave_lds_sync();
        fft_stages<N, NS * R>(a, off, tw, s, lane);
    }
}

// In place on the padded column (col, off); tw: e^{-2 pi i q / N}, q < N.
// The caller makes the column's data visible to the wave first.
template <int N>
THX_DEV void wave_fft(float2* col, int off, const float2* __restrict__ tw, float s, int lane)
{
    fft_stages<N, 1>(col, off, tw, s, lane);
}

}  // namespace thx
