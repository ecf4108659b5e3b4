// dcte_passes.h -- per-lane row / column passes of the energy-map kernels.
//
// Host+device (see dcte_math.h): the gfx950 kernel and the host emulation in
// tests/emu run this exact code, so their fp32 results are bit-identical.
//
// ring[slot][ch] holds the last N row transforms (first pass, along x -- the
// reference's first index, src/fft2d/shrtdct.c:62-89) of the lane's output
// column; slot O is the oldest.  A column pass runs the second-pass transforms
// (along y) over the ring and folds |C| into
//     m_e = max(|C01|, |C10|)   (edge atoms, src/dct.c:34-41 LUT)
//     m_t = max over the other non-DC coefficients.
#pragma once

#include "dcte_math.h"

#if defined(__HIPCC__)
#define DCTE_HD_MEMBER __host__ __device__ __forceinline__ static
#else
#define DCTE_HD_MEMBER static inline
#endif

namespace dcte {

template <int N>
struct Lanes {
    static constexpr int S = (N == 16) ? 2 : 1;   // lanes per output column
    static constexpr int CH = N / S;              // k1 channels per lane
};

// ------------------------------------------------------------------ column pass
// Per-lane column stage: fold this lane's channels into (m_t, m_e).
template <int N>
struct Cols;

template <>
struct Cols<8> {
    // ring[s][k1]; oldest row in slot O
    template <int O>
    DCTE_HD_MEMBER void run(const float (&ring)[8][8], int /*lane_p*/,
                                               float& mt, float& me)
    {
        float col[8];
        float e0, e1;
        mt = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; j++) col[j] = ring[(O + j) & 7][0];
        mt = dct8_k0_max(col, mt, e0);
#pragma unroll
        for (int j = 0; j < 8; j++) col[j] = ring[(O + j) & 7][1];
        mt = dct8_k1_max(col, mt, e1);
#pragma unroll
        for (int k = 2; k < 8; k++) {
#pragma unroll
            for (int j = 0; j < 8; j++) col[j] = ring[(O + j) & 7][k];
            mt = dct8_tex_max(col, mt);
        }
        me = fmaxf(e0, e1);
    }
};

template <int N>
struct ColsSmall {
    template <int O>
    DCTE_HD_MEMBER void run(const float (&ring)[N][N], int, float& mt, float& me)
    {
        mt = 0.0f;
        me = 0.0f;
#pragma unroll
        for (int k = 0; k < N; k++) {
            float col[N], X[N];
#pragma unroll
            for (int j = 0; j < N; j++) col[j] = ring[(O + j) % N][k];
            if constexpr (N == 4) dct4(col, X); else dct2(col, X);
#pragma unroll
            for (int q = 0; q < N; q++) {
                if (k == 0 && q == 0) continue;                 // DC
                if ((k == 0 && q == 1) || (k == 1 && q == 0)) me = fmaxf(me, fabsf(X[q]));
                else mt = fmaxf(mt, fabsf(X[q]));
            }
        }
    }
};
template <> struct Cols<4> : ColsSmall<4> {};
template <> struct Cols<2> : ColsSmall<2> {};

template <>
struct Cols<16> {
    // lane parity p: channel m holds k1 = 2m + p
    template <int O>
    DCTE_HD_MEMBER void run(const float (&ring)[16][8], int p, float& mt, float& me)
    {
        mt = 0.0f;
        me = 0.0f;
#pragma unroll
        for (int m = 0; m < 8; m++) {
            float col[16], X[16];
#pragma unroll
            for (int j = 0; j < 16; j++) col[j] = ring[(O + j) & 15][m];
            if (m == 0) {
                // k1 = 0 column (p = 0) carries exact row sums: centre it on one
                // of its own samples (exact) so no large partial sum forms.  The
                // k1 = 1 column (p = 1) must keep its X0 (edge atom C10).
                float ref = p ? 0.0f : col[7];
#pragma unroll
                for (int j = 0; j < 16; j++) col[j] -= ref;
            }
            dct16(col, X);
            if (m == 0) {
                me = p ? fabsf(X[0]) : fabsf(X[1]);
                float x1 = p ? fabsf(X[1]) : 0.0f;
                mt = fmaxf(mt, x1);
#pragma unroll
                for (int q = 2; q < 16; q++) mt = fmaxf(mt, fabsf(X[q]));
            } else {
#pragma unroll
                for (int q = 0; q < 16; q++) mt = fmaxf(mt, fabsf(X[q]));
            }
        }
    }
};

// ------------------------------------------------------------------ row pass
template <int N>
DCTE_HD void row_pass(const float* lrow, int c, int p, float (&dst)[Lanes<N>::CH])
{
    if constexpr (N == 8) {
        float x[8];
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = lrow[c + j];
        dct8(x, dst);
    } else if constexpr (N == 4) {
        float x[4];
#pragma unroll
        for (int j = 0; j < 4; j++) x[j] = lrow[c + j];
        dct4(x, dst);
    } else if constexpr (N == 2) {
        float x[2] = {lrow[c], lrow[c + 1]};
        dct2(x, dst);
    } else {
        float s[8], d[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            float a = lrow[c + j], b = lrow[c + 15 - j];
            s[j] = a + b;
            d[j] = a - b;
        }
        if (p == 0) {
            dct8(s, dst);                 // k1 = 0, 2, ..., 14
        } else {
            float X[16];
            dct16_odd(d, X);              // k1 = 1, 3, ..., 15
#pragma unroll
            for (int m = 0; m < 8; m++) dst[m] = X[2 * m + 1];
        }
    }
}

}  // namespace dcte
