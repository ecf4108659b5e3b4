// dcte_passes.h -- per-lane row / column passes of the energy-map kernels.
//
// Host+device (see dcte_math.h): the gfx950 kernel and the host emulation in
// tests/emu run this exact code, so their fp32 results are bit-identical.
//
// ring[slot][ch] holds the last N row transforms (first pass, along x -- the
// reference's first index, src/fft2d/shrtdct.c:62-89) of the lane's output
// column; slot O is the oldest.  A column pass runs the second-pass transforms
// (along y) over the ring and folds |C| into
//     m_e = max(|C01|, |C10|)   (edge atoms, src/dct.c:18-25 LUT)
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
    static constexpr int S = (N == 16) ? 4 : 1;   // lanes (N=16: waves) per output column
    static constexpr int CH = N / S;              // k1 channels per lane
};

// N = 16: wave q of the workgroup owns the four horizontal frequencies
//   q = 0: k1 = 0, 4, 8, 12    (even part of the 8-point transform of s)
//   q = 1: k1 = 2, 6, 10, 14   (odd part of the 8-point transform of s)
//   q = 2: k1 = 1, 5, 9, 13    (odd half of the 16-point transform)
//   q = 3: k1 = 3, 7, 11, 15
// with s_j = x_j + x_{15-j}; channel c of wave q holds k1 = 4c + {0,2,1,3}[q].
// Roles are wave-uniform, so nothing diverges; the four partial maxima of a
// pixel meet in LDS (dcte_map, N = 16).

// ------------------------------------------------------------------ column pass
// Per-lane column stage: fold this lane's channels into (m_t, m_e).
template <int N>
struct Cols;

template <>
struct Cols<8> {
    // ring[s][k1]; oldest row in slot O.  All eight columns in scaled form
    // (dct8_col_sc, dct8_k0_sc), each folded into the running maxima m1
    // (scale 1), mE, mA, mQ as soon as it is formed; k1 = 1 seeds them and
    // k1 = 0 comes last (fewer live registers than seeding from k1 = 0)
    template <int O>
    DCTE_HD_MEMBER void run(const float (&ring)[8][8], int /*lane_p*/, float& mt, float& me)
    {
        float col[8];
        float e0, e1;
        float v1, ye[2], ya[2], pq, unused;
        col_at<O>(ring, 1, col);
        dct8_col_sc<true>(col, v1, ye, ya, pq, e1);
        float m1 = fabsf(v1), mQ = pq;
        float mE = fmaxf(fabsf(ye[0]), fabsf(ye[1])), mA = fmaxf(fabsf(ya[0]), fabsf(ya[1]));
#pragma unroll
        for (int k = 2; k < 8; k++) {
            col_at<O>(ring, k, col);
            dct8_col_sc<false>(col, v1, ye, ya, pq, unused);
            m1 = fmaxf(m1, v1);
            mQ = fmaxf(mQ, pq);
            mE = max2in(mE, ye[0], ye[1]);
            mA = max2in(mA, ya[0], ya[1]);
        }
        col_at<O>(ring, 0, col);
        dct8_k0_sc(col, m1, mE, mA, mQ, e0);
        mt = max2in(max2in(m1, mQ * k8sPQ, mE * k8sE), mA * k8sA, 0.0f);
        me = fmaxf(e1, e0 * k8sPQ);
    }

    template <int O>
    DCTE_HD_MEMBER void col_at(const float (&ring)[8][8], int k, float (&col)[8])
    {
#pragma unroll
        for (int j = 0; j < 8; j++) col[j] = ring[(O + j) & 7][k];
    }
};

// N = 2: the plain 2-point transforms, every coefficient folded
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
            dct2(col, X);
#pragma unroll
            for (int q = 0; q < N; q++) {
                if (k == 0 && q == 0) continue;                 // DC
                if ((k == 0 && q == 1) || (k == 1 && q == 0)) me = fmaxf(me, fabsf(X[q]));
                else mt = fmaxf(mt, fabsf(X[q]));
            }
        }
    }
};
// N = 4 in scaled form: X2 = H (s0 - s1) and the rotation X1 = A (d0 + r d1),
// X3 = A (r d0 - d1), r = B / A, feed running maxima scaled once per pixel
// (8 VALU ops per column instead of 11).  Edge atoms: X1 of k1 = 0 (scale A)
// and X0 of k1 = 1 (scale 1).
template <>
struct Cols<4> {
    template <int O>
    DCTE_HD_MEMBER void run(const float (&ring)[4][4], int, float& mt, float& me)
    {
        float m1 = 0.0f, mH = 0.0f, mA = 0.0f, e0 = 0.0f, e1 = 0.0f;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            float c[4];
#pragma unroll
            for (int j = 0; j < 4; j++) c[j] = ring[(O + j) & 3][k];
            const float s0 = c[0] + c[3], d0 = c[0] - c[3];
            const float s1 = c[1] + c[2], d1 = c[1] - c[2];
            mH = fmaxf(mH, fabsf(s0 - s1));
            const float x1 = fmaf(d1, k4rBA, d0), x3 = fmaf(d0, k4rBA, -d1);
            if (k == 0) {
                e0 = fabsf(x1);
                mA = fabsf(x3);
            } else {
                mA = max2in(mA, x1, x3);
                if (k == 1) e1 = fabsf(s0 + s1); else m1 = fmaxf(m1, fabsf(s0 + s1));
            }
        }
        mt = max2in(m1, mH * k4H, mA * k4A);
        me = fmaxf(e1, e0 * k4A);
    }
};
template <> struct Cols<2> : ColsSmall<2> {};

template <>
struct Cols<16> {
    template <int O>
    DCTE_HD_MEMBER void run(const float (&ring)[16][4], int q, float& mt, float& me)
    {
        float col[16];
        mt = 0.0f;
        me = 0.0f;
        float mE = 0.0f, mA = 0.0f, mQ = 0.0f, m2 = 0.0f;   // scaled running maxima (dct16_tex_sc)
        float mO = 0.0f, mEO = 0.0f;                         // ... of the odd halves
        // channel 0: k1 = 4q' ... special roles for k1 = 0 (q = 0) and k1 = 1 (q = 2)
#pragma unroll
        for (int j = 0; j < 16; j++) col[j] = ring[(O + j) & 15][0];
        if (q == 0 || q == 2) {
            // the two edge columns in the scaled forms as well: q = 0 holds
            // k1 = 0 (exact integer row sums, centred on one of its own
            // samples so no large partial sum forms; the DC is excluded, X1 =
            // C01 is the odd half's sqrt2 Re U0), q = 2 holds k1 = 1 (X0 = C10
            // is the even half's a + b)
            if (q == 0) {
                const float ref = col[7];
#pragma unroll
                for (int j = 0; j < 16; j++) col[j] -= ref;
            }
            float s[8], d[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                s[j] = col[j] + col[15 - j];
                d[j] = col[j] - col[15 - j];
            }
            float v1, ye[2], ya[2], pq, e_even, e_odd;
            dct8_col_sc<true>(s, v1, ye, ya, pq, e_even);
            mt = fabsf(v1);
            mE = max2in(mE, ye[0], ye[1]);
            mA = max2in(mA, ya[0], ya[1]);
            mQ = pq;
            if (q == 0) {
                dct16_odd_sc<true>(d, mO, mEO, m2, &e_odd);
                me = e_odd * k16o2;
            } else {
                dct16_odd_sc<false>(d, mO, mEO, m2);
                me = e_even;
            }
        } else {
            dct16_tex_sc(col, mt, mE, mA, mQ, mO, mEO, m2);
        }
#pragma unroll
        for (int c = 1; c < 4; c++) {
#pragma unroll
            for (int j = 0; j < 16; j++) col[j] = ring[(O + j) & 15][c];
            dct16_tex_sc(col, mt, mE, mA, mQ, mO, mEO, m2);
        }
        mt = max2in(max2in(max2in(mt, mQ * k8sPQ, mE * k8sE), mA * k8sA, m2 * k16o2), mO * k16oM, mEO * k16oE);
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
        // N = 16, wave q (see Lanes): 4 of the 16 frequencies of this row
        float s[8], d[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            float a = lrow[c + j], b = lrow[c + 15 - j];
            s[j] = a + b;
            d[j] = a - b;
        }
        if (p == 0 || p == 1) {
            float t0 = s[0] + s[7], t1 = s[1] + s[6], t2 = s[2] + s[5], t3 = s[3] + s[4];
            if (p == 0) {                   // k1 = 0, 4, 8, 12 (exact sums for 0, 8)
                float a = t0 + t3, b = t1 + t2, cc = t0 - t3, e = t1 - t2;
                dst[0] = a + b;
                dst[1] = fmaf(cc, k8E, e * k8F);
                dst[2] = a - b;
                dst[3] = fmaf(cc, k8F, -(e * k8E));
            } else {                        // k1 = 2, 6, 10, 14
                dct8_odd(s[0] - s[7], s[1] - s[6], s[2] - s[5], s[3] - s[4],
                         dst[0], dst[1], dst[2], dst[3]);
            }
        } else {
            dct16_odd_rows(d, p == 2 ? 1 : 3, dst);   // k1 = 1,5,9,13 or 3,7,11,15
        }
    }
}

}  // namespace dcte
