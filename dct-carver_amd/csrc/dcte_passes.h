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

#ifndef DCTE_SC
#define DCTE_SC 1    // N = 8: columns in scaled form (dct8_k0_sc, dct8_col_sc), four running maxima
#endif
#ifndef DCTE_SC4
#define DCTE_SC4 1   // N = 4: second pass in scaled form (Cols<4>)
#endif
#ifndef DCTE_SC16
#define DCTE_SC16 1  // N = 16: even halves of the texture columns in scaled form (dct16_tex_sc)
#endif
#ifndef DCTE_PQ2
#define DCTE_PQ2 1   // N = 8: fold |X1|, |X7| through their own chain (dct8_col_parts)
#endif

#ifndef DCTE_MFMA8
#define DCTE_MFMA8 0     // N = 8: texture columns k1 = 8 - DCTE_MFMA8 .. 7 on the matrix pipe (0..6)
#endif
#ifndef DCTE_MFMA8_SYM
#define DCTE_MFMA8_SYM 1 // 1: the VALU forms x_t +- x_{7-t}, 2 x 4 MFMAs per column; 0: 2 x 8 MFMAs on x
#endif

namespace dcte {

// ------------------------------------------------------------------ matrix pipe
// A texture column of the N = 8 second pass on the matrix pipe, co-issued with
// the VALU columns.  v_mfma_f32_4x4x1_16b_f32 is 16 independent 4x4 outer
// products per wave: D[r] of lane l += A(lane 4 (l / 4) + r) * B(lane l) --
// with B = the lane's own ring value and A = a per-lane constant (lane l holds
// row l & 3 of the transform matrix) every lane accumulates four outputs of
// ITS OWN column, one fmaf per output per instruction (the MFMA is bit-for-bit
// an fmaf chain in program order).  The host side evaluates the same chains
// with fmaf, so tests/emu stays bit-identical to the device.
// Hat units as dct8: X[0] = sum x_j, X[k] = sqrt2 sum x_j cos(pi (2j+1) k / 16).
//   kMe[r][t]: X[2r] from s_t = x_t + x_{7-t};  kMo[r][t]: X[2r+1] from d_t = x_t - x_{7-t}
constexpr float kMe[4][4] = {{1.0f, 1.0f, 1.0f, 1.0f},
                             {k8E, k8F, -k8F, -k8E},
                             {1.0f, -1.0f, -1.0f, 1.0f},
                             {k8F, -k8E, k8E, -k8F}};
constexpr float kMo[4][4] = {{k8A, k8B, k8C, k8D},
                             {k8B, -k8D, -k8A, -k8C},
                             {k8C, -k8A, k8D, k8B},
                             {k8D, -k8C, k8B, -k8A}};

struct Mfma8K {
    float e[4], o[4];    // device: this lane's A operands (row lane & 3); unused on the host
};

#if defined(__HIP_DEVICE_COMPILE__)
typedef float dcte_v4f __attribute__((ext_vector_type(4)));
#endif
#if defined(__HIPCC__)
// this lane's A operands, made opaque so they stay in 8 registers for the
// whole kernel (not re-derived or re-loaded from a table per row)
__device__ __forceinline__ Mfma8K mfma8_consts()
{
    Mfma8K k{};
#if defined(__HIP_DEVICE_COMPILE__)
    const int r = __lane_id() & 3;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        k.e[t] = r == 0 ? kMe[0][t] : (r == 1 ? kMe[1][t] : (r == 2 ? kMe[2][t] : kMe[3][t]));
        k.o[t] = r == 0 ? kMo[0][t] : (r == 1 ? kMo[1][t] : (r == 2 ? kMo[2][t] : kMo[3][t]));
        asm volatile("" : "+v"(k.e[t]), "+v"(k.o[t]));
    }
#endif
    return k;
}
#endif

// The eight outputs of texture column x (all texture atoms: order irrelevant).
// MATRIX (device, every lane of the wave active, mk from mfma8_consts): on the
// matrix pipe; otherwise the same fmaf chains on the VALU (host emulation,
// and device kernels whose lanes may be inactive: dcte_pixel.h) -- identical
// bits either way.
template <bool MATRIX>
DCTE_HD void col_mfma8(const float x[8], const Mfma8K& mk, float out[8])
{
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (MATRIX) {
        dcte_v4f ev = {0.f, 0.f, 0.f, 0.f}, od = {0.f, 0.f, 0.f, 0.f};
#if DCTE_MFMA8_SYM
        float sv[4], dv[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            sv[t] = x[t] + x[7 - t];
            dv[t] = x[t] - x[7 - t];
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
            ev = __builtin_amdgcn_mfma_f32_4x4x1f32(mk.e[t], sv[t], ev, 0, 0, 0);
            od = __builtin_amdgcn_mfma_f32_4x4x1f32(mk.o[t], dv[t], od, 0, 0, 0);
        }
#else
#pragma unroll
        for (int t = 0; t < 4; t++) {
            ev = __builtin_amdgcn_mfma_f32_4x4x1f32(mk.e[t], x[t], ev, 0, 0, 0);
            od = __builtin_amdgcn_mfma_f32_4x4x1f32(mk.o[t], x[t], od, 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
            ev = __builtin_amdgcn_mfma_f32_4x4x1f32(mk.e[3 - t], x[4 + t], ev, 0, 0, 0);
            od = __builtin_amdgcn_mfma_f32_4x4x1f32(-mk.o[3 - t], x[4 + t], od, 0, 0, 0);
        }
#endif
#pragma unroll
        for (int r = 0; r < 4; r++) {
            out[r] = ev[r];
            out[4 + r] = od[r];
        }
        return;
    }
#endif
    (void)mk;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        float e = 0.0f, o = 0.0f;
#if DCTE_MFMA8_SYM
#pragma unroll
        for (int t = 0; t < 4; t++) {
            e = fmaf(kMe[r][t], x[t] + x[7 - t], e);
            o = fmaf(kMo[r][t], x[t] - x[7 - t], o);
        }
#else
#pragma unroll
        for (int t = 0; t < 4; t++) {
            e = fmaf(kMe[r][t], x[t], e);
            o = fmaf(kMo[r][t], x[t], o);
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
            e = fmaf(kMe[r][3 - t], x[4 + t], e);
            o = fmaf(-kMo[r][3 - t], x[4 + t], o);
        }
#endif
        out[r] = e;
        out[4 + r] = o;
    }
}

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
    // ring[s][k1]; oldest row in slot O.  k1 = 0 first (m starts at 0)
    // MATRIX: the DCTE_MFMA8 texture columns on the matrix pipe (dcte_map,
    // mk = mfma8_consts()); otherwise their fmaf chains on the VALU, same bits
    template <int O, bool MATRIX = false>
    DCTE_HD_MEMBER void run(const float (&ring)[8][8], int /*lane_p*/, float& mt, float& me,
                            const Mfma8K& mk = Mfma8K{})
    {
        float col[8];
        float e0, e1;
#if DCTE_SC
        // all eight columns in scaled form (dct8_col_sc, dct8_k0_sc), each
        // folded into the running maxima m1 (scale 1), mE, mA, mQ as soon as
        // it is formed; k1 = 1 seeds them and k1 = 0 comes last (fewer live
        // registers than seeding from k1 = 0)
        float v1, ye[2], ya[2], pq, unused;
#if DCTE_MFMA8 > 0
        // the matrix-pipe columns first: their chains run while the VALU
        // columns below are computed, and are folded last
        constexpr int KM = 8 - DCTE_MFMA8;
        float mx[DCTE_MFMA8][8];
#pragma unroll
        for (int k = KM; k < 8; k++) {
            col_at<O>(ring, k, col);
            col_mfma8<MATRIX>(col, mk, mx[k - KM]);
        }
#else
        constexpr int KM = 8;
#endif
        col_at<O>(ring, 1, col);
        dct8_col_sc<true>(col, v1, ye, ya, pq, e1);
        float m1 = fabsf(v1), mQ = pq;
        float mE = fmaxf(fabsf(ye[0]), fabsf(ye[1])), mA = fmaxf(fabsf(ya[0]), fabsf(ya[1]));
#pragma unroll
        for (int k = 2; k < KM; k++) {
            col_at<O>(ring, k, col);
            dct8_col_sc<false>(col, v1, ye, ya, pq, unused);
            m1 = fmaxf(m1, v1);
            mQ = fmaxf(mQ, pq);
            mE = max2in(mE, ye[0], ye[1]);
            mA = max2in(mA, ya[0], ya[1]);
        }
        col_at<O>(ring, 0, col);
        dct8_k0_sc(col, m1, mE, mA, mQ, e0);
#if DCTE_MFMA8 > 0
        // matrix-pipe outputs are plain hat-unit coefficients: scale-1 chain
#pragma unroll
        for (int k = 0; k < DCTE_MFMA8; k++)
#pragma unroll
            for (int r = 0; r < 8; r += 2) m1 = max2in(m1, mx[k][r], mx[k][r + 1]);
#endif
        mt = max2in(max2in(m1, mQ * k8sPQ, mE * k8sE), mA * k8sA, 0.0f);
        me = fmaxf(e1, e0 * k8sPQ);
#else
        col_at<O>(ring, 0, col);
        mt = dct8_k0_max(col, 0.0f, e0);
#if DCTE_PQ2
        // k1 = 1..7 as parts (dct8_col_parts): two columns' magnitudes per
        // fold10, the seven pq in a chain of their own, scaled once
        float va[5], vb[5], pq[7], unused;
        col_at<O>(ring, 1, col);
        dct8_col_parts<true>(col, va, pq[0], e1);
        col_at<O>(ring, 2, col);
        dct8_col_parts<false>(col, vb, pq[1], unused);
        mt = fold10(mt, va, vb);
        col_at<O>(ring, 3, col);
        dct8_col_parts<false>(col, va, pq[2], unused);
        col_at<O>(ring, 4, col);
        dct8_col_parts<false>(col, vb, pq[3], unused);
        mt = fold10(mt, va, vb);
        col_at<O>(ring, 5, col);
        dct8_col_parts<false>(col, va, pq[4], unused);
        col_at<O>(ring, 6, col);
        dct8_col_parts<false>(col, vb, pq[5], unused);
        mt = fold10(mt, va, vb);
        col_at<O>(ring, 7, col);
        dct8_col_parts<false>(col, va, pq[6], unused);
        mt = max2in(max2in(mt, va[0], va[1]), va[2], va[3]);
        mt = fmaxf(mt, fabsf(va[4]));
        float q = fmaxf(fmaxf(pq[0], pq[1]), pq[2]);
        q = fmaxf(fmaxf(q, pq[3]), pq[4]);
        q = fmaxf(fmaxf(q, pq[5]), pq[6]);
        mt = fmaxf(mt, q * k8R);
#else
#pragma unroll
        for (int j = 0; j < 8; j++) col[j] = ring[(O + j) & 7][1];
        mt = dct8_k1_max(col, mt, e1);
#pragma unroll
        for (int k = 2; k < 8; k++) {
#pragma unroll
            for (int j = 0; j < 8; j++) col[j] = ring[(O + j) & 7][k];
            mt = dct8_tex_max(col, mt);
        }
#endif
        me = fmaxf(e0, e1);
#endif
    }

    template <int O>
    DCTE_HD_MEMBER void col_at(const float (&ring)[8][8], int k, float (&col)[8])
    {
#pragma unroll
        for (int j = 0; j < 8; j++) col[j] = ring[(O + j) & 7][k];
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
#if DCTE_SC4
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
#else
template <> struct Cols<4> : ColsSmall<4> {};
#endif
template <> struct Cols<2> : ColsSmall<2> {};

template <>
struct Cols<16> {
    template <int O>
    DCTE_HD_MEMBER void run(const float (&ring)[16][4], int q, float& mt, float& me)
    {
        float col[16];
        mt = 0.0f;
        me = 0.0f;
#if DCTE_SC16
        float mE = 0.0f, mA = 0.0f, mQ = 0.0f, m2 = 0.0f;   // scaled running maxima (dct16_tex_sc)
#endif
        // channel 0: k1 = 4q' ... special roles for k1 = 0 (q = 0) and k1 = 1 (q = 2)
#pragma unroll
        for (int j = 0; j < 16; j++) col[j] = ring[(O + j) & 15][0];
#if DCTE_SC16 && DCTE_ODD16SC
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
                dct16_odd_sc<true>(d, mt, mE, m2, &e_odd);
                me = e_odd * k16s2c;
            } else {
                dct16_odd_sc<false>(d, mt, mE, m2);
                me = e_even;
            }
        } else {
            dct16_tex_sc(col, mt, mE, mA, mQ, m2);
        }
#else
        float X[16];
        if (q == 0) {
            // exact integer row sums: centre on one of its own samples (exact)
            // so no large partial sum forms; X0 is the DC (excluded), X1 = C01
            const float ref = col[7];
#pragma unroll
            for (int j = 0; j < 16; j++) col[j] -= ref;
            dct16(col, X);
            me = fabsf(X[1]);
#pragma unroll
            for (int k = 2; k < 16; k += 2) mt = fmaxf(fmaxf(mt, fabsf(X[k])), fabsf(X[k + 1]));
        } else if (q == 2) {
            dct16(col, X);                 // X0 = C10 (edge)
            me = fabsf(X[0]);
#pragma unroll
            for (int k = 1; k < 15; k += 2) mt = fmaxf(fmaxf(mt, fabsf(X[k])), fabsf(X[k + 1]));
            mt = fmaxf(mt, fabsf(X[15]));
        } else {
#if DCTE_SC16
            dct16_tex_sc(col, mt, mE, mA, mQ, m2);
#else
            mt = dct16_tex_max(col, mt);
#endif
        }
#endif
#pragma unroll
        for (int c = 1; c < 4; c++) {
#pragma unroll
            for (int j = 0; j < 16; j++) col[j] = ring[(O + j) & 15][c];
#if DCTE_SC16
            dct16_tex_sc(col, mt, mE, mA, mQ, m2);
#else
            mt = dct16_tex_max(col, mt);
#endif
        }
#if DCTE_SC16
        mt = max2in(max2in(mt, mQ * k8sPQ, mE * k8sE), mA * k8sA, m2 * k16s2c);
#endif
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
