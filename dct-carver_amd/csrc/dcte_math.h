// dcte_math.h -- fp32 transform arithmetic of the energy-map kernels.
//
// Shared, unchanged, by the gfx950 kernels (dcte_kernels.hip) and by the
// host-side emulation used in tests (tests/emu/), so that CPU tests can check
// the exact fp32 operation sequence the GPU runs.  Both sides compile with
// -ffp-contract=off and every fused multiply-add is an explicit fmaf(), so
// host and device results are bit-identical.
//
// Units ("hat" scaling).  A 1-D transform of length N returns
//     X[0] = sum_j x_j                         (unscaled DC)
//     X[k] = g * sum_j x_j cos(pi (2j+1) k / 2N),   k >= 1
// with g = sqrt(2) for the orthonormal family (N = 8, 16: ddct8x8s /
// ddct16x16s, src/fft2d/shrtdct.c:18-28,189-193) and g = 1 for the
// unnormalised family (N = 2, 4: ddct2d, src/fft2d/fftsg2d.c:204-209).
// Then every 2-D coefficient is C[k1][k2] * S with one global S (N for the
// orthonormal family, 1 for the unnormalised one), so comparisons between
// coefficients -- all that the weighted max needs (src/dct.c:96-110) -- are
// unaffected, and the kernel folds 1/S and the luma scale into the weights.
//
// Exactness.  Inputs are integer-valued luma samples biased into
// [-637500, 637500] (dcte_luma.h), so every sum/difference of the first
// butterfly stages is an exact fp32 integer (< 2^24).  Rounding therefore only
// enters through the rotations, whose operands scale with the window's local
// contrast, never with its mean brightness.  The DC column (k1 = 0) of the
// second pass is kept free of large partial sums (see col_dc_*).
#pragma once

#include <math.h>

#if defined(__HIPCC__)
#define DCTE_HD __host__ __device__ __forceinline__
#else
#define DCTE_HD static inline
#endif

namespace dcte {

// running max folding two more magnitudes in: one v_max3_f32 (abs modifiers)
DCTE_HD float max2in(float m, float a, float b) { return fmaxf(fmaxf(m, fabsf(a)), fabsf(b)); }

// ---------------------------------------------------------------- N = 8
// g * cos(pi (2j+1) k / 16) magnitudes (g = sqrt 2)
constexpr float k8A = 1.3870398453221475f;   // cos(1 pi/16)
constexpr float k8B = 1.1758756024193588f;   // cos(3 pi/16)
constexpr float k8C = 0.7856949583871023f;   // cos(5 pi/16)
constexpr float k8D = 0.2758993792829431f;   // cos(7 pi/16)
constexpr float k8E = 1.3065629648763766f;   // cos(2 pi/16)
constexpr float k8F = 0.5411961001461971f;   // cos(6 pi/16)

// odd outputs X1, X3, X5, X7 from d_j = x_j - x_{7-j}
DCTE_HD void dct8_odd(float d0, float d1, float d2, float d3,
                      float& X1, float& X3, float& X5, float& X7)
{
    X1 = fmaf(d3, k8D, fmaf(d2, k8C, fmaf(d1, k8B, d0 * k8A)));
    X3 = fmaf(d3, -k8C, fmaf(d2, -k8A, fmaf(d1, -k8D, d0 * k8B)));
    X5 = fmaf(d3, k8B, fmaf(d2, k8D, fmaf(d1, -k8A, d0 * k8C)));
    X7 = fmaf(d3, -k8A, fmaf(d2, k8B, fmaf(d1, -k8C, d0 * k8D)));
}

// scaled-form constants (see dct8_col_sc)
constexpr float k8rEF = 0.41421356237309503f;  // F / E = tan(pi/8)
constexpr float k8rCB = 0.66817863791929891f;  // C / B = tan(3 pi/16)
constexpr float k8rDA = 0.19891236737965800f;  // D / A = tan(pi/16)
constexpr float k8rBA = 0.84775906502257351f;  // B / A = cos(3 pi/16) / cos(pi/16)
constexpr float k8sA = 1.3870398453221475f;    // A (scale of the ya chain)
constexpr float k8sE = 1.3065629648763766f;    // E (scale of the ye chain)
constexpr float k8sPQ = 0.98078528040323043f;  // A / sqrt2 = cos(pi/16) (scale of the pq chain)

// full 8-point transform (row pass of N = 8; inside the N = 16 transforms).
// The odd half goes through the scaled form of dct8_col_sc and is then
// materialised: 14 VALU ops instead of the 16 of dct8_odd.
DCTE_HD void dct8(const float x[8], float X[8])
{
    float s0 = x[0] + x[7], d0 = x[0] - x[7];
    float s1 = x[1] + x[6], d1 = x[1] - x[6];
    float s2 = x[2] + x[5], d2 = x[2] - x[5];
    float s3 = x[3] + x[4], d3 = x[3] - x[4];
    float a = s0 + s3, b = s1 + s2, c = s0 - s3, e = s1 - s2;
    X[0] = a + b;
    X[4] = a - b;
    X[2] = fmaf(c, k8E, e * k8F);
    X[6] = fmaf(c, k8F, -(e * k8E));
    float u0 = fmaf(d0, k8rCB, d3);
    float u3 = fmaf(d3, k8rCB, -d0);
    float u1 = fmaf(d1, k8rDA, d2);
    float u2 = fmaf(d2, k8rDA, -d1);
    float pp = fmaf(u3, -k8rBA, u1), qq = fmaf(u0, k8rBA, -u2);
    X[1] = (pp + qq) * k8sPQ;
    X[3] = fmaf(u3, k8rBA, u1) * -k8sA;
    X[5] = fmaf(u0, k8rBA, u2) * k8sA;
    X[7] = (pp - qq) * k8sPQ;
}

// A k1 >= 1 column in SCALED form: every output magnitude is a known constant
// times a cheaper value, and values sharing a constant go to one running max
// that is multiplied by it once per pixel (max_i fl(K y_i) == fl(K max_i y_i):
// rounding is monotone).  Rotations by a fixed angle then cost one FMA per
// output instead of a multiply and an FMA:
//   X2 = E (c + r e), X6 = E (r c - e)                  r = F/E = tan(pi/8)
//   t0 = B u0, t3 = B u3 with u0 = (C/B) d0 + d3, u3 = (C/B) d3 - d0
//   t1 = A u1, t2 = A u2 with u1 = (D/A) d1 + d2, u2 = (D/A) d2 - d1
//   X3 = -A (u1 + (B/A) u3), X5 = A (u2 + (B/A) u0)
//   max(|X1|, |X7|) = (|P| + |Q|) / sqrt2 = (A / sqrt2) (|p| + |q|),
//     p = u1 - (B/A) u3, q = (B/A) u0 - u2
// 24 VALU ops per column instead of 30.  Outputs:
//   v1 -> scale 1 (|a| + |b| for X0/X4, or a - b = X4 alone when X0 is the
//         edge atom C10, EDGE);  ye[2] -> scale E;  ya[2] -> scale A;
//   pq -> scale A / sqrt2.
template <bool EDGE>
DCTE_HD void dct8_col_sc(const float x[8], float& v1, float ye[2], float ya[2], float& pq,
                         float& edge)
{
    float s0 = x[0] + x[7], d0 = x[0] - x[7];
    float s1 = x[1] + x[6], d1 = x[1] - x[6];
    float s2 = x[2] + x[5], d2 = x[2] - x[5];
    float s3 = x[3] + x[4], d3 = x[3] - x[4];
    float a = s0 + s3, b = s1 + s2, c = s0 - s3, e = s1 - s2;
    if constexpr (EDGE) {
        edge = fabsf(a + b);
        v1 = a - b;
    } else {
        v1 = fabsf(a) + fabsf(b);
    }
    ye[0] = fmaf(e, k8rEF, c);
    ye[1] = fmaf(c, k8rEF, -e);
    float u0 = fmaf(d0, k8rCB, d3);
    float u3 = fmaf(d3, k8rCB, -d0);
    float u1 = fmaf(d1, k8rDA, d2);
    float u2 = fmaf(d2, k8rDA, -d1);
    ya[0] = fmaf(u3, k8rBA, u1);
    ya[1] = fmaf(u0, k8rBA, u2);
    pq = fabsf(fmaf(u3, -k8rBA, u1)) + fabsf(fmaf(u0, k8rBA, -u2));
}

// k1 = 0 column in scaled form (inputs: exact integer row sums), folded into
// the four running maxima.  The DC is never formed; X4 = (s0 - s1) + (s3 - s2)
// (exact integer partial sums).  X1 (the edge atom C01) = (A / sqrt2)(p + q) and
// X7 = (A / sqrt2)(p - q) with p, q as in dct8_col_sc; e0 = |p + q| carries
// the scale A / sqrt2.  25 VALU ops instead of 33.
DCTE_HD void dct8_k0_sc(const float x[8], float& m1, float& mE, float& mA, float& mQ, float& e0)
{
    float s0 = x[0] + x[7], d0 = x[0] - x[7];
    float s1 = x[1] + x[6], d1 = x[1] - x[6];
    float s2 = x[2] + x[5], d2 = x[2] - x[5];
    float s3 = x[3] + x[4], d3 = x[3] - x[4];
    float c = s0 - s3, e = s1 - s2;
    m1 = fmaxf(m1, fabsf((s0 - s1) + (s3 - s2)));
    mE = max2in(mE, fmaf(e, k8rEF, c), fmaf(c, k8rEF, -e));
    float u0 = fmaf(d0, k8rCB, d3);
    float u3 = fmaf(d3, k8rCB, -d0);
    float u1 = fmaf(d1, k8rDA, d2);
    float u2 = fmaf(d2, k8rDA, -d1);
    mA = max2in(mA, fmaf(u3, k8rBA, u1), fmaf(u0, k8rBA, u2));
    float pp = fmaf(u3, -k8rBA, u1), qq = fmaf(u0, k8rBA, -u2);
    e0 = fabsf(pp + qq);
    mQ = fmaxf(mQ, fabsf(pp - qq));
}

// ---------------------------------------------------------------- N = 4, 2
// unnormalised family (g = 1): cos(pi/4), cos(pi/8), cos(3 pi/8)
constexpr float k4H = 0.7071067811865476f;
constexpr float k4A = 0.9238795325112867f;
constexpr float k4B = 0.38268343236508984f;
constexpr float k4rBA = 0.41421356237309503f;  // k4B / k4A = tan(pi/8)

DCTE_HD void dct4(const float x[4], float X[4])
{
    float s0 = x[0] + x[3], d0 = x[0] - x[3];
    float s1 = x[1] + x[2], d1 = x[1] - x[2];
    X[0] = s0 + s1;
    X[2] = (s0 - s1) * k4H;
    X[1] = fmaf(d1, k4B, d0 * k4A);
    X[3] = fmaf(d1, -k4A, d0 * k4B);
}

DCTE_HD void dct2(const float x[2], float X[2])
{
    X[0] = x[0] + x[1];
    X[1] = (x[0] - x[1]) * k4H;
}

// ---------------------------------------------------------------- N = 16
// odd-part matrix g * cos(pi (2j+1) k / 32), k odd, j = 0..7 (g = sqrt 2)
constexpr float k16a0 = 1.4074037375263826f;  // cos( 1 pi/32)
constexpr float k16a1 = 1.3533180011743526f;  // cos( 3 pi/32)
constexpr float k16a2 = 1.2472250129866713f;  // cos( 5 pi/32)
constexpr float k16a3 = 1.0932018670017576f;  // cos( 7 pi/32)
constexpr float k16a4 = 0.8971675863426364f;  // cos( 9 pi/32)
constexpr float k16a5 = 0.6666556584777468f;  // cos(11 pi/32)
constexpr float k16a6 = 0.41052452752235735f; // cos(13 pi/32)
constexpr float k16a7 = 0.1386171691990917f;  // cos(15 pi/32)

// Four odd outputs X[k0], X[k0+4], X[k0+8], X[k0+12] (k0 = 1 or 3) of the
// 16-point transform from d_j = x_j - x_{15-j}: the rows of dct16_odd.
DCTE_HD void dct16_odd_rows(const float d[8], int k0, float out[4])
{
    float X[16];
    const float A0 = k16a0, A1 = k16a1, A2 = k16a2, A3 = k16a3;
    const float A4 = k16a4, A5 = k16a5, A6 = k16a6, A7 = k16a7;
#define DCTE_ROW(o, c0, c1, c2, c3, c4, c5, c6, c7)                                   \
    X[o] = fmaf(d[7], c7, fmaf(d[6], c6, fmaf(d[5], c5, fmaf(d[4], c4,                \
           fmaf(d[3], c3, fmaf(d[2], c2, fmaf(d[1], c1, d[0] * c0)))))));
    if (k0 == 1) {
        DCTE_ROW(1,  A0,  A1,  A2,  A3,  A4,  A5,  A6,  A7)
        DCTE_ROW(5,  A2,  A7, -A3, -A1, -A6,  A4,  A0,  A5)
        DCTE_ROW(9,  A4, -A2, -A6,  A0, -A7, -A1,  A5,  A3)
        DCTE_ROW(13, A6, -A3,  A0, -A2,  A5,  A7, -A4,  A1)
        out[0] = X[1]; out[1] = X[5]; out[2] = X[9]; out[3] = X[13];
    } else {
        DCTE_ROW(3,  A1,  A4,  A7, -A5, -A2, -A0, -A3, -A6)
        DCTE_ROW(7,  A3, -A5, -A1,  A7,  A0,  A6, -A2, -A4)
        DCTE_ROW(11, A5, -A0,  A4,  A6, -A1,  A3,  A7, -A2)
        DCTE_ROW(15, A7, -A6,  A5, -A4,  A3, -A2,  A1, -A0)
        out[0] = X[3]; out[1] = X[7]; out[2] = X[11]; out[3] = X[15];
    }
#undef DCTE_ROW
}

// Odd half of the 16-point transform for the max only: the DCT-IV of size 8
// of d (X[2m+1] = sqrt2 * Y_m) through a 4-point complex DFT,
//   v_n = d_{2n} + i d_{7-2n},  u_n = v_n exp(-i pi (4n+1)/32)      (pre-twiddle)
//   U_k = sum_n u_n exp(-2 pi i n k / 4)                            (DFT-4)
//   Y_{2k} = Re W_k, Y_{7-2k} = -Im W_k,  W_k = U_k exp(-i pi k / 8)  (post-twiddle)
// all in scaled form (r05): each pre-twiddle is one FMA per output with its
// larger factor sigma_n = max(cos, sin) pulled out (ratio t_n <= 1), and the
// DFT's additions absorb the ratios of those factors (sigma_2 / sigma_0,
// sigma_3 / sigma_1, sigma_1 / sigma_0) as one FMA each, so every U_k comes
// out at the common scale sigma_0 = cos(pi/32).  The post-twiddle as before:
// k = 0 free (chain m2, scale sqrt2 sigma_0); k = 1 and 3 one FMA per output
// with tan(pi/8) (chain mE, scale E sigma_0); k = 2 max(|Ur + Ui|, |Ur - Ui|)
// = |Ur| + |Ui| (chain m, scale sigma_0).  The chains are the odd half's own
// (their scales differ from the even half's by sigma_0): 33 VALU ops, r04's
// form (two per pre-twiddle output) took 41.
constexpr float k16t0 = 0.09849140335716425f;   // tan( 1 pi/32)         (sigma_0 = cos)
constexpr float k16t1 = 0.5345111359507916f;    // tan( 5 pi/32)         (sigma_1 = cos)
constexpr float k16t2 = 0.8206787908286602f;    // cot( 9 pi/32)         (sigma_2 = sin)
constexpr float k16t3 = 0.30334668360734235f;   // cot(13 pi/32)         (sigma_3 = sin)
constexpr float k16r02 = 0.7767507203889779f;   // sigma_2 / sigma_0
constexpr float k16r13 = 1.085063230037077f;    // sigma_3 / sigma_1
constexpr float k16r01 = 0.8861885042161126f;   // sigma_1 / sigma_0
constexpr float k16s2c = 1.4142135623730951f;   // sqrt2
constexpr float k16oM = 0.9951847266721969f;    // sigma_0: scale of the odd m chain
constexpr float k16oE = 1.300271507080512f;     // E sigma_0: the odd mE chain
constexpr float k16o2 = 1.4074037375263826f;    // sqrt2 sigma_0: the m2 chain (and the C01 edge)

template <bool EDGE = false>
DCTE_HD void dct16_odd_sc(const float d[8], float& m, float& mE, float& m2, float* edge = nullptr)
{
    // u_n / sigma_n: (a + t b) + i (b - t a) for sigma = cos, (t a + b) + i (t b - a) for sigma = sin
    const float R0 = fmaf(d[7], k16t0, d[0]), I0 = fmaf(d[0], -k16t0, d[7]);
    const float R1 = fmaf(d[5], k16t1, d[2]), I1 = fmaf(d[2], -k16t1, d[5]);
    const float R2 = fmaf(d[4], k16t2, d[3]), I2 = fmaf(d[3], k16t2, -d[4]);
    const float R3 = fmaf(d[6], k16t3, d[1]), I3 = fmaf(d[1], k16t3, -d[6]);
    // DFT-4 at scale sigma_0 (s = u0 + u2, dd = u0 - u2 at sigma_0; t = u1 + u3, e = u1 - u3 at sigma_1)
    const float sr = fmaf(R2, k16r02, R0), si = fmaf(I2, k16r02, I0);
    const float dr = fmaf(R2, -k16r02, R0), di = fmaf(I2, -k16r02, I0);
    const float tr = fmaf(R3, k16r13, R1), ti = fmaf(I3, k16r13, I1);
    const float er = fmaf(R3, -k16r13, R1), ei = fmaf(I3, -k16r13, I1);
    // U0 = (s + t), U2 = (s - t), U1 = (dr + ei) + i (di - er), U3 = (dr - ei) + i (di + er)
    const float u0r = fmaf(tr, k16r01, sr), u0i = fmaf(ti, k16r01, si);
    if constexpr (EDGE) {                       // X1 = sqrt2 Re U0 is the edge atom C01
        *edge = fabsf(u0r);
        m2 = fmaxf(m2, fabsf(u0i));
    } else {
        m2 = max2in(m2, u0r, u0i);
    }
    m = fmaxf(m, fabsf(fmaf(tr, -k16r01, sr)) + fabsf(fmaf(ti, -k16r01, si)));
    const float u1r = fmaf(ei, k16r01, dr), u1i = fmaf(er, -k16r01, di);
    const float u3r = fmaf(ei, -k16r01, dr), u3i = fmaf(er, k16r01, di);
    mE = max2in(mE, fmaf(u1i, k8rEF, u1r), fmaf(u1r, k8rEF, -u1i));
    mE = max2in(mE, fmaf(u3r, k8rEF, u3i), fmaf(u3i, -k8rEF, u3r));
}

// An all-texture column of the N = 16 second pass: the even half (the 8-point transform of s, same hat
// units) in the scaled form of dct8_col_sc and the odd half through
// dct16_odd_sc: magnitudes go to the running maxima m (scale 1), mE, mA, mQ
// (even half) and mO, mEO, m2 (odd half, scales k16oM, k16oE, k16o2).
DCTE_HD void dct16_tex_sc(const float x[16], float& m, float& mE, float& mA, float& mQ,
                          float& mO, float& mEO, float& m2)
{
    float s[8], d[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        s[j] = x[j] + x[15 - j];
        d[j] = x[j] - x[15 - j];
    }
    float v1, ye[2], ya[2], pq, unused;
    dct8_col_sc<false>(s, v1, ye, ya, pq, unused);
    mE = max2in(mE, ye[0], ye[1]);
    mA = max2in(mA, ya[0], ya[1]);
    mQ = fmaxf(mQ, pq);
    m = fmaxf(m, v1);
    dct16_odd_sc<false>(d, mO, mEO, m2);
}

}  // namespace dcte
