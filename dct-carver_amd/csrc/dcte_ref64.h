// dcte_ref64.h -- fp64 "tie refinement" arithmetic (device + host).
//
// The fast fp32 path (dcte_math.h) agrees with the reference to ~1e-6
// relative, but the edge/texture class of a pixel is a comparison
// (src/dct.c:100-109: last maximum wins, so "edge" iff max|C01|,|C10| is
// strictly larger than every texture atom).  Pixels whose two candidates are
// within the fp32 error band are recomputed here in fp64, in the reference's
// own operation order, so the class -- and the value -- equal the reference's:
//   - luma     : liblqr LQR_ER_LUMA in double [liblqr, unverified]
//   - gather   : src/render.c:122-157 (replicate clamp, window[dx][dy])
//   - N = 8    : ddct8x8s forward,   src/fft2d/shrtdct.c:61-117
//   - N = 16   : ddct16x16s forward, src/fft2d/shrtdct.c:238-386
//   - N = 2, 4 : ddct2d -> ddct(-1)  src/fft2d/fftsg2d.c:566-627,
//                src/fft2d/fftsg.c:349-402 (cftx020, dctsub), twiddles from
//                makect (fftsg.c:724-740) evaluated on the host with libm and
//                passed in, exactly as the reference evaluates them
//   - max      : src/dct.c:96-110
// The TU is compiled with -ffp-contract=off so no multiply-add is fused.
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define DCTE_HD64 __host__ __device__ __forceinline__
#else
#define DCTE_HD64 static inline
#endif

namespace dcte {
namespace r64 {

// binary64 values of Ooura's literals (shrtdct.c:45-52, 211-227)
struct K8 {
    static constexpr double c1 = 0x1.f6297cff75cb0p-2, s1 = 0x1.8f8b83c69a60bp-4;
    static constexpr double c2 = 0x1.d906bcf328d46p-2, s2 = 0x1.87de2a6aea963p-3;
    static constexpr double c3 = 0x1.a9b66290ea1a3p-2, s3 = 0x1.1c73b39ae68c8p-2;
    static constexpr double c4 = 0x1.6a09e667f3bcdp-2, w4 = 0x1.6a09e667f3bcdp-1;
};
struct K16 {
    static constexpr double c1 = 0x1.684b9c80f1a8bp-2, s1 = 0x1.1be35182fe5aap-5;
    static constexpr double c2 = 0x1.63150b15e8536p-2, s2 = 0x1.1a855dec071b5p-4;
    static constexpr double c3 = 0x1.5a730c6c21c67p-2, s3 = 0x1.a4608aafa8527p-4;
    static constexpr double c4 = 0x1.4e7ae9144f0fcp-2, s4 = 0x1.1517a7bdb3895p-3;
    static constexpr double c5 = 0x1.3f4a237187eafp-2, s5 = 0x1.5553e3f5b5e58p-3;
    static constexpr double c6 = 0x1.2d062ef88e319p-2, s6 = 0x1.92469c0dcf32dp-3;
    static constexpr double c7 = 0x1.17dc13dab2dd6p-2, s7 = 0x1.cb598cc4beea0p-3;
    static constexpr double c8 = 0x1.0000000000000p-2;
    static constexpr double w4c = 0x1.d906bcf328d46p-1, w4s = 0x1.87de2a6aea963p-2;
    static constexpr double w8 = 0x1.6a09e667f3bcdp-1;
};

// 8-point forward step on v[0], v[st], ..., one iteration of shrtdct.c:62-89
DCTE_HD64 void step8(double* v, int st)
{
    double t0 = v[0] + v[7 * st], u0 = v[0] - v[7 * st];
    double t1 = v[2 * st] + v[5 * st], u1 = v[2 * st] - v[5 * st];
    double t2 = v[4 * st] + v[3 * st], u2 = v[4 * st] - v[3 * st];
    double t3 = v[6 * st] + v[st], u3 = v[6 * st] - v[st];
    double p = t0 + t2, q = t1 + t3;
    v[0] = K8::c4 * (p + q);
    v[4 * st] = K8::c4 * (p - q);
    p = t0 - t2;
    q = t1 - t3;
    v[2 * st] = K8::c2 * p - K8::s2 * q;
    v[6 * st] = K8::c2 * q + K8::s2 * p;
    p = K8::w4 * (u1 - u3);
    u1 = K8::w4 * (u1 + u3);
    u3 = u1 - u2;
    u1 += u2;
    u2 = u0 - p;
    u0 += p;
    v[st] = K8::c1 * u0 - K8::s1 * u1;
    v[7 * st] = K8::c1 * u1 + K8::s1 * u0;
    v[3 * st] = K8::c3 * u2 - K8::s3 * u3;
    v[5 * st] = K8::c3 * u3 + K8::s3 * u2;
}

// Pass 2 of ddct8x8s on coefficient row k1 (step8's operations in its order,
// no C00; the exact maps and the N = 8 refinement) (shrtdct.c:90-117: a[k1][0..7] ->
// C_k1,0..7), folded into the scan's maxima.  v[j] = a[k1][j] after pass 1.
//   ROLE 0 (k1 = 0): a01 = |C01|, m0 = max |C0,2..7| (C00 is never scanned)
//   ROLE 1 (k1 = 1): a10 = |C10| (into a01's slot), mp = max(mp, |C1,1..7|)
//   ROLE 2 (k1 >= 2): mp = max(mp, |C_k1,0..7|)
template <int ROLE>
DCTE_HD64 void col8(double v0, double v1, double v2, double v3, double v4, double v5,
                                     double v6, double v7, double& a, double& m)
{
    const double x0r = v0 + v7, x1r = v0 - v7;
    const double x0i = v2 + v5, x1i = v2 - v5;
    const double x2r = v4 + v3, x3r = v4 - v3;
    const double x2i = v6 + v1, x3i = v6 - v1;
    double xr = x0r + x2r, xi = x0i + x2i;
    double acc;
    if constexpr (ROLE == 0) {
        acc = fabs(K8::c4 * (xr - xi));                       // C04
    } else if constexpr (ROLE == 1) {
        a = fabs(K8::c4 * (xr + xi));                          // C10
        acc = fmax(m, fabs(K8::c4 * (xr - xi)));               // C14
    } else {
        acc = fmax(m, K8::c4 * (fabs(xr) + fabs(xi)));         // max(|C_k1,0|, |C_k1,4|)
    }
    xr = x0r - x2r;
    xi = x0i - x2i;
    acc = fmax(acc, fabs(K8::c2 * xr - K8::s2 * xi));          // C_k1,2
    acc = fmax(acc, fabs(K8::c2 * xi + K8::s2 * xr));          // C_k1,6
    xr = K8::w4 * (x1i - x3i);
    const double y1i = K8::w4 * (x1i + x3i);
    const double y3i = y1i - x3r;
    const double z1i = y1i + x3r;
    const double y3r = x1r - xr;
    const double y1r = x1r + xr;
    const double c1 = K8::c1 * y1r - K8::s1 * z1i;             // C_k1,1
    if constexpr (ROLE == 0) {
        a = fabs(c1);
    } else {
        acc = fmax(acc, fabs(c1));
    }
    acc = fmax(acc, fabs(K8::c1 * z1i + K8::s1 * y1r));        // C_k1,7
    acc = fmax(acc, fabs(K8::c3 * y3r - K8::s3 * y3i));        // C_k1,3
    acc = fmax(acc, fabs(K8::c3 * y3i + K8::s3 * y3r));        // C_k1,5
    m = acc;
}

// 16-point forward step, one iteration of shrtdct.c:239-313
DCTE_HD64 void step16(double* v, int st)
{
    double r0, i0, r1, i1, r2, i2, r3, i3, r4, i4, r5, i5, r6, i6, r7, i7, p, q;
    r4 = v[0] - v[15 * st];       p = v[0] + v[15 * st];
    i4 = v[8 * st] - v[7 * st];   q = v[8 * st] + v[7 * st];
    r0 = p + q;  i0 = p - q;
    r5 = v[2 * st] - v[13 * st];  p = v[2 * st] + v[13 * st];
    i5 = v[10 * st] - v[5 * st];  q = v[10 * st] + v[5 * st];
    r1 = p + q;  i1 = p - q;
    r6 = v[4 * st] - v[11 * st];  p = v[4 * st] + v[11 * st];
    i6 = v[12 * st] - v[3 * st];  q = v[12 * st] + v[3 * st];
    r2 = p + q;  i2 = p - q;
    r7 = v[6 * st] - v[9 * st];   p = v[6 * st] + v[9 * st];
    i7 = v[14 * st] - v[st];      q = v[14 * st] + v[st];
    r3 = p + q;  i3 = p - q;
    p = r0 + r2;  q = r1 + r3;
    v[0] = K16::c8 * (p + q);
    v[8 * st] = K16::c8 * (p - q);
    p = r0 - r2;  q = r1 - r3;
    v[4 * st] = K16::c4 * p - K16::s4 * q;
    v[12 * st] = K16::c4 * q + K16::s4 * p;
    r0 = K16::w8 * (i1 - i3);
    r2 = K16::w8 * (i1 + i3);
    p = i0 + r0;  q = r2 + i2;
    v[2 * st] = K16::c2 * p - K16::s2 * q;
    v[14 * st] = K16::c2 * q + K16::s2 * p;
    p = i0 - r0;  q = r2 - i2;
    v[6 * st] = K16::c6 * p - K16::s6 * q;
    v[10 * st] = K16::c6 * q + K16::s6 * p;
    p = K16::w8 * (r6 - i6);
    q = K16::w8 * (i6 + r6);
    r6 = r4 - p;  i6 = i4 - q;
    r4 += p;      i4 += q;
    p = K16::w4s * r7 - K16::w4c * i7;
    q = K16::w4s * i7 + K16::w4c * r7;
    r7 = K16::w4c * r5 - K16::w4s * i5;
    i7 = K16::w4c * i5 + K16::w4s * r5;
    r5 = r7 + p;  i5 = i7 + q;
    r7 -= p;      i7 -= q;
    p = r4 + r5;  q = i5 + i4;
    v[st] = K16::c1 * p - K16::s1 * q;
    v[15 * st] = K16::c1 * q + K16::s1 * p;
    p = r4 - r5;  q = i5 - i4;
    v[7 * st] = K16::c7 * p - K16::s7 * q;
    v[9 * st] = K16::c7 * q + K16::s7 * p;
    p = r6 - i7;  q = r7 + i6;
    v[5 * st] = K16::c5 * p - K16::s5 * q;
    v[11 * st] = K16::c5 * q + K16::s5 * p;
    p = r6 + i7;  q = r7 - i6;
    v[3 * st] = K16::c3 * p - K16::s3 * q;
    v[13 * st] = K16::c3 * q + K16::s3 * p;
}

// ddct(n, -1) for n = 2, 4 on a strided vector; ct = makect(n) twiddles
DCTE_HD64 void step_small(int n, double* v, int st, const double* ct)
{
    if (n == 2) {
        double t = v[st];
        v[st] = v[0] - t;
        v[0] += t;
        v[st] *= ct[0];
        return;
    }
    double a0 = v[0], a1 = v[st], a2 = v[2 * st], a3 = v[3 * st];
    double t = a3;
    a3 = a2 - a1;
    a2 += a1;
    a1 = a0 - t;
    a0 += t;
    double x0r = a0 - a2, x0i = a1 - a3;  // cftx020
    a0 += a2;
    a1 += a3;
    a2 = x0r;
    a3 = x0i;
    double wkr = ct[1] - ct[3], wki = ct[1] + ct[3];  // dctsub
    double xr = wki * a1 - wkr * a3;
    a1 = wkr * a1 + wki * a3;
    a3 = xr;
    a2 *= ct[0];
    v[0] = a0; v[st] = a1; v[2 * st] = a2; v[3 * st] = a3;
}

// in-place 2-D transform of d[i*n + j] (i = dx), dctNxN order
DCTE_HD64 void transform(int n, double* d, const double* ct)
{
    if (n == 8) {
        for (int i = 0; i < 8; i++) step8(d + i, 8);
        for (int i = 0; i < 8; i++) step8(d + 8 * i, 1);
    } else if (n == 16) {
        for (int i = 0; i < 16; i++) step16(d + i, 16);
        for (int i = 0; i < 16; i++) step16(d + 16 * i, 1);
    } else {
        for (int i = 0; i < n; i++) step_small(n, d + n * i, 1, ct);
        for (int i = 0; i < n; i++) step_small(n, d + i, n, ct);
    }
}

DCTE_HD64 float weighted_max(int n, const double* d, float edges, float textures)
{
    int b1 = 0, b2 = 0;
    double m = 0;
    for (int k1 = 0; k1 < n; k1++)
        for (int k2 = 0; k2 < n; k2++) {
            double v = d[k1 * n + k2];
            v = v < 0 ? -v : v;
            if (m <= v && (k1 || k2)) {
                m = v;
                b1 = k1;
                b2 = k2;
            }
        }
    bool edge = (b1 == 0 && b2 == 1) || (b1 == 1 && b2 == 0);
    return edge ? (float)(m * (double)edges) : (float)(m * (double)textures);
}

DCTE_HD64 double luma(const uint8_t* p, int bpp)
{
    if (bpp == 1) return (double)p[0] / 255;
    double r = (double)p[0] / 255, g = (double)p[1] / 255, b = (double)p[2] / 255;
    return 0.2126 * r + 0.7152 * g + 0.0722 * b;
}

}  // namespace r64
}  // namespace dcte
