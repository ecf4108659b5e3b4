// tau_bound.cpp -- a DERIVED bound on the fp32 error the refinement margin
// tau must cover (TEST INFRASTRUCTURE, built into libdcte_emu.so).
//
// The fast map decides edge vs texture by m_e > m_t on fp32 maxima and sends
// a pixel to the fp64 refinement when lo > (1 - tau) hi (dcte_kernels.hip,
// emit).  A pixel can only leave with the wrong class if the errors of the
// two maxima (against the reference's values) together exceed the margin, so
// tau is safe once  tau - 2u >= (delta_e + delta_t)(1 + delta)  (u = 2^-24),
// delta_x bounding |m_x(fp32) - m_x(reference)| / M for every window, M =
// the window's largest non-DC coefficient.
//
// delta_e, delta_t are derived here, not searched: the kernels' OWN pass code
// (dcte_passes.h / dcte_math.h) is compiled with `float` replaced by a
// tracking type and run on a symbolic N x N window.  Every intermediate
// carries its exact linear form a over the window samples (with the fp32
// constants the code uses, as reals).  Integer intermediates (sums and
// differences of the biased integer luma, dcte_luma.h) are exact while their
// magnitude bound stays below 2^24; every other operation is a rounding
// event k with error d_k v_k, |d_k| <= u, and must act on a form without DC
// component (else its error would scale with the window's brightness; the
// derivation fails -- it does not).  Such a v_k = a_k.x is bounded by the
// window's coefficients: a_k = sum_c alpha_c b_c over the orthogonal hat-unit
// basis b_c (dcte_math.h), so |v_k| <= |alpha|_1 M.  Each intermediate also
// carries the gains g_k of every event on its own error (first order), so an
// output's error is sum_k d_k g_k v_k, bounded two ways and the smaller taken:
//   l1:  u sum_k |g_k| |alpha_k|_1 M;
//   CS:  u sqrt(sum_k |g_k|) sqrt(lambda_max(sum_k |g_k| a_k a_k^T)) ||x_AC||,
//        ||x_AC|| <= c_N M (Parseval), lambda_max certified by a Cholesky
//        factorisation of (lambda I - Q) -- events of different window rows
//        lie along near-orthogonal directions, and Cauchy-Schwarz does not
//        add them up in one direction the way the l1 bound does;
// plus the second-order terms (u times the operands' own error bounds).
// Magnitudes (fabs, max, |a| + |b| = max(|a + b|, |a - b|), a max times its
// scale) carry the set of linear forms they are the maximum of; at the end
// that set must be exactly the reference's coefficients -- m_e: C01 and C10;
// m_t: every other non-DC coefficient -- up to the fp32 constants, whose
// deviation is added (in units of M).
//
// The reference side (tau_ref_error): its fp64 transform in its own operation
// order (dcte_ref64.h) tracked the same way on unbiased samples |x| <= xmax,
// where every operation rounds (unit 2^-53) and errors scale with the
// brightness: relative to the smallest M of a non-flat integer window this
// adds rho_64; liblqr's luma (0.2126 * (R / 255) + ... in double) is off the
// integer luma by <= 5 * 2^-53 per sample, which adds rho_luma.  The test
// (tests/test_tau_bound.py) combines the terms.
//
// Reference arithmetic: src/fft2d/shrtdct.c:61-117, 238-386,
// src/fft2d/fftsg2d.c:566-627; decision src/dct.c:100-109.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <utility>
#include <vector>

namespace tb {

constexpr int kMaxK = 256;          // window samples (N = 16)
constexpr double kU = 5.9604644775390625e-08;   // 2^-24
static int g_K = 64;                // samples of the window being analysed
static double g_xmax = 637500;      // max |sample|
static int g_fail = 0;              // derivation failures (see the header)
// "abs" mode: the reference's fp64 transform on unbiased samples (every op
// rounds; |value| <= ||a||_1 xmax; no contrast argument), unit 2^-53
static bool g_abs = false;
static double g_u = kU;

struct Form {
    double a[kMaxK];
};
using Gains = std::vector<std::pair<int, double>>;   // (event, gain), sorted by event
struct Event {
    int form;      // the rounded value's exact form
    double ein;    // l1 bound of its operands' accumulated error (units of M)
};
struct Entry {     // one linear error combination of a magnitude, plus a scalar part
    int gv;
    double s;
};

// the tracking type that stands in for `float` (and, for the reference, `double`)
struct TF {
    enum Kind : int { CONST, LIN, MAG };
    int kind = CONST;
    double val = 0;                 // CONST: the constant
    int form = -1;                  // LIN: index into the form pool
    int gv = -1;                    // LIN: gains of the events on its error (-1: none)
    double err = 0;                 // l1 error bound (units of M; abs mode: absolute)
    bool exact = false;             // LIN: exactly an integer (no rounding so far)
    double mag = 0;                 // MAG: |true value| <= mag M
    int cands = -1;                 // MAG: candidate forms
    int eset = -1;                  // MAG: error entries
    constexpr TF() {}
    constexpr TF(float v) : val(v) {}
    constexpr TF(double v) : val(v) {}
    constexpr TF(int v) : val(v) {}
    constexpr TF(unsigned char v) : val(v) {}
    explicit operator float() const { g_fail += 1000; return 0; }
};

static std::vector<Form> g_forms;
static std::vector<std::vector<int>> g_candsets;
static std::vector<Gains> g_gains;
static std::vector<Event> g_events;
static std::vector<std::vector<Entry>> g_esets;
static double g_basis[kMaxK][kMaxK];   // hat-unit basis b_c, c = k2 N + k1
static double g_bnorm2[kMaxK];

static int new_form() { g_forms.push_back(Form{}); return (int)g_forms.size() - 1; }
static int new_form_from(const double* src)
{
    int f = new_form();
    memcpy(g_forms[f].a, src, sizeof(double) * kMaxK);
    return f;
}
static double norm2(const double* a) { double s = 0; for (int i = 0; i < g_K; i++) s += a[i] * a[i]; return sqrt(s); }
static double sum1(const double* a) { double s = 0; for (int i = 0; i < g_K; i++) s += a[i]; return s; }
static double norm1(const double* a) { double s = 0; for (int i = 0; i < g_K; i++) s += fabs(a[i]); return s; }
// |alpha|_1 over the non-DC coefficients: |a.x| <= coef_l1(a) M for AC forms
static double coef_l1(const double* a)
{
    double s = 0;
    for (int c = 1; c < g_K; c++) {
        double d = 0;
        for (int i = 0; i < g_K; i++) d += a[i] * g_basis[c][i];
        s += fabs(d) / g_bnorm2[c];
    }
    return s;
}
static bool has_dc(const double* a) { return fabs(sum1(a)) > 1e-9 * (norm1(a) + 1); }

static int gains_combine(double c1, int g1, double c2, int g2)
{
    Gains out;
    const Gains empty;
    const Gains& A = g1 >= 0 ? g_gains[g1] : empty;
    const Gains& B = g2 >= 0 ? g_gains[g2] : empty;
    size_t i = 0, j = 0;
    while (i < A.size() || j < B.size()) {
        if (j == B.size() || (i < A.size() && A[i].first < B[j].first)) {
            out.push_back({A[i].first, c1 * A[i].second});
            i++;
        } else if (i == A.size() || B[j].first < A[i].first) {
            out.push_back({B[j].first, c2 * B[j].second});
            j++;
        } else {
            const double v = c1 * A[i].second + c2 * B[j].second;
            if (v != 0) out.push_back({A[i].first, v});
            i++;
            j++;
        }
    }
    g_gains.push_back(std::move(out));
    return (int)g_gains.size() - 1;
}

// a linear value c1 x + c2 y (forms and gains), not yet rounded
static TF lin(double c1, const TF* x, double c2, const TF* y)
{
    double tmp[kMaxK];
    for (int i = 0; i < g_K; i++)
        tmp[i] = (x ? c1 * g_forms[x->form].a[i] : 0.0) + (y ? c2 * g_forms[y->form].a[i] : 0.0);
    const int gx = x ? x->gv : -1, gy = y ? y->gv : -1;
    TF r;
    r.kind = TF::LIN;
    r.form = new_form_from(tmp);
    r.gv = gains_combine(c1, gx, c2, gy);
    return r;
}

// the rounding of a LIN result whose operands' errors add up to e_in
static void round_lin(TF& r, double e_in, bool operands_exact)
{
    const double* a = g_forms[r.form].a;
    if (g_abs) {
        r.exact = false;
        r.err = e_in + g_u * (norm1(a) * g_xmax + e_in);
        return;
    }
    if (operands_exact && norm1(a) * g_xmax < 16777216.0) {   // integer below 2^24: exact
        r.exact = true;
        r.err = 0;
        return;
    }
    r.exact = false;
    if (has_dc(a)) g_fail++;
    r.err = e_in + g_u * (coef_l1(a) + e_in);
    g_events.push_back({r.form, e_in});
    const int k = (int)g_events.size() - 1;
    g_gains[r.gv].push_back({k, 1.0});   // the newest event has the largest id
}

static TF as_lin(const TF& x)
{
    if (x.kind == TF::LIN) return x;
    if (x.kind == TF::CONST && x.val == 0) {   // the literal 0 as data: the zero form
        TF r;
        r.kind = TF::LIN;
        r.form = new_form();
        r.exact = true;
        return r;
    }
    g_fail += 1000;   // a magnitude or a nonzero constant where a linear value was expected
    return x;
}

static int eset_new(std::vector<Entry> e)
{
    g_esets.push_back(std::move(e));
    return (int)g_esets.size() - 1;
}
static int cands_new(std::vector<int> c)
{
    g_candsets.push_back(std::move(c));
    return (int)g_candsets.size() - 1;
}

static TF add(const TF& x0, const TF& y0, double sy)
{
    if (x0.kind == TF::CONST && y0.kind == TF::CONST) return TF(x0.val + sy * y0.val);
    TF x = as_lin(x0), y = as_lin(y0);
    TF r = lin(1.0, &x, sy, &y);
    round_lin(r, x.err + y.err, x.exact && y.exact);
    return r;
}

inline TF operator+(const TF& x, const TF& y)
{
    if (x.kind == TF::MAG && y.kind == TF::MAG) {
        // |a| + |b| = max(|a + b|, |a - b|): candidates a +- b; the error of
        // |a'| + |b'| is at most |E_a| + |E_b| = max(|E_a + E_b|, |E_a - E_b|)
        const std::vector<int> A = g_candsets[x.cands], B = g_candsets[y.cands];
        const std::vector<Entry> EA = g_esets[x.eset], EB = g_esets[y.eset];
        if (A.size() != 1 || B.size() != 1 || EA.size() != 1 || EB.size() != 1) g_fail += 1000;
        TF r;
        r.kind = TF::MAG;
        std::vector<int> c;
        double m = 0;
        for (int sgn = -1; sgn <= 1; sgn += 2) {
            double tmp[kMaxK];
            for (int i = 0; i < g_K; i++) tmp[i] = g_forms[A[0]].a[i] + sgn * g_forms[B[0]].a[i];
            c.push_back(new_form_from(tmp));
            m = std::max(m, coef_l1(tmp));
        }
        r.mag = m;
        r.err = x.err + y.err + g_u * (m + x.err + y.err);
        const double s = EA[0].s + EB[0].s + g_u * (m + x.err + y.err);
        r.cands = cands_new(c);
        const int gp = gains_combine(1.0, EA[0].gv, 1.0, EB[0].gv);
        const int gm = gains_combine(1.0, EA[0].gv, -1.0, EB[0].gv);
        r.eset = eset_new({{gp, s}, {gm, s}});
        return r;
    }
    return add(x, y, 1.0);
}
inline TF operator-(const TF& x, const TF& y) { return add(x, y, -1.0); }
inline TF operator-(const TF& x)
{
    if (x.kind == TF::CONST) return TF(-x.val);
    TF l = as_lin(x);
    TF r = lin(-1.0, &l, 0.0, nullptr);
    r.err = l.err;
    r.exact = l.exact;
    return r;
}
inline TF& operator-=(TF& x, const TF& y) { x = x - y; return x; }
inline TF& operator+=(TF& x, const TF& y) { x = x + y; return x; }

// c * x (x data, c a constant), rounded once
static TF scale(const TF& x, double c)
{
    if (x.kind == TF::MAG) {
        if (c < 0) g_fail += 1000;
        TF r = x;
        std::vector<int> cs;
        for (int f : g_candsets[x.cands]) {
            double tmp[kMaxK];
            for (int i = 0; i < g_K; i++) tmp[i] = c * g_forms[f].a[i];
            cs.push_back(new_form_from(tmp));
        }
        r.cands = cands_new(cs);
        r.mag = x.mag * c;
        const double rnd = g_u * (c * x.mag + c * x.err);
        r.err = c * x.err + rnd;
        std::vector<Entry> es;
        const std::vector<Entry> src = g_esets[x.eset];
        for (const Entry& e : src) {
            const int g = gains_combine(c, e.gv, 0.0, -1);
            es.push_back({g, c * e.s + rnd});
        }
        r.eset = eset_new(es);
        return r;
    }
    TF l = as_lin(x);
    TF r = lin(c, &l, 0.0, nullptr);
    round_lin(r, fabs(c) * l.err, false);
    return r;
}
inline TF operator*(const TF& x, const TF& y)
{
    if (x.kind == TF::CONST && y.kind == TF::CONST) return TF(x.val * y.val);
    if (y.kind == TF::CONST) return scale(x, y.val);
    if (x.kind == TF::CONST) return scale(y, x.val);
    g_fail += 1000;   // data * data never occurs in the passes
    return x;
}
inline TF& operator*=(TF& x, const TF& y) { x = x * y; return x; }
// compile-only (the reference header's luma / scan, never called here)
inline TF operator/(const TF& x, int) { g_fail += 1000; return x; }
inline bool operator<(const TF&, int) { g_fail += 1000; return false; }
inline bool operator<=(const TF&, const TF&) { g_fail += 1000; return false; }

// fmaf with one constant factor: one rounding
inline TF fmaf(const TF& x, const TF& y, const TF& z)
{
    const TF& c = x.kind == TF::CONST ? x : y;
    const TF& d = x.kind == TF::CONST ? y : x;
    if (c.kind != TF::CONST || d.kind == TF::CONST) { g_fail += 1000; return z; }
    TF dl = as_lin(d), zl = as_lin(z);
    TF r = lin(c.val, &dl, 1.0, &zl);
    round_lin(r, fabs(c.val) * dl.err + zl.err, false);
    return r;
}

inline TF fabsf(const TF& x)
{
    if (x.kind == TF::MAG) return x;
    if (x.kind == TF::CONST) return TF(fabs(x.val));
    const double* a = g_forms[x.form].a;
    if (has_dc(a)) g_fail++;   // |a.x| not bounded by the contrast
    TF r;
    r.kind = TF::MAG;
    r.mag = coef_l1(a);
    r.err = x.err;
    r.cands = cands_new({x.form});
    r.eset = eset_new({{x.gv, 0.0}});
    return r;
}

inline TF fmaxf(const TF& x, const TF& y)
{
    if (x.kind == TF::CONST && x.val == 0) return fabsf(y);   // max with 0 (magnitudes only)
    if (y.kind == TF::CONST && y.val == 0) return fabsf(x);
    if (x.kind != TF::MAG || y.kind != TF::MAG) g_fail += 1000;
    TF r;
    r.kind = TF::MAG;
    r.mag = std::max(x.mag, y.mag);
    r.err = std::max(x.err, y.err);
    std::vector<int> c = g_candsets[x.cands];
    c.insert(c.end(), g_candsets[y.cands].begin(), g_candsets[y.cands].end());
    r.cands = cands_new(c);
    std::vector<Entry> e = g_esets[x.eset];
    e.insert(e.end(), g_esets[y.eset].begin(), g_esets[y.eset].end());
    r.eset = eset_new(e);
    return r;
}

#define float TF
#include "dcte_passes.h"
#undef float
#define double TF
#include "dcte_ref64.h"
#undef double

// exact hat-unit basis h_k(i) (dcte_math.h units)
static long double hat(int n, int k, int i)
{
    const long double pi = 3.141592653589793238462643383279502884L;
    const long double g = n >= 8 ? sqrtl(2.0L) : 1.0L;
    return k == 0 ? 1.0L : g * cosl(pi * (2 * i + 1) * k / (2.0L * n));
}

// lambda_max of Q = sum_k |g_k| a_k a_k^T (over the window samples): power
// iteration, then a Cholesky factorisation of (t I - Q) certifies t
static double lambda_max_certified(const Gains& ev)
{
    const int K = g_K;
    std::vector<double> Q((size_t)K * K, 0.0);
    for (const auto& e : ev) {
        const double* a = g_forms[g_events[e.first].form].a;
        const double w = fabs(e.second);
        for (int i = 0; i < K; i++) {
            if (a[i] == 0) continue;
            const double wa = w * a[i];
            for (int j = 0; j < K; j++) Q[(size_t)i * K + j] += wa * a[j];
        }
    }
    double trace = 0;
    for (int i = 0; i < K; i++) trace += Q[(size_t)i * K + i];
    if (trace == 0) return 0;
    std::vector<double> v(K), q(K);
    for (int i = 0; i < K; i++) v[i] = 1.0 + 0.01 * i;
    double lam = 0;
    for (int it = 0; it < 300; it++) {
        double nrm = 0;
        for (int i = 0; i < K; i++) {
            double s = 0;
            for (int j = 0; j < K; j++) s += Q[(size_t)i * K + j] * v[j];
            q[i] = s;
            nrm += s * s;
        }
        nrm = sqrt(nrm);
        if (nrm == 0) return 0;
        lam = nrm;
        for (int i = 0; i < K; i++) v[i] = q[i] / nrm;
    }
    std::vector<double> L((size_t)K * K);
    for (double t = lam * 1.001 + 1e-12 * trace; t < trace * 1.001 + 1e-300; t *= 1.02) {
        // Cholesky of t I - Q: all pivots positive iff t > lambda_max
        bool ok = true;
        for (int j = 0; j < K && ok; j++) {
            double d = t - Q[(size_t)j * K + j];
            for (int p = 0; p < j; p++) d -= L[(size_t)j * K + p] * L[(size_t)j * K + p];
            if (!(d > 1e-10 * t)) {
                ok = false;
                break;
            }
            const double ljj = sqrt(d);
            L[(size_t)j * K + j] = ljj;
            for (int i = j + 1; i < K; i++) {
                double s = -Q[(size_t)i * K + j];
                for (int p = 0; p < j; p++) s -= L[(size_t)i * K + p] * L[(size_t)j * K + p];
                L[(size_t)i * K + j] = s / ljj;
            }
        }
        if (ok) return t;
    }
    return trace;   // lambda_max <= trace(Q) always
}

// the bound of one error entry (units of M)
static double entry_bound(const Entry& e, double cN)
{
    if (e.gv < 0) return e.s;
    const Gains& g = g_gains[e.gv];
    double l1 = 0, sg = 0, second = 0;
    for (const auto& p : g) {
        const Event& ev = g_events[p.first];
        l1 += fabs(p.second) * coef_l1(g_forms[ev.form].a);
        sg += fabs(p.second);
        second += fabs(p.second) * ev.ein;
    }
    double cs = 1e300;
    if (!g.empty()) cs = sqrt(sg) * sqrt(lambda_max_certified(g)) * cN;
    return g_u * (std::min(l1, cs) + second) + e.s;
}

// one symbolic window through the kernel's passes (pixel_maxima, dcte_pixel.h)
template <int N>
static int analyse(double xmax, double* out)
{
    g_forms.clear();
    g_candsets.clear();
    g_gains.clear();
    g_events.clear();
    g_esets.clear();
    g_K = N * N;
    g_xmax = xmax;
    g_fail = 0;
    g_abs = false;
    g_u = kU;
    for (int k1 = 0; k1 < N; k1++)
        for (int k2 = 0; k2 < N; k2++) {
            const int c = k2 * N + k1;
            double n2 = 0;
            for (int j = 0; j < N; j++)
                for (int i = 0; i < N; i++) {
                    g_basis[c][j * N + i] = (double)(hat(N, k1, i) * hat(N, k2, j));
                    n2 += g_basis[c][j * N + i] * g_basis[c][j * N + i];
                }
            g_bnorm2[c] = n2;
        }
    constexpr int CH = dcte::Lanes<N>::CH, S = dcte::Lanes<N>::S;
    TF mt = 0.0f, me = 0.0f;
    for (int lp = 0; lp < S; lp++) {
        TF lrow[N];
        TF ring[N][CH];
        for (int j = 0; j < N; j++) {          // window row j (y), sample i (x): index j N + i
            for (int i = 0; i < N; i++) {
                TF s;
                s.kind = TF::LIN;
                s.form = new_form();
                g_forms[s.form].a[j * N + i] = 1.0;
                s.exact = true;
                lrow[i] = s;
            }
            dcte::row_pass<N>(lrow, 0, lp, ring[j]);
        }
        TF t_, e_;
        dcte::Cols<N>::template run<0>(ring, lp, t_, e_);
        mt = fmaxf(mt, t_);
        me = fmaxf(me, e_);
    }
    // the candidate sets against the reference's coefficients
    std::vector<std::vector<double>> exact_e, exact_t;
    for (int k1 = 0; k1 < N; k1++)
        for (int k2 = 0; k2 < N; k2++) {
            if (!k1 && !k2) continue;
            ((k1 + k2 == 1) ? exact_e : exact_t).push_back(
                std::vector<double>(g_basis[k2 * N + k1], g_basis[k2 * N + k1] + g_K));
        }
    // every candidate is +-(some coefficient of its class) up to the fp32
    // constants, and every coefficient has a candidate
    auto match = [&](const TF& m, std::vector<std::vector<double>>& ex, double& dev) {
        if (m.kind != TF::MAG) return -1;
        std::vector<int> hit(ex.size(), 0);
        dev = 0;
        for (int f : g_candsets[m.cands]) {
            const double* a = g_forms[f].a;
            int best = -1;
            double bd = 1e300;
            for (size_t q = 0; q < ex.size(); q++)
                for (int sg = -1; sg <= 1; sg += 2) {
                    double d = 0;
                    for (int i = 0; i < g_K; i++) d += (a[i] - sg * ex[q][i]) * (a[i] - sg * ex[q][i]);
                    if (d < bd) {
                        bd = d;
                        best = (int)q;
                    }
                }
            if (sqrt(bd) > 1e-5 * norm2(ex[best].data())) return -2;
            hit[best] = 1;
            double diff[kMaxK] = {}, sg = 0;
            for (int i = 0; i < g_K; i++) sg += a[i] * ex[best][i];
            sg = sg >= 0 ? 1.0 : -1.0;
            for (int i = 0; i < g_K; i++) diff[i] = a[i] - sg * ex[best][i];
            dev = std::max(dev, coef_l1(diff));
        }
        for (int h : hit)
            if (!h) return -3;
        return 0;
    };
    double dev_e = 0, dev_t = 0;
    const int rc_e = match(me, exact_e, dev_e), rc_t = match(mt, exact_t, dev_t);
    const double cN = N >= 8 ? sqrt((double)N * N - 1) / N : 2.0 * sqrt((double)N * N - 1) / N;
    double be = 0, bt = 0;
    if (rc_e == 0 && rc_t == 0) {
        for (const Entry& e : g_esets[me.eset]) be = std::max(be, entry_bound(e, cN));
        for (const Entry& e : g_esets[mt.eset]) bt = std::max(bt, entry_bound(e, cN));
    }
    double l1 = 0;
    for (auto& b : exact_t) l1 = std::max(l1, norm1(b.data()));
    for (auto& b : exact_e) l1 = std::max(l1, norm1(b.data()));
    out[0] = std::min(be, me.err);         // fp32 rounding, in units of M
    out[1] = std::min(bt, mt.err);
    out[2] = dev_e;                        // fp32 constants, in units of M
    out[3] = dev_t;
    out[4] = l1;                           // max ||basis||_1 (hat units)
    out[5] = (double)g_candsets[me.cands].size();
    out[6] = (double)g_candsets[mt.cands].size();
    out[7] = sqrt(1.0 - 1.0 / (N * N)) / cN;   // M_min of a non-flat integer window (hat units)
    out[8] = (double)g_fail;
    out[9] = (double)(rc_e * 10 + rc_t);
    out[10] = me.err;                      // the forward l1 bounds alone
    out[11] = mt.err;
    out[12] = (double)g_events.size();
    return g_fail == 0 && rc_e == 0 && rc_t == 0 ? 0 : -1;
}

// The reference's own fp64 transform (dcte_ref64.h: ddct8x8s / ddct16x16s /
// ddct2d in Ooura's operation order, src/fft2d/shrtdct.c:61-117, 238-386,
// fftsg2d.c:566-627) on a symbolic window of samples |x| <= xmax: the largest
// absolute error of a non-DC coefficient, in the reference's units (ortho
// for N = 8, 16; unnormalised for N = 2, 4), unit 2^-53, plus the deviation
// of its fp64 constants.
template <int N>
static double ref_error(double xmax)
{
    g_forms.clear();
    g_candsets.clear();
    g_gains.clear();
    g_events.clear();
    g_esets.clear();
    g_K = N * N;
    g_xmax = xmax;
    g_fail = 0;
    g_abs = true;
    g_u = 1.1102230246251565e-16;
    struct Restore {
        ~Restore()
        {
            g_abs = false;
            g_u = kU;
        }
    } restore_;
    double ctd[4] = {0, 0, 0, 0};               // makect(n) as the reference builds it
    if (N == 2 || N == 4) {
        const int nch = N >> 1;
        const double delta = atan(1.0) / nch;
        ctd[0] = cos(delta * nch);
        ctd[nch] = 0.5 * ctd[0];
        for (int j = 1; j < nch; j++) {
            ctd[j] = 0.5 * cos(delta * j);
            ctd[N - j] = 0.5 * sin(delta * j);
        }
    }
    TF ct[4] = {TF(ctd[0]), TF(ctd[1]), TF(ctd[2]), TF(ctd[3])};
    TF d[N * N];
    for (int i = 0; i < N; i++)                 // d[i N + j]: i = dx (first index), j = dy
        for (int j = 0; j < N; j++) {
            TF s;
            s.kind = TF::LIN;
            s.form = new_form();
            g_forms[s.form].a[i * N + j] = 1.0;
            d[i * N + j] = s;
        }
    dcte::r64::transform(N, d, ct);
    const long double pi = 3.141592653589793238462643383279502884L;
    auto basis = [&](int k, int i) -> long double {
        const long double c = cosl(pi * (2 * i + 1) * k / (2.0L * N));
        if (N <= 4) return c;                                          // unnormalised
        return k == 0 ? sqrtl(1.0L / N) : sqrtl(2.0L / N) * c;        // orthonormal
    };
    double worst = 0;
    for (int k1 = 0; k1 < N; k1++)
        for (int k2 = 0; k2 < N; k2++) {
            if (!k1 && !k2) continue;
            const TF& v = d[k1 * N + k2];
            if (v.kind != TF::LIN) return -1;
            double dev = 0;
            for (int i = 0; i < N; i++)
                for (int j = 0; j < N; j++)
                    dev += fabs(g_forms[v.form].a[i * N + j] - (double)(basis(k1, i) * basis(k2, j)));
            if (dev > 1e-9) {
                fprintf(stderr, "ref_error N=%d: (%d,%d) off its basis by %g\n", N, k1, k2, dev);
                return -1;
            }
            worst = std::max(worst, v.err + dev * xmax);
        }
    if (g_fail) fprintf(stderr, "ref_error N=%d: %d failures\n", N, g_fail);
    return g_fail ? -1 : worst;
}

}  // namespace tb

extern "C" {

// out[13]: delta_e, delta_t (fp32 rounding, the smaller of the two bounds);
// constants delta_e, delta_t (all in units of M); max ||basis||_1;
// candidates of m_e, m_t; M_min of a non-flat integer window (hat units);
// failures; match codes; the forward l1 bounds of m_e, m_t; rounding events.
// xmax: max |biased luma| (637500 liblqr, 128 preview).  0 = derivation holds.
int tau_bound(int n, double xmax, double* out)
{
    switch (n) {
    case 2: return tb::analyse<2>(xmax, out);
    case 4: return tb::analyse<4>(xmax, out);
    case 8: return tb::analyse<8>(xmax, out);
    case 16: return tb::analyse<16>(xmax, out);
    default: return -9;
    }
}

// The reference's fp64 error bound (ref_error) for N at sample bound xmax.
double tau_ref_error(int n, double xmax)
{
    switch (n) {
    case 2: return tb::ref_error<2>(xmax);
    case 4: return tb::ref_error<4>(xmax);
    case 8: return tb::ref_error<8>(xmax);
    case 16: return tb::ref_error<16>(xmax);
    default: return -1;
    }
}
}
