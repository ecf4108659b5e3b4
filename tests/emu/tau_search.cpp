// tau_search.cpp -- adversarial search for the fp32 error the refinement
// margin tau must cover (TEST INFRASTRUCTURE, built into libdcte_emu.so).
//
// The kernel decides edge vs texture by comparing its fp32 maxima m_e and
// m_t (src/dct.c:100-109 reduced to m_e > m_t) and hands a pixel to the fp64
// refinement when the two lie within tau of each other.  A pixel can leave
// with the wrong class only if one candidate's fp32 value is off its exact
// value by more than tau/2 of the window's max coefficient.  This searches
// integer-luma windows for the largest
//     delta = max(|m_e32 - m_e|, |m_t32 - m_t|) / max(m_e, m_t)
// with random restarts and hill climbing over the window's pixel bytes.  The
// fp32 side is the map kernel's own code on one window (dcte_pixel.h ->
// dcte_passes.h / dcte_math.h); the exact side is the separable 2-D DCT-II of
// the same integer luma in long double, in the kernel's "hat" units
// (dcte_math.h: X0 = sum x, Xk = g sum x cos(pi (2j+1) k / 2N), g = sqrt2 for
// N = 8, 16 and 1 for N = 2, 4) -- the reference transforms
// (src/fft2d/shrtdct.c:61-117, 238-386; src/fft2d/fftsg2d.c:566-627) up to
// that global scale.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "dcte_pixel.h"

using namespace dcte;

namespace {

struct Rng {   // xorshift64*
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 1) {}
    uint64_t next()
    {
        s ^= s >> 12;
        s ^= s << 25;
        s ^= s >> 27;
        return s * 0x2545F4914F6CDD1Dull;
    }
    int below(int n) { return (int)((next() >> 33) % (uint64_t)n); }
};

template <int N>
struct Exact {
    long double cs[N][N];   // g_k cos(pi (2j+1) k / 2N), [k][j]
    explicit Exact()
    {
        const long double pi = 3.141592653589793238462643383279502884L;
        const long double g = N >= 8 ? sqrtl(2.0L) : 1.0L;
        for (int k = 0; k < N; k++)
            for (int j = 0; j < N; j++)
                cs[k][j] = k == 0 ? 1.0L : g * cosl(pi * (2 * j + 1) * k / (2.0L * N));
    }
    // m_e, m_t of an N x N luma window x[row][col]
    void maxima(const long double (&x)[N][N], long double& me, long double& mt) const
    {
        long double r[N][N];                     // row transforms r[row][k2]
        for (int i = 0; i < N; i++)
            for (int k = 0; k < N; k++) {
                long double s = 0;
                for (int j = 0; j < N; j++) s += cs[k][j] * x[i][j];
                r[i][k] = s;
            }
        me = mt = 0;
        for (int k1 = 0; k1 < N; k1++)
            for (int k2 = 0; k2 < N; k2++) {
                if (!k1 && !k2) continue;
                long double s = 0;
                for (int i = 0; i < N; i++) s += cs[k1][i] * r[i][k2];
                s = fabsl(s);
                if ((k1 == 0 && k2 == 1) || (k1 == 1 && k2 == 0)) me = me > s ? me : s;
                else mt = mt > s ? mt : s;
            }
    }
};

template <int N>
double delta(const Exact<N>& ex, const uint8_t* win, int bpp, int sem, double* me_o, double* mt_o)
{
    const int HL = halo_left(N, sem);
    float mt32, me32;
    pixel_maxima<N>(win, (long long)N * bpp, 0, N, N, bpp, sem, HL, HL, mt32, me32);
    long double x[N][N];
    for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++) x[i][j] = luma_biased(win + (i * N + j) * bpp, bpp, sem);
    long double me, mt;
    ex.maxima(x, me, mt);
    const long double hi = me > mt ? me : mt;
    if (me_o) *me_o = (double)me;
    if (mt_o) *mt_o = (double)mt;
    // a window without AC content: the exact side is 0 up to the long double
    // rounding of the cosines (~1e-13 here), the kernel's exact-integer
    // stages give 0, and nothing is compared (the map is 0, ATOL covers it)
    if (hi < 1e-3L) return 0.0;
    long double de = fabsl((long double)me32 - me), dt = fabsl((long double)mt32 - mt);
    return (double)((de > dt ? de : dt) / hi);
}

// initial windows of several kinds
void seed_window(Rng& r, uint8_t* w, int n, int bpp)
{
    const int cnt = n * n * bpp;
    const int kind = r.below(6);
    const int base = r.below(256), amp = 1 + r.below(kind == 0 ? 255 : 12);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++)
            for (int c = 0; c < bpp; c++) {
                int v;
                switch (kind) {
                case 0: v = r.below(256); break;                                  // uniform
                case 1: v = r.below(40) == 0 ? r.below(256) : base; break;        // sparse dots
                case 2: v = base + r.below(2 * amp + 1) - amp; break;             // low-contrast noise
                case 3: v = base + (amp * (i + 2 * j)) / 3 - amp * n / 2; break;  // ramp
                case 4: v = ((i + j) & 1) ? base : base + amp; break;             // checker
                default: v = (i < n / 2) != (j < r.below(n + 1)) ? base : 255 - base; break;  // step
                }
                w[(i * n + j) * bpp + c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
            }
    (void)cnt;
}

template <int N>
double search(int sem, int bpp, int restarts, int iters, uint64_t seed, uint8_t* best_w,
              double* best_me, double* best_mt)
{
    static const Exact<N> ex;
    Rng r(seed);
    const int cnt = N * N * bpp;
    uint8_t cur[16 * 16 * 4], cand[16 * 16 * 4];
    double best = -1.0;
    for (int k = 0; k < restarts; k++) {
        if (k % 4 == 3 && best >= 0) memcpy(cur, best_w, cnt);   // exploit the best so far
        else seed_window(r, cur, N, bpp);
        double dc = delta<N>(ex, cur, bpp, sem, nullptr, nullptr);
        for (int it = 0; it < iters; it++) {
            memcpy(cand, cur, cnt);
            const int m = 1 + r.below(3);
            for (int q = 0; q < m; q++) {
                const int p = r.below(cnt);
                int v = cand[p];
                v = r.below(4) == 0 ? r.below(256) : v + r.below(9) - 4;
                cand[p] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
            }
            const double dn = delta<N>(ex, cand, bpp, sem, nullptr, nullptr);
            if (dn >= dc) {
                dc = dn;
                memcpy(cur, cand, cnt);
            }
        }
        if (dc > best) {
            best = dc;
            memcpy(best_w, cur, cnt);
        }
    }
    delta<N>(ex, best_w, bpp, sem, best_me, best_mt);
    return best;
}

}  // namespace

extern "C" {

// Largest delta found; the window (N x N x bpp bytes, evaluated at its own
// pixel (HL, HL), so no clamping) and its exact maxima are written out.
double emu_tau_search(int n, int sem, int bpp, int restarts, int iters, unsigned long long seed,
                      uint8_t* best_window, double* best_me, double* best_mt)
{
    switch (n) {
    case 2: return search<2>(sem, bpp, restarts, iters, seed, best_window, best_me, best_mt);
    case 4: return search<4>(sem, bpp, restarts, iters, seed, best_window, best_me, best_mt);
    case 8: return search<8>(sem, bpp, restarts, iters, seed, best_window, best_me, best_mt);
    case 16: return search<16>(sem, bpp, restarts, iters, seed, best_window, best_me, best_mt);
    default: return -1.0;
    }
}

// delta of one given window (for checking a found window against the oracle)
double emu_window_delta(int n, int sem, int bpp, const uint8_t* win, double* me, double* mt)
{
    switch (n) {
    case 2: { static const Exact<2> e; return delta<2>(e, win, bpp, sem, me, mt); }
    case 4: { static const Exact<4> e; return delta<4>(e, win, bpp, sem, me, mt); }
    case 8: { static const Exact<8> e; return delta<8>(e, win, bpp, sem, me, mt); }
    case 16: { static const Exact<16> e; return delta<16>(e, win, bpp, sem, me, mt); }
    default: return -1.0;
    }
}
}
