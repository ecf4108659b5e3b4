// dcte_host.cpp -- the context-free CPU entry points of include/dctenergy.h
// (SURVEY §8b): plain host C++, no HIP, so the same file also builds with
// g++ under AddressSanitizer / UBSan (tests/asan).  The GPU entry points
// never fall back to these.
#include <math.h>
#include <string.h>

#include "../../include/dctenergy.h"
#include "dcte_host.h"
#include "dcte_normkey.h"
#include "dcte_ref64.h"

namespace dcte {

// the reference's makect (src/fft2d/fftsg.c:724-740) for nc = n, with libm,
// exactly as the reference evaluates it; used by the fp64 refinement and the
// exact kernels (N = 2, 4)
void small_twiddles(int n, double ct[4])
{
    ct[0] = ct[1] = ct[2] = ct[3] = 0.0;
    if (n != 2 && n != 4) return;
    int nch = n >> 1;
    double delta = atan(1.0) / nch;
    ct[0] = cos(delta * nch);
    ct[nch] = 0.5 * ct[0];
    for (int j = 1; j < nch; j++) {
        ct[j] = 0.5 * cos(delta * j);
        ct[n - j] = 0.5 * sin(delta * j);
    }
}

}  // namespace dcte

extern "C" {

int dcte_energy_window(int n, const double* win, float edges, float textures, float* out)
{
    if (!(n == 2 || n == 4 || n == 8 || n == 16) || !win || !out) return DCTE_EINVAL;
    double d[16 * 16];
    memcpy(d, win, sizeof(double) * (size_t)n * (size_t)n);
    double ct[4];
    dcte::small_twiddles(n, ct);
    dcte::r64::transform(n, d, ct);
    *out = dcte::r64::weighted_max(n, d, edges, textures);
    return DCTE_OK;
}

int dcte_normalize_u8_host(const float* E, size_t n, int mode, int channels, uint8_t* out)
{
    if (!E || !out || n == 0 || !((mode == DCTE_NORM_LQR || mode == DCTE_NORM_PREVIEW) &&
                                  channels >= 1 && channels <= 4))
        return DCTE_EINVAL;
    unsigned kmin = 0xffffffffu, kmax = 0u;
    for (size_t i = 0; i < n; i++) {
        const unsigned k = dcte::norm_fkey(E[i]);
        kmin = k < kmin ? k : kmin;
        kmax = k > kmax ? k : kmax;
    }
    const float mn = dcte::norm_funkey(kmin), mx = dcte::norm_funkey(kmax);
    for (size_t i = 0; i < n; i++) {
        const uint8_t v = dcte::norm_one(E[i], mn, mx, mode);
        for (int c = 0; c < channels; c++) out[i * (size_t)channels + c] = v;
    }
    return DCTE_OK;
}

}  // extern "C"
