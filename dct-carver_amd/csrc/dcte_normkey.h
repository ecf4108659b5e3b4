// dcte_normkey.h -- the energy -> u8 arithmetic shared by the device kernels
// (dcte_norm.hip) and the host entry point (dcte_host.cpp, dcte_normalize_u8_
// host), so both give the same bytes.  No HIP headers: the host file also
// builds with a plain C++ compiler (tests/asan).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define DCTE_NORM_HD __host__ __device__ inline
#else
#define DCTE_NORM_HD inline
#endif

namespace dcte {

constexpr int kNormLqr = 0;      // DCTE_NORM_LQR
constexpr int kNormPreview = 1;  // DCTE_NORM_PREVIEW

// order-preserving float <-> uint key (total order on non-NaN floats)
DCTE_NORM_HD unsigned norm_fkey(float f)
{
    unsigned b = __builtin_bit_cast(unsigned, f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
DCTE_NORM_HD float norm_funkey(unsigned k)
{
    return __builtin_bit_cast(float, (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
// one energy -> u8 with the frame's {min, max} (modes: dcte_norm.hip)
DCTE_NORM_HD uint8_t norm_one(float d, float mn, float mx, int mode)
{
    if (!(mx > mn)) return 0;
    if (mode == kNormPreview) {
        double v = 255.0 * (((double)d - (double)mn) / ((double)mx - (double)mn));
        return (uint8_t)(int)(v + 0.5);
    }
    float v = (d - mn) / (mx - mn);
    return (uint8_t)(int)(v * 255.0f);
}

}  // namespace dcte
