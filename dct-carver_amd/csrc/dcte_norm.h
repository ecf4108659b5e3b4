// dcte_norm.h -- launchers of the energy-map -> u8 kernels (dcte_norm.hip).
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

namespace dcte {

constexpr int kNormLqr = 0;      // DCTE_NORM_LQR
constexpr int kNormPreview = 1;  // DCTE_NORM_PREVIEW

// Shared by the device kernels and the host entry point
// (dcte_normalize_u8_host), so both give the same bytes.
// order-preserving float <-> uint key (total order on non-NaN floats)
__host__ __device__ inline unsigned norm_fkey(float f)
{
    unsigned b = __builtin_bit_cast(unsigned, f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__host__ __device__ inline float norm_funkey(unsigned k)
{
    return __builtin_bit_cast(float, (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
// one energy -> u8 with the frame's {min, max} (modes: dcte_norm.hip)
__host__ __device__ inline uint8_t norm_one(float d, float mn, float mx, int mode)
{
    if (!(mx > mn)) return 0;
    if (mode == kNormPreview) {
        double v = 255.0 * (((double)d - (double)mn) / ((double)mx - (double)mn));
        return (uint8_t)(int)(v + 0.5);
    }
    float v = (d - mn) / (mx - mn);
    return (uint8_t)(int)(v * 255.0f);
}

// keys: 2 device uints of scratch; minmax: 2 device floats {min, max}
hipError_t launch_minmax(const float* e, long long n, unsigned* keys, float* minmax, hipStream_t s);
hipError_t launch_to_u8(const float* e, long long n, const float* minmax, int mode, int channels,
                        uint8_t* out, hipStream_t s);

// u8 frame (rows x cols x bpp) -> its transpose (cols x rows x bpp)
hipError_t launch_transpose_u8(const uint8_t* src, long long src_pitch, int rows, int cols, int bpp,
                               uint8_t* dst, long long dst_pitch, hipStream_t s);

}  // namespace dcte
