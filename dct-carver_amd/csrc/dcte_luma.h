// dcte_luma.h -- integer luma domain shared by kernels and host emulation.
//
// liblqr's LQR_ER_LUMA read for 8-bit pixels (requested by the plug-in at
// src/render.c:315) is, in double [liblqr, unverified]:
//     RGB : 0.2126 R/255 + 0.7152 G/255 + 0.0722 B/255
//     grey: v/255
// Since 0.2126 = 1063/5000, 0.7152 = 3576/5000, 0.0722 = 361/5000, that is
// exactly  L / 1275000  with the integer  L = 1063 R + 3576 G + 361 B  (grey:
// L = 5000 v), 0 <= L <= 1275000.  The kernels work on L - 637500, an exact
// fp32 integer in [-637500, 637500]; the bias only moves the DC coefficient,
// which the energy never looks at (src/dct.c:103, "k1 || k2").
#pragma once

#if defined(__HIPCC__)
#define DCTE_LUMA_HD __host__ __device__ __forceinline__
#else
#define DCTE_LUMA_HD static inline
#endif

namespace dcte {

// energy semantics (DCTE_LQR / DCTE_PREVIEW in include/dctenergy.h)
constexpr int kSemLqr = 0;
constexpr int kSemPreview = 1;

// Preview semantics: convert_row_to_luminance (src/render.c:62-79) with
// RGB2LUMINANCE (src/render.h:5), evaluated in double left to right (the TU
// is compiled without contraction) and truncated to guchar; grey copies the
// byte.  The kernels work on L - 128, exact in fp32.
constexpr int kPreviewBias = 128;
DCTE_LUMA_HD unsigned preview_luma(unsigned r, unsigned g, unsigned b, int bpp)
{
    if (bpp == 1) return r;
    return (unsigned char)(16.0 + r * 0.2568 + g * 0.5041 + b * 0.0979);
}

constexpr int kLumaR = 1063, kLumaG = 3576, kLumaB = 361, kLumaGrey = 5000;
constexpr int kLumaBias = 637500;
constexpr double kLumaScale = 1275000.0;  // L / kLumaScale = liblqr luma

}  // namespace dcte
