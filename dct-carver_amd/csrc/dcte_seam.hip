// dcte_seam.hip -- seam removal with energy update, and energies at listed
// pixels (liblqr's carve + update_emap, and the batched
// per-window API the seam update needs).
//
// A carver step removes one pixel per row (the seam s[y]) and then needs the
// energy of the narrower frame.  Only pixels whose window straddles the seam
// change: pixel (x, y) of the new (w-1)-wide frame reads rows
// R(y) = clamp(y - HL .. y + HR) and, per row y', columns x - HL .. x + HR.
// With lo / hi = min / max of s over R(y):
//   x + HR <  lo   every window column lies left of the seam: the window is
//                  the old window of (x, y)       -> E' = E[y][x]
//   min(x - HL, w - 2) >= hi
//                  every (clamped) column lies right of it: the window is
//                  the old window of (x + 1, y), clamps included (the right
//                  border moved by one too)      -> E' = E[y][x + 1]
//                  (the min matters when HL < 0, preview N = 2: a window
//                  clamped onto the last column reads left of a seam there)
//   otherwise      recomputed (<= N - 1 + (hi - lo) pixels per row).
// Recomputed pixels go through pixel_maxima (dcte_pixel.h), the map kernel's
// own passes, and the same tie flagging + fp64 refinement as dcte_map, so
// K incremental steps give exactly the map of the carved frame.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dcte_kernels.h"
#include "dcte_pixel.h"

namespace dcte {

__device__ __forceinline__ void seam_span(const int* __restrict__ seam, int w, int h, int n, int sem,
                                          int y, int& lo, int& hi)
{
    const int HL = halo_left(n, sem);
    lo = w;
    hi = -1;
    for (int j = 0; j < n; j++) {
        const int s = clamp_px(seam[clamp_px(y - HL + j, 0, h - 1)], 0, w - 1);
        lo = min(lo, s);
        hi = max(hi, s);
    }
}

// new frame + the map pixels that only move: one thread per new pixel
template <int BPP>
__global__ __launch_bounds__(256) void dcte_seam_shift(const SeamParams p)
{
    const int y = blockIdx.y;
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int w1 = p.w - 1;
    if (x >= w1) return;
    const int s = clamp_px(p.seam[y], 0, p.w - 1);
    const int xs = x + (x >= s ? 1 : 0);
    const uint8_t* src = p.px + (long long)y * p.rowstride + (long long)xs * BPP;
    uint8_t* dst = p.px_out + (long long)y * p.out_rowstride + (long long)x * BPP;
#pragma unroll
    for (int c = 0; c < BPP; c++) dst[c] = src[c];
    int lo, hi;
    seam_span(p.seam, p.w, p.h, p.n, p.sem, y, lo, hi);
    const int HL = halo_left(p.n, p.sem), HR = p.n - 1 - HL;
    if (x + HR < lo)
        p.map_out[(long long)y * p.map_out_stride + x] = p.map[(long long)y * p.map_stride + x];
    else if (min(x - HL, p.w - 2) >= hi)
        p.map_out[(long long)y * p.map_out_stride + x] = p.map[(long long)y * p.map_stride + x + 1];
}

__device__ __forceinline__ void emit_pixel(const SeamParams& p, float mt, float me, float* dst,
                                           unsigned fix_index)
{
    const float hi = fmaxf(me, mt), lo = fminf(me, mt);
    *dst = hi * (me > mt ? p.we : p.wt);        // the map kernel's decision (dcte_map emit)
    if ((p.we != p.wt && lo > (1.0f - p.tie_tau) * hi) || p.tie_tau >= 1.0f) {
        const unsigned k = atomicAdd(p.fix_count, 1u);
        if (k < p.fix_cap) p.fix_list[k] = fix_index;
    }
}

// recomputed band: one wave per row of the new frame
template <int N, int BPP, int SEM>
__global__ __launch_bounds__(256) void dcte_seam_band(const SeamParams p)
{
    const int y = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (y >= p.h) return;
    constexpr int HL = SEM == kSemLqr ? N / 2 - 1 : (N - 1) / 2 - 1, HR = N - 1 - HL;
    const int w1 = p.w - 1;
    int lo, hi;
    seam_span(p.seam, p.w, p.h, N, SEM, y, lo, hi);
    const int a = max(0, lo - HR), b = hi <= p.w - 2 ? min(w1 - 1, hi + HL - 1) : w1 - 1;
    for (int x = a + lane; x <= b; x += 64) {
        float mt, me;
        pixel_maxima<N>(p.px_out, p.out_rowstride, 0, w1, p.h, BPP, SEM, x, y, mt, me);
        emit_pixel(p, mt, me, p.map_out + (long long)y * p.map_out_stride + x,
                   (unsigned)(y * w1 + x));
    }
}

// energies at listed pixels: one thread per point
template <int N, int BPP, int SEM>
__global__ __launch_bounds__(256) void dcte_points(const SeamParams p)
{
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= p.count) return;
    const int x = clamp_px(p.pts[2 * k], 0, p.w - 1), y = clamp_px(p.pts[2 * k + 1], 0, p.h - 1);
    float mt, me;
    pixel_maxima<N>(p.px, p.rowstride, p.in_row0, p.w, p.h, BPP, SEM, x, y, mt, me);
    emit_pixel(p, mt, me, p.map_out + k, (unsigned)k);
}

// ------------------------------------------------------------------ launchers
#define DCTE_SEM_BPP_SWITCH(KERNEL, N, grid, block, s, p)                                        \
    do {                                                                                        \
        if ((p).sem == kSemLqr) {                                                               \
            if ((p).bpp == 1) { hipLaunchKernelGGL((KERNEL<N, 1, kSemLqr>), grid, block, 0, s, p); break; }     \
            if ((p).bpp == 3) { hipLaunchKernelGGL((KERNEL<N, 3, kSemLqr>), grid, block, 0, s, p); break; }     \
        } else {                                                                                \
            if ((p).bpp == 1) { hipLaunchKernelGGL((KERNEL<N, 1, kSemPreview>), grid, block, 0, s, p); break; } \
            if ((p).bpp == 3) { hipLaunchKernelGGL((KERNEL<N, 3, kSemPreview>), grid, block, 0, s, p); break; } \
            if ((p).bpp == 4) { hipLaunchKernelGGL((KERNEL<N, 4, kSemPreview>), grid, block, 0, s, p); break; } \
        }                                                                                       \
        return hipErrorInvalidValue;                                                            \
    } while (0)

template <int N>
static hipError_t launch_band_n(const SeamParams& p, hipStream_t s)
{
    dim3 grid((p.h + 3) / 4), block(256);
    DCTE_SEM_BPP_SWITCH(dcte_seam_band, N, grid, block, s, p);
    return hipGetLastError();
}

template <int N>
static hipError_t launch_points_n(const SeamParams& p, hipStream_t s)
{
    dim3 grid((p.count + 255) / 256), block(256);
    DCTE_SEM_BPP_SWITCH(dcte_points, N, grid, block, s, p);
    return hipGetLastError();
}

hipError_t launch_seam_carve(const SeamParams& p, hipStream_t s)
{
    if (p.w < 2 || p.h < 1) return hipErrorInvalidValue;
    dim3 grid((p.w - 1 + 255) / 256, p.h), block(256);
    switch (p.bpp) {
    case 1: hipLaunchKernelGGL(dcte_seam_shift<1>, grid, block, 0, s, p); break;
    case 3: hipLaunchKernelGGL(dcte_seam_shift<3>, grid, block, 0, s, p); break;
    case 4: hipLaunchKernelGGL(dcte_seam_shift<4>, grid, block, 0, s, p); break;
    default: return hipErrorInvalidValue;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    switch (p.n) {
    case 2: return launch_band_n<2>(p, s);
    case 4: return launch_band_n<4>(p, s);
    case 8: return launch_band_n<8>(p, s);
    case 16: return launch_band_n<16>(p, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_points(const SeamParams& p, hipStream_t s)
{
    if (p.count <= 0) return hipSuccess;
    switch (p.n) {
    case 2: return launch_points_n<2>(p, s);
    case 4: return launch_points_n<4>(p, s);
    case 8: return launch_points_n<8>(p, s);
    case 16: return launch_points_n<16>(p, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace dcte
