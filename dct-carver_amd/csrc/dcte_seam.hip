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

constexpr unsigned kRawBufFlags = 0x00020000u;   // gfx9 raw buffer dword3 (as dcte_map)
constexpr int kShiftThreads = 256;
#ifndef DCTE_SHIFT_VEC
#define DCTE_SHIFT_VEC 2                    // 16-byte blocks per thread per pass (8 KB per pass)
#endif
constexpr int kShiftVec = DCTE_SHIFT_VEC;

// One workgroup per row.  New row bytes [o0, o1) come from old byte
// b + (b >= s*bpp ? bpp : 0); new map entries x come from old x (left of the
// recomputed band) or x + 1 (right of it).  Both move in 16-byte destination
// blocks: a frame block's 16 source bytes (any alignment) are one dwordx4 +
// one dword from the aligned dword below them, funnel-shifted
// (v_alignbyte); a map block's 4 source floats are one dword-aligned
// dwordx4.  INPLACE (px_out == px, same row stride; map likewise): only the
// part right of the seam moves (o0 = s*bpp), every pass loads all its sources
// before the barrier and stores after it, and a pass never reads bytes an
// earlier pass wrote (sources lie at or right of the destinations); the
// <= 15 unaligned head bytes (<= 3 head floats) are loaded first and the
// <= 15 tail bytes (<= 3 floats), read as sources by the last blocks, are
// stored last.
template <int BPP, bool INPLACE>
__global__ __launch_bounds__(kShiftThreads) void dcte_seam_shift(const SeamParams p)
{
    using u4 = unsigned int __attribute__((ext_vector_type(4)));
    const int y = blockIdx.x;
    const int tx = threadIdx.x;
    const int w = p.w, w1 = w - 1;
    const int s = clamp_px(p.seam[y], 0, w - 1);
    int lo, hi;
    seam_span(p.seam, w, p.h, p.n, p.sem, y, lo, hi);
    const int HL = halo_left(p.n, p.sem), HR = p.n - 1 - HL;

    // ---- frame bytes
    const uintptr_t ib = reinterpret_cast<uintptr_t>(p.px);
    const uint32_t iofs = (uint32_t)(ib & 3u);
    // records rounded up to whole dwords: every load below lies inside them
    // (a block's sources end at most at the row's end), and the aligned
    // dword holding the frame's last byte never crosses a page
    const uint32_t nrec =
        (iofs + (uint32_t)((long long)(p.h - 1) * p.rowstride) + (uint32_t)(w * BPP) + 3u) & ~3u;
    __amdgpu_buffer_rsrc_t in = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(ib - iofs), (short)0, (int)nrec, (int)kRawBufFlags);
    const uint32_t irow = iofs + (uint32_t)((long long)y * p.rowstride);   // row y in `in`
    uint8_t* orow = p.px_out + (long long)y * p.out_rowstride;
    const int sb = s * BPP;
    const int o0 = INPLACE ? sb : 0, o1 = w1 * BPP;
    auto src = [&](int b) -> uint32_t { return irow + (uint32_t)(b + (b >= sb ? BPP : 0)); };
    // 16 bytes starting at byte q of `in`
    auto load16 = [&](uint32_t q) -> u4 {
        const uint32_t a = q & ~3u, sh = q & 3u;
        const u4 v = __builtin_amdgcn_raw_buffer_load_b128(in, (int)a, 0, 0);
        const uint32_t e = __builtin_amdgcn_raw_buffer_load_b32(in, (int)(a + 16u), 0, 0);
        u4 r;
        r.x = __builtin_amdgcn_alignbyte(v.y, v.x, sh);
        r.y = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
        r.z = __builtin_amdgcn_alignbyte(v.w, v.z, sh);
        r.w = __builtin_amdgcn_alignbyte(e, v.w, sh);
        return r;
    };
    // 16-byte-aligned destination blocks [d0, d1), head [o0, d0), tail [d1, o1)
    const int mis = (int)(reinterpret_cast<uintptr_t>(orow) & 15u);
    int d0 = o0 + ((16 - ((mis + o0) & 15)) & 15);
    if (d0 > o1) d0 = o1;
    const int d1 = d0 + ((o1 - d0) & ~15);
    uint8_t edge_v = 0;                               // one head/tail byte per thread < 30
    int edge_b = -1;
    if (tx < 15 && o0 + tx < d0) edge_b = o0 + tx;
    if (tx >= 15 && tx < 30 && d1 + (tx - 15) < o1) edge_b = d1 + (tx - 15);
    if (edge_b >= 0) edge_v = (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(in, (int)src(edge_b), 0, 0);
    for (int base = d0; base < d1; base += 16 * kShiftThreads * kShiftVec) {
        u4 v[kShiftVec];
#pragma unroll
        for (int k = 0; k < kShiftVec; k++) {
            const int b = base + 16 * (tx + k * kShiftThreads);
            v[k] = u4{0u, 0u, 0u, 0u};
            if (b < d1) {
                if (INPLACE || b >= sb) {
                    v[k] = load16(irow + (uint32_t)(b + BPP));
                } else if (b + 16 <= sb) {
                    v[k] = load16(irow + (uint32_t)b);
                } else {                                   // the block straddling the seam
                    uint32_t d[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                    for (int j = 0; j < 16; j++)
                        d[j >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(in, (int)src(b + j), 0, 0)
                                     << (8 * (j & 3));
                    v[k] = u4{d[0], d[1], d[2], d[3]};
                }
            }
        }
        if constexpr (INPLACE) __syncthreads();
#pragma unroll
        for (int k = 0; k < kShiftVec; k++) {
            const int b = base + 16 * (tx + k * kShiftThreads);
            if (b < d1) *reinterpret_cast<u4*>(orow + b) = v[k];
        }
    }

    // ---- map: rows of floats (4-byte aligned)
    const float* mrow = p.map + (long long)y * p.map_stride;
    float* nrow = p.map_out + (long long)y * p.map_out_stride;
    // the source row through a buffer resource: dword-aligned dwordx4 loads
    __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(mrow), (short)0,
                                                                   w * 4, (int)kRawBufFlags);
    // left part [0, lo - HR) keeps x; right part [r0, w1) takes x + 1
    const int lend = max(0, min(w1, lo - HR));
    int r0 = hi + HL;                                  // first x with min(x - HL, w - 2) >= hi
    if (hi > w - 2) r0 = w1;
    r0 = max(r0, 0);
    if constexpr (!INPLACE) {
        for (int x = tx; x < lend; x += kShiftThreads) nrow[x] = mrow[x];
    }
    // 4-float destination blocks [x0, x1) (16-byte aligned), head [r0, x0), tail [x1, w1)
    const int mmis = (int)((reinterpret_cast<uintptr_t>(nrow) >> 2) & 3u);
    int x0 = r0 + ((4 - ((mmis + r0) & 3)) & 3);
    if (x0 > w1) x0 = w1;
    const int x1 = x0 + ((w1 - x0) & ~3);
    float medge_v = 0.0f;                              // one head/tail float per thread in [32, 38)
    int medge_x = -1;
    if (tx >= 32 && tx < 35 && r0 + (tx - 32) < x0) medge_x = r0 + (tx - 32);
    if (tx >= 35 && tx < 38 && x1 + (tx - 35) < w1) medge_x = x1 + (tx - 35);
    if (medge_x >= 0) medge_v = mrow[medge_x + 1];
    for (int base = x0; base < x1; base += 4 * kShiftThreads * kShiftVec) {
        u4 v[kShiftVec];
#pragma unroll
        for (int k = 0; k < kShiftVec; k++) {
            const int x = base + 4 * (tx + k * kShiftThreads);
            v[k] = x < x1 ? __builtin_amdgcn_raw_buffer_load_b128(mr, (x + 1) * 4, 0, 0) : u4{0u, 0u, 0u, 0u};
        }
        if constexpr (INPLACE) __syncthreads();
#pragma unroll
        for (int k = 0; k < kShiftVec; k++) {
            const int x = base + 4 * (tx + k * kShiftThreads);
            if (x < x1) *reinterpret_cast<u4*>(nrow + x) = v[k];
        }
    }
    if constexpr (INPLACE) __syncthreads();
    if (edge_b >= 0) orow[edge_b] = edge_v;
    if (medge_x >= 0) nrow[medge_x] = medge_v;
}

__device__ __forceinline__ void emit_pixel(const SeamParams& p, float mt, float me, float* dst,
                                           unsigned fix_index)
{
    const bool edge = me > mt;                      // as in dcte_map's emit
    const float hi = edge ? me : mt, lo = edge ? mt : me;
    *dst = hi * (edge ? p.we : p.wt);        // the map kernel's decision (dcte_map emit)
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

// Band of one carver step (dcte_carver_step): after seam s removed from a
// frame, row y of the carved w-wide frame keeps, from column x0[y] on, `bw`
// energies and pixels -- x0[y] = lo - 2R - 1 clamped to [0, max(0, w - bw)],
// lo = min of s over rows y - 2R .. y + 2R.  The band holds every pixel
// liblqr re-evaluates after the step (columns min s - R .. max s + R - 1 over
// the seam rows within R [liblqr, unverified]) AND every pixel of those
// pixels' N x N reading windows (render.c:146-152: x - (R - 1) .. x + R, rows
// likewise), so the plug-in hook can check a callback's whole window against
// the mirror before it serves: the seam moves <= 1 column per row, so over
// the 4R + 1 rows that decide x0[y] it spans <= 4R columns, and bw = 8 R + 4
// covers it.  One wave per row.
__global__ __launch_bounds__(64) void dcte_band_gather(const BandParams p)
{
    const int y = blockIdx.x, l = threadIdx.x;
    int lo = p.w;
    for (int j = -2 * p.r; j <= 2 * p.r; j++) lo = min(lo, p.seam[clamp_px(y + j, 0, p.h - 1)]);
    const int x0 = clamp_px(lo - 2 * p.r - 1, 0, max(0, p.w - p.bw));
    if (l == 0) p.x0[y] = x0;
    for (int k = l; k < p.bw; k += 64) {
        const int x = min(x0 + k, p.w - 1);
        p.e[(long long)y * p.bw + k] = p.map[(long long)y * p.map_stride + x];
        for (int c = 0; c < p.bpp; c++)
            p.pxb[((long long)y * p.bw + k) * p.bpp + c] = p.px[(long long)y * p.rowstride + (long long)x * p.bpp + c];
    }
}

hipError_t launch_band_gather(const BandParams& p, hipStream_t s)
{
    if (p.h <= 0) return hipSuccess;
    hipLaunchKernelGGL(dcte_band_gather, dim3(p.h), dim3(64), 0, s, p);
    return hipGetLastError();
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
    dim3 grid(p.h), block(kShiftThreads);
    const bool inplace = p.px_out == p.px && p.out_rowstride == p.rowstride &&
                         p.map_out == p.map && p.map_out_stride == p.map_stride;
#define DCTE_SHIFT(B)                                                                        \
    case B:                                                                                  \
        if (inplace) hipLaunchKernelGGL((dcte_seam_shift<B, true>), grid, block, 0, s, p);  \
        else hipLaunchKernelGGL((dcte_seam_shift<B, false>), grid, block, 0, s, p);         \
        break;
    switch (p.bpp) {
        DCTE_SHIFT(1)
        DCTE_SHIFT(3)
        DCTE_SHIFT(4)
    default: return hipErrorInvalidValue;
    }
#undef DCTE_SHIFT
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
