// dcte_kernels.hip -- gfx950 kernels for the dct-carver energy map.
//
// What is computed (reference: src/render.c:134-157 + src/dct.c:77-110):
// for every pixel (x, y) the N x N luma window with offsets -(N/2-1)..N/2 in
// both axes (replicate-clamped at the image border), its 2-D DCT-II, and
//     E = m_e > m_t ? m_e * edges : m_t * textures
// with m_e = max(|C01|, |C10|) and m_t = max over the other non-DC
// coefficients -- the reference's last-maximum scan reduced to a comparison
// (SURVEY.md §0.5).
//
// How (VALU-bound design, no MFMA -- see DESIGN.md §3):
//  * A workgroup owns a strip of TW output columns x tile_h output rows and
//    walks DOWN it.  Each input row is DCT-transformed along x exactly once
//    (row pass) and kept in a register ring of the last N row transforms;
//    every output pixel then only needs the N column transforms over the
//    ring (N + 1 one-dimensional transforms per pixel instead of 2N).
//  * Pixels arrive as raw bytes: one 32-bit buffer load per lane per row
//    (bounds-checked buffer resource, no over-read), prefetched one group of
//    G rows ahead in registers, staged through LDS, converted to the exact
//    integer luma domain (dcte_luma.h), staged again, and read back as the
//    N-wide row windows.  For N <= 8 both stages are double-buffered: one
//    barrier per group of G rows.
//  * N = 16 splits the 16 horizontal frequencies of a column over the four
//    waves of a workgroup (4 k1 channels each: a 16 x 4 register ring).
//  * Pixels whose edge/texture decision falls inside the fp32 error band are
//    appended to a list and recomputed by dcte_fix in fp64, in the
//    reference's operation order.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <utility>

#include "dcte_kernels.h"
#include "dcte_luma.h"
#include "dcte_math.h"
#include "dcte_passes.h"
#include "dcte_ref64.h"

namespace dcte {

// Build-time tuning values.  Each can be overridden with -D (tools/variants.sh
// builds such variants for A/Bs on the GPU; tests/test_knob_builds.py compiles
// every one of them with a non-default value).  The losing code paths of
// earlier A/Bs are gone from the source; their records stay in profiles/.
#ifndef DCTE_WG8
#define DCTE_WG8 256       // threads per workgroup (= strip width) at N = 8 (64: +0.3 %, 4x the halo reads)
#endif
#ifndef DCTE_TILE_H
#define DCTE_TILE_H 128    // output rows per map workgroup, N <= 8
#endif
#ifndef DCTE_TILE_H16
#define DCTE_TILE_H16 128  // ... N = 16
#endif
#ifndef DCTE_G8
#define DCTE_G8 8          // rows per staging group for N = 8 (multiple of 8)
#endif
#ifndef DCTE_MIN_WAVES
#define DCTE_MIN_WAVES 4   // __launch_bounds__ minimum waves per SIMD (<= 128 VGPRs)
#endif
#ifndef DCTE_MIN_WAVES16
#define DCTE_MIN_WAVES16 4 // the same for N = 16 (it would take 134 VGPRs and 3 waves: -2 % with the cap)
#endif
#ifndef DCTE_TSTAMP
#define DCTE_TSTAMP 0      // timing-probe builds: per-workgroup timestamps (tools/tstamp.py)
#endif
#ifndef DCTE_PF2_MAXN
#define DCTE_PF2_MAXN 4    // N <= this: raw rows prefetched two groups ahead (else one)
#endif
constexpr int kPrio = 1;   // wave priority while staging / converting a group (A/B: -2 % at N = 8 and 16)
constexpr unsigned kBufFlags = 0x00020000u;  // gfx9 raw buffer dword3

// refinement (below): strips with at most kFixDirect<N> flagged pixels are
// "sparse" (dcte_fix_strips gathers their windows directly), the rest dense
#ifndef DCTE_FIX_DIRECT4
#define DCTE_FIX_DIRECT4 16u    // N = 4 (lane walk since r04)
#endif
#ifndef DCTE_FIX_DIRECT8
#define DCTE_FIX_DIRECT8 16u    // N = 8: most flagged pixels a strip may hold and still be sparse (128 before: dots +47 %, text +4 %; profiles/r03/fix_direct_ab.jsonl)
#endif
// (N = 2, 4 keep r02's 128: their dense strips take the band path of
// dcte_fix_strips, which that value was tuned for, profiles/r02/fix_direct.jsonl)
template <int N>
constexpr unsigned kFixDirect = N == 16 ? 32u : (N == 8 ? (unsigned)DCTE_FIX_DIRECT8
                                                          : (N == 4 ? (unsigned)DCTE_FIX_DIRECT4 : 128u));
// dense strips walked by a lane-per-pixel (N = 4, 8, fix_dense_lane) /
// lane-quad-per-pixel (N = 16 liblqr, fix_dense16_flat) walk rather than the
// band path of dcte_fix_strips
template <int N, int SEM>
constexpr bool kDenseOwn = N == 8 || N == 4 || N == 16;
// ... N = 16 from the flat list the map kernel numbers (MapParams::dense_list)
template <int N, int SEM>
constexpr bool kDenseFlat = N == 16 && kDenseOwn<N, SEM>;
// entries per refinement batch of the flat list (a quad of lanes per pixel)
constexpr unsigned kDenseBatch16 = 16u;
static_assert(kFixDirect<16> >= kDenseBatch16, "N = 16 dense batches");

// SEM = kSemLqr    : liblqr callback window, offsets -(N/2-1)..N/2
//                    (src/render.c:146-152), liblqr luma (dcte_luma.h)
// SEM = kSemPreview: GTK preview window, offsets -(c-1)..N-c with
//                    c = (N-1)/2 (src/dct.h:8-9, src/render.c:43-44, 461),
//                    u8 luma RGB2LUMINANCE (src/render.h:5)
template <int N>
struct MapThreads {
    static constexpr int value = N == 8 ? DCTE_WG8 : 256;
    // 4 waves per SIMD: <= 128 VGPRs (N = 8 needs 113; N = 16 would take 134
    // and drop to 3 waves: A/B -2 % with the cap)
    static constexpr int min_waves = N == 16 ? DCTE_MIN_WAVES16 : DCTE_MIN_WAVES;
};

template <int N, int SEM>
struct Geo {
    static constexpr int T = MapThreads<N>::value;       // threads per workgroup
    static constexpr int S = Lanes<N>::S;                // lanes per output column
    static constexpr int CH = Lanes<N>::CH;              // k1 channels per lane
    static constexpr int TW = T / S;              // output columns per WG
    static constexpr int HL = SEM == kSemLqr ? N / 2 - 1 : (N - 1) / 2 - 1;   // halo left / top
    static constexpr int HR = N - 1 - HL;                                     // halo right / bottom
    static constexpr int LW = TW + N - 1;                // luma columns per row
    static constexpr int LWP = LW | 1;                   // odd row pitch
    static constexpr int G = (N < 8) ? 8 : (N == 8 ? DCTE_G8 : N);  // rows per group (multiple of N)
    template <int BPP>
    static constexpr int ndw() { return (LW * BPP + 3) / 4 + 1; }  // dwords per raw row
    template <int BPP>
    static constexpr int dpt() { return (ndw<BPP>() + T - 1) / T; }  // per lane
};

template <int... Is, class F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, Is...>, F&& f)
{
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int Count, class F>
__device__ __forceinline__ void static_for(F&& f)
{
    static_for_impl(std::make_integer_sequence<int, Count>{}, f);
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// forward declarations (refinement section below)
template <int N, class Line>
__device__ __forceinline__ void refine_group_f(Line&& line, double* w, int l, double& best, bool& edge);

// N = 8: the sparse strips of a map tile refined by the map launch itself,
// after its last row (a small frame's call paid a second
// launch for a few hundred flagged pixels).  Wave w owns strip w of the tile
// (cnt flagged pixels at el[0 .. cnt), cnt <= kFixDirect: the rest go to
// dcte_fix_strips as before).  Four pixels per pass, one 8-lane group each
// (lanes 32-63 repeat lanes 0-31's pixels: same values into the same LDS);
// the window gathered from the frame with the replicate clamp of
// src/render.c:146-152, liblqr luma in double [liblqr, unverified] / the
// preview's RGB2LUMINANCE, ddct8x8s and the last-maximum scan in the
// reference's order (refine_group_f) -- the bits dcte_fix_strips produces.
// lds: the map's luma buffer, free after its last barrier (>= 256 + waves x
// 4 x 72 doubles).  Every thread of the workgroup calls it.
template <int N, int BPP, int SEM>
__device__ __forceinline__ void map_refine_sparse(const MapParams& p, double* lds, unsigned cnt,
                                                  const unsigned* el, int sx0, int ys, int tx, int nthreads)
{
    constexpr int HL = Geo<N, SEM>::HL;
    double* const lut = lds;                         // v / 255 (liblqr)
    for (int v = tx; v < 256; v += nthreads) lut[v] = (double)v / 255;
    __syncthreads();
    if (cnt - 1u >= (unsigned)kFixDirect<N>) return;   // uniform per wave: nothing, or dcte_fix_strips'
    const int lane = tx & 63, l = lane & (N - 1), grp = (lane / N) & 3;
    double* const w = lds + 256 + ((tx >> 6) * 4 + grp) * (N * (N + 1));
    auto luma = [&](const uint8_t* q) -> double {
        if constexpr (SEM == kSemLqr) {
            if constexpr (BPP == 1) return lut[q[0]];
            else return 0.2126 * lut[q[0]] + 0.7152 * lut[q[1]] + 0.0722 * lut[q[2]];
        } else {
            return (double)preview_luma(q[0], BPP > 1 ? q[1] : 0u, BPP > 1 ? q[2] : 0u, BPP);
        }
    };
    for (unsigned e0 = 0; e0 < cnt; e0 += 4) {       // uniform
        const unsigned e = e0 + (unsigned)grp;
        const bool valid = e < cnt;
        const unsigned loc = el[valid ? e : 0u];
        const int x = sx0 + (int)(loc & 63u), y = ys + (int)(loc >> 6);
        double best;
        bool edge;
        // lane l: liblqr data[i][l] = pixel (x - HL + i, y - HL + l); preview
        // data[i][l] = data[dy = i][dx = l]
        refine_group_f<N>([&](int i) {
            const int ox = SEM == kSemLqr ? i : l, oy = SEM == kSemLqr ? l : i;
            const int gx = clampi(x - HL + ox, 0, p.w - 1), gy = clampi(y - HL + oy, 0, p.h - 1);
            return luma(p.px + (long long)(gy - p.in_row0) * p.rowstride + (long long)gx * BPP);
        }, w, l, best, edge);
        if (valid && l == 0 && lane < 32)
            p.out[(long long)(y - p.y0) * p.out_stride + x] =
                edge ? (float)(best * (double)p.edges) : (float)(best * (double)p.textures);
    }
    if (p.fix_total && lane == 0) atomicAdd(p.fix_total, cnt);
}

// ------------------------------------------------------------------ main kernel
template <int N, int BPP, int SEM>
__global__ __launch_bounds__((Geo<N, SEM>::T), MapThreads<N>::min_waves) void dcte_map(const MapParams p)
{
    using Gm = Geo<N, SEM>;
    constexpr int kThreads = Gm::T;
    constexpr int S = Gm::S, CH = Gm::CH, TW = Gm::TW, HL = Gm::HL;
    constexpr int LW = Gm::LW, LWP = Gm::LWP, G = Gm::G;
    constexpr int NDW = Gm::template ndw<BPP>();
    constexpr int DPT = Gm::template dpt<BPP>();         // raw dwords per lane per row

    // N <= 8: raw / lum double-buffered, so a row group needs one barrier
    // (N = 16 keeps one buffer and three barriers per group: double-buffered
    // luma and partial maxima with one barrier per group measured no faster,
    // staged (+0.1 %) or with direct loads (+2.5 %), profiles/r05/n16_pipeline_ab.jsonl --
    // this kernel is VALU-bound, not barrier-bound)
    constexpr bool kDB = S == 1;
    constexpr int NB = kDB ? 2 : 1;
    // the direct loads (below) need no raw stage
    // raw rows two groups ahead (N <= 4; N = 4 colour layers take the direct
    // loads below instead: 16384^2 RGB 0.534 -> 0.486 ms; grey and N = 2 are
    // faster two groups ahead, profiles/r05/small_n_direct_ab.jsonl)
    constexpr bool kPF2 = S == 1 && N <= DCTE_PF2_MAXN && !(N == 4 && BPP >= 3);
    constexpr bool kDirectLds = S == 1 && kDB && !kPF2 &&
                                LW - kThreads > 0 && (LW - kThreads) * G <= 64;
    __shared__ uint32_t raw[kDirectLds ? 1 : NB][kDirectLds ? 1 : G][kDirectLds ? 1 : NDW];
    __shared__ __attribute__((aligned(16))) float lum[NB][G][LWP];
    // S = 4 (N = 16): the group's rows' maxima over the four waves, met by
    // LDS atomic max on the bits (non-negative floats order as their bits);
    // only the waves owning k1 = 0 (q = 0) and k1 = 1 (q = 2) carry an edge
    // candidate.  Zero between uses (the combine resets what it read).  One
    // slot per pixel and ds_max instead of a slot per wave and three fmax:
    // -0.7 % per launch (profiles/r05/n16_pipeline_ab.jsonl)
    __shared__ uint32_t part_t[S == 4 ? G : 1][S == 4 ? 64 : 1];
    __shared__ uint32_t part_e[S == 4 ? G : 1][S == 4 ? 64 : 1];
    // refinement lists per 64-column strip (one wave's columns; N = 16: the tile)
    constexpr int SPT = S == 1 ? TW / 64 : 1;        // strips per tile
    __shared__ unsigned nflag[SPT];                  // pixels each strip flagged
    // N = 8: a strip with at most kFixDirect flagged pixels is refined by its
    // own wave after the last row (map_refine_sparse), not by dcte_fix_strips;
    // its entries are kept here as well
    constexpr bool kEpi = N == 8 && S == 1;
    constexpr unsigned kEpiMax = kFixDirect<N>;
    __shared__ unsigned elist[kEpi ? SPT : 1][kEpi ? kEpiMax : 1];

    const int tx = threadIdx.x;
    const int lane_p = (S == 4) ? (tx >> 6) : 0;     // N = 16: wave index = k1 class
    const int c = (S == 4) ? (tx & 63) : tx;         // output column within the strip
    // Workgroups are dealt round-robin over the 8 XCDs in dispatch order; the
    // remap gives each XCD a contiguous run of tiles (strips of a row band in
    // order), so the N - 1 halo columns two neighbouring strips both read
    // come from one L2 instead of being fetched twice.
#if DCTE_TSTAMP
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
    int bx = blockIdx.x, by = blockIdx.y;
    {
        const int nwg = gridDim.x * gridDim.y, L = blockIdx.x + gridDim.x * blockIdx.y;
        const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
        const int T = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
        bx = T % gridDim.x;
        by = T / gridDim.x;
    }
    const int x0 = bx * TW;
    const int x = x0 + c;
    const int ys = tile_row0(p, by);
    const int ye = tile_row1(p, by);
    const int n_in = (ye - ys) + N - 1;
    const int ngroups = (n_in + G - 1) / G;
    const int w = p.w, h = p.h;

    // raw byte span of one input row: columns [xs, xs + span) of the strip
    const int xs = min(max(0, x0 - HL), w - 1);
    // buffer resource over the readable rows (aligned base; OOB loads read 0)
    const uintptr_t pbase = reinterpret_cast<uintptr_t>(p.px);
    const uint32_t base_off = (uint32_t)(pbase & 3u);
    const unsigned nrec = base_off + (unsigned)((long long)(p.in_rows - 1) * p.rowstride) +
                          (unsigned)(w * BPP);
    const unsigned nrec4 = nrec & ~3u;                // bytes covered by whole dwords
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(pbase - base_off), (short)0, (int)nrec, (int)kBufFlags);

    auto row_start = [&](int i) -> uint32_t {       // byte offset of (xs, row i)
        int t = clampi(ys - HL + i, 0, h - 1);
        return base_off + (uint32_t)((long long)(t - p.in_row0) * p.rowstride) +
               (uint32_t)(xs * BPP);
    };

    // A dword straddling the end of the readable bytes reads as 0 (buffer
    // bounds are checked per dword).  The workgroups whose span reaches the
    // last readable row's last pixel fetch those <= 3 tail bytes once here and
    // patch them in when staging raw rows.
    const bool tail_wg = (nrec & 3u) != 0u && x0 + TW + Gm::HR - 1 >= w - 1 &&
                         min(h - 1, ye - 1 + Gm::HR) >= p.in_row0 + p.in_rows - 1;
    uint32_t tail = 0;
    if (tail_wg) {
        for (uint32_t b = 0; b < (nrec & 3u); b++)
            tail |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, (int)(nrec4 + b), 0, 0) << (8u * b);
    }

    // raw rows in flight: PFD groups ahead (two register buffers for the
    // small blocks, whose launches are bound by loads in flight, not VALU)
    constexpr int PFD = kPF2 ? 2 : 1;
    uint32_t pref[PFD][G][DPT];
    auto issue = [&](int g, auto PB) {
#pragma unroll
        for (int u = 0; u < G; u++) {
            int i = g * G + u;
            uint32_t a = row_start(i < n_in ? i : n_in - 1) & ~3u;
#pragma unroll
            for (int q = 0; q < DPT; q++) {
                const int dw = tx + q * kThreads;
                pref[PB][u][q] = (dw < NDW) ? __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)(a + 4u * dw), 0, 0) : 0u;
            }
        }
    };

    // Direct loads (N = 8): no raw stage in LDS.  Each lane fetches the bytes
    // of its own column of each row of a group with one 8-byte buffer load
    // (any alignment: the pixel's <= 4 bytes lie inside it), one group ahead,
    // and converts them straight from registers; the last wave's lanes also
    // fetch the N - 1 halo columns' pixels (one (row, column) each, as in
    // convert()).
    // The convert phase then waits on no LDS reads.
    constexpr int XH = LW - kThreads;                  // halo columns past one per lane
    constexpr bool kDirect = S == 1 && kDB && PFD == 1 && XH > 0 && XH * G <= 64;
    static_assert(kDirect == kDirectLds, "raw stage sizing");
    uint32_t dlo[kDirect ? G : 1], dhi[kDirect ? G : 1];
    uint32_t xlo = 0, xhi = 0;
    const int hlane = tx - (kThreads - 64);
    const bool has_halo = kDirect && hlane >= 0 && hlane < XH * G;
    const int hrow = has_halo ? hlane / XH : 0, hcc = has_halo ? kThreads + hlane % XH : 0;
    auto col_bytes = [&](int cc) -> uint32_t {         // byte offset of column cc from xs
        return (uint32_t)((clampi(x0 - HL + cc, 0, w - 1) - xs) * BPP);
    };
    auto fetch2 = [&](uint32_t a) __attribute__((always_inline)) {
        const uint32_t a4 = a & ~3u;
        auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)a4, 0, 0);
        if (tail_wg) {                                  // uniform; a handful of WGs
            if (a4 == nrec4) v[0] = tail;
            else if (a4 + 4u == nrec4) v[1] = tail;
        }
        return v;
    };
    auto issue_direct = [&](int g) __attribute__((always_inline)) {
        if constexpr (kDirect) {
#pragma unroll
            for (int u = 0; u < G; u++) {
                const int i = g * G + u;
                const auto v = fetch2(row_start(i < n_in ? i : n_in - 1) + col_bytes(tx));
                dlo[u] = v[0];
                dhi[u] = v[1];
            }
            if (has_halo) {
                const int i = g * G + hrow;
                const auto v = fetch2(row_start(i < n_in ? i : n_in - 1) + col_bytes(hcc));
                xlo = v[0];
                xhi = v[1];
            }
        }
    };
    auto luma_bytes = [&](uint32_t wd) -> float {       // exact integer luma (biased) of a pixel's bytes
        const uint32_t c0 = wd & 255u, c1 = BPP >= 3 ? (wd >> 8) & 255u : 0u, c2 = BPP >= 3 ? (wd >> 16) & 255u : 0u;
        int L;
        if constexpr (SEM == kSemLqr && BPP >= 3) {
            // L = 1063 R + 3576 G + 361 B - 637500 with the byte dot products:
            // the weights split into 256 hi + lo (4 / 39, 13 / 248, 1 / 105),
            // the bias in the lo sum's accumulator (mod 2^32); the fourth byte
            // weighs 0.  Exact, the same integer as below
            constexpr uint32_t kLo = 39u | 248u << 8 | 105u << 16, kHi = 4u | 13u << 8 | 1u << 16;
            static_assert(39 + 4 * 256 == kLumaR && 248 + 13 * 256 == kLumaG && 105 + 1 * 256 == kLumaB, "split weights");
            const uint32_t lo = __builtin_amdgcn_udot4(wd, kLo, (uint32_t)-kLumaBias, false);
            const uint32_t hi = __builtin_amdgcn_udot4(wd, kHi, 0u, false);
            return (float)(int)((hi << 8) + lo);
        } else if constexpr (SEM == kSemLqr) {
            L = (BPP == 1) ? kLumaGrey * (int)c0
                           : kLumaR * (int)c0 + kLumaG * (int)c1 + kLumaB * (int)c2;
            L -= kLumaBias;
        } else {
            L = (int)preview_luma(c0, c1, c2, BPP) - kPreviewBias;
        }
        return (float)L;
    };
    auto convert_direct = [&](int g, int b) __attribute__((always_inline)) {
        if constexpr (kDirect) {
#pragma unroll
            for (int u = 0; u < G; u++) {
                const int i = g * G + u;
                const uint32_t off = (row_start(i < n_in ? i : n_in - 1) + col_bytes(tx)) & 3u;
                lum[b][u][tx] = luma_bytes(__builtin_amdgcn_alignbyte(dhi[u], dlo[u], off));
            }
            if (has_halo) {
                const int i = g * G + hrow;
                const uint32_t off = (row_start(i < n_in ? i : n_in - 1) + col_bytes(hcc)) & 3u;
                lum[b][hrow][hcc] = luma_bytes(__builtin_amdgcn_alignbyte(xhi, xlo, off));
            }
        }
    };

    float ring[N][CH];
    const float we = p.we, wt = p.wt;
    // output rows [ys, ye) of this workgroup through one buffer resource
    const int ostride4 = (int)(p.out_stride * 4);
    const uint32_t orec = (unsigned)(max(ye - ys - 1, 0)) * (unsigned)ostride4 + (unsigned)w * 4u;
    __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        p.out + (long long)(ys - p.y0) * p.out_stride, (short)0, (int)orec, (int)kBufFlags);
    // refinement lists of this tile's strips (dcte_fix_strips); nflag is set
    // before the first barrier and read after the last one
    const int sc = S == 1 ? c >> 6 : 0;              // this thread's strip in the tile
    const unsigned strip = (unsigned)(by * gridDim.x + bx) * SPT + sc;
    unsigned* strip_list = p.fix_list + (size_t)strip * (size_t)(64 * p.tile_h);
    const int sx0 = x0 + 64 * sc;                    // first column of the strip
    if (tx < SPT) nflag[tx] = 0;
    if constexpr (S == 4) {
        for (int e = tx; e < G * 64; e += kThreads) {
            (&part_t[0][0])[e] = 0u;
            (&part_e[0][0])[e] = 0u;
        }
    }
    // the next launch's dirty-strip and dense counters (stream order: nothing
    // reads them before this launch ends) -- in every launch, whatever its N
    // or semantics: the phases alternate over all launches of the stream
    if (tx == 0 && blockIdx.x == 0 && blockIdx.y == 0) {
        *p.dirty_next = 0u;
        *p.dense_next = 0ull;
    }
    const bool check_ties = we != wt;                // uniform
    const bool force_all = p.tie_tau >= 1.0f;        // uniform
    const float keep = 1.0f - p.tie_tau;             // |me - mt| <= tau * hi  <=>  lo >= (1 - tau) hi

    // decision + store (+ refinement flag) of output pixel (x, y)
    auto emit = [&](int y, int xx, float mt, float me) {
        // no branch on the column: a lane past the frame's last column stores
        // at the resource's size, which the bounds check drops (the wave's
        // row offset rides in soffset, so the sum stays below 2^32)
        const bool inside = xx < w;
        const uint32_t voff = inside ? (uint32_t)xx * 4u : orec;
        const bool edge = me > mt;
        // the product, then the select (the weights stay in SGPRs)
        const float e_out = me * we, t_out = mt * wt;
        // row offset is wave-uniform (soffset), column offset per lane
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(edge ? e_out : t_out), orsrc,
                                              (int)voff, (y - ys) * ostride4, 0);
        // refine in fp64 when the class is uncertain: the smaller maximum
        // within the fp32 error band of the larger, lo > (1 - tau) hi, i.e.
        // me > keep mt AND mt > keep me (never for all-zero windows); every
        // pixel when tie_tau >= 1 (testing)
        if (inside && ((check_ties && me > keep * mt && mt > keep * me) || force_all)) {
            const unsigned k = atomicAdd(&nflag[sc], 1u);      // < 64 * tile_h
            const unsigned loc = (unsigned)((y - ys) * 64 + (xx - sx0));
            strip_list[k] = loc;
            if constexpr (kEpi)
                if (k < kEpiMax) elist[sc][k] = loc;   // (read only when p.epi)
        }
    };

    // raw dwords of group gg (prefetched in pref[PB]) -> raw[b]
    auto stage = [&](int gg, int b, auto PB) {
#pragma unroll
        for (int q = 0; q < DPT; q++) {
            const int dw = tx + q * kThreads;
            if (dw < NDW) {
#pragma unroll
                for (int u = 0; u < G; u++) {
                    uint32_t v = pref[PB][u][q];
                    if (tail_wg) {                 // uniform; a handful of WGs
                        int i = gg * G + u;
                        uint32_t a = (row_start(i < n_in ? i : n_in - 1) & ~3u) + 4u * dw;
                        if (a == nrec4) v = tail;
                    }
                    raw[b][u][dw] = v;
                }
            }
        }
    };
    // bytes -> exact integer luma (biased) of row u of group gg, column cc
    auto luma_at = [&](int gg, int b, int u, int cc) {
        const int xc = clampi(x0 - HL + cc, 0, w - 1);
        const uint32_t off = (row_start(gg * G + u) & 3u) + (uint32_t)((xc - xs) * BPP);
        const uint8_t* rb = reinterpret_cast<const uint8_t*>(&raw[b][u][0]);
        uint32_t c0 = rb[off], c1 = 0, c2 = 0;
        if constexpr (BPP >= 3) {
            c1 = rb[off + 1];
            c2 = rb[off + 2];
        }
        int L;
        if constexpr (SEM == kSemLqr) {
            L = (BPP == 1) ? kLumaGrey * (int)c0
                           : kLumaR * (int)c0 + kLumaG * (int)c1 + kLumaB * (int)c2;
            L -= kLumaBias;
        } else {
            L = (int)preview_luma(c0, c1, c2, BPP) - kPreviewBias;
        }
        lum[b][u][cc] = (float)L;
    };
    auto convert = [&](int gg, int b) {
        constexpr int X = LW - kThreads;                 // halo columns past one per lane
        if constexpr (X > 0 && X * G <= 64) {
            // one column per lane for all G rows; the X * G halo conversions
            // go one per lane to the last wave instead of G rows to X lanes
            // of the first (which would hold the whole workgroup at the barrier)
#pragma unroll
            for (int u = 0; u < G; u++) luma_at(gg, b, u, tx);
            const int l = tx - (kThreads - 64);
            if (l >= 0 && l < X * G) luma_at(gg, b, l / X, kThreads + l % X);
        } else {
            for (int cc = tx; cc < LW; cc += kThreads) {
#pragma unroll
                for (int u = 0; u < G; u++) luma_at(gg, b, u, cc);
            }
        }
    };
    // row pass + column pass for the G rows of group g (luma in lum[b])
    auto compute = [&](int g, int b) __attribute__((always_inline)) {
        static_for<G>([&](auto U) {
            constexpr int u = decltype(U)::value;
            const int i = g * G + u;
            if (i < n_in) {
                if constexpr (N == 8) {
                    // the lane's row base, opaque to the optimiser: its 8 reads
                    // then pair into ds_read2 off ONE base (offsets 0..7)
                    // instead of one address add per pair
                    using lds_cfloat = const __attribute__((address_space(3))) float;
                    uint32_t a = (uint32_t)(uintptr_t)(lds_cfloat*)&lum[b][u][c];
                    asm volatile("" : "+v"(a));
                    row_pass<N>((const float*)(lds_cfloat*)(uintptr_t)a, 0, lane_p, ring[u % N]);
                } else {
                    row_pass<N>(&lum[b][u][0], c, lane_p, ring[u % N]);
                }
                if (i >= N - 1) {
                    float mt, me;
                    Cols<N>::template run<(u + 1) % N>(ring, lane_p, mt, me);
                    if constexpr (S == 4) {
                        atomicMax(&part_t[u][c], __float_as_uint(mt));
                        if ((lane_p & 1) == 0) atomicMax(&part_e[u][c], __float_as_uint(me));
                    } else {
                        emit(ys + i - (N - 1), x, mt, me);
                    }
                }
            }
        });
    };
    // N = 16: the four waves' maxima of group g (complete after a barrier
    // that follows every wave's compute(g)); wave q finishes rows u = q mod 4
    // and zeroes what it read
    auto combine = [&](int g) __attribute__((always_inline)) {
        if constexpr (S == 4) {
#pragma unroll
            for (int u = lane_p; u < G; u += 4) {
                const int i = g * G + u;
                if (i >= N - 1 && i < n_in)
                    emit(ys + i - (N - 1), x, __uint_as_float(part_t[u][c]), __uint_as_float(part_e[u][c]));
                part_t[u][c] = 0u;
                part_e[u][c] = 0u;
            }
        }
    };

    // Wave priority.  A wave stages and converts a group at a raised
    // priority so its workgroup reaches the barrier sooner (kPrio).  In
    // launches of one or two rounds (p.fair > 0, set by the host) the level
    // also falls as the workgroup gets through its tile: the hardware
    // otherwise favours the OLDEST waves of a SIMD, so of the workgroups
    // sharing a CU the first-dispatched finishes long before the last, and
    // the CU runs the launch's tail below occupancy (tools/tstamp.py, one
    // round of 128-row tiles: 115-202 us for identical tiles, 137-185 with
    // the falling level).
    const int fair = N == 8 ? p.fair : 0;            // uniform; the host sets it for N = 8 only
    auto set_prio = [&](bool staging, int g) __attribute__((always_inline)) {
        int lvl = staging ? kPrio : 0;
        if (fair > 0) lvl += (fair - 1) - min(fair - 1, g * fair / ngroups);
        if (lvl >= 3) __builtin_amdgcn_s_setprio(3);
        else if (lvl == 2) __builtin_amdgcn_s_setprio(2);
        else if (lvl == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    };
    constexpr std::integral_constant<int, 0> P0{};
    if constexpr (!kDirect) issue(0, P0);
    if constexpr (kDB && PFD == 2) {
        // As below, with groups g + 2 AND g + 3 in flight while group g is
        // computed: the group staged next comes from pref[(g + 1) & 1], which
        // is refilled with group g + 3 right after (loop unrolled by two so
        // the register buffers are indexed statically).
        constexpr std::integral_constant<int, 1> P1{};
        if (ngroups > 1) issue(1, P1);
        stage(0, 0, P0);
        if (ngroups > 2) issue(2, P0);
        __syncthreads();
        auto step = [&](int g, int b, auto PB) __attribute__((always_inline)) {
            set_prio(true, g);
            convert(g, b);
            if (g + 1 < ngroups) {
                stage(g + 1, b ^ 1, PB);
                if (g + 3 < ngroups) issue(g + 3, PB);
            }
            __syncthreads();
            set_prio(false, g);
            compute(g, b);
        };
        for (int g = 0; g < ngroups; g += 2) {
            step(g, 0, P1);
            if (g + 1 >= ngroups) break;
            step(g + 1, 1, P0);
        }
    } else if constexpr (kDirect) {
        // As below without the raw stage: group g's bytes are in registers
        // (loaded during group g - 1's passes), converted into lum[b], then
        // group g + 1's loads go out; one barrier; group g's passes.
        issue_direct(0);
        for (int g = 0; g < ngroups; g++) {
            const int b = g & 1;
            set_prio(true, g);
            convert_direct(g, b);
            if (g + 1 < ngroups) issue_direct(g + 1);
            __syncthreads();
            set_prio(false, g);
            compute(g, b);
        }
    } else if constexpr (kDB) {
        // One barrier per group: group g is converted and group g + 1 staged
        // before it, group g's passes run after it.  raw[b] / lum[b] are
        // rewritten only after every wave has passed the barrier that follows
        // their last reads (convert(g - 1) / compute(g - 2)).
        stage(0, 0, P0);
        if (ngroups > 1) issue(1, P0);
        __syncthreads();
        for (int g = 0; g < ngroups; g++) {
            const int b = g & 1;
            set_prio(true, g);
            convert(g, b);
            if (g + 1 < ngroups) {
                stage(g + 1, b ^ 1, P0);
                if (g + 2 < ngroups) issue(g + 2, P0);
            }
            __syncthreads();
            set_prio(false, g);
            compute(g, b);
        }
    } else {
        for (int g = 0; g < ngroups; g++) {
            // stage raw bytes of group g, then prefetch group g + 1
            set_prio(true, g);
            stage(g, 0, P0);
            if (g + 1 < ngroups) issue(g + 1, P0);
            __syncthreads();
            convert(g, 0);
            __syncthreads();
            set_prio(false, g);
            compute(g, 0);
            if constexpr (S == 4) {
                __syncthreads();
                combine(g);
            }
        }
    }
    __syncthreads();
    bool epi = false;                                // uniform
    if constexpr (kEpi) {
        epi = p.epi != 0;
        bool any = false;                            // uniform over the workgroup
#pragma unroll
        for (int s2 = 0; s2 < SPT; s2++) any = any || (nflag[s2] - 1u < kEpiMax);
        if (epi && any) {
            static_assert(sizeof(lum) >= sizeof(double) * (256 + SPT * 4 * N * (N + 1)), "epilogue LDS");
            map_refine_sparse<N, BPP, SEM>(p, reinterpret_cast<double*>(&lum[0][0][0]), nflag[sc], elist[sc],
                                           sx0, ys, tx, kThreads);
        }
    }
    if (tx < SPT) {
        const unsigned cnt = nflag[tx];
        if (cnt && !(epi && cnt <= kEpiMax)) {
            const unsigned st = strip - sc + tx;
            p.tile_count[st] = cnt;
            p.dirty_list[atomicAdd(p.dirty_count, 1u)] = st;
            if (kDenseFlat<N, SEM> && cnt > kFixDirect<N>) {
                const unsigned long long r = atomicAdd(p.dense_ctr, (1ull << 32) | cnt);
                const unsigned slot = (unsigned)(r >> 32), off = (unsigned)r;
                // a launch holds gridDim.x * gridDim.y * SPT strips (the guard only
                // matters if the counter did not start at zero)
                if (slot < gridDim.x * gridDim.y * SPT) p.dense_list[slot] = make_uint2(st, off);
            }
        }
    }
#if DCTE_TSTAMP
    // timing probe builds only (tools/tstamp.py): the workgroup's start /
    // end on the 100 MHz real-time counter and its hardware slot, into a
    // buffer of their own (the map itself stays right)
    if (tx == 0 && p.stamps) {
        const unsigned L = blockIdx.x + gridDim.x * blockIdx.y;
        unsigned long long* ts = p.stamps;
        ts[3 * L] = t_start;
        ts[3 * L + 1] = __builtin_amdgcn_s_memrealtime();
        ts[3 * L + 2] = (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
    }
#endif
}

// ------------------------------------------------------------------ refinement
// Flagged pixels (and points-mode entries) are recomputed in fp64 in the
// reference's own operation order (dcte_ref64.h): liblqr luma, the window
// gather of src/render.c:146-152 (data[dx][dy]; preview data[dy][dx],
// src/render.c:49), ddct8x8s / ddct16x16s / ddct2d, and the last-maximum scan
// of src/dct.c:100-108 -- identical class AND value to the reference.
//
// Tie-dense frames (line art, isolated dots: exact edge/texture ties in real
// arithmetic, decided only by the reference's rounding) flag a few % of all
// pixels, so this is a throughput kernel, not a cleanup pass:
//  * N <= 8: one LANE per pixel, the whole window in registers (N = 8: 64
//    doubles), the transform and the scan fully unrolled;
//  * N = 16: one 16-lane group per pixel (4 pixels per wave) -- 256 doubles do
//    not fit a lane's registers -- with the window in LDS: each lane gathers 16
//    elements, runs one line of each pass, scans one coefficient row, and the
//    group reduces (max, last index) with shuffles.
// liblqr luma divides each channel by 255 in double; the 256 quotients are
// tabulated in LDS once per workgroup (bit-identical to dividing).
constexpr int kFixThreads = 256;

struct Pix {
    int x, y;
    long long o;   // output element
};

__device__ __forceinline__ Pix fix_pixel(const FixParams& p, unsigned k)
{
    const unsigned idx = p.fix_list[k];
    Pix r;
    if (p.pts) {                                   // points mode
        r.x = clampi(p.pts[2 * idx], 0, p.w - 1);
        r.y = clampi(p.pts[2 * idx + 1], 0, p.h - 1);
        r.o = idx;
    } else {
        r.y = p.y0 + (int)(idx / (unsigned)p.w);
        r.x = (int)(idx % (unsigned)p.w);
        r.o = (long long)(r.y - p.y0) * p.out_stride + r.x;
    }
    return r;
}

// window element (i, j) of pixel q: liblqr data[dx][dy] (i = column offset),
// preview data[dy][dx]
template <int N, int SEM>
__device__ __forceinline__ double fix_elem(const FixParams& p, const double* lut, const Pix& q,
                                           int i, int j)
{
    constexpr int HL = Geo<N, SEM>::HL;
    const int ox = SEM == kSemLqr ? i : j, oy = SEM == kSemLqr ? j : i;
    const int xx = clampi(q.x + ox - HL, 0, p.w - 1);
    const int yy = clampi(q.y + oy - HL, 0, p.h - 1);
    const uint8_t* px = p.px + (long long)(yy - p.in_row0) * p.rowstride + (long long)xx * p.bpp;
    if constexpr (SEM == kSemLqr) {
        if (p.bpp == 1) return lut[px[0]];
        return 0.2126 * lut[px[0]] + 0.7152 * lut[px[1]] + 0.0722 * lut[px[2]];
    } else {
        return (double)preview_luma(px[0], p.bpp > 1 ? px[1] : 0u, p.bpp > 1 ? px[2] : 0u, p.bpp);
    }
}

__device__ __forceinline__ void fix_store(const FixParams& p, const Pix& q, double m, bool edge)
{
    p.out[q.o] = edge ? (float)(m * (double)p.edges) : (float)(m * (double)p.textures);
}

// The reference transform + last-maximum scan of one window held in
// The reference's last-maximum scan (src/dct.c:100-108) as plain maxima, no
// index tracking: the winner is the LAST index holding M = max |C| over the
// non-DC coefficients, and only two indices are edge atoms (src/dct.c:18-25),
// 1 = (0,1) and N = (1,0).  With a01 = |C01|, a10 = |C10|, mb = max over
// indices 2 .. N-1 and ma = max over indices > N (-1 for an empty set):
//     edge  <=>  ma < M  and  (a10 == M  or  (mb < M  and  a01 == M))
// -- exact comparisons of the very doubles the scan compares, so the class
// is the scan's (the all-zero window: ma == M == 0, texture, as the scan).
__device__ __forceinline__ void lastmax_decide(double a01, double a10, double mb, double ma,
                                               double& m, bool& edge)
{
    m = fmax(fmax(ma, a10), fmax(mb, a01));
    edge = !(ma == m) && (a10 == m || (!(mb == m) && a01 == m));
}

// Group form: lane l of an N-lane group holds coefficient row k1 = l in
// v[0..N-1]; the decision is valid on the group's lane 0.
template <int N>
__device__ __forceinline__ void lastmax_group(const double* v, int l, double& m, bool& edge)
{
    double mb = -1.0;
#pragma unroll
    for (int k = 2; k < N; k++) mb = fmax(mb, fabs(v[k]));
    const double v0 = fabs(v[0]), v1 = fabs(v[1]);
    double pa = fmax(mb, v1);                      // row l from k2 = 1
    pa = l >= 2 ? fmax(pa, v0) : (l == 1 ? pa : -1.0);   // indices > N
#pragma unroll
    for (int o = N / 2; o > 0; o >>= 1) pa = fmax(pa, __shfl_xor(pa, o, N));
    const double a10 = __shfl(v0, 1, N);           // lane 1's |C10|
    lastmax_decide(v1, a10, mb, pa, m, edge);
}

// registers (N <= 8): ddct8x8s along the first index, then the second;
// ddct2d (N = 2, 4) the second index first.  The scan keeps the LAST maximum
// (src/dct.c:103, "max <= currval"); edge atoms (0,1), (1,0) (src/dct.c:18-25).
#ifndef DCTE_FIX_IL
#define DCTE_FIX_IL 1    // N = 8 register path: 8-point steps the scheduler may interleave
#endif
template <int N, int IL = DCTE_FIX_IL>
__device__ __forceinline__ void refine_regs(double (&d)[N * N], const double* ct, double& m, bool& edge)
{
    if constexpr (N == 8) {
        // IL 8-point steps at a time: interleaving all eight would need their
        // temporaries live beside the 64-element window (> 256 registers)
#pragma unroll
        for (int i = 0; i < 8; i++) {
            r64::step8(d + i, 8);
            if ((i + 1) % IL == 0) __builtin_amdgcn_sched_barrier(0);
        }
        // pass 2 folded into the scan (r64::col8: step8's operations on row
        // k1 in its order, C00 never formed, max(|C_k1,0|, |C_k1,4|) as one
        // exact product for k1 >= 2 -- the exact maps' form, bit-identical;
        // line art RGB -1.4 %, profiles/r06/refine_col8_grey_ab.jsonl)
        double a01, a10, mb, ma = -1.0;
        r64::col8<0>(d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], a01, mb);
        r64::col8<1>(d[8], d[9], d[10], d[11], d[12], d[13], d[14], d[15], a10, ma);
#pragma unroll
        for (int i = 2; i < 8; i++) {
            double unused;
            r64::col8<2>(d[8 * i], d[8 * i + 1], d[8 * i + 2], d[8 * i + 3], d[8 * i + 4], d[8 * i + 5],
                         d[8 * i + 6], d[8 * i + 7], unused, ma);
            if ((i + 1) % IL == 0) __builtin_amdgcn_sched_barrier(0);
        }
        lastmax_decide(a01, a10, mb, ma, m, edge);
        return;
    } else {
#pragma unroll
        for (int i = 0; i < N; i++) r64::step_small(N, d + N * i, 1, ct);
#pragma unroll
        for (int i = 0; i < N; i++) r64::step_small(N, d + i, N, ct);
    }
    double mb = -1.0, ma = -1.0;
#pragma unroll
    for (int e = 2; e < N; e++) mb = fmax(mb, fabs(d[e]));
#pragma unroll
    for (int e = N + 1; e < N * N; e++) ma = fmax(ma, fabs(d[e]));
    lastmax_decide(fabs(d[1]), fabs(d[N]), mb, ma, m, edge);
}

__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// N = 16: the 16-lane group of lane l owns the window d[0..255] (LDS, filled
// and made visible by the caller): ddct16x16s, then row k1 = l's last
// maximum (lastmax_group).  Every lane of the
// wave must call it (wave barriers inside).
__device__ __forceinline__ void refine16_group(double* d, int l, double& best, bool& edge)
{
    r64::step16(d + l, 16);                  // along the first index ...
    wave_sync_lds();
    r64::step16(d + 16 * l, 1);              // ... then the second
    wave_sync_lds();
    double v[16];
#pragma unroll
    for (int c = 0; c < 16; c++) v[c] = d[l * 16 + c];
    lastmax_group<16>(v, l, best, edge);
}

template <int N, int SEM>
__global__ __launch_bounds__(kFixThreads) void dcte_fix(const FixParams p)
{
    __shared__ double lut[256];
    constexpr int LDS_PIX = N == 16 ? kFixThreads / 16 : 1;
    __shared__ double win[LDS_PIX][N == 16 ? 256 : 1];
    const unsigned cnt = min(*p.fix_count, p.fix_cap);
    if (p.fix_total && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(p.fix_total, cnt);
    if (blockIdx.x * (unsigned)(kFixThreads / (N == 16 ? 16 : 1)) >= cnt) return;   // uniform
    lut[threadIdx.x] = (double)threadIdx.x / 255;
    __syncthreads();

    if constexpr (N <= 8) {
        for (unsigned k = blockIdx.x * kFixThreads + threadIdx.x; k < cnt; k += gridDim.x * kFixThreads) {
            const Pix q = fix_pixel(p, k);
            double d[N * N];
#pragma unroll
            for (int i = 0; i < N; i++)
#pragma unroll
                for (int j = 0; j < N; j++) d[i * N + j] = fix_elem<N, SEM>(p, lut, q, i, j);
            double m;
            bool edge;
            refine_regs<N>(d, p.ct, m, edge);
            fix_store(p, q, m, edge);
        }
    } else {
        // 16 lanes per pixel, 4 pixels per wave; every lane runs every wave
        // barrier (invalid groups compute on stale LDS and store nothing)
        const int l = threadIdx.x & 15;
        const int slot = threadIdx.x >> 4;                        // pixel slot in the block
        double* d = win[slot];
        const unsigned per_pass = gridDim.x * (kFixThreads / 16);
        const unsigned rounds = (cnt + per_pass - 1) / per_pass;   // uniform
        for (unsigned r = 0; r < rounds; r++) {
            const unsigned k = r * per_pass + blockIdx.x * (kFixThreads / 16) + slot;
            const bool valid = k < cnt;
            Pix q{};
            if (valid) {
                q = fix_pixel(p, k);
#pragma unroll
                for (int t = 0; t < 16; t++) d[t * 16 + l] = fix_elem<16, SEM>(p, lut, q, t, l);
            }
            wave_sync_lds();
            double best;
            bool edge;
            refine16_group(d, l, best, edge);
            if (valid && l == 0) fix_store(p, q, best, edge);
            wave_sync_lds();
        }
    }
}

// Refinement of a map launch: one wave per batch of 64-column STRIPs with
// flagged pixels (dcte_map keeps a list per strip -- one wave's columns at
// N <= 8, the whole 64-column tile at N = 16 -- in the row order it emitted
// them).  Tie-dense frames (line art, dots on flat ground) flag a few % of
// all pixels over most strips; read straight from HBM, one scattered byte per
// lane, their windows were bound by the texture addresser (17 ms for 7.2 M
// pixels at 16384^2, profiles/r02).  So each wave works alone (no workgroup
// barriers; several waves per CU hide each other's latency):
//  * the sparse strips of a batch (cnt <= kFixDirect<N>) are refined side by
//    side, one lane group per strip, windows gathered from global memory --
//    natural frames flag ~1 pixel per dirty strip, text-like frames a few;
//  * a denser strip is walked by the whole wave in bands of SBH output rows:
//    the band's input rows + window halo are copied to LDS with coalesced
//    dword loads (clamped per pixel only in strips at the left / right frame
//    border), converted there ONCE to the reference's fp64 luma, and every
//    window element is one 8-byte LDS read.  Entries come in row-group order,
//    so the wave steps through them 64 at a time and stages each band once;
//    the next band's list chunk and raw rows load during this band's work.
// One lane per pixel for N <= 4 (the window in registers), one N-lane group
// per pixel for N = 8, 16 (the window in LDS).
// Strips with at most kFixDirect<N> flagged pixels take the direct path: N <= 8
// at 16 since the lane-per-pixel dense walk (dots on flat ground, 0.37 %
// flagged at 16384^2: 0.17 ms vs 0.24 at 128, 0.16 at 8 where text loses
// 10 %; profiles/r03/fix_direct_ab.jsonl -- with the band path of r02 the
// best was 128), N = 16 at 32 (profiles/r02/fix_direct.jsonl).

template <int N, int SEM>
struct FixStrip {
    static constexpr int LW = 64 + N - 1;             // luma columns of a strip
    static constexpr int G = Geo<N, SEM>::G;          // map kernel rows per group
#ifndef DCTE_FIX_GPS
#define DCTE_FIX_GPS 2   // A/B at N = 8 vs 1: line art -6 % (grey) / -1 % (RGB), 8-px grid -10 %; 3, 4: +20-50 % (profiles/r02/fix_gps_ab.jsonl)
#endif
    static constexpr int GPS = N == 16 ? 1 : DCTE_FIX_GPS;   // map row groups per band
    static constexpr int SBH = GPS * G;               // output rows per band (16; N = 16: 16)
    static constexpr int LR = SBH + N - 1;            // input rows staged per band
};

__device__ __forceinline__ unsigned wave_max_u(unsigned v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (unsigned)__shfl_xor((int)v, o));
    return v;
}

// One pixel's refinement by a group of N lanes (N = 8, 16) from the band's
// fp64 luma in LDS: lane l runs the reference's first pass on window line l
// (ddct8x8s / ddct16x16s transform along the first index for each second
// index), the lines meet in the group's window buffer w, lane l runs the
// second pass on coefficient row l and scans it (last maximum,
// src/dct.c:103, as maxima: lastmax_group).  `at` =
// the lum index of window element (0, 0); w holds N rows of N + 1 doubles
// (the pad keeps both passes' accesses on distinct LDS banks).  Every lane
// of the wave calls it.
template <int N, class Line>
__device__ __forceinline__ void refine_group_f(Line&& line, double* w, int l, double& best, bool& edge)
{
    double v[N];
#pragma unroll
    for (int i = 0; i < N; i++) v[i] = line(i);
    if constexpr (N == 8) r64::step8(v, 1); else r64::step16(v, 1);
#pragma unroll
    for (int i = 0; i < N; i++) w[i * (N + 1) + l] = v[i];   // rows padded: no bank conflicts
    wave_sync_lds();
#pragma unroll
    for (int k = 0; k < N; k++) v[k] = w[l * (N + 1) + k];
    wave_sync_lds();                                   // w may be refilled after this
    if constexpr (N == 8) r64::step8(v, 1); else r64::step16(v, 1);
    lastmax_group<N>(v, l, best, edge);
}

template <int N, int SEM>
__device__ __forceinline__ void refine_group(const double* lum, int LW, int at, double* w, int l,
                                             double& best, bool& edge)
{
    // d[i][l]: liblqr data[dx][dy] (row l, column i); preview data[dy][dx]
    refine_group_f<N>([&](int i) { return SEM == kSemLqr ? lum[at + l * LW + i] : lum[at + i * LW + l]; },
                      w, l, best, edge);
}

// The dense walks' waves: up to DCTE_DENSE_OVERSUB x the resident wave slots
// (N = 8: one wave per dirty strip; N = 16: one per 16-entry batch up to that
// cap), so the hardware hands out strips as slots free up instead of each
// resident wave striding over a fixed tenth of them -- the launch's tail is one
// strip.  16 vs 1 (r03): line art RGB 0.436 -> 0.393 ms, the 8-px grid 3.44 ->
// 2.86, dots -10 %, N = 16 line art RGB 0.760 -> 0.695 (profiles/r04/
// dense_oversub_ab.jsonl).  Splitting a strip into interleaved pieces, or the
// same for the sparse walk, measured slower (dense_oversub_ab2.jsonl).
#ifndef DCTE_DENSE_OVERSUB
#define DCTE_DENSE_OVERSUB 16
#endif
// N = 8 grey layers (the window memo): fewer waves, each walking several
// strips, keep their memo tables warm -- 4 vs 16: line art 0.283 -> 0.269 ms,
// the 8-px grid 1.565 -> 1.49; 8, 2, 1 in between or slower
// (profiles/r04/memo_oversub_ab.jsonl)
#ifndef DCTE_DENSE_OVERSUB_MEMO
#define DCTE_DENSE_OVERSUB_MEMO 4
#endif
// N = 8 with the two-way memo (r05): 2 vs 4: line art 0.265 -> 0.251 ms, dots
// -7 %, text -1 %, the grid +2 %; N = 4 keeps 4 (2: line art +7 %, dots +4 %)
// (profiles/r05/memo_oversub_ab.jsonl)
#ifndef DCTE_DENSE_OVERSUB_MEMO8
#define DCTE_DENSE_OVERSUB_MEMO8 2
#endif
// ... on launches of fewer pixels than DCTE_MEMO8_BIG_PX, 1: each wave then
// walks more strips with its memo warm -- 1 vs 2 (r06), the four grey frames
// of tools/fix_study.py summed: 2048^2 -8 %, 4096^2 -12 % (line art -18 %,
// the 8-px grid -17 %; preview -12 %), 6144^2 -4 %, 8192^2 -2 %, 11584^2
// -3 %, but 16384^2 +2 % (liblqr and preview; profiles/r06/memo_oversub1_ab.jsonl,
// memo_oversub1_sizes.jsonl)
#ifndef DCTE_MEMO8_BIG_PX
#define DCTE_MEMO8_BIG_PX 192000000LL
#endif
// grey layers at N <= 4 fit 128 VGPRs: 4 waves per SIMD (the LDS allows them)
#ifndef DCTE_FIX_MINW
#define DCTE_FIX_MINW 4
#endif
#ifndef DCTE_FIX_MINW_LANES
#define DCTE_FIX_MINW_LANES 2   // N = 8 (lane-per-pixel dense strips in the same launch): the window alone is 128 VGPRs
#endif
#ifndef DCTE_FIX_MINW_RGB8
#define DCTE_FIX_MINW_RGB8 1    // N = 8 RGB layers
#endif
template <int N, int BPP>
constexpr int kFixMinWaves = (BPP == 1 && N <= 8) ? (N == 8 ? DCTE_FIX_MINW_LANES : DCTE_FIX_MINW)
                                                  : (N == 8 && BPP == 3 ? DCTE_FIX_MINW_RGB8 : 1);

// Dense strips at N = 8 (more than kFixDirect<8> flagged pixels; the sparse
// ones stay with dcte_fix_strips): one lane per flagged pixel, its whole
// window in registers.  The eight window rows come straight from the frame as
// whole dwords (neighbouring windows share rows: L1 / L2 hits), each byte is
// converted through the LDS tables, and refine_regs runs both passes of
// ddct8x8s and the last-maximum scan with no LDS round trip and no cross-lane
// step -- eight independent 8-point transforms per pass keep the lane busy
// where the group-per-window form of dcte_fix_strips waited on LDS transposes
// (line art RGB at 16384^2: 1.27 -> 0.46 ms, profiles/r03/fix_lanes_ab.jsonl).
// Extra blocks of the dcte_fix_strips launch: no band staging, so only the
// tables take LDS.  Waves take dirty strips in turn.
// the 256 liblqr channel quotients v / 255 (pre-weighted per channel for
// liblqr RGB: kTab), as the reference divides (bit-identical); kTab also
// fills lut[768 + v] = the luma of the grey pixel (v, v, v), summed in the
// reference's order ((k_r v + k_g v) + k_b v): what the three tables give for
// it, bit for bit (the dense N = 8 walk's grey-RGB path)
template <bool kTab>
__device__ __forceinline__ void fill_luma_lut(double* lut, int lane)
{
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int v = lane + 64 * t;
        const double q = (double)v / 255;
        if constexpr (kTab) {
            lut[v] = 0.2126 * q;
            lut[256 + v] = 0.7152 * q;
            lut[512 + v] = 0.0722 * q;
            lut[768 + v] = lut[v] + lut[256 + v] + lut[512 + v];
        } else {
            lut[v] = q;
        }
    }
}

// Preview RGB / RGBA (the lane walks): RGB2LUMINANCE (src/render.h:5, preview_
// in dcte_luma.h) is ((16 + 0.2568 r) + 0.5041 g) + 0.0979 b in double, then
// truncated to u8: the three terms tabulated as computed (no contraction), so
// (lut[r] + lut[256 + g]) + lut[512 + b] is the same double; lut[768 + v] is
// the u8 luma of the grey pixel (v, v, v)
__device__ __forceinline__ void fill_preview_lut(double* lut, int lane)
{
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int v = lane + 64 * t;
        lut[v] = 16.0 + v * 0.2568;
        lut[256 + v] = v * 0.5041;
        lut[512 + v] = v * 0.0979;
        lut[768 + v] = (double)preview_luma((unsigned)v, (unsigned)v, (unsigned)v, 3);
    }
}

// RGB bytes of a window line (8 pixels in 6 dwords, wd): every pixel grey
// (R = G = B)?  d = the stream XOR itself shifted by one byte; within each
// pixel's three bytes the first two of d are zero iff the channels agree.
template <int K>
__device__ __forceinline__ bool rgb_line_grey(const uint32_t (&wd)[K])
{
    static_assert(K % 3 == 0, "whole pixels: 4 per 3 dwords");
    constexpr uint32_t M[3] = {0xFF00FFFFu, 0xFFFF00FFu, 0x00FFFF00u};
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < K; j++) {
        const uint32_t nx = __builtin_amdgcn_alignbyte(j < K - 1 ? wd[j + 1] : 0u, wd[j], 1u);
        acc |= (wd[j] ^ nx) & M[j % 3];
    }
    return acc == 0u;
}

// The same test over a whole window, cheaper: the lines' differences are
// OR-ed per dword class (j mod 3) across all lines and masked once at the end
// (6 + 6 + 3 operations per 8-pixel line instead of 24)
template <int K>
__device__ __forceinline__ void rgb_grey_acc(const uint32_t (&wd)[K], uint32_t (&acc)[3])
{
    static_assert(K % 3 == 0, "whole pixels: 4 per 3 dwords");
#pragma unroll
    for (int j = 0; j < K; j++) {
        const uint32_t nx = __builtin_amdgcn_alignbyte(j < K - 1 ? wd[j + 1] : 0u, wd[j], 1u);
        acc[j % 3] |= wd[j] ^ nx;
    }
}
__device__ __forceinline__ bool rgb_grey_done(const uint32_t (&acc)[3])
{
    return ((acc[0] & 0xFF00FFFFu) | (acc[1] & 0xFFFF00FFu) | (acc[2] & 0x00FFFF00u)) == 0u;
}

// Window memo of the dense lane walks, N = 4 and 8 (r04).  Tie-dense frames are regular:
// their flagged windows repeat (straight strokes, grid lines, flat fills, the
// same glyph), and a window's refined energy depends only on its bytes.  Each
// wave keeps the windows it refined in an LDS table -- kMemoSlots entries
// (the sparse walk's window buffers, grown to hold them),
// direct-mapped on a hash of the key, key = the window's N^2 bytes (liblqr /
// preview grey; RGB: the R bytes of a window whose every pixel has R = G = B,
// which then fix its luma) and the output's bits -- and answers a flagged pixel
// whose window equals an entry's key in all its bytes from the entry.  Misses
// queue in LDS and are refined 64 at a time, full waves across strip
// boundaries.  Entries are written by one elected lane per slot and read only
// after the wave's refinement phase, so none is ever seen half-written.
// Grey layers only: for RGB (keyed by the R bytes of windows whose pixels are
// all grey) the probe's 56-dword row loads, loaded again for every miss, cost
// more than the hits save -- with this hash and 3 waves per SIMD: grey line
// art stored as RGB +7 %, colour strokes +22 %, dots +17 %
// (profiles/r04/memo_ab.jsonl); with r05's two ways (r06, 1-3 waves per
// SIMD): line art RGB -1.6 %, colour strokes +28 %, dots +18 %
// (profiles/r06/memo_rgb_ab.jsonl).
// 128 slots (8.7 KB with the queue, the block's LDS 11 KB: 3 waves per SIMD
// still fit): vs 64 the grid 1.50 -> 1.39 ms, line art 0.269 -> 0.265, dots
// -7 %; 256 costs occupancy (grid 1.62) (profiles/r04/memo_slots_ab.jsonl).
// Two ways (r05): a key may sit in its slot or the slot's pair partner (s ^ 1),
// an empty way filled first; the 8-px grid (many distinct windows per slot)
// 1.415 -> 1.18 ms at N = 8, line art and dots within +-1.5 %; four ways
// (s ^ 0 .. 3) 1.19
// (profiles/r05/memo_ways_ab.jsonl)
#ifndef DCTE_MEMO_SLOTS
#define DCTE_MEMO_SLOTS 128
#endif
#ifndef DCTE_MEMO_WAYS
#define DCTE_MEMO_WAYS 2
#endif
constexpr int kMemoWays = DCTE_MEMO_WAYS;              // 1: direct-mapped; W: the slots s ^ 0 .. s ^ (W - 1)
static_assert(kMemoWays == 1 || kMemoWays == 2 || kMemoWays == 4, "memo ways");
constexpr int kMemoSlots = DCTE_MEMO_SLOTS;            // a power of two
static_assert((kMemoSlots & (kMemoSlots - 1)) == 0 && kMemoSlots >= 64, "memo slots");
template <int N>
constexpr int kMemoKey = N * N / 4;                    // key dwords (N^2 bytes)
template <int N>
constexpr int kMemoStride = kMemoKey<N> + 1;           // key + the output's bits
constexpr uint32_t kMemoEmpty = 0xFFFFFFFFu;           // a NaN: never an output
constexpr int kMemoPend = 128;                         // misses waiting for a full batch (< 64 + 64)
template <int N>
constexpr int kMemoDwords = kMemoSlots * kMemoStride<N> + kMemoPend;

// slot of a key: FNV-1a over its dwords, then a murmur finaliser, top bits.
// (A rotate-xor fold is linear over GF(2) and maps the 0x00 / 0xFF byte
// patterns of line art onto few slots.)
template <int KD>
__device__ __forceinline__ int memo_slot(const uint32_t (&key)[KD])
{
    uint32_t h = 0x811c9dc5u;
#pragma unroll
    for (int j = 0; j < KD; j++) h = (h ^ key[j]) * 0x01000193u;
    h ^= h >> 15;
    h *= 0x2c1b3c6du;
    h ^= h >> 12;
    return (int)(h >> (32 - __builtin_ctz((unsigned)kMemoSlots)));
}

// The dense-strip walk of one wave, N = 4 or 8: wave `blk` of `nblk` takes
// dirty strips blk, blk + nblk, ...; `lut` filled by fill_luma_lut; `memo`
// the wave's kMemoDwords<N> of LDS.
template <int N, int BPP, int SEM>
__device__ __forceinline__ void fix_dense_lane(const TileFixParams& tp, const double* lut, uint32_t* memo,
                                               unsigned blk, unsigned nblk)
{
    static_assert(N == 4 || N == 8, "lane walk: N = 4, 8");
    constexpr int HL = Geo<N, SEM>::HL;
    constexpr int KD = kMemoKey<N>, MS = kMemoStride<N>, KW = N / 4;   // key dwords, entry, per row
    constexpr bool kMemo = BPP == 1;                // grey layers (RGB: see above)
    const MapParams& p = tp.m;
    const unsigned ndirty = *p.dirty_count;
    const int lane = threadIdx.x;
    const uintptr_t pbase = reinterpret_cast<uintptr_t>(p.px);
    const uint32_t base_off = (uint32_t)(pbase & 3u);
    const unsigned nrec = base_off + (unsigned)((long long)(p.in_rows - 1) * p.rowstride) +
                          (unsigned)(p.w * BPP);
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(pbase - base_off), (short)0, (int)nrec, (int)kBufFlags);
    // liblqr luma (src/render.c:315, LQR_ER_LUMA) [liblqr, unverified] in the
    // reference's order ((k_r r + k_g g) + k_b b); preview: RGB2LUMINANCE
    // (colour layers through the per-channel tables of fill_preview_lut)
    auto luma3 = [&](uint32_t c0, uint32_t c1, uint32_t c2) -> double {
        if constexpr (SEM == kSemLqr) {
            if constexpr (BPP == 1) return lut[c0];
            else return lut[c0] + lut[256 + c1] + lut[512 + c2];
        } else if constexpr (BPP >= 3) {
            return (double)(unsigned char)((lut[c0] + lut[256 + c1]) + lut[512 + c2]);
        } else {
            return (double)preview_luma(c0, c1, c2, BPP);
        }
    };
    const unsigned spt = (unsigned)tp.tile_w / 64u;   // strips per map tile
    constexpr int NW = (N * BPP + 3) / 4 + 1;         // dwords of a row's N pixels, any alignment
    uint32_t* const pend = memo + kMemoSlots * MS;
    if constexpr (kMemo) {
        for (int s = lane; s < kMemoSlots; s += 64) memo[s * MS + KD] = kMemoEmpty;
        wave_sync_lds();
    }

    // the window's N image rows as whole dwords (fast: unclamped and inside
    // the buffer; otherwise the loads return zeros)
    auto load_rows = [&](bool active, int x, int y, uint32_t (&fv)[N][NW], uint32_t (&foff)[N], bool (&fast)[N]) {
        const int gx0 = x - HL;
        const bool inside = active && gx0 >= 0 && gx0 + N <= p.w;
#pragma unroll
        for (int rr = 0; rr < N; rr++) {
            const int gy = clampi(y - HL + rr, 0, p.h - 1);
            const uint32_t s0 = base_off + (uint32_t)((long long)(gy - p.in_row0) * p.rowstride) +
                                (uint32_t)(gx0 * BPP);
            fast[rr] = inside && ((s0 + N * BPP - 1) | 3u) < nrec;
            foff[rr] = s0 & 3u;
            const uint32_t a = fast[rr] ? (s0 & ~3u) : 0x7ffffff0u;   // past num_records: zeros
#pragma unroll
            for (int j = 0; j < NW; j++)
                fv[rr][j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)(a + 4u * j), 0, 0);
        }
    };
    // the rows' bytes from their first pixel on (aligned once: the raw dwords
    // die here)
    auto align_rows = [&](const uint32_t (&fv)[N][NW], const uint32_t (&foff)[N], uint32_t (&wa)[N][NW - 1]) {
#pragma unroll
        for (int rr = 0; rr < N; rr++)
#pragma unroll
            for (int j = 0; j < NW - 1; j++) wa[rr][j] = __builtin_amdgcn_alignbyte(fv[rr][j + 1], fv[rr][j], foff[rr]);
    };
    // the window's memo key; false: it has none (a clamped row, or RGB with a
    // pixel whose channels differ)
    auto make_key = [&](const uint32_t (&wa)[N][NW - 1], const bool (&fast)[N], uint32_t (&key)[KD]) -> bool {
        bool ok = true;
#pragma unroll
        for (int rr = 0; rr < N; rr++) {
            const uint32_t (&wd)[NW - 1] = wa[rr];
            ok = ok && fast[rr];
            if constexpr (BPP == 1) {
#pragma unroll
                for (int j = 0; j < KW; j++) key[KW * rr + j] = wd[j];
            } else {
                uint32_t g[3 * KW];
#pragma unroll
                for (int j = 0; j < 3 * KW; j++) g[j] = wd[j];
                ok = ok && rgb_line_grey(g);
                auto byte = [&](int b) { return (wd[b >> 2] >> (8 * (b & 3))) & 255u; };
#pragma unroll
                for (int j = 0; j < KW; j++)
                    key[KW * rr + j] = byte(12 * j) | byte(12 * j + 3) << 8 | byte(12 * j + 6) << 16 |
                                       byte(12 * j + 9) << 24;
            }
        }
        return ok;
    };

    // refine the pixel of each active lane from its loaded rows (fp64, the
    // reference's order) and, with `ins` (uniform), enter its window into the
    // memo
    auto refine_rows = [&](bool active, int x, int y, const uint32_t (&wa)[N][NW - 1], const bool (&fast)[N],
                           bool ins) {
        if (!active) return;
        int slot = -1;                                   // the memo slot this lane fills
        if (kMemo && ins) {
            uint32_t key[KD];
            const bool keyed = make_key(wa, fast, key);
            int s = 0;
            if (keyed) {
                s = memo_slot(key);
                if constexpr (kMemoWays > 1) {
                    // the first empty way; all full: the way this lane's
                    // position picks
                    int pick = -1;
#pragma unroll
                    for (int w = 0; w < kMemoWays; w++)
                        if (pick < 0 && memo[(s ^ w) * MS + KD] == kMemoEmpty) pick = w;
                    s ^= pick >= 0 ? pick : ((lane ^ y) & (kMemoWays - 1));
                }
                memo[s * MS + KD] = (uint32_t)lane;                 // one lane per slot wins
            }
            wave_sync_lds();
            if (keyed && memo[s * MS + KD] == (uint32_t)lane) {
#pragma unroll
                for (int j = 0; j < KD; j++) memo[s * MS + j] = key[j];
                slot = s;                                // its value follows the refinement
            }
        }
        // RGB: when every window pixel of every lane is grey (scanned
        // documents, line art stored as RGB), one table read per element
        // (lut[768 + v], the same double the three reads and two adds give --
        // liblqr -- or the same u8 luma -- preview) instead of three
        bool grey = false;
        if constexpr (BPP == 3) {
            bool all_fast = true;
#pragma unroll
            for (int rr = 0; rr < N; rr++) all_fast = all_fast && fast[rr];
            // one test over the window (rgb_grey_acc), the first row alone
            // first: a colour window on any lane ends the test for the wave
            // there (uniform branch) -- line art RGB -2.6 % with col8 below,
            // colour strokes -2.9 % (profiles/r06/refine_col8_grey_ab.jsonl)
            auto acc_row = [&](int rr, uint32_t (&acc)[3]) {
                uint32_t wd[3 * KW];
#pragma unroll
                for (int j = 0; j < 3 * KW; j++) wd[j] = wa[rr][j];
                rgb_grey_acc(wd, acc);
            };
            uint32_t acc[3] = {0u, 0u, 0u};
            acc_row(0, acc);
            if (__all(all_fast && rgb_grey_done(acc))) {     // uniform
#pragma unroll
                for (int rr = 1; rr < N; rr++) acc_row(rr, acc);
                grey = __all(rgb_grey_done(acc));          // uniform
            }
        }
        double d[N * N];
        const int gx0 = x - HL;
#pragma unroll
        for (int r = 0; r < N; r++) {
            double lv[N];
            if (fast[r]) {
                const uint32_t (&wd)[NW - 1] = wa[r];
                auto byte = [&](int b) { return (wd[b >> 2] >> (8 * (b & 3))) & 255u; };
                if (grey) {
#pragma unroll
                    for (int c = 0; c < N; c++) lv[c] = lut[768 + byte(c * BPP)];
                } else {
#pragma unroll
                    for (int c = 0; c < N; c++)
                        lv[c] = luma3(byte(c * BPP), BPP > 1 ? byte(c * BPP + 1) : 0u, BPP > 1 ? byte(c * BPP + 2) : 0u);
                }
            } else {
                // clamped at the left / right frame border, or at the frame's
                // last bytes: per-pixel reads
                const int gy = clampi(y - HL + r, 0, p.h - 1);
                const uint8_t* row = p.px + (long long)(gy - p.in_row0) * p.rowstride;
#pragma unroll
                for (int c = 0; c < N; c++) {
                    const uint8_t* q8 = row + (long long)clampi(gx0 + c, 0, p.w - 1) * BPP;
                    lv[c] = luma3(q8[0], BPP > 1 ? q8[1] : 0u, BPP > 1 ? q8[2] : 0u);
                }
            }
            // image row r, pixel c: liblqr data[c][r], preview data[r][c]
#pragma unroll
            for (int c = 0; c < N; c++) d[SEM == kSemLqr ? c * N + r : r * N + c] = lv[c];
        }
        double m;
        bool edge;
        refine_regs<N>(d, tp.ct, m, edge);
        const float v = edge ? (float)(m * (double)p.edges) : (float)(m * (double)p.textures);
        p.out[(long long)(y - p.y0) * p.out_stride + x] = v;
        if (kMemo && slot >= 0) memo[slot * MS + KD] = __float_as_uint(v);
    };

    // (without the memo, the direct walk: queueing RGB entries for full
    // batches across strips was slower -- line art +6 %, dots +-2 %,
    // profiles/r04/memo_ab.jsonl)
    if constexpr (!kMemo) {
        for (unsigned k = blk; k < ndirty; k += nblk) {   // uniform
            const unsigned strip = p.dirty_list[k];
            const unsigned cnt = p.tile_count[strip];
            if (cnt <= kFixDirect<N>) continue;            // sparse: dcte_fix_strips' own walk
            const unsigned tile = strip / spt;
            const int bx = (int)(tile % (unsigned)tp.tiles_x), by = (int)(tile / (unsigned)tp.tiles_x);
            const int sx0 = bx * tp.tile_w + 64 * (int)(strip % spt);
            const int ys = tile_row0(p, by);
            const unsigned* list = p.fix_list + (size_t)strip * (size_t)(64 * p.tile_h);
            for (unsigned q0 = 0; q0 < cnt; q0 += 64) {   // uniform
                const unsigned q = q0 + (unsigned)lane;
                if (q >= cnt) continue;
                const unsigned loc = list[q];
                const int x = sx0 + (int)(loc & 63), y = ys + (int)(loc >> 6);
                uint32_t fv[N][NW];
                uint32_t foff[N];
                bool fast[N];
                load_rows(true, x, y, fv, foff, fast);
                uint32_t wa[N][NW - 1];
                align_rows(fv, foff, wa);
                refine_rows(true, x, y, wa, fast, false);
            }
        }
        return;
    } else {
    // misses wait in pend[0 .. np) as (y - y0) * w + x (< 2^32: the launch's
    // output span, checked by the host)
    const unsigned uw = (unsigned)p.w;
    unsigned np = 0;                                       // uniform
    bool use = true;                                       // uniform: this wave's windows repeat
    unsigned tries = 0, hits = 0;                          // uniform: windows probed, answered
    // a step probes the current strip's next 64 entries and queues the misses
    // (after 512 windows with fewer than one in eight answered, the wave
    // queues without probing); a full batch of misses (at the end: what is
    // left) is loaded again and refined.  One refinement site.
    unsigned k = blk, q0 = 0, cnt = 0;                     // uniform
    int sx0 = 0, ys = 0;
    const unsigned* list = nullptr;
    bool have = false;                                     // strip k has entries from q0 on
    for (;;) {
        while (!have && k < ndirty) {                      // uniform
            const unsigned strip = p.dirty_list[k];
            cnt = p.tile_count[strip];
            if (cnt <= kFixDirect<N>) {                    // sparse: dcte_fix_strips' own walk
                k += nblk;
                continue;
            }
            const unsigned tile = strip / spt;
            const int bx = (int)(tile % (unsigned)tp.tiles_x), by = (int)(tile / (unsigned)tp.tiles_x);
            sx0 = bx * tp.tile_w + 64 * (int)(strip % spt);
            ys = tile_row0(p, by);
            list = p.fix_list + (size_t)strip * (size_t)(64 * p.tile_h);
            q0 = 0;
            have = true;
        }
        if (have && np < 64) {                             // uniform
            const unsigned q = q0 + (unsigned)lane;
            const bool act = q < cnt;
            const unsigned loc = act ? list[q] : 0u;
            const int x = sx0 + (int)(loc & 63), y = ys + (int)(loc >> 6);
            bool hit = false;
            if (use) {
                uint32_t fv[N][NW];
                uint32_t foff[N];
                bool fast[N];
                load_rows(act, x, y, fv, foff, fast);
                uint32_t wa[N][NW - 1];
                align_rows(fv, foff, wa);
                uint32_t key[KD];
                if (act && make_key(wa, fast, key)) {
                    const int s0 = memo_slot(key);
                    const uint32_t* ent = memo + s0 * MS;
                    uint32_t val = ent[KD];
                    uint32_t diff = val == kMemoEmpty ? 1u : 0u;
#pragma unroll
                    for (int j = 0; j < KD; j++) diff |= ent[j] ^ key[j];
                    // the next ways (filled only after this one)
#pragma unroll
                    for (int w = 1; w < kMemoWays; w++)
                        if (diff != 0u && val != kMemoEmpty) {
                            ent = memo + (s0 ^ w) * MS;
                            val = ent[KD];
                            diff = val == kMemoEmpty ? 1u : 0u;
#pragma unroll
                            for (int j = 0; j < KD; j++) diff |= ent[j] ^ key[j];
                        }
                    if (diff == 0u) {
                        p.out[(long long)(y - p.y0) * p.out_stride + x] = __uint_as_float(val);
                        hit = true;
                    }
                }
            }
            const unsigned long long bal = __ballot(act && !hit);
            if (act && !hit)
                pend[np + (unsigned)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u))] =
                    (uint32_t)(y - p.y0) * uw + (uint32_t)x;
            const unsigned nmiss = (unsigned)__popcll(bal);
            if (use) {
                const unsigned nact = (unsigned)__popcll(__ballot(act));
                tries += nact;
                hits += nact - nmiss;
                if (tries >= 512 && hits * 8 < tries) use = false;
            }
            np += nmiss;
            wave_sync_lds();
            q0 += 64u;
            if (q0 >= cnt) {
                have = false;
                k += nblk;
            }
        }
        const bool done = !have && k >= ndirty;
        if (np >= 64 || (done && np > 0)) {                // refine pend[0 .. c)
            const unsigned c = np >= 64 ? 64u : np;
            const bool act = (unsigned)lane < c;
            const uint32_t e = act ? pend[lane] : 0u;
            wave_sync_lds();
            if ((unsigned)lane < np - c) pend[lane] = pend[c + (unsigned)lane];   // the rest moves down
            np -= c;
            unsigned yr = (unsigned)((double)e / (double)uw);
            if ((unsigned long long)yr * uw > e) yr--;     // the quotient rounded up
            const int x = (int)(e - yr * uw), y = p.y0 + (int)yr;
            if (act) {
                uint32_t fv[N][NW];
                uint32_t foff[N];
                bool fast[N];
                load_rows(true, x, y, fv, foff, fast);
                uint32_t wa[N][NW - 1];
                align_rows(fv, foff, wa);
                refine_rows(true, x, y, wa, fast, use);
            }
            wave_sync_lds();
        }
        if (done && np == 0) break;
    }
    }
}

// Cursor over the flat dense list (N = 16) for one wave: batches of EPB entries,
// the wave taking batches blk, blk + nblk, ... -- the waves resident at one
// time work on neighbouring batches (neighbouring strips, so their window rows
// share the L2), every wave gets the same number of full batches whatever the
// strips' counts.  A batch's first strip comes from the map kernel's batch
// map (MapParams::dense_batch); a batch spans at most two strips (a dense
// strip holds more than kFixDirect >= EPB entries), the second one is the
// next slot of dense_list.
#ifndef DCTE_DENSE_CHUNK
#define DCTE_DENSE_CHUNK 1      // consecutive refinement batches per wave before it strides on (N = 16: 1 -4 %, 8 +0, 32 +7..14 % vs 8, profiles/r03/dense16_ab.jsonl)
#endif
template <int EPB>
struct DenseWalk {
    const TileFixParams* tp;
    unsigned total, nb, b0, step, per_strip, chunk;

    // false: no batch for this wave
    __device__ __forceinline__ bool init(const TileFixParams& t, unsigned blk, unsigned nblk)
    {
        tp = &t;
        const MapParams& p = t.m;
        const unsigned long long dc = *p.dense_ctr;
        const unsigned nd = (unsigned)(dc >> 32);
        total = (unsigned)dc;
        per_strip = 64u * (unsigned)p.tile_h;
        // the map launch numbered at most this many strips (a counter that did
        // not start at zero must not send the walk past the lists)
        const unsigned nstrips = (unsigned)t.tiles_x * ((unsigned)t.tile_w / 64u) * (unsigned)p.tiles_y;
        if (nd > nstrips || total > nstrips * per_strip) return false;   // uniform
        nb = (total + EPB - 1) / EPB;
        // chunks of up to DCTE_DENSE_CHUNK consecutive batches while every
        // wave still gets several (fewer batches: one at a time, all waves busy)
        chunk = min(max(nb / nblk, 1u), (unsigned)DCTE_DENSE_CHUNK);
        b0 = blk * chunk;
        step = nblk;
        return b0 < nb;
    }

    // the wave's batch after b (>= nb: none): chunk blk, blk + nblk, ... of
    // `chunk` consecutive batches -- a chunk's batches share window rows in
    // the wave's L1, the resident waves' chunks neighbour each other in the L2
    __device__ __forceinline__ unsigned next(unsigned b) const
    {
        return ((b + 1) % chunk != 0 && b + 1 < nb) ? b + 1 : (b / chunk + step) * chunk;
    }

    // batch b's entry of the batch map (b < nb): {first column, first output
    // row, strip, offset of its first entry in the flat list} of the strip
    // holding entry EPB b; loaded a batch ahead of its list()
    __device__ __forceinline__ uint4 info(unsigned b) const { return tp->m.dense_batch[b]; }

    // batch b's list word of entry EPB b + q (q < EPB); A = info(b), B =
    // info(b + 1) (b + 1 < nb; else A): a batch whose last entries lie in the
    // next strip finds that strip as the first one of batch b + 1 (a dense
    // strip holds more than EPB entries)
    __device__ __forceinline__ void list(unsigned b, const uint4& A, const uint4& B, unsigned q, unsigned& loc,
                                         int& sx0, int& ys, bool& valid) const
    {
        const unsigned e = b * EPB + q;
        valid = e < total;
        const bool up = B.z != A.z && e >= B.w;
        sx0 = (int)(up ? B.x : A.x);
        ys = (int)(up ? B.y : A.y);
        const unsigned idx = up ? B.z * per_strip + (e - B.w) : A.z * per_strip + (e - A.w);
        loc = tp->m.fix_list[valid ? idx : A.z * per_strip];
    }
};

// The batch map of a flat dense list, between the map launch and its
// refinement (a pass of its own: written from the map kernel's tail it cost
// the N = 16 map kernel a spilled register): wave k takes dense slot k and
// writes, for every batch of EPB entries whose first entry lies in that
// strip, {first column, first output row, strip, offset}.
template <int EPB>
__global__ __launch_bounds__(256) void dcte_dense_index(const TileFixParams tp)
{
    const MapParams& p = tp.m;
    const unsigned slot = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const unsigned nd = (unsigned)(*p.dense_ctr >> 32);
    const unsigned spt = (unsigned)tp.tile_w / 64u;
    const unsigned nstrips = (unsigned)tp.tiles_x * spt * (unsigned)p.tiles_y;
    if (slot >= nd || nd > nstrips) return;            // uniform per wave
    const uint2 v = p.dense_list[slot];
    const unsigned strip = v.x, off = v.y, cnt = p.tile_count[strip], tile = strip / spt;
    const uint4 di = make_uint4((unsigned)((int)(tile % (unsigned)tp.tiles_x) * tp.tile_w + 64 * (int)(strip % spt)),
                                (unsigned)tile_row0(p, (int)(tile / (unsigned)tp.tiles_x)), strip, off);
    const unsigned first = (off + EPB - 1u) / EPB, last = (off + cnt - 1u) / EPB;
    for (unsigned b = first + lane; b <= last; b += 64u) p.dense_batch[b] = di;
}

// ---- N = 16 dense strips (liblqr): four lanes per pixel ----------------
// 256 doubles do not fit one lane, so a window is split over the four rows
// (16 lanes each) of the wave: lane 16 q + w holds window lines 4q .. 4q + 3
// of pixel slot w (liblqr data[dx][dy]: line j = image row y - 7 + j, 16
// pixels along x), 64 doubles in registers.  The reference's first pass
// (ddct16x16s along the first index for each line, src/fft2d/shrtdct.c:
// 239-313) needs only the lane's own lines; the second pass needs whole
// coefficient rows k1, so the 16 x 16 block of first-pass outputs is
// transposed across the four rows with the gfx950 row swaps
// (v_permlane32_swap: rows 2-3 of one register <-> rows 0-1 of another;
// v_permlane16_swap: odd rows <-> even rows), 4 x 4 blocks of doubles at a
// time, no LDS: afterwards lane 16 q + w holds rows k1 = 4q .. 4q + 3.  The
// last-maximum scan (src/dct.c:100-108) reduces the four rows' maxima.

// the register swaps of one double (two dwords each)
__device__ __forceinline__ void swap_rows32(double& x, double& y)
{
    const unsigned long long a = (unsigned long long)__double_as_longlong(x);
    const unsigned long long b = (unsigned long long)__double_as_longlong(y);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)a, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(a >> 32), (unsigned)(b >> 32), false, false);
    x = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
    y = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}
__device__ __forceinline__ void swap_rows16(double& x, double& y)
{
    const unsigned long long a = (unsigned long long)__double_as_longlong(x);
    const unsigned long long b = (unsigned long long)__double_as_longlong(y);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)a, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(a >> 32), (unsigned)(b >> 32), false, false);
    x = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
    y = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}

// One window quarter: X[K][kk][jj] (K, kk, jj in 0..3) starts as the lane's
// first-pass outputs a[4K + kk][4q + jj] (its lines j = 4q + jj) and ends as
// a[4q + kk][4K + jj].  Stage 1 exchanges blocks between rows {0, 1} and
// {2, 3}, stage 2 within the pairs (0, 1), (2, 3).
__device__ __forceinline__ void transpose_quad(double (&X)[4][4][4])
{
#pragma unroll
    for (int kk = 0; kk < 4; kk++)
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
            swap_rows32(X[0][kk][jj], X[2][kk][jj]);
            swap_rows32(X[1][kk][jj], X[3][kk][jj]);
        }
#pragma unroll
    for (int kk = 0; kk < 4; kk++)
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
            swap_rows16(X[0][kk][jj], X[1][kk][jj]);
            swap_rows16(X[2][kk][jj], X[3][kk][jj]);
        }
}

template <int BPP>
struct D16Rows {
    static constexpr int NW = (16 * BPP + 3) / 4 + 1;  // dwords of a line's 16 pixels, any alignment
    uint32_t fv[4][NW];
    uint32_t foff;      // 2 bits per line
    uint32_t fast;      // bit per line
    int x, y;
    bool valid;
};

template <int BPP, int SEM>
__device__ __forceinline__ void fix_dense16_flat(const TileFixParams& tp, const double* lut,
                                                 unsigned blk, unsigned nblk)
{
    constexpr int N = 16;
    constexpr int HL = Geo<N, SEM>::HL;
    constexpr int NW = D16Rows<BPP>::NW;
    const MapParams& p = tp.m;
    DenseWalk<16> dw;
    if (!dw.init(tp, blk, nblk)) return;               // uniform
    const unsigned b0 = dw.b0, nb = dw.nb;
    const int lane = threadIdx.x, q = lane >> 4, slot = lane & 15;
    const uintptr_t pbase = reinterpret_cast<uintptr_t>(p.px);
    const uint32_t base_off = (uint32_t)(pbase & 3u);
    const unsigned nrec = base_off + (unsigned)((long long)(p.in_rows - 1) * p.rowstride) +
                          (unsigned)(p.w * BPP);
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(pbase - base_off), (short)0, (int)nrec, (int)kBufFlags);
    // liblqr luma (src/render.c:315, LQR_ER_LUMA) [liblqr, unverified]:
    // grey v / 255; RGB (k_r r + k_g g) + k_b b through the pre-weighted tables.
    // Preview: RGB2LUMINANCE (colour through fill_preview_lut's tables)
    auto luma3 = [&](uint32_t c0, uint32_t c1, uint32_t c2) -> double {
        if constexpr (SEM == kSemLqr) {
            if constexpr (BPP == 1) return lut[c0];
            else return lut[c0] + lut[256 + c1] + lut[512 + c2];
        } else if constexpr (BPP >= 3) {
            return (double)(unsigned char)((lut[c0] + lut[256 + c1]) + lut[512 + c2]);
        } else {
            return (double)preview_luma(c0, c1, c2, BPP);
        }
    };
    // this lane's four lines: image rows y - HL + 4q + jj, pixels x - HL .. x - HL + 15
    auto row_stage = [&](unsigned loc, int sx0, int ys, bool valid, D16Rows<BPP>& R) {
        R.x = sx0 + (int)(loc & 63u);
        R.y = ys + (int)(loc >> 6);
        R.valid = valid;
        const int gx0 = R.x - HL;
        const bool inside = valid && gx0 >= 0 && gx0 + 16 <= p.w;
        R.fast = 0;
        R.foff = 0;
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
            const int gy = clampi(R.y - HL + 4 * q + jj, 0, p.h - 1);
            const uint32_t s0 = base_off + (uint32_t)((long long)(gy - p.in_row0) * p.rowstride) +
                                (uint32_t)(gx0 * BPP);
            const bool fast = inside && ((s0 + 16 * BPP - 1) | 3u) < nrec;
            R.fast |= (uint32_t)fast << jj;
            R.foff |= (s0 & 3u) << (2 * jj);
            const uint32_t a = fast ? (s0 & ~3u) : 0x7ffffff0u;   // past num_records: zeros
#pragma unroll
            for (int j = 0; j < NW; j++)
                R.fv[jj][j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)(a + 4u * j), 0, 0);
        }
    };
    // X[K][kk][jj] = luma of line jj, pixel 4K + kk (the first index)
    auto convert = [&](const D16Rows<BPP>& R, double (&X)[4][4][4]) {
        const int gx0 = R.x - HL;
        // RGB: every pixel of every lane's lines grey (R = G = B) -> one
        // table read per element (lut[768 + v], the same double as the
        // three reads and two adds; fill_luma_lut) instead of three
        bool grey = false;
        if constexpr (BPP == 3) {
            bool mine = true;
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const uint32_t fo = (R.foff >> (2 * jj)) & 3u;
                uint32_t wd[12];
#pragma unroll
                for (int j = 0; j < 12; j++) wd[j] = __builtin_amdgcn_alignbyte(R.fv[jj][j + 1], R.fv[jj][j], fo);
                mine = mine && ((((R.fast >> jj) & 1u) && rgb_line_grey(wd)) || !R.valid);
            }
            grey = __all(mine);                          // uniform
        }
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
            double lv[16];
            // lanes without an entry decode their (zero) fetch like a fast line
            if (((R.fast >> jj) & 1u) || !R.valid) {
                const uint32_t fo = (R.foff >> (2 * jj)) & 3u;
                uint32_t wd[NW - 1];
#pragma unroll
                for (int j = 0; j < NW - 1; j++) wd[j] = __builtin_amdgcn_alignbyte(R.fv[jj][j + 1], R.fv[jj][j], fo);
                auto byte = [&](int b) { return (wd[b >> 2] >> (8 * (b & 3))) & 255u; };
                if (grey) {
#pragma unroll
                    for (int c = 0; c < 16; c++) lv[c] = lut[768 + byte(c * BPP)];
                } else {
#pragma unroll
                    for (int c = 0; c < 16; c++)
                        lv[c] = luma3(byte(c * BPP), BPP > 1 ? byte(c * BPP + 1) : 0u, BPP > 1 ? byte(c * BPP + 2) : 0u);
                }
            } else {
                // clamped at the left / right border, or at the frame's last
                // bytes (opaque copies: keep these addresses inside the branch)
                int xs = gx0, yr = R.y - HL + 4 * q + jj;
                asm volatile("" : "+v"(xs), "+v"(yr));
                const int gy = clampi(yr, 0, p.h - 1);
                const uint8_t* row = p.px + (long long)(gy - p.in_row0) * p.rowstride;
#pragma unroll
                for (int c = 0; c < 16; c++) {
                    const uint8_t* q8 = row + (long long)clampi(xs + c, 0, p.w - 1) * BPP;
                    lv[c] = luma3(q8[0], BPP > 1 ? q8[1] : 0u, BPP > 1 ? q8[2] : 0u);
                }
            }
#pragma unroll
            for (int c = 0; c < 16; c++) X[c >> 2][c & 3][jj] = lv[c];
        }
    };

    // batch-map entries of the next list16's batch b and of b + 1
    uint4 infA = dw.info(b0), infB = b0 + 1 < nb ? dw.info(b0 + 1) : infA;
    auto list16 = [&](unsigned b, unsigned& loc, int& sx0, int& ys, bool& valid) {
        const uint4 A = infA, B = infB;
        const unsigned bn = dw.next(b);
        if (bn < nb) {                                 // uniform
            infA = dw.info(bn);
            infB = bn + 1 < nb ? dw.info(bn + 1) : infA;
        }
        dw.list(b, A, B, (unsigned)slot, loc, sx0, ys, valid);
    };
    unsigned locN = 0;
    int sxN = 0, ysN = 0;
    bool vN = false;
    // a batch's lines load during the previous batch (without: +2 %)
    D16Rows<BPP> R;
    {
        unsigned loc0;
        int sx, ys;
        bool v;
        list16(b0, loc0, sx, ys, v);
        if (dw.next(b0) < nb) list16(dw.next(b0), locN, sxN, ysN, vN);
        row_stage(loc0, sx, ys, v, R);
    }
    for (unsigned b = b0; b < nb; b = dw.next(b)) {    // uniform
        double X[4][4][4];
        convert(R, X);
        const int x = R.x, y = R.y;
        const bool v = R.valid;
        // the next batch's loads reuse R's registers: not above the convert
        __builtin_amdgcn_sched_barrier(0);
        const unsigned bn = dw.next(b);
        if (bn < nb) {                                 // uniform
            row_stage(locN, sxN, ysN, vN, R);
            if (dw.next(bn) < nb) list16(dw.next(bn), locN, sxN, ysN, vN);
        }
        double rmax[4], c01 = 0.0, c10 = 0.0, r0_2 = -1.0, r1_1 = -1.0;
        // the maxima of coefficient row k1 = 4q + kk after its second pass
        auto row_max = [&](int kk, const double (&line)[16]) {
            double m2 = -1.0;
#pragma unroll
            for (int k2 = 2; k2 < 16; k2++) m2 = fmax(m2, fabs(line[k2]));
            if (kk == 0) {
                c01 = fabs(line[1]);
                r0_2 = m2;
            } else if (kk == 1) {
                c10 = fabs(line[0]);
                r1_1 = fmax(m2, fabs(line[1]));
            }
            rmax[kk] = fmax(fmax(fabs(line[0]), fabs(line[1])), m2);
        };
        if constexpr (SEM == kSemLqr) {
            // first pass: the lane's four lines along the first index (x)
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                double line[16];
#pragma unroll
                for (int c = 0; c < 16; c++) line[c] = X[c >> 2][c & 3][jj];
                r64::step16(line, 1);
#pragma unroll
                for (int c = 0; c < 16; c++) X[c >> 2][c & 3][jj] = line[c];
                __builtin_amdgcn_sched_barrier(0);
            }
            transpose_quad(X);
            // second pass: coefficient rows k1 = 4q + kk along the second index
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                double line[16];
#pragma unroll
                for (int j = 0; j < 16; j++) line[j] = X[j >> 2][kk][j & 3];
                r64::step16(line, 1);
                row_max(kk, line);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
            // preview data[r][c]: the first index is the image row, so the
            // lane first takes pixels 4q .. 4q + 3 with all 16 rows (the same
            // exchange), runs the first pass down them, and the exchange back
            // leaves it first-pass rows k1 = 4q + jj across all pixels
            transpose_quad(X);
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                double line[16];
#pragma unroll
                for (int l = 0; l < 16; l++) line[l] = X[l >> 2][kk][l & 3];
                r64::step16(line, 1);
#pragma unroll
                for (int l = 0; l < 16; l++) X[l >> 2][kk][l & 3] = line[l];
                __builtin_amdgcn_sched_barrier(0);
            }
            transpose_quad(X);
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                double line[16];
#pragma unroll
                for (int c = 0; c < 16; c++) line[c] = X[c >> 2][c & 3][jj];
                r64::step16(line, 1);
                row_max(jj, line);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // indices past N = (1, 0) in the scan order: rows 1 (from k2 = 1), 2, 3 of
        // quarter 0, every row of the others
        double ma = q == 0 ? fmax(r1_1, fmax(rmax[2], rmax[3]))
                           : fmax(fmax(rmax[0], rmax[1]), fmax(rmax[2], rmax[3]));
        ma = fmax(ma, __shfl_xor(ma, 16));
        ma = fmax(ma, __shfl_xor(ma, 32));
        double m;
        bool edge;
        lastmax_decide(c01, c10, r0_2, ma, m, edge);
        if (v && q == 0)
            p.out[(long long)(y - p.y0) * p.out_stride + x] =
                edge ? (float)(m * (double)p.edges) : (float)(m * (double)p.textures);
    }
}

template <int N, int BPP, int SEM>
__global__ __launch_bounds__(64, (kFixMinWaves<N, BPP>)) void dcte_fix_strips(const TileFixParams tp)
{
    using FS = FixStrip<N, SEM>;
    constexpr int LW = FS::LW, G = FS::G, SBH = FS::SBH, LR = FS::LR;
    constexpr int HL = Geo<N, SEM>::HL;
    const int TW = tp.tile_w;                          // the map launch's tile width
    const unsigned SPT = Lanes<N>::S == 1 ? (unsigned)TW / 64u : 1u;   // strips per tile
    constexpr int PB = ((LW * BPP + 3) & ~3) + 4;      // raw row pitch: the span + misalignment
    constexpr int PDW = PB / 4;
    constexpr bool kGroup = N >= 8;                    // N lanes per pixel (else one lane)
    constexpr int PPW = kGroup ? 64 / N : 64;          // pixels per wave pass
    // kOtf (grey layers): window elements converted from the band's raw bytes
    // as they are read -- one byte and one table read each -- instead of a
    // staged fp64 luma band: fewer LDS bytes, more waves per CU (line art
    // N = 8: 1.02 -> 0.67 ms, N = 16: 1.28 -> 0.96; profiles/r02/fix_otf_ab.jsonl).
    // RGB keeps the staged band: three bytes, three table reads and five fp64
    // operations per element read would cost more than the occupancy wins
    // (N = 16: 1.66 -> 1.93 ms).
    // liblqr RGB at N = 8 reads elements from the raw band too, with the three
    // weighted quotients k_c (v / 255) tabulated so a luma is two fp64 adds
    // ((k_r r + k_g g) + k_b b, the reference's order): line art RGB 1.41 ->
    // 1.33 ms; at N = 16 the same costs +30 % (profiles/r02/fix_otf_ab.jsonl)
    constexpr bool kTab = SEM == kSemLqr && BPP == 3 && (N == 8 || N == 4);
    constexpr bool kOtf = BPP == 1 || kTab;
    // dense strips go to fix_dense_lane / fix_dense16_flat (kDenseOwn): no band
    // staging here, and the N = 16 RGB dense blocks want pre-weighted tables
    constexpr bool kOwn = kDenseOwn<N, SEM>;
    constexpr bool kTab16 = N == 16 && kOwn && BPP == 3 && SEM == kSemLqr;
    constexpr bool kTabP = SEM == kSemPreview && kOwn && BPP >= 3;   // fill_preview_lut
    __shared__ double lut[(kTab || kTab16 || kTabP) ? 4 * 256 : 256];
    __shared__ double lum[(kOtf || kOwn) ? 1 : LR * LW];   // fp64 luma of one band (+ halo), needed columns
    __shared__ unsigned char mis[LR];                  // byte offset of each raw row's first pixel
    __shared__ unsigned char colidx[(kOtf || kOwn) ? 1 : LW];   // the needed luma columns, ascending
    // per group: N rows of N + 1 doubles, plus a pad that starts consecutive
    // groups 16 banks apart
    constexpr int WS = kGroup ? (N * (N + 1) + 7) / 8 * 8 + 8 : 1;
    // the band's raw rows and the groups' window buffers: one region when raw
    // is read only by the luma conversion (the windows only after it)
    // (no dense band here when the dense strips have a kernel of their own)
    constexpr int RAW_D = kOwn ? 0 : (LR * PDW + 1) / 2, WIN_D = (kGroup ? PPW : 1) * WS;
    constexpr int RW_D0 = kOtf ? RAW_D + WIN_D : (RAW_D > WIN_D ? RAW_D : WIN_D);
    constexpr int MEMO_D = N <= 8 && kOwn && BPP == 1 ? (kMemoDwords<N> + 1) / 2 : 0;   // the lane walk's memo (grey)
    constexpr int RW_D = RW_D0 > MEMO_D ? RW_D0 : MEMO_D;
    __shared__ __attribute__((aligned(16))) double rw_lds[RW_D];
    uint32_t* const raw = reinterpret_cast<uint32_t*>(rw_lds);
    double (*const win)[WS] = reinterpret_cast<double (*)[WS]>(rw_lds + (kOtf ? RAW_D : 0));
    const MapParams& p = tp.m;
    const unsigned ndirty = *p.dirty_count;
    if constexpr (kOwn) {
        // one launch for both: blocks past tp.sparse_blocks walk the dense strips
        if (blockIdx.x >= (unsigned)tp.sparse_blocks) {
            const unsigned blk = blockIdx.x - (unsigned)tp.sparse_blocks;
            const unsigned nblk = gridDim.x - (unsigned)tp.sparse_blocks;
            if constexpr (N <= 8) {
                if (blk >= ndirty) return;             // uniform
                if constexpr (kTabP) fill_preview_lut(lut, threadIdx.x);
                else fill_luma_lut<kTab>(lut, threadIdx.x);
                wave_sync_lds();
                // the window buffers of the sparse walk hold the dense walk's memo
                static_assert(BPP != 1 || sizeof(rw_lds) >= kMemoDwords<N> * sizeof(uint32_t), "memo fits");
                fix_dense_lane<N, BPP, SEM>(tp, lut, reinterpret_cast<uint32_t*>(rw_lds), blk, nblk);
            } else {
                if constexpr (kTabP) fill_preview_lut(lut, threadIdx.x);
                else fill_luma_lut<kTab16>(lut, threadIdx.x);
                wave_sync_lds();
                fix_dense16_flat<BPP, SEM>(tp, lut, blk, nblk);
            }
            return;
        }
    }
    constexpr int SB = kGroup ? PPW : 8;               // strips per batch (below)
    if (blockIdx.x * SB >= ndirty) return;             // uniform
    const int lane = threadIdx.x;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int v = lane + 64 * t;
        const double q = (double)v / 255;
        if constexpr (kTab) {
            lut[v] = 0.2126 * q;
            lut[256 + v] = 0.7152 * q;
            lut[512 + v] = 0.0722 * q;
        } else {
            lut[v] = q;
        }
    }
    wave_sync_lds();

    // the frame through a bounds-checked buffer resource (as dcte_map)
    const uintptr_t pbase = reinterpret_cast<uintptr_t>(p.px);
    const uint32_t base_off = (uint32_t)(pbase & 3u);
    const unsigned nrec = base_off + (unsigned)((long long)(p.in_rows - 1) * p.rowstride) +
                          (unsigned)(p.w * BPP);
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(pbase - base_off), (short)0, (int)nrec, (int)kBufFlags);

    // liblqr luma of a pixel (src/render.c:315, LQR_ER_LUMA) [liblqr, unverified];
    // preview: the u8 RGB2LUMINANCE (src/render.h:5)
    auto luma3 = [&](uint32_t c0, uint32_t c1, uint32_t c2) -> double {
        if constexpr (SEM == kSemLqr) {
            if constexpr (BPP == 1) return lut[c0];
            else if constexpr (kTab) return lut[c0] + lut[256 + c1] + lut[512 + c2];
            else return 0.2126 * lut[c0] + 0.7152 * lut[c1] + 0.0722 * lut[c2];
        } else {
            return (double)preview_luma(c0, c1, c2, BPP);
        }
    };
    auto luma = [&](const uint8_t* q) -> double {
        return luma3(q[0], BPP > 1 ? q[1] : 0u, BPP > 1 ? q[2] : 0u);
    };
    auto pixel = [&](int gx, int gy) {
        return p.px + (long long)(gy - p.in_row0) * p.rowstride + (long long)gx * BPP;
    };
    // window element (i, j): liblqr data[dx][dy] (src/render.c:150), preview
    // data[dy][dx] (src/render.c:49)
    auto offs = [](int i, int j, int& ox, int& oy) {
        ox = SEM == kSemLqr ? i : j;
        oy = SEM == kSemLqr ? j : i;
    };
    auto band_of = [](unsigned loc) { return (((int)(loc >> 6) + N - 1) / G) / FS::GPS; };

    // strip geometry: first column, output rows [ys, ye), refinement list
    struct StripGeo {
        int sx0, ys, ye;
        const unsigned* list;
    };
    auto geo = [&](unsigned strip) {
        StripGeo g;
        const unsigned tile = strip / SPT;
        const int bx = (int)(tile % (unsigned)tp.tiles_x), by = (int)(tile / (unsigned)tp.tiles_x);
        g.sx0 = bx * TW + 64 * (int)(strip % SPT);
        g.ys = tile_row0(p, by);
        g.ye = tile_row1(p, by);
        g.list = p.fix_list + (size_t)strip * (size_t)(64 * p.tile_h);
        return g;
    };
    auto store_at = [&](const StripGeo& g, int lx, int ly, double m, bool edge) {
        p.out[(long long)(g.ys + ly - p.y0) * p.out_stride + g.sx0 + lx] =
            edge ? (float)(m * (double)p.edges) : (float)(m * (double)p.textures);
    };

    // Dirty strips in batches of SB, one group of GL lanes per strip.  The
    // batch's sparse strips (cnt <= kFixDirect<N>) are refined side by side, their
    // windows gathered straight from global memory, so their latency chains
    // (dirty list -> count -> entries -> window bytes) overlap; its dense
    // strips follow one at a time, each walked by the whole wave.
    constexpr int GL = 64 / SB;
    const int sgi = lane / GL, sl = lane % GL;
    // the sparse walk's blocks: in a merged launch only the first
    // tp.sparse_blocks (the rest walk the dense strips), so they stride by
    // that many -- striding by gridDim.x skipped every strip batch past
    // sparse_blocks * SB in launches with more dirty strips than that
    const unsigned nsparse = kOwn ? (unsigned)tp.sparse_blocks : gridDim.x;
    for (unsigned k0 = blockIdx.x * SB; k0 < ndirty; k0 += nsparse * SB) {   // uniform
        const unsigned kk = k0 + sgi;
        unsigned my_strip = 0, my_cnt = 0;
        if (kk < ndirty) {
            my_strip = p.dirty_list[kk];
            my_cnt = p.tile_count[my_strip];
        }
        if (tp.fix_total && sl == 0 && my_cnt) atomicAdd(tp.fix_total, my_cnt);
        const bool sparse = my_cnt <= kFixDirect<N>;
        const StripGeo sg = geo(my_strip);
        const unsigned smax = wave_max_u(sparse ? my_cnt : 0u);
        if constexpr (!kGroup) {
            // lane sl of the group: entries sl, sl + GL, ... of its strip
            for (unsigned i0 = 0; i0 < smax; i0 += GL) {                 // uniform
                const unsigned i = i0 + sl;
                if (sparse && i < my_cnt) {
                    const unsigned loc = sg.list[i];
                    const int ly = (int)(loc >> 6), lx = (int)(loc & 63);
                    double d[N * N];
#pragma unroll
                    for (int ii = 0; ii < N; ii++)
#pragma unroll
                        for (int j = 0; j < N; j++) {
                            int ox, oy;
                            offs(ii, j, ox, oy);
                            d[ii * N + j] = luma(pixel(clampi(sg.sx0 + lx + ox - HL, 0, p.w - 1),
                                                       clampi(sg.ys + ly + oy - HL, 0, p.h - 1)));
                        }
                    double m;
                    bool edge;
                    refine_regs<N>(d, tp.ct, m, edge);
                    store_at(sg, lx, ly, m, edge);
                }
            }
        } else {
            // the group (GL = N lanes) takes its strip's entries one at a
            // time, software-pipelined through ONE fetch buffer: entry i's
            // bytes go to LDS first, then entry i + 1's loads (and entry
            // i + 2's list word) are issued and fly while entry i is
            // transformed.  Lane l fetches image row l of the window as whole
            // dwords (the row's N pixels: 3 dwords grey, 7 RGB at N = 8)
            // through the frame's buffer resource; windows clamped at the
            // left / right frame border, or whose last dword would straddle
            // the end of the readable bytes, gather per pixel instead (rare).
            // The loads are unconditional (an invalid or per-pixel entry
            // reads past the buffer's end: zeros, no access), so the wait
            // counts are the same on every path; list words are clamped
            // into the strip's own entries.
            const int l = sl;
            double* d = win[sgi];
            constexpr int NW = (N * BPP + 3) / 4;              // dwords of a row's N pixels
            constexpr int K = NW + 1;                          // loaded: any byte alignment
            uint32_t fv[K];
            uint32_t foff = 0;
            bool fwide = false;
            auto list_at = [&](unsigned i) {
                return sg.list[min(i, my_cnt > 0 ? my_cnt - 1 : 0u)];
            };
            auto fetch = [&](bool valid, unsigned loc) {
                const int ly = (int)(loc >> 6), lx = (int)(loc & 63);
                const int gx0 = sg.sx0 + lx - HL;
                const int gy = clampi(sg.ys + ly + l - HL, 0, p.h - 1);
                const uint32_t s = base_off + (uint32_t)((long long)(gy - p.in_row0) * p.rowstride) +
                                   (uint32_t)(gx0 * BPP);
                fwide = valid && gx0 >= 0 && gx0 + N <= p.w && ((s + N * BPP - 1) | 3u) < nrec;
                foff = s & 3u;
                const uint32_t a = fwide ? (s & ~3u) : 0x7ffffff0u;     // past num_records: zeros
#pragma unroll
                for (int j = 0; j < K; j++)
                    fv[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)(a + 4u * j), 0, 0);
            };
            unsigned lcur = list_at(0), lnext = list_at(1);
            fetch(sparse && my_cnt > 0, lcur);
            for (unsigned i = 0; i < smax; i++) {                         // uniform
                const bool valid = sparse && i < my_cnt;
                const int ly = (int)(lcur >> 6), lx = (int)(lcur & 63);
                if (valid) {
                    double lv[N];
                    if (fwide) {
                        uint32_t wd[NW];
#pragma unroll
                        for (int j = 0; j < NW; j++) wd[j] = __builtin_amdgcn_alignbyte(fv[j + 1], fv[j], foff);
#pragma unroll
                        for (int t = 0; t < N; t++) {
                            auto byte = [&](int k) { return (wd[k >> 2] >> (8 * (k & 3))) & 255u; };
                            lv[t] = luma3(byte(t * BPP), BPP > 1 ? byte(t * BPP + 1) : 0u,
                                          BPP > 1 ? byte(t * BPP + 2) : 0u);
                        }
                    } else {
                        const int gy = clampi(sg.ys + ly + l - HL, 0, p.h - 1);
#pragma unroll
                        for (int t = 0; t < N; t++)
                            lv[t] = luma(pixel(clampi(sg.sx0 + lx + t - HL, 0, p.w - 1), gy));
                    }
                    // image row l, pixel t: liblqr data[t][l], preview data[l][t]
#pragma unroll
                    for (int t = 0; t < N; t++) d[SEM == kSemLqr ? t * (N + 1) + l : l * (N + 1) + t] = lv[t];
                }
                // entry i + 1's bytes and entry i + 2's list word in flight
                const unsigned lafter = list_at(i + 2);
                fetch(sparse && i + 1 < my_cnt, lnext);
                wave_sync_lds();
                // the group transforms its window in place (d[i][j] = d[i * (N + 1) + j])
                if constexpr (N == 8) r64::step8(d + l, N + 1); else r64::step16(d + l, N + 1);
                wave_sync_lds();
                if constexpr (N == 8) r64::step8(d + (N + 1) * l, 1); else r64::step16(d + (N + 1) * l, 1);
                wave_sync_lds();
                double v[N];
#pragma unroll
                for (int c = 0; c < N; c++) v[c] = d[l * (N + 1) + c];
                double best;
                bool edge;
                lastmax_group<N>(v, l, best, edge);
                if (valid && l == 0) store_at(sg, lx, ly, best, edge);
                wave_sync_lds();
                lcur = lnext;
                lnext = lafter;
            }
        }

        // the batch's dense strips, one at a time (N = 8, N = 16 liblqr: the
        // dense walks of the extra blocks instead)
        uint64_t dense_mask = kOwn ? 0ull : __ballot(!sparse && sl == 0);
        while (dense_mask) {                                              // uniform
            const int leader = __builtin_ctzll(dense_mask);             // lane 0 of its group
            dense_mask &= dense_mask - 1;
            const unsigned strip = __shfl(my_strip, leader);
            const unsigned cnt = __shfl(my_cnt, leader);
            const StripGeo dg = geo(strip);
            const int sx0 = dg.sx0, ys = dg.ys, ye = dg.ye;
            const unsigned* list = dg.list;
            auto store = [&](int lx, int ly, double m, bool edge) { store_at(dg, lx, ly, m, edge); };

            // dense strip, band by band.  The entries are sorted by band (the map
            // kernel emits them group by group; band = group / GPS), so a band's
            // entries are a contiguous run [pos, end) of the list.  Software
            // pipelined: the next run's first list chunk and (interior strips) its
            // band's raw rows are in flight while this band converts and computes.
            const bool interior = sx0 - HL >= 0 && (sx0 - HL + LW) * BPP + 3 <= p.w * BPP;
            constexpr int SPAN = LW * BPP;
            constexpr int U = (LR * PDW + 63) / 64;
            // fp64 luma of band row r, span column c
            // raw pixel (r, c) of the band: its bytes through the one or two
            // ALIGNED dwords holding them (byte-wise reads got merged into
            // unaligned 64-bit LDS reads: a third of the LDS cycles stalled)
            auto px_at = [&](int r, int c) -> uint32_t {
                const uint32_t o = (uint32_t)(r * PB) + mis[r] + (uint32_t)(c * BPP);
                if constexpr (BPP == 1) {
                    return reinterpret_cast<const uint8_t*>(raw)[o];
                } else {
                    const uint32_t lo = raw[o >> 2], hi = raw[(o >> 2) + 1];
                    return __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
                }
            };
            auto luma_px = [&](uint32_t v) -> double {
                return luma3(v & 255u, (v >> 8) & 255u, (v >> 16) & 255u);
            };
            auto lum_at = [&](int r, int c) -> double {
                if constexpr (kOtf)
                    return luma_px(px_at(r, c));
                else
                    return lum[r * LW + c];
            };
            // liblqr: the N pixels of band row r from column c on (a lane's
            // window line) as whole aligned dwords
            auto line_at = [&](int r, int c, double (&lv)[N]) {
                constexpr int NW = (N * BPP + 3) / 4;
                const uint32_t o = (uint32_t)(r * PB) + mis[r] + (uint32_t)(c * BPP);
                const uint32_t* q = raw + (o >> 2);
                uint32_t v[NW + 1];
#pragma unroll
                for (int j = 0; j <= NW; j++) v[j] = q[j];
                uint32_t wd[NW];
#pragma unroll
                for (int j = 0; j < NW; j++) wd[j] = __builtin_amdgcn_alignbyte(v[j + 1], v[j], o & 3u);
#pragma unroll
                for (int t = 0; t < N; t++) {
                    auto byte = [&](int k) { return (wd[k >> 2] >> (8 * (k & 3))) & 255u; };
                    lv[t] = luma3(byte(t * BPP), BPP > 1 ? byte(t * BPP + 1) : 0u,
                                  BPP > 1 ? byte(t * BPP + 2) : 0u);
                }
            };
            auto band_rows = [&](int bb, int& r0, int& nrows) {
                // band bb: output rows [max(A, 0), min(A + SBH, ye - ys)), A = bb SBH - (N - 1);
                // input rows from r0 = max(A, 0) - HL (tile-relative)
                const int A = bb * SBH - (N - 1);
                r0 = max(A, 0) - HL;
                nrows = min(A + SBH, ye - ys) - max(A, 0) + N - 1;
            };
            uint32_t v[U];
            // raw dwords of band bb -> v (interior strips: every row's span is in
            // the frame); each row's misalignment -> mis
            // byte offset of the span's first pixel in frame row gy
            auto row_addr = [&](int gy) -> uint32_t {
                return base_off + (uint32_t)((long long)(gy - p.in_row0) * p.rowstride) +
                       (uint32_t)((sx0 - HL) * BPP);
            };
            auto issue_raw = [&](int bb) {
                int r0, nrows;
                band_rows(bb, r0, nrows);
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int e = lane + 64 * u;
                    const int r = e / PDW, dw = e - r * PDW;
                    v[u] = 0;
                    if (r < nrows) {
                        const int gy = clampi(ys + r0 + r, 0, p.h - 1);
                        const uint32_t a = row_addr(gy);
                        if (dw * 4 < (int)(a & 3u) + SPAN)
                            v[u] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)((a & ~3u) + 4u * dw), 0, 0);
                    }
                }
            };
            unsigned loc = (unsigned)lane < cnt ? list[lane] : 0u;      // the first run's first chunk
            int b = band_of(__shfl(loc, 0));
            if (interior) issue_raw(b);
            for (unsigned pos = 0; pos < cnt;) {                           // uniform
                // the run's end and the luma columns its windows need (a 128-bit
                // mask); a run of <= 64 entries stays in registers (loc0)
                unsigned end = pos;
                const unsigned loc0 = loc;
                bool single = true;
                uint64_t mlo = 0, mhi = 0;
                for (int chunk = 0;; chunk++) {
                    const unsigned q = end + lane;
                    const unsigned lc = chunk == 0 ? loc : (q < cnt ? list[q] : 0u);
                    const bool in = q < cnt && band_of(lc) == b;
                    if (in) {
                        constexpr uint64_t bits = (1ull << N) - 1;
                        const int lx = (int)(lc & 63);
                        mlo |= bits << lx;
                        if (lx + N > 64) mhi |= bits >> (64 - lx);
                    }
                    const int nin = __popcll(__ballot(in));     // a prefix of the lanes
                    end += nin;
                    if (nin < 64) break;
                    single = false;
                }
                // the next run's first chunk, in flight through this band
                const unsigned locN = end + lane < cnt ? list[end + lane] : 0u;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    mlo |= __shfl_xor(mlo, o);
                    mhi |= __shfl_xor(mhi, o);
                }
                const uint32_t m0 = (uint32_t)mlo, m1 = (uint32_t)(mlo >> 32), m2 = (uint32_t)mhi;
                int r0, nrows;
                band_rows(b, r0, nrows);
                // raw bytes of the band's rows
                if (interior) {
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const int e = lane + 64 * u;
                        if (e < nrows * PDW) {
                            raw[e] = v[u];
                            // each row's misalignment, written with its bytes (the
                            // next band's loads are issued while this band's
                            // windows still read mis)
                            const int r = e / PDW;
                            if (e == r * PDW)
                                mis[r] = (unsigned char)(row_addr(clampi(ys + r0 + r, 0, p.h - 1)) & 3u);
                        }
                    }
                } else {
                    for (int e = lane; e < nrows * LW; e += 64) {
                        const int r = e / LW, c = e - r * LW;
                        const uint8_t* src = pixel(clampi(sx0 - HL + c, 0, p.w - 1), clampi(ys + r0 + r, 0, p.h - 1));
                        uint8_t* dst = reinterpret_cast<uint8_t*>(&raw[r * PDW]) + c * BPP;
#pragma unroll
                        for (int ch = 0; ch < BPP; ch++) dst[ch] = src[ch];
                        if (c == 0) mis[r] = 0;
                    }
                }
                if constexpr (!kOtf) {
                // the needed columns, compacted
                const int n0 = __popc(m0), n1 = __popc(m1);
                const int ncols = n0 + n1 + __popc(m2);
                for (int c = lane; c < LW; c += 64) {
                    const uint32_t word = c < 32 ? m0 : (c < 64 ? m1 : m2);
                    const int bit = c & 31;
                    if ((word >> bit) & 1u) {
                        const int before = (c < 32 ? 0 : (c < 64 ? n0 : n0 + n1)) +
                                           __popc(word & ((1u << bit) - 1u));
                        colidx[before] = (unsigned char)c;
                    }
                }
                wave_sync_lds();
                // fp64 luma of the needed columns, kConv elements per lane at a time
                // (their LDS round trips overlap)
                constexpr int kConv = 4;
                const float inv = 1.0f / (float)max(ncols, 1);
                const int total = nrows * ncols;
                for (int e0 = lane; e0 < total; e0 += 64 * kConv) {
                    int at[kConv], cc[kConv];
#pragma unroll
                    for (int k = 0; k < kConv; k++) {
                        const int e = min(e0 + 64 * k, total - 1);  // tail: repeat the last element
                        int r = (int)((float)e * inv);             // e / ncols, corrected (e < 2^12)
                        r += (r + 1) * ncols <= e;
                        r -= r * ncols > e;
                        at[k] = r;
                        cc[k] = e - r * ncols;
                    }
#pragma unroll
                    for (int k = 0; k < kConv; k++) cc[k] = colidx[cc[k]];
                    double lv[kConv];
#pragma unroll
                    for (int k = 0; k < kConv; k++)
                        lv[k] = luma(reinterpret_cast<const uint8_t*>(&raw[at[k] * PDW]) + mis[at[k]] + cc[k] * BPP);
#pragma unroll
                    for (int k = 0; k < kConv; k++) lum[at[k] * LW + cc[k]] = lv[k];
                }
                }   // !kOtf
                wave_sync_lds();
                // the next run's band: its raw rows in flight through this band's compute
                int bN = b;
                if (end < cnt) {                                       // uniform
                    bN = band_of(__shfl(locN, 0));
                    if (interior) issue_raw(bN);
                }
                // element (i, j) of pixel (lx, ly): lum row ly + oy - HL - r0, column lx + ox
                if constexpr (!kGroup) {
                    for (unsigned q = pos + lane; q < end; q += 64) {
                        const unsigned lc = single ? loc0 : list[q];
                        const int ly = (int)(lc >> 6), lx = (int)(lc & 63);
                        double d[N * N];
#pragma unroll
                        for (int i = 0; i < N; i++)
#pragma unroll
                            for (int j = 0; j < N; j++) {
                                int ox, oy;
                                offs(i, j, ox, oy);
                                d[i * N + j] = lum_at(ly - HL - r0 + oy, lx + ox);
                            }
                        double m;
                        bool edge;
                        refine_regs<N>(d, tp.ct, m, edge);
                        store(lx, ly, m, edge);
                    }
                } else {
                    const int l = lane & (N - 1), grp = lane / N;
                    for (unsigned q0 = pos; q0 < end; q0 += PPW) {        // uniform
                        const unsigned q = q0 + grp;
                        const bool valid = q < end;
                        const unsigned lq = __shfl(loc0, (int)(q - pos) & 63);
                        const unsigned lc = single ? (valid ? lq : loc0) : list[valid ? q : pos];
                        const int ly = (int)(lc >> 6), lx = (int)(lc & 63);
                        double best;
                        bool edge;
                        const int rr = ly - HL - r0;
                        if constexpr (kOtf && SEM == kSemLqr) {
                            // liblqr: lane l reads window row l (contiguous bytes)
                            double lv[N];
                            line_at(rr + l, lx, lv);
                            refine_group_f<N>([&](int i) { return lv[i]; }, win[grp], l, best, edge);
                        } else if constexpr (kOtf) {
                            // liblqr: lane l reads window row l; preview: window column l
                            refine_group_f<N>([&](int i) {
                                return SEM == kSemLqr ? lum_at(rr + l, lx + i) : lum_at(rr + i, lx + l);
                            }, win[grp], l, best, edge);
                        } else {
                            refine_group<N, SEM>(lum, LW, rr * LW + lx, win[grp], l, best, edge);
                        }
                        if (valid && l == 0) store(lx, ly, best, edge);
                    }
                }
                wave_sync_lds();                           // lum / raw / colidx free for the next band
                pos = end;
                loc = locN;
                b = bN;
            }
        }
    }
}

// ------------------------------------------------------------------ windows
// dctNxN + weighted_max_dct_correlation (src/dct.c:77-110) on windows the
// caller filled -- the per-window form of the callback (src/render.c:146-155
// fills data[dx][dy] and calls exactly these two) -- in fp64 in the
// reference's operation order: bit-identical to the reference.  One lane per
// window for N <= 8 (registers), one 16-lane group for N = 16 (LDS).
template <int N>
__global__ __launch_bounds__(kFixThreads) void dcte_windows(const WinParams p)
{
    __shared__ double win[N == 16 ? kFixThreads / 16 : 1][N == 16 ? 256 : 1];
    if constexpr (N <= 8) {
        for (long long k = blockIdx.x * (long long)kFixThreads + threadIdx.x; k < p.count;
             k += (long long)gridDim.x * kFixThreads) {
            const double* src = p.win + k * (N * N);
            double d[N * N];
#pragma unroll
            for (int e = 0; e < N * N; e++) d[e] = src[e];
            double m;
            bool edge;
            refine_regs<N>(d, p.ct, m, edge);
            p.out[k] = edge ? (float)(m * (double)p.edges) : (float)(m * (double)p.textures);
        }
    } else {
        const int l = threadIdx.x & 15, slot = threadIdx.x >> 4;
        double* d = win[slot];
        const long long per_pass = (long long)gridDim.x * (kFixThreads / 16);
        const long long rounds = (p.count + per_pass - 1) / per_pass;   // uniform
        for (long long r = 0; r < rounds; r++) {
            const long long k = r * per_pass + blockIdx.x * (kFixThreads / 16) + slot;
            const bool valid = k < p.count;
            if (valid) {
#pragma unroll
                for (int t = 0; t < 16; t++) d[t * 16 + l] = p.win[k * 256 + t * 16 + l];
            }
            wave_sync_lds();
            double m;
            bool edge;
            refine16_group(d, l, m, edge);
            if (valid && l == 0) p.out[k] = edge ? (float)(m * (double)p.edges) : (float)(m * (double)p.textures);
            wave_sync_lds();
        }
    }
}

// ------------------------------------------------------------------ launchers
int map_tile_w(int n)
{
    return n == 16 ? Geo<16, kSemLqr>::TW
                   : (n == 8 ? Geo<8, kSemLqr>::TW : (n == 4 ? Geo<4, kSemLqr>::TW : Geo<2, kSemLqr>::TW));
}
int map_default_tile_h(int n) { return n == 16 ? DCTE_TILE_H16 : DCTE_TILE_H; }
int map_tiles_x(int n, int w) { return (w + map_tile_w(n) - 1) / map_tile_w(n); }
int map_tiles_y(int n, int rows, int tile_h) { return (rows + tile_h - 1) / tile_h; }
int map_strips_per_tile(int n) { return n == 16 ? 1 : map_tile_w(n) / 64; }

// workgroups of dcte_map<N, BPP, SEM> one CU holds at once (the launch-shape
// model of the host, dcte_capi.cpp pick_tile_h); cached per instantiation
template <int N, int BPP, int SEM>
static int map_blocks_per_cu_t()
{
    static std::atomic<int> cache{0};
    int v = cache.load(std::memory_order_relaxed);
    if (!v) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_map<N, BPP, SEM>, Geo<N, SEM>::T, 0) != hipSuccess || v <= 0)
            v = 1;
        cache.store(v, std::memory_order_relaxed);
    }
    return v;
}
template <int N>
static int map_blocks_per_cu_n(int bpp, int sem)
{
    if (sem == kSemLqr) return bpp == 1 ? map_blocks_per_cu_t<N, 1, kSemLqr>() : map_blocks_per_cu_t<N, 3, kSemLqr>();
    if (bpp == 1) return map_blocks_per_cu_t<N, 1, kSemPreview>();
    return bpp == 3 ? map_blocks_per_cu_t<N, 3, kSemPreview>() : map_blocks_per_cu_t<N, 4, kSemPreview>();
}
int map_blocks_per_cu(int n, int bpp, int sem)
{
    switch (n) {
    case 2: return map_blocks_per_cu_n<2>(bpp, sem);
    case 4: return map_blocks_per_cu_n<4>(bpp, sem);
    case 8: return map_blocks_per_cu_n<8>(bpp, sem);
    default: return map_blocks_per_cu_n<16>(bpp, sem);
    }
}

// With ev_a / ev_b (DCTE_OPT_PROFILE), the launch itself records the kernel's
// start and end (hipExtLaunchKernel: timestamps of the dispatch, no marker
// packets of their own -- two hipEventRecord calls around the launch cost a
// 4096^2 call ~6 us, r06)
template <int N, int BPP, int SEM>
static hipError_t launch_map_t(const MapParams& p, hipStream_t s, hipEvent_t ev_a, hipEvent_t ev_b)
{
    constexpr int TW = Geo<N, SEM>::TW;
    dim3 grid((p.w + TW - 1) / TW, p.tiles_y);
    if (ev_a || ev_b) {
        MapParams arg = p;
        void* args[] = {&arg};
        return hipExtLaunchKernel(reinterpret_cast<const void*>(&dcte_map<N, BPP, SEM>), grid,
                                  dim3(Geo<N, SEM>::T), args, 0, s, ev_a, ev_b, 0);
    }
    hipLaunchKernelGGL((dcte_map<N, BPP, SEM>), grid, dim3(Geo<N, SEM>::T), 0, s, p);
    return hipGetLastError();
}

template <int N>
static hipError_t launch_map_n(int bpp, int sem, const MapParams& p, hipStream_t s, hipEvent_t a, hipEvent_t b)
{
    if (sem == kSemLqr) {
        if (bpp == 1) return launch_map_t<N, 1, kSemLqr>(p, s, a, b);
        if (bpp == 3) return launch_map_t<N, 3, kSemLqr>(p, s, a, b);
    } else if (sem == kSemPreview) {
        if (bpp == 1) return launch_map_t<N, 1, kSemPreview>(p, s, a, b);
        if (bpp == 3) return launch_map_t<N, 3, kSemPreview>(p, s, a, b);
        if (bpp == 4) return launch_map_t<N, 4, kSemPreview>(p, s, a, b);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_map(int n, int bpp, int sem, const MapParams& p, hipStream_t s, hipEvent_t ev_a,
                      hipEvent_t ev_b)
{
    if (p.tiles_y <= 0) {
        // nothing to launch: the events still mark this point of the stream
        hipError_t e = hipSuccess;
        if (ev_a) e = hipEventRecord(ev_a, s);
        if (e == hipSuccess && ev_b) e = hipEventRecord(ev_b, s);
        return e;
    }
    switch (n) {
    case 2: return launch_map_n<2>(bpp, sem, p, s, ev_a, ev_b);
    case 4: return launch_map_n<4>(bpp, sem, p, s, ev_a, ev_b);
    case 8: return launch_map_n<8>(bpp, sem, p, s, ev_a, ev_b);
    case 16: return launch_map_n<16>(bpp, sem, p, s, ev_a, ev_b);
    default: return hipErrorInvalidValue;
    }
}

template <int N>
static void launch_fix_n(const FixParams& p, hipStream_t s)
{
    // enough blocks for the most pixels this launch can flag, capped at ~8
    // waves per CU; blocks past the device-side count return at once
    const unsigned per_block = kFixThreads / (N == 16 ? 16 : 1);
    unsigned blocks = (p.max_items + per_block - 1) / per_block;
    blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
    if (p.sem == kSemLqr)
        hipLaunchKernelGGL((dcte_fix<N, kSemLqr>), dim3(blocks), dim3(kFixThreads), 0, s, p);
    else
        hipLaunchKernelGGL((dcte_fix<N, kSemPreview>), dim3(blocks), dim3(kFixThreads), 0, s, p);
}

constexpr int kMaxDevices = 64;

template <int N, int BPP, int SEM>
static hipError_t launch_fix_tiles_t(const TileFixParams& p, hipStream_t s)
{
    if (p.m.tile_h < 1 || p.tile_w != map_tile_w(N) || p.tiles_x != (p.m.w + p.tile_w - 1) / p.tile_w)
        return hipErrorInvalidValue;
    const int nstrips = p.tiles_x * map_strips_per_tile(N) * p.m.tiles_y;
    // one wave per block, as many as the device holds at once (LDS-bound:
    // ~10 per CU at N = 8 RGB); each walks the dirty list in strip batches.
    // Cached per device (CU counts may differ between devices).
    static std::atomic<int> cache[kMaxDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    int resident = dev >= 0 && dev < kMaxDevices ? cache[dev].load(std::memory_order_relaxed) : 0;
    if (!resident) {
        int cus = 0, per_cu = 0;
        if (dev >= 0 &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dcte_fix_strips<N, BPP, SEM>, 64, 0) ==
                hipSuccess && cus > 0 && per_cu > 0)
            resident = cus * per_cu;
        else
            resident = 2048;
        if (dev >= 0 && dev < kMaxDevices) cache[dev].store(resident, std::memory_order_relaxed);
    }
    // the sparse walk takes SB strips per block and pass (dcte_fix_strips):
    // more blocks than batches only launch to exit (a band's edge ranges)
    constexpr int SB = N >= 8 ? 64 / N : 8;            // = dcte_fix_strips' SB
    const int batches = (nstrips + SB - 1) / SB;
    const int blocks = batches < resident ? batches : resident;
    if constexpr (kDenseFlat<N, SEM>) {
        // the flat list's batch map first (one wave per possible listed strip)
        hipLaunchKernelGGL((dcte_dense_index<kDenseBatch16>), dim3((nstrips + 3) / 4), dim3(256), 0, s, p);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    if constexpr (kDenseOwn<N, SEM>) {
        // the dense strips' walk: extra blocks of the same launch, up to one
        // wave per batch the flat list could hold (N = 16) or per strip (N = 8)
        const long long most = kDenseFlat<N, SEM>
                                   ? ((long long)nstrips * 64 * p.m.tile_h + kDenseBatch16 - 1) / kDenseBatch16
                                   : nstrips;
        const long long npx = (long long)p.m.w * ((p.m.y1 - p.m.y0) + (p.m.yb1 - p.m.yb0));
        const int memo8 = npx < DCTE_MEMO8_BIG_PX ? 1 : DCTE_DENSE_OVERSUB_MEMO8;
        const long long dmax = (long long)resident * (N <= 8 && BPP == 1 ? (N == 8 ? memo8 : DCTE_DENSE_OVERSUB_MEMO)
                                                                     : DCTE_DENSE_OVERSUB);
        const int dblocks = (int)(most < dmax ? most : dmax);
        TileFixParams q = p;
        q.sparse_blocks = blocks;
        hipLaunchKernelGGL((dcte_fix_strips<N, BPP, SEM>), dim3(blocks + dblocks), dim3(64), 0, s, q);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((dcte_fix_strips<N, BPP, SEM>), dim3(blocks), dim3(64), 0, s, p);
    return hipGetLastError();
}

template <int N>
static hipError_t launch_fix_tiles_n(int bpp, int sem, const TileFixParams& p, hipStream_t s)
{
    if (sem == kSemLqr) {
        if (bpp == 1) return launch_fix_tiles_t<N, 1, kSemLqr>(p, s);
        if (bpp == 3) return launch_fix_tiles_t<N, 3, kSemLqr>(p, s);
    } else if (sem == kSemPreview) {
        if (bpp == 1) return launch_fix_tiles_t<N, 1, kSemPreview>(p, s);
        if (bpp == 3) return launch_fix_tiles_t<N, 3, kSemPreview>(p, s);
        if (bpp == 4) return launch_fix_tiles_t<N, 4, kSemPreview>(p, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_fix_tiles(int n, int bpp, int sem, const TileFixParams& p, hipStream_t s)
{
    if (p.m.tiles_y <= 0) return hipSuccess;
    switch (n) {
    case 2: return launch_fix_tiles_n<2>(bpp, sem, p, s);
    case 4: return launch_fix_tiles_n<4>(bpp, sem, p, s);
    case 8: return launch_fix_tiles_n<8>(bpp, sem, p, s);
    case 16: return launch_fix_tiles_n<16>(bpp, sem, p, s);
    default: return hipErrorInvalidValue;
    }
}

int dense_batch_entries(int n, int sem)
{
    if (n == 16) return (sem == kSemLqr ? kDenseFlat<16, kSemLqr> : kDenseFlat<16, kSemPreview>) ? (int)kDenseBatch16 : 0;
    return 0;
}

hipError_t launch_windows(const WinParams& p, hipStream_t s)
{
    if (p.count <= 0) return hipSuccess;
    const long long per_block = p.n == 16 ? kFixThreads / 16 : kFixThreads;
    const long long want = (p.count + per_block - 1) / per_block;
    const dim3 grid((unsigned)(want < 2048 ? want : 2048)), block(kFixThreads);
    switch (p.n) {
    case 2: hipLaunchKernelGGL((dcte_windows<2>), grid, block, 0, s, p); break;
    case 4: hipLaunchKernelGGL((dcte_windows<4>), grid, block, 0, s, p); break;
    case 8: hipLaunchKernelGGL((dcte_windows<8>), grid, block, 0, s, p); break;
    case 16: hipLaunchKernelGGL((dcte_windows<16>), grid, block, 0, s, p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_fix(const FixParams& p, hipStream_t s)
{
    switch (p.n) {
    case 2: launch_fix_n<2>(p, s); break;
    case 4: launch_fix_n<4>(p, s); break;
    case 8: launch_fix_n<8>(p, s); break;
    case 16: launch_fix_n<16>(p, s); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace dcte
