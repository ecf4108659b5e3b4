// dcte_exact.hip -- the energy map in the reference's own fp64 arithmetic,
// bit-identical to dct_pixel_energy for every pixel (DCTE_OPT_EXACT).
//
// What the reference computes per pixel (src/render.c:134-157, src/dct.c:
// 77-110): the N x N window data[dx][dy] of liblqr luma (double), dctNxN, and
// the last-maximum scan.  For N = 8 dctNxN is ddct8x8s(-1, data)
// (src/fft2d/shrtdct.c:55-117): pass 1 transforms along the FIRST index for
// every second index j (shrtdct.c:62-89) -- the first index is dx, so pass 1
// is an 8-point transform along one image row, the same doubles for every
// pixel of that column whose window holds the row; pass 2 transforms each
// coefficient row k1 along dy (shrtdct.c:90-117).
//
// So the sliding-window structure of the fp32 map (dcte_kernels.hip) holds in
// fp64 bit for bit: a lane owns one output column and walks DOWN a strip; each
// input row's pass-1 transform is computed ONCE and kept in a register ring of
// the last 8 rows (64 doubles); each output pixel then runs the 8 pass-2
// steps over the ring.  Every operation is the reference's own (same operands,
// same order, no contraction: the Makefile builds with -ffp-contract=off), so
// every coefficient is the reference's double.  The scan is decided from
// maxima of the scan's own doubles (lastmax_decide, as in dcte_kernels.hip),
// with one exact shortcut: for k1 >= 2, max(|C_k1,0|, |C_k1,4|) =
// fl(C8_4R * fl(|xr| + |xi|)) (rounding is monotone and sign-symmetric, so the
// larger of fl(c * fl(xr + xi)) and fl(c * fl(xr - xi)) in magnitude is that
// value), and both coefficients sit on the same side of (1,0) in the scan.
//
// Cost (fp64 VALU lane-ops per pixel): pass 1 42, pass 2 364 - 42 + 40 ...:
// 42 + 40 (k1 = 0, C00 never formed) + 42 (k1 = 1) + 6 x 40 = 364 transform
// ops, 53 maxima, 7 for the decision and the weight: ~426 -- against ~860 for
// refining one window from scratch (dcte_fix*), which is what the r04 exact
// mode (tie_tau = 1) paid per pixel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <utility>

#include "dcte_kernels.h"
#include "dcte_luma.h"
#include "dcte_ref64.h"

namespace dcte {
namespace {

#ifndef DCTE_EX_TILE_H
#define DCTE_EX_TILE_H 128   // output rows per workgroup
#endif
#ifndef DCTE_EX_MINW
#define DCTE_EX_MINW 2       // N = 8: waves per SIMD the register budget is cut for (<= 256 VGPRs)
#endif
#ifndef DCTE_EX16_MINW
#define DCTE_EX16_MINW 4     // N = 16 (8-wave workgroups: 4 = two of them per CU, <= 128 VGPRs)
#endif

constexpr unsigned kRawFlags = 0x00020000u;   // gfx9 raw buffer dword3

template <int... Is, class F>
__device__ __forceinline__ void sfor_impl(std::integer_sequence<int, Is...>, F&& f)
{
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int Count, class F>
__device__ __forceinline__ void sfor(F&& f)
{
    sfor_impl(std::make_integer_sequence<int, Count>{}, f);
}

__device__ __forceinline__ int clampx(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// the weight of a decision: edges or textures, selected in registers.  The
// operands go through an empty asm so the optimiser cannot turn the select
// into a load through a selected address (it did: the weights live in the
// lambdas' closures, and a select between two loads from them became a
// dynamically indexed closure, i.e. scratch memory)
__device__ __forceinline__ double weight(bool edge, double we, double wt)
{
    asm volatile("" : "+v"(we), "+v"(wt));
    return edge ? we : wt;
}

using r64::K8;

using r64::col8;

// Frame bytes through one bounds-checked buffer resource over the readable
// rows (a dword straddling the end reads as 0: the <= 3 tail bytes are fetched
// once by the workgroups that reach them and patched in).
struct Frame {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t base_off, nrec4, tail;
    long long rowstride;
    int in_row0;
    bool tail_wg;

    __device__ __forceinline__ void init(const MapParams& p, int bpp, bool reaches_end)
    {
        const uintptr_t pbase = reinterpret_cast<uintptr_t>(p.px);
        rowstride = p.rowstride;
        in_row0 = p.in_row0;
        base_off = (uint32_t)(pbase & 3u);
        const unsigned nrec = base_off + (unsigned)((long long)(p.in_rows - 1) * p.rowstride) +
                              (unsigned)(p.w * bpp);
        nrec4 = nrec & ~3u;
        rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(pbase - base_off), (short)0,
                                                 (int)nrec, (int)kRawFlags);
        tail_wg = (nrec & 3u) != 0u && reaches_end;
        tail = 0;
        if (tail_wg) {
            for (uint32_t b = 0; b < (nrec & 3u); b++)
                tail |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, (int)(nrec4 + b), 0, 0) << (8u * b);
        }
    }
    // byte offset (from the aligned base) of pixel (x, global row y)
    __device__ __forceinline__ uint32_t at(int x, int y, int bpp) const
    {
        return base_off + (uint32_t)((long long)(y - in_row0) * rowstride) + (uint32_t)(x * bpp);
    }
    // the 8 bytes from the dword holding byte a on
    __device__ __forceinline__ uint2 fetch(uint32_t a) const
    {
        const uint32_t a4 = a & ~3u;
        auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)a4, 0, 0);
        if (tail_wg) {
            if (a4 == nrec4) v[0] = tail;
            else if (a4 + 4u == nrec4) v[1] = tail;
        }
        return make_uint2(v[0], v[1]);
    }
};

// liblqr luma tables (LQR_ER_LUMA [liblqr, unverified], as dcte_ref64.h's
// luma): grey lut[v] = v / 255; RGB lut[c * 256 + v] = k_c * (v / 255), so
// (lut[r] + lut[256 + g]) + lut[512 + b] is the reference's double
template <int BPP>
__device__ __forceinline__ void fill_lut(double* lut, int tx, int nthreads)
{
    for (int v = tx; v < 256; v += nthreads) {
        const double q = (double)v / 255;
        if constexpr (BPP == 1) {
            lut[v] = q;
        } else {
            lut[v] = 0.2126 * q;
            lut[256 + v] = 0.7152 * q;
            lut[512 + v] = 0.0722 * q;
        }
    }
}
template <int BPP>
__device__ __forceinline__ double luma_of(const double* lut, uint32_t wd)
{
    if constexpr (BPP == 1) return lut[wd & 255u];
    else return (lut[wd & 255u] + lut[256 + ((wd >> 8) & 255u)]) + lut[512 + ((wd >> 16) & 255u)];
}

// first / one-past-last output row of tile row by (tile_row0 / tile_row1 of
// dcte_kernels.h) in arithmetic: a select between two fields of the kernel
// argument is folded into a load through a selected address, which keeps the
// whole argument block in scratch memory
__device__ __forceinline__ void tile_rows(const MapParams& p, int by, int& ys, int& ye)
{
    const int second = by >= p.tiles_a;                // 0 / 1
    const int r0 = p.y0 + second * (p.yb0 - p.y0), e = p.y1 + second * (p.yb1 - p.y1);
    ys = r0 + (by - second * p.tiles_a) * p.tile_h;
    ye = min(ys + p.tile_h, e);
}

// XCD-aware tile order (as dcte_map): each XCD gets a contiguous run of tiles
__device__ __forceinline__ void xcd_tile(int& bx, int& by)
{
    const int nwg = gridDim.x * gridDim.y, L = blockIdx.x + gridDim.x * blockIdx.y;
    const int q = nwg / 8, r = nwg % 8, xcd = L % 8;
    const int T = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + L / 8;
    bx = T % gridDim.x;
    by = T / gridDim.x;
}

// ------------------------------------------------------------------ N = 8
// One workgroup = 256 lanes = 256 output columns x tile_h output rows.  Per
// group of 8 input rows: every lane fetches its column's bytes (one 8-byte
// buffer load a group ahead), converts them to the reference's fp64 luma
// through the LDS tables into lum[b] (the last wave also converts the 7 halo
// columns), one barrier, then per row: pass 1 on the lane's window line
// lum[b][u][tx .. tx + 7] -> ring slot u, and for every complete window the
// 8 pass-2 steps and the decision.  lum is double-buffered, so a group needs
// one barrier.
constexpr int kEx8T = 256;
constexpr int kEx8LW = kEx8T + 7;

template <int BPP>
__global__ __launch_bounds__(kEx8T, DCTE_EX_MINW) void dcte_exact8(const MapParams p)
{
    constexpr int N = 8, HL = 3, HR = 4, G = 8, T = kEx8T, LW = kEx8LW;
    constexpr int XH = LW - T;                        // halo columns past one per lane
    __shared__ double lut[BPP == 1 ? 256 : 768];
    __shared__ double lum[2][G][LW];

    const int tx = threadIdx.x;
    int bx, by;
    xcd_tile(bx, by);
    const int x0 = bx * T, x = x0 + tx;
    int ys, ye;
    tile_rows(p, by, ys, ye);
    const int n_in = (ye - ys) + N - 1;
    const int ngroups = (n_in + G - 1) / G;
    const int w = p.w, h = p.h;

    Frame fr;
    fr.init(p, BPP, x0 + T + HR - 1 >= w - 1 && min(h - 1, ye - 1 + HR) >= p.in_row0 + p.in_rows - 1);
    fill_lut<BPP>(lut, tx, T);

    // input row i of the tile = global row clamp(ys - HL + i)
    auto row_of = [&](int i) { return clampx(ys - HL + (i < n_in ? i : n_in - 1), 0, h - 1); };
    const int xc = clampx(x - HL, 0, w - 1);          // this lane's luma column
    const int hl = tx - (T - 64);                     // last wave: halo conversions
    const bool has_halo = hl >= 0 && hl < XH * G;
    const int hrow = has_halo ? hl / XH : 0;
    const int hxc = clampx(x0 + T - HL + (has_halo ? hl % XH : 0), 0, w - 1);

    uint2 pend[G], hpend = make_uint2(0u, 0u);
    auto issue = [&](int g) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < G; u++) pend[u] = fr.fetch(fr.at(xc, row_of(g * G + u), BPP));
        if (has_halo) hpend = fr.fetch(fr.at(hxc, row_of(g * G + hrow), BPP));
    };
    auto convert = [&](int g, int b) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < G; u++) {
            const uint32_t off = fr.at(xc, row_of(g * G + u), BPP) & 3u;
            lum[b][u][tx] = luma_of<BPP>(lut, __builtin_amdgcn_alignbyte(pend[u].y, pend[u].x, off));
        }
        if (has_halo) {
            const uint32_t off = fr.at(hxc, row_of(g * G + hrow), BPP) & 3u;
            lum[b][hrow][T + hl % XH] = luma_of<BPP>(lut, __builtin_amdgcn_alignbyte(hpend.y, hpend.x, off));
        }
    };

    const double we = (double)p.edges, wt = (double)p.textures;
    float* const orow = p.out + (long long)(ys - p.y0) * p.out_stride + x;
    const bool inside = x < w;
    double ring[N][N];                                // ring[slot][k1], slot = input row mod 8

    auto compute = [&](int g, int b) __attribute__((always_inline)) {
        sfor<G>([&](auto U) __attribute__((always_inline)) {
            constexpr int u = decltype(U)::value;
            const int i = g * G + u;
            if (i < n_in) {
                // pass 1 (shrtdct.c:62-89) on window line (y = row i): a[0..7][j]
                double* r = ring[u];
#pragma unroll
                for (int k = 0; k < N; k++) r[k] = lum[b][u][tx + k];
                r64::step8(r, 1);
                if (i >= N - 1) {
                    // pass 2 over the ring: line j = input row i - 7 + j = slot (u + 1 + j) % 8
                    constexpr int s0 = (u + 1) % 8, s1 = (u + 2) % 8, s2 = (u + 3) % 8, s3 = (u + 4) % 8;
                    constexpr int s4 = (u + 5) % 8, s5 = (u + 6) % 8, s6 = (u + 7) % 8, s7 = u;
                    double a01, m0, a10, mp = 0.0;
#define DCTE_COL(ROLE, K, A, M) \
    col8<ROLE>(ring[s0][K], ring[s1][K], ring[s2][K], ring[s3][K], ring[s4][K], ring[s5][K], ring[s6][K], ring[s7][K], A, M)
                    DCTE_COL(0, 0, a01, m0);
                    DCTE_COL(1, 1, a10, mp);
                    double dummy;
                    DCTE_COL(2, 2, dummy, mp);
                    DCTE_COL(2, 3, dummy, mp);
                    DCTE_COL(2, 4, dummy, mp);
                    DCTE_COL(2, 5, dummy, mp);
                    DCTE_COL(2, 6, dummy, mp);
                    DCTE_COL(2, 7, dummy, mp);
#undef DCTE_COL
                    // the scan's last maximum (src/dct.c:100-108) from maxima:
                    // edge iff nothing after (1,0) holds M and (|C10| = M, or
                    // nothing in (0,2..7) holds it and |C01| = M)
                    const double M = fmax(fmax(mp, a10), fmax(m0, a01));
                    const bool edge = !(mp == M) && (a10 == M || (!(m0 == M) && a01 == M));
                    const float e = (float)(M * weight(edge, we, wt));
                    if (inside) orow[(long long)(i - (N - 1)) * p.out_stride] = e;
                }
            }
        });
    };

    // (loads issued just before their conversion instead -- nothing in
    // flight across the passes: 178 VGPRs, no faster at 2 waves, and at the
    // 3-wave cap (spilling) +3.5 %, profiles/r05/exact_occupancy_ab.jsonl)
    issue(0);
    __syncthreads();                                  // lut
    for (int g = 0; g < ngroups; g++) {
        const int b = g & 1;
        convert(g, b);
        if (g + 1 < ngroups) issue(g + 1);
        __syncthreads();
        compute(g, b);
    }
}

template <int BPP>
hipError_t launch_exact8(const MapParams& p, hipStream_t s)
{
    dim3 grid((p.w + kEx8T - 1) / kEx8T, p.tiles_y);
    hipLaunchKernelGGL((dcte_exact8<BPP>), grid, dim3(kEx8T), 0, s, p);
    return hipGetLastError();
}


// ------------------------------------------------------------------ N = 16
// ddct16x16s (shrtdct.c:231-386): the same sliding structure with a 16-row
// ring of 16 channels per column -- 256 doubles, so a column is split over
// EIGHT waves, wave q holding the two channels (k1) one rotation of the
// reference's pass-1 step produces together:
//   q = 0: k1 = 0, 8    q = 1: 4, 12    q = 2: 2, 14    q = 3: 6, 10
//   q = 4: 1, 15        q = 5: 7, 9     q = 6: 5, 11    q = 7: 3, 13
// (a 2 x 16 register ring, 64 VGPRs).  Each wave runs only the part of the
// pass-1 step its pair needs (sums for q < 4, differences for q >= 4, then its
// rotation; 18-40 of the step's 114 operations), and the pass-2 steps of its
// two channels.  The eight partial maxima of a pixel meet in LDS: the post-
// (1,0) maximum by a 64-bit LDS atomic max on the (non-negative) doubles'
// bits, |C01|, max |C0,2..15| and |C10| in slots of their own; after the
// group's barrier wave q decides rows u = q, q + 8 of the group.
constexpr int kEx16W = 8;                          // waves per workgroup
constexpr int kEx16T = 64 * kEx16W;
constexpr int kEx16LW = 64 + 15;                   // luma columns of a 64-column strip
constexpr int kEx16G = 16;                         // rows per group (= ring depth)
constexpr int kEx16Conv = (kEx16G * kEx16LW + kEx16T - 1) / kEx16T;   // conversions per lane and group

using r64::K16;

// pass 1 of ddct16x16s (shrtdct.c:239-313) on window line v, only the two
// outputs of wave q (k1 = kA, kB above); q is wave-uniform
__device__ __forceinline__ void row16_pair(int q, const double (&v)[16], double& oa, double& ob)
{
    double xr, xi;
    if (q < 4) {
        const double s0 = v[0] + v[15], t0 = v[8] + v[7];
        const double s1 = v[2] + v[13], t1 = v[10] + v[5];
        const double s2 = v[4] + v[11], t2 = v[12] + v[3];
        const double s3 = v[6] + v[9], t3 = v[14] + v[1];
        if (q < 2) {
            const double x0r = s0 + t0, x1r = s1 + t1, x2r = s2 + t2, x3r = s3 + t3;
            if (q == 0) {                                  // k1 = 0, 8
                xr = x0r + x2r;
                xi = x1r + x3r;
                oa = K16::c8 * (xr + xi);
                ob = K16::c8 * (xr - xi);
            } else {                                       // k1 = 4, 12
                xr = x0r - x2r;
                xi = x1r - x3r;
                oa = K16::c4 * xr - K16::s4 * xi;
                ob = K16::c4 * xi + K16::s4 * xr;
            }
        } else {
            const double x0i = s0 - t0, x1i = s1 - t1, x2i = s2 - t2, x3i = s3 - t3;
            const double y0r = K16::w8 * (x1i - x3i), y2r = K16::w8 * (x1i + x3i);
            if (q == 2) {                                  // k1 = 2, 14
                xr = x0i + y0r;
                xi = y2r + x2i;
                oa = K16::c2 * xr - K16::s2 * xi;
                ob = K16::c2 * xi + K16::s2 * xr;
            } else {                                       // k1 = 6, 10
                xr = x0i - y0r;
                xi = y2r - x2i;
                oa = K16::c6 * xr - K16::s6 * xi;
                ob = K16::c6 * xi + K16::s6 * xr;
            }
        }
    } else {
        const double x4r = v[0] - v[15], x4i = v[8] - v[7];
        const double x5r = v[2] - v[13], x5i = v[10] - v[5];
        const double x6r = v[4] - v[11], x6i = v[12] - v[3];
        const double x7r = v[6] - v[9], x7i = v[14] - v[1];
        xr = K16::w8 * (x6r - x6i);
        xi = K16::w8 * (x6i + x6r);
        const double y6r = x4r - xr, y6i = x4i - xi, y4r = x4r + xr, y4i = x4i + xi;
        xr = K16::w4s * x7r - K16::w4c * x7i;
        xi = K16::w4s * x7i + K16::w4c * x7r;
        const double y7r = K16::w4c * x5r - K16::w4s * x5i;
        const double y7i = K16::w4c * x5i + K16::w4s * x5r;
        const double y5r = y7r + xr, y5i = y7i + xi, z7r = y7r - xr, z7i = y7i - xi;
        double c, sn;
        if (q == 4) {                                      // k1 = 1, 15
            xr = y4r + y5r;
            xi = y5i + y4i;
            c = K16::c1;
            sn = K16::s1;
        } else if (q == 5) {                               // k1 = 7, 9
            xr = y4r - y5r;
            xi = y5i - y4i;
            c = K16::c7;
            sn = K16::s7;
        } else if (q == 6) {                               // k1 = 5, 11
            xr = y6r - z7i;
            xi = z7r + y6i;
            c = K16::c5;
            sn = K16::s5;
        } else {                                           // k1 = 3, 13
            xr = y6r + z7i;
            xi = z7r - y6i;
            c = K16::c3;
            sn = K16::s3;
        }
        oa = c * xr - sn * xi;
        ob = c * xi + sn * xr;
    }
}

// pass 2 of ddct16x16s (shrtdct.c:314-386) on coefficient row k1 (v[j] =
// a[k1][j]): acc = max over |C_k1,k2| for k2 in {2..7, 9..15}; x0 / x1 = the
// pair C_k1,0 = c8 (x0 + x1), C_k1,8 = c8 (x0 - x1) is formed from; c1 = C_k1,1
__device__ __forceinline__ void col16(const double (&v)[16], double& acc, double& x0, double& x1, double& c1)
{
    const double x4r = v[0] - v[15], sr0 = v[0] + v[15];
    const double x4i = v[8] - v[7], si0 = v[8] + v[7];
    const double x0r = sr0 + si0, x0i = sr0 - si0;
    const double x5r = v[2] - v[13], sr1 = v[2] + v[13];
    const double x5i = v[10] - v[5], si1 = v[10] + v[5];
    const double x1r = sr1 + si1, x1i = sr1 - si1;
    const double x6r = v[4] - v[11], sr2 = v[4] + v[11];
    const double x6i = v[12] - v[3], si2 = v[12] + v[3];
    const double x2r = sr2 + si2, x2i = sr2 - si2;
    const double x7r = v[6] - v[9], sr3 = v[6] + v[9];
    const double x7i = v[14] - v[1], si3 = v[14] + v[1];
    const double x3r = sr3 + si3, x3i = sr3 - si3;
    x0 = x0r + x2r;
    x1 = x1r + x3r;
    double xr = x0r - x2r, xi = x1r - x3r;
    double a = fmax(fabs(K16::c4 * xr - K16::s4 * xi), fabs(K16::c4 * xi + K16::s4 * xr));   // C4, C12
    const double y0r = K16::w8 * (x1i - x3i), y2r = K16::w8 * (x1i + x3i);
    xr = x0i + y0r;
    xi = y2r + x2i;
    a = fmax(a, fabs(K16::c2 * xr - K16::s2 * xi));        // C2
    a = fmax(a, fabs(K16::c2 * xi + K16::s2 * xr));        // C14
    xr = x0i - y0r;
    xi = y2r - x2i;
    a = fmax(a, fabs(K16::c6 * xr - K16::s6 * xi));        // C6
    a = fmax(a, fabs(K16::c6 * xi + K16::s6 * xr));        // C10
    xr = K16::w8 * (x6r - x6i);
    xi = K16::w8 * (x6i + x6r);
    const double y6r = x4r - xr, y6i = x4i - xi, y4r = x4r + xr, y4i = x4i + xi;
    xr = K16::w4s * x7r - K16::w4c * x7i;
    xi = K16::w4s * x7i + K16::w4c * x7r;
    const double y7r = K16::w4c * x5r - K16::w4s * x5i;
    const double y7i = K16::w4c * x5i + K16::w4s * x5r;
    const double y5r = y7r + xr, y5i = y7i + xi, z7r = y7r - xr, z7i = y7i - xi;
    xr = y4r + y5r;
    xi = y5i + y4i;
    c1 = K16::c1 * xr - K16::s1 * xi;                      // C1
    a = fmax(a, fabs(K16::c1 * xi + K16::s1 * xr));        // C15
    xr = y4r - y5r;
    xi = y5i - y4i;
    a = fmax(a, fabs(K16::c7 * xr - K16::s7 * xi));        // C7
    a = fmax(a, fabs(K16::c7 * xi + K16::s7 * xr));        // C9
    xr = y6r - z7i;
    xi = z7r + y6i;
    a = fmax(a, fabs(K16::c5 * xr - K16::s5 * xi));        // C5
    a = fmax(a, fabs(K16::c5 * xi + K16::s5 * xr));        // C11
    xr = y6r + z7i;
    xi = z7r - y6i;
    a = fmax(a, fabs(K16::c3 * xr - K16::s3 * xi));        // C3
    a = fmax(a, fabs(K16::c3 * xi + K16::s3 * xr));        // C13
    acc = a;
}

template <int BPP>
__global__ __launch_bounds__(kEx16T, DCTE_EX16_MINW) void dcte_exact16(const MapParams p)
{
    constexpr int N = 16, HL = 7, HR = 8, G = kEx16G, LW = kEx16LW, T = kEx16T;
    __shared__ double lut[BPP == 1 ? 256 : 768];
    __shared__ double lum[G][LW];
    __shared__ unsigned long long pmax[G][64];      // max |C| after (1,0), as bits (atomic max)
    __shared__ double pe[G][3][64];                 // |C01|, max |C0,2..15|, |C10|

    const int tx = threadIdx.x, c = tx & 63;
    const int q = __builtin_amdgcn_readfirstlane(tx >> 6);   // wave = channel pair
    int bx, by;
    xcd_tile(bx, by);
    const int x0 = bx * 64, x = x0 + c;
    int ys, ye;
    tile_rows(p, by, ys, ye);
    const int n_in = (ye - ys) + N - 1;
    const int ngroups = (n_in + G - 1) / G;
    const int w = p.w, h = p.h;

    Frame fr;
    fr.init(p, BPP, x0 + 64 + HR - 1 >= w - 1 && min(h - 1, ye - 1 + HR) >= p.in_row0 + p.in_rows - 1);
    fill_lut<BPP>(lut, tx, T);
    for (int e = tx; e < G * 64; e += T) pmax[e / 64][e % 64] = 0ull;

    auto row_of = [&](int i) { return clampx(ys - HL + (i < n_in ? i : n_in - 1), 0, h - 1); };
    // the lane's luma conversions of a group: (row, column) pairs e = tx + T k
    int crow[kEx16Conv], ccol[kEx16Conv], cxc[kEx16Conv];
#pragma unroll
    for (int k = 0; k < kEx16Conv; k++) {
        const int e = tx + T * k;
        crow[k] = e < G * LW ? e / LW : -1;
        ccol[k] = e < G * LW ? e % LW : 0;
        cxc[k] = clampx(x0 - HL + ccol[k], 0, w - 1);
    }
    uint2 pend[kEx16Conv];
    auto issue = [&](int g) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < kEx16Conv; k++)
            if (crow[k] >= 0) pend[k] = fr.fetch(fr.at(cxc[k], row_of(g * G + crow[k]), BPP));
    };
    auto convert = [&](int g) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < kEx16Conv; k++) {
            if (crow[k] >= 0) {
                const uint32_t off = fr.at(cxc[k], row_of(g * G + crow[k]), BPP) & 3u;
                lum[crow[k]][ccol[k]] = luma_of<BPP>(lut, __builtin_amdgcn_alignbyte(pend[k].y, pend[k].x, off));
            }
        }
    };

    const double we = (double)p.edges, wt = (double)p.textures;
    double ring[N][2];

    auto compute = [&](int g) __attribute__((always_inline)) {
        sfor<G>([&](auto U) __attribute__((always_inline)) {
            constexpr int u = decltype(U)::value;
            const int i = g * G + u;
            if (i < n_in) {
                double v[16];
#pragma unroll
                for (int k = 0; k < 16; k++) v[k] = lum[u][c + k];
                row16_pair(q, v, ring[u][0], ring[u][1]);
                if (i >= N - 1) {
                    // window line j = input row i - 15 + j = slot (u + 1 + j) % 16
                    double va[16], vb[16];
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        va[j] = ring[(u + 1 + j) % 16][0];
                        vb[j] = ring[(u + 1 + j) % 16][1];
                    }
                    double accb, b0, b1, bc1;
                    col16(vb, accb, b0, b1, bc1);      // channel B: never an edge atom's row
                    double mp = fmax(fmax(accb, fabs(bc1)), K16::c8 * (fabs(b0) + fabs(b1)));
                    double acca, a0, a1, ac1;
                    col16(va, acca, a0, a1, ac1);
                    if (q == 0) {                      // k1 = 0: C01 and C0,2..15 (C00 not scanned)
                        pe[u][0][c] = fabs(ac1);
                        pe[u][1][c] = fmax(acca, fabs(K16::c8 * (a0 - a1)));
                    } else if (q == 4) {               // k1 = 1: C10 apart
                        pe[u][2][c] = fabs(K16::c8 * (a0 + a1));
                        mp = fmax(mp, fmax(fmax(acca, fabs(ac1)), fabs(K16::c8 * (a0 - a1))));
                    } else {
                        mp = fmax(mp, fmax(fmax(acca, fabs(ac1)), K16::c8 * (fabs(a0) + fabs(a1))));
                    }
                    atomicMax(&pmax[u][c], (unsigned long long)__double_as_longlong(mp));
                }
            }
        });
    };
    auto finalize = [&](int g) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const int u = q + 8 * r, i = g * G + u;
            if (i >= N - 1 && i < n_in) {
                const double mp = __longlong_as_double((long long)pmax[u][c]);
                const double a01 = pe[u][0][c], m0 = pe[u][1][c], a10 = pe[u][2][c];
                const double M = fmax(fmax(mp, a10), fmax(m0, a01));
                const bool edge = !(mp == M) && (a10 == M || (!(m0 == M) && a01 == M));
                if (x < w) p.out[(long long)(ys + i - (N - 1) - p.y0) * p.out_stride + x] = (float)(M * weight(edge, we, wt));
            }
            pmax[u][c] = 0ull;
        }
    };

    issue(0);
    for (int g = 0; g < ngroups; g++) {
        convert(g);
        if (g + 1 < ngroups) issue(g + 1);
        __syncthreads();             // lum of g; the previous group's decisions done
        compute(g);
        __syncthreads();             // partials of g; every read of lum done
        finalize(g);
    }
}

template <int BPP>
hipError_t launch_exact16(const MapParams& p, hipStream_t s)
{
    dim3 grid((p.w + 63) / 64, p.tiles_y);
    hipLaunchKernelGGL((dcte_exact16<BPP>), grid, dim3(kEx16T), 0, s, p);
    return hipGetLastError();
}


// ------------------------------------------------------------------ N = 2, 4
// dctNxN calls ddct2d here (src/dct.c:82-85, src/fft2d/fftsg2d.c:566-627):
// ddct (fftsg.c:349-402) along the SECOND index first -- dy, a vertical
// transform of each window column -- then along the first.  The vertical
// transform V(x', y) of image column x' over the window rows is the same
// doubles for the N pixels x' - HR .. x' + HL whose windows hold that column,
// so it is computed once per (column, row) and shared ACROSS lanes: a wave owns
// 64 consecutive columns, lane l computes V of its column from a register ring
// of the column's last N luma values, the wave swaps the V vectors through a
// wave-private LDS row, and lanes 0 .. 64 - N each run the N horizontal
// transforms of their pixel (the last N - 1 lanes only supply V).  No
// workgroup barrier after the luma tables.
constexpr int kExST = 256;                         // 4 independent waves

// ddct(n, -1) on v[0..n-1] (dcte_ref64.h step_small: fftsg.c ddct with
// cftx020 / dctsub for n = 4, the makect twiddles ct)
template <int N>
__device__ __forceinline__ void ddct_small(double (&v)[N], const double* ct, double wkr, double wki)
{
    if constexpr (N == 2) {
        const double t = v[1];
        v[1] = v[0] - t;
        v[0] += t;
        v[1] *= ct[0];
    } else {
        double a0 = v[0], a1 = v[1], a2 = v[2], a3 = v[3];
        const double t = a3;
        a3 = a2 - a1;
        a2 += a1;
        a1 = a0 - t;
        a0 += t;
        const double x0r = a0 - a2, x0i = a1 - a3;    // cftx020
        a0 += a2;
        a1 += a3;
        a2 = x0r;
        a3 = x0i;
        const double xr = wki * a1 - wkr * a3;        // dctsub
        a1 = wkr * a1 + wki * a3;
        a3 = xr;
        a2 *= ct[0];
        v[0] = a0;
        v[1] = a1;
        v[2] = a2;
        v[3] = a3;
    }
}

template <int N, int BPP>
__global__ __launch_bounds__(kExST) void dcte_exact_small(const MapParams p)
{
    constexpr int HL = N / 2 - 1, HR = N / 2, G = 8, OW = 64 - (N - 1);
    __shared__ double lut[BPP == 1 ? 256 : 768];
    __shared__ double vrow[kExST / 64][2][N][64];   // per wave, by row parity: V[k2][lane]

    const int tx = threadIdx.x, l = tx & 63, wv = tx >> 6;
    int bx, by;
    xcd_tile(bx, by);
    const int xs = (bx * (kExST / 64) + wv) * OW;      // first output column of the wave
    const int x = xs + l;
    int ys, ye;
    tile_rows(p, by, ys, ye);
    const int n_in = (ye - ys) + N - 1;
    const int ngroups = (n_in + G - 1) / G;
    const int w = p.w, h = p.h;
    const int xcol = clampx(x - HL, 0, w - 1);         // lane l's column: x - HL

    Frame fr;
    fr.init(p, BPP, (bx + 1) * (kExST / 64) * OW + 64 >= w && min(h - 1, ye - 1 + HR) >= p.in_row0 + p.in_rows - 1);
    fill_lut<BPP>(lut, tx, kExST);
    const double ct[2] = {p.ct[0], 0.0};
    const double wkr = p.ct[1] - p.ct[3], wki = p.ct[1] + p.ct[3];   // dctsub's k = 1 twiddle
    const double we = (double)p.edges, wt = (double)p.textures;
    __syncthreads();
    if (xs >= w) return;                               // wave-uniform; no barrier follows

    auto row_of = [&](int i) { return clampx(ys - HL + (i < n_in ? i : n_in - 1), 0, h - 1); };
    uint2 pend[2][G];
    auto issue = [&](int g, int b) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < G; u++) pend[b][u] = fr.fetch(fr.at(xcol, row_of(g * G + u), BPP));
    };
    double ring[N];                                    // luma of the column's last N input rows
    const bool emits = l < OW && x < w;
    float* const orow = p.out + (long long)(ys - p.y0) * p.out_stride + x;

    auto compute = [&](int g, int b) __attribute__((always_inline)) {
        sfor<G>([&](auto U) __attribute__((always_inline)) {
            constexpr int u = decltype(U)::value;
            const int i = g * G + u;
            if (i < n_in) {
                const uint32_t off = fr.at(xcol, row_of(i), BPP) & 3u;
                ring[u % N] = luma_of<BPP>(lut, __builtin_amdgcn_alignbyte(pend[b][u].y, pend[b][u].x, off));
                if (i >= N - 1) {
                    // pass 1 along dy: window line j = input row i - N + 1 + j
                    double v[N];
#pragma unroll
                    for (int j = 0; j < N; j++) v[j] = ring[(u + 1 + j) % N];
                    ddct_small<N>(v, ct, wkr, wki);
                    double* vr = &vrow[wv][u & 1][0][0];
#pragma unroll
                    for (int k = 0; k < N; k++) vr[k * 64 + l] = v[k];
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    // pass 2 along dx for each k2, over lanes l .. l + N - 1
                    const int ll = l < OW ? l : OW - 1;
                    double a01 = 0.0, m0 = -1.0, a10 = 0.0, mp = 0.0;
#pragma unroll
                    for (int k2 = 0; k2 < N; k2++) {
                        double hv[N];
#pragma unroll
                        for (int j = 0; j < N; j++) hv[j] = vr[k2 * 64 + ll + j];
                        ddct_small<N>(hv, ct, wkr, wki);
                        // C[k1][k2] = hv[k1]; scan order k1 outer, k2 inner
#pragma unroll
                        for (int k1 = 0; k1 < N; k1++) {
                            const double a = fabs(hv[k1]);
                            if (k1 == 0 && k2 == 0) continue;              // C00 is not scanned
                            if (k1 == 0 && k2 == 1) a01 = a;
                            else if (k1 == 0) m0 = fmax(m0, a);
                            else if (k1 == 1 && k2 == 0) a10 = a;
                            else mp = fmax(mp, a);
                        }
                    }
                    const double M = fmax(fmax(mp, a10), fmax(m0, a01));
                    const bool edge = !(mp == M) && (a10 == M || (!(m0 == M) && a01 == M));
                    if (emits) orow[(long long)(i - (N - 1)) * p.out_stride] = (float)(M * weight(edge, we, wt));
                }
            }
        });
    };

    issue(0, 0);
    for (int g = 0; g < ngroups; g += 2) {
        if (g + 1 < ngroups) issue(g + 1, 1);
        compute(g, 0);
        if (g + 1 >= ngroups) break;
        if (g + 2 < ngroups) issue(g + 2, 0);
        compute(g + 1, 1);
    }
}

template <int N, int BPP>
hipError_t launch_exact_small(const MapParams& p, hipStream_t s)
{
    constexpr int per_wg = (kExST / 64) * (64 - (N - 1));
    dim3 grid((p.w + per_wg - 1) / per_wg, p.tiles_y);
    hipLaunchKernelGGL((dcte_exact_small<N, BPP>), grid, dim3(kExST), 0, s, p);
    return hipGetLastError();
}

// ------------------------------------------------------------------ preview
// The GTK preview's energies (dct_energy_preview_rows, src/render.c:31-79,
// 421-479): the luma is RGB2LUMINANCE truncated to guchar (src/render.h:5,
// convert_row_to_luminance :62-79) -- a small integer, as a double -- the
// window data[dy][dx] with offsets -(c - 1) .. N - c, c = (N - 1) / 2
// (src/dct.h:8-9, src/render.c:43-49), clamped to the region, then the same
// dctNxN and last-maximum scan.  The window is stored the other way round
// from liblqr's data[dx][dy], so the shareable pass swaps direction and the
// kernels turn the liblqr ones on their side:
//  * N = 8, 16 (dcte_exact_pv8t, dcte_exact_pv16t): ddct8x8s / ddct16x16s
//    pass 1 runs along the FIRST index -- dy here -- so a lane owns an output
//    ROW and walks RIGHT with dcte_exact8's / dcte_exact16's register ring
//    (one pass-1 transform per (row, column)).  r05's first preview kernels
//    shared V across lanes through LDS as dcte_exact_small does (4.22 ms at
//    16384^2 N = 8, 5.79 ms at 8192^2 N = 16, against 3.75 / 4.90 now:
//    profiles/r05/exact_preview8_transposed_ab.jsonl, exact_preview16_transposed_ab.jsonl).
//  * N = 2, 4 (dcte_exact_pvs): ddct2d transforms along the SECOND index
//    first -- dx here: a horizontal transform of each window row, the same
//    doubles for the N pixels below each other: a register ring down the
//    strip, as dcte_exact8.
template <int BPP>
__device__ __forceinline__ void fill_lut_pv(double* lut, int tx, int nthreads)
{
    if constexpr (BPP >= 3) {
        for (int v = tx; v < 256; v += nthreads) {   // RGB2LUMINANCE's terms, left to right
            lut[v] = 16.0 + v * 0.2568;
            lut[256 + v] = v * 0.5041;
            lut[512 + v] = v * 0.0979;
        }
    }
}
template <int BPP>
__device__ __forceinline__ double luma_pv(const double* lut, uint32_t wd)
{
    if constexpr (BPP == 1) return (double)(wd & 255u);
    else return (double)(unsigned char)((lut[wd & 255u] + lut[256 + ((wd >> 8) & 255u)]) + lut[512 + ((wd >> 16) & 255u)]);
}

// N = 8, transposed (dcte_exact_pv8t, r05): dcte_exact8 turned on its side.
// A lane owns one output ROW of a 256-row tile and walks RIGHT along a
// 128-column strip; per input column it runs pass 1 (along dy: the column's
// 8 window lumas, staged in LDS as lumT[column][row]) into slot `column mod
// 8` of a 64-double register ring and, for every complete window, the 8
// pass-2 steps over the ring (col8, along dx) and the decision.  Every lane
// emits (no halo lanes), nothing crosses lanes, and pass 1 runs once per
// (row, column) as in dcte_exact8.
// (16384^2 RGB 4.22 -> 3.75 ms against r05's first, lane-shared preview
// kernel, grey 4.07 -> 3.59: profiles/r05/exact_preview8_transposed_ab.jsonl)
constexpr int kExPTT = 256;                        // lanes = output rows per tile
constexpr int kExPTW = 128;                        // output columns per workgroup

template <int BPP>
__global__ __launch_bounds__(kExPTT, DCTE_EX_MINW) void dcte_exact_pv8t(const MapParams p)
{
    constexpr int N = 8, C = (N - 1) / 2, HL = C - 1, HR = N - C, G = 8, T = kExPTT, TW = kExPTW;
    constexpr int LR = T + N - 1;                      // luma rows staged per column
    // input column i = global column x0 - HL - 1 + i (one column before the
    // first window, so that group g >= 1 completes the windows of output
    // columns x0 + 8 (g - 1) .. + 7: a lane stores them as two aligned float4)
    constexpr int NC = TW + N;
    constexpr int CONV = (G * LR + T - 1) / T;         // conversions per thread and group
    __shared__ double lut[BPP == 1 ? 1 : 768];
    __shared__ double lumT[2][G][LR];                  // [buffer][column of the group][row]

    const int tx = threadIdx.x;
    int bx, by;
    xcd_tile(bx, by);
    const int x0 = bx * TW;
    int ys, ye;
    tile_rows(p, by, ys, ye);
    const int w = p.w, h = p.h;
    const int ngroups = (NC + G - 1) / G;

    Frame fr;
    fr.init(p, BPP, x0 + TW + HR - 1 >= w - 1 && min(h - 1, ys + LR - 1 - HL) >= p.in_row0 + p.in_rows - 1);
    fill_lut_pv<BPP>(lut, tx, T);

    // conversion k of a group: element e = tx + T k -> row e / G, column e % G
    // (a wave's loads cover 8 neighbouring columns of 8 rows)
    auto col_of = [&](int g, int c) { return clampx(x0 - HL - 1 + g * G + c, 0, w - 1); };
    auto row_of = [&](int r) { return clampx(ys - HL + r, 0, h - 1); };
    uint2 pend[CONV];
    auto issue = [&](int g) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < CONV; k++) {
            const int e = tx + T * k;
            if (CONV * T == G * LR || e < G * LR) pend[k] = fr.fetch(fr.at(col_of(g, e % G), row_of(e / G), BPP));
        }
    };
    auto convert = [&](int g, int b) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < CONV; k++) {
            const int e = tx + T * k;
            if (CONV * T == G * LR || e < G * LR) {
                const uint32_t off = fr.at(col_of(g, e % G), row_of(e / G), BPP) & 3u;
                lumT[b][e % G][e / G] = luma_pv<BPP>(lut, __builtin_amdgcn_alignbyte(pend[k].y, pend[k].x, off));
            }
        }
    };

    const double we = (double)p.edges, wt = (double)p.textures;
    const int y = ys + tx;
    const bool row_ok = y < ye;
    float* const orow = p.out + (long long)((row_ok ? y : ys) - p.y0) * p.out_stride;
    double ring[N][N];                                // ring[slot][k1], slot = input column mod 8
    float res[G];                                     // the group's outputs (columns x0 + 8 (g - 1) + u)

    auto compute = [&](int g, int b) __attribute__((always_inline)) {
        sfor<G>([&](auto U) __attribute__((always_inline)) {
            constexpr int u = decltype(U)::value;          // input column g G + u
            static_assert(NC % G == 0, "whole groups");
            {
                // pass 1 along dy (the first index): window line of the column,
                // rows y - HL .. y + HR = staged rows tx .. tx + 7
                double* r = ring[u];
#pragma unroll
                for (int k = 0; k < N; k++) r[k] = lumT[b][u][tx + k];
                r64::step8(r, 1);
                if (g > 0) {
                    // pass 2 along dx over the ring: window column j = input column i - 7 + j
                    constexpr int s0 = (u + 1) % 8, s1 = (u + 2) % 8, s2 = (u + 3) % 8, s3 = (u + 4) % 8;
                    constexpr int s4 = (u + 5) % 8, s5 = (u + 6) % 8, s6 = (u + 7) % 8, s7 = u;
                    double a01, m0, a10, mp = 0.0;
#define DCTE_COL(ROLE, K, A, M) \
    col8<ROLE>(ring[s0][K], ring[s1][K], ring[s2][K], ring[s3][K], ring[s4][K], ring[s5][K], ring[s6][K], ring[s7][K], A, M)
                    DCTE_COL(0, 0, a01, m0);
                    DCTE_COL(1, 1, a10, mp);
                    double dummy;
                    DCTE_COL(2, 2, dummy, mp);
                    DCTE_COL(2, 3, dummy, mp);
                    DCTE_COL(2, 4, dummy, mp);
                    DCTE_COL(2, 5, dummy, mp);
                    DCTE_COL(2, 6, dummy, mp);
                    DCTE_COL(2, 7, dummy, mp);
#undef DCTE_COL
                    const double M = fmax(fmax(mp, a10), fmax(m0, a01));
                    const bool edge = !(mp == M) && (a10 == M || (!(m0 == M) && a01 == M));
                    res[u] = (float)(M * weight(edge, we, wt));
                }
            }
        });
        if (g > 0 && row_ok) {
            const int xa = x0 + G * (g - 1);
            float* o = orow + xa;
            if (xa + G <= w && (reinterpret_cast<uintptr_t>(o) & 15u) == 0) {
                reinterpret_cast<float4*>(o)[0] = make_float4(res[0], res[1], res[2], res[3]);
                reinterpret_cast<float4*>(o)[1] = make_float4(res[4], res[5], res[6], res[7]);
            } else {
#pragma unroll
                for (int u = 0; u < G; u++)
                    if (xa + u < w) o[u] = res[u];
            }
        }
    };

    issue(0);
    __syncthreads();                                  // lut
    for (int g = 0; g < ngroups; g++) {
        const int b = g & 1;
        convert(g, b);
        if (g + 1 < ngroups) issue(g + 1);
        __syncthreads();
        compute(g, b);
    }
}

template <int BPP>
hipError_t launch_exact_pv8t(const MapParams& p, hipStream_t s)
{
    dim3 grid((p.w + kExPTW - 1) / kExPTW, p.tiles_y);
    hipLaunchKernelGGL((dcte_exact_pv8t<BPP>), grid, dim3(kExPTT), 0, s, p);
    return hipGetLastError();
}

// N = 16, transposed (dcte_exact_pv16t, r05): dcte_exact16 on its side, as
// dcte_exact_pv8t is dcte_exact8 on its side.  A workgroup of 8 waves owns 64
// output ROWS (lane = row) and walks right along a strip in groups of 16
// input columns; wave q keeps the two channels (k1 = the vertical frequency
// here) of dcte_exact16's pairing in a 16-column ring, runs the part of pass
// 1 (along dy) its pair needs on the column's 16 staged lumas, and pass 2
// (along dx) over its ring; the eight partial maxima meet in LDS as in
// dcte_exact16, and after the group's barrier all 512 threads decide the
// group's 64 rows x 16 columns and write them row by row.
constexpr int kExP16TW = 128;                      // output columns per workgroup

template <int BPP>
__global__ __launch_bounds__(kEx16T, DCTE_EX16_MINW) void dcte_exact_pv16t(const MapParams p)
{
    constexpr int N = 16, C = (N - 1) / 2, HL = C - 1, HR = N - C, G = 16, T = kEx16T, TW = kExP16TW;
    constexpr int LR = 64 + N - 1;                     // luma rows staged per column
    constexpr int NC = TW + N;                         // input columns (one before the first window)
    static_assert(NC % G == 0, "whole groups");
    constexpr int CONV = (G * LR + T - 1) / T;         // conversions per thread and group
    __shared__ double lut[BPP == 1 ? 1 : 768];
    __shared__ double lumT[G][LR];                     // [column of the group][row]
    __shared__ unsigned long long pmax[G][64];         // max |C| after (1,0), as bits (atomic max)
    __shared__ double pe[G][3][64];                    // |C01|, max |C0,2..15|, |C10|

    const int tx = threadIdx.x, c = tx & 63;
    const int q = __builtin_amdgcn_readfirstlane(tx >> 6);   // wave = channel pair
    int bx, by;
    xcd_tile(bx, by);
    const int x0 = bx * TW;
    int ys, ye;
    tile_rows(p, by, ys, ye);
    const int w = p.w, h = p.h;
    constexpr int ngroups = NC / G;

    Frame fr;
    fr.init(p, BPP, x0 + TW + HR - 1 >= w - 1 && min(h - 1, ys + LR - 1 - HL) >= p.in_row0 + p.in_rows - 1);
    fill_lut_pv<BPP>(lut, tx, T);
    for (int e = tx; e < G * 64; e += T) pmax[e / 64][e % 64] = 0ull;

    // conversion k of a group: element e = tx + T k -> row e / G, column e % G
    auto col_of = [&](int g, int cc) { return clampx(x0 - HL - 1 + g * G + cc, 0, w - 1); };
    auto row_of = [&](int r) { return clampx(ys - HL + r, 0, h - 1); };
    uint2 pend[CONV];
    auto issue = [&](int g) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < CONV; k++) {
            const int e = tx + T * k;
            if (CONV * T == G * LR || e < G * LR) pend[k] = fr.fetch(fr.at(col_of(g, e % G), row_of(e / G), BPP));
        }
    };
    auto convert = [&](int g) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < CONV; k++) {
            const int e = tx + T * k;
            if (CONV * T == G * LR || e < G * LR) {
                const uint32_t off = fr.at(col_of(g, e % G), row_of(e / G), BPP) & 3u;
                lumT[e % G][e / G] = luma_pv<BPP>(lut, __builtin_amdgcn_alignbyte(pend[k].y, pend[k].x, off));
            }
        }
    };

    const double we = (double)p.edges, wt = (double)p.textures;
    double ring[N][2];                                 // ring[slot][channel], slot = input column mod 16

    auto compute = [&](int g) __attribute__((always_inline)) {
        sfor<G>([&](auto U) __attribute__((always_inline)) {
            constexpr int u = decltype(U)::value;
            // pass 1 along dy (the first index): the column's window line, rows c .. c + 15
            double v[16];
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = lumT[u][c + k];
            row16_pair(q, v, ring[u][0], ring[u][1]);
            if (g > 0) {
                // pass 2 along dx: window column j = input column g G + u - 15 + j = slot (u + 1 + j) % 16
                double va[16], vb[16];
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    va[j] = ring[(u + 1 + j) % 16][0];
                    vb[j] = ring[(u + 1 + j) % 16][1];
                }
                double accb, b0, b1, bc1;
                col16(vb, accb, b0, b1, bc1);          // channel B: never an edge atom's row
                double mp = fmax(fmax(accb, fabs(bc1)), K16::c8 * (fabs(b0) + fabs(b1)));
                double acca, a0, a1, ac1;
                col16(va, acca, a0, a1, ac1);
                if (q == 0) {                          // k1 = 0: C01 and C0,2..15 (C00 not scanned)
                    pe[u][0][c] = fabs(ac1);
                    pe[u][1][c] = fmax(acca, fabs(K16::c8 * (a0 - a1)));
                } else if (q == 4) {                   // k1 = 1: C10 apart
                    pe[u][2][c] = fabs(K16::c8 * (a0 + a1));
                    mp = fmax(mp, fmax(fmax(acca, fabs(ac1)), fabs(K16::c8 * (a0 - a1))));
                } else {
                    mp = fmax(mp, fmax(fmax(acca, fabs(ac1)), K16::c8 * (fabs(a0) + fabs(a1))));
                }
                atomicMax(&pmax[u][c], (unsigned long long)__double_as_longlong(mp));
            }
        });
    };
    // the group's 64 rows x 16 columns, row by row: thread t -> row t / 8,
    // columns 2 (t % 8) and 2 (t % 8) + 1 (a wave writes 8 rows x 64 bytes)
    auto finalize = [&](int g) __attribute__((always_inline)) {
        const int r = tx >> 3, y = ys + r, xa = x0 + G * (g - 1) + 2 * (tx & 7);
        float o[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int u = 2 * (tx & 7) + k;
            const double mp = __longlong_as_double((long long)pmax[u][r]);
            const double a01 = pe[u][0][r], m0 = pe[u][1][r], a10 = pe[u][2][r];
            const double M = fmax(fmax(mp, a10), fmax(m0, a01));
            const bool edge = !(mp == M) && (a10 == M || (!(m0 == M) && a01 == M));
            o[k] = (float)(M * weight(edge, we, wt));
            pmax[u][r] = 0ull;
        }
        if (y < ye) {
            float* const dst = p.out + (long long)(y - p.y0) * p.out_stride + xa;
            if (xa < w) dst[0] = o[0];
            if (xa + 1 < w) dst[1] = o[1];
        }
    };

    issue(0);
    for (int g = 0; g < ngroups; g++) {
        convert(g);
        if (g + 1 < ngroups) issue(g + 1);
        __syncthreads();             // lumT of g; the previous group's decisions done
        compute(g);
        __syncthreads();             // partials of g; every read of lumT done
        if (g > 0) finalize(g);
    }
}

template <int BPP>
hipError_t launch_exact_pv16t(const MapParams& p, hipStream_t s)
{
    dim3 grid((p.w + kExP16TW - 1) / kExP16TW, p.tiles_y);
    hipLaunchKernelGGL((dcte_exact_pv16t<BPP>), grid, dim3(kEx16T), 0, s, p);
    return hipGetLastError();
}

// N = 2, 4: lane = output column, walking down the strip (dcte_exact8's
// structure): per input row the horizontal ddct of the lane's window row
// (lum[b][u][tx .. tx + N - 1]) into slot `row mod N` of an N x N ring, then
// for each k2 the vertical ddct over the ring and the scan
template <int N, int BPP>
__global__ __launch_bounds__(kEx8T) void dcte_exact_pvs(const MapParams p)
{
    constexpr int C = (N - 1) / 2, HL = C - 1, G = 8, T = kEx8T, LW = T + N - 1;
    constexpr int HR = N - C;
    constexpr int XH = LW - T;                        // halo columns past one per lane
    __shared__ double lut[BPP == 1 ? 1 : 768];
    __shared__ double lum[2][G][LW];

    const int tx = threadIdx.x;
    int bx, by;
    xcd_tile(bx, by);
    const int x0 = bx * T, x = x0 + tx;
    int ys, ye;
    tile_rows(p, by, ys, ye);
    const int n_in = (ye - ys) + N - 1;
    const int ngroups = (n_in + G - 1) / G;
    const int w = p.w, h = p.h;

    Frame fr;
    fr.init(p, BPP, x0 + T + HR - 1 >= w - 1 && min(h - 1, ye - 1 + HR) >= p.in_row0 + p.in_rows - 1);
    fill_lut_pv<BPP>(lut, tx, T);
    const double ct[2] = {p.ct[0], 0.0};
    const double wkr = p.ct[1] - p.ct[3], wki = p.ct[1] + p.ct[3];   // dctsub's k = 1 twiddle

    auto row_of = [&](int i) { return clampx(ys - HL + (i < n_in ? i : n_in - 1), 0, h - 1); };
    const int xc = clampx(x - HL, 0, w - 1);
    const int hl = tx - (T - 64);                     // last wave: halo conversions
    const bool has_halo = hl >= 0 && hl < XH * G;
    const int hrow = has_halo ? hl / XH : 0;
    const int hxc = clampx(x0 + T - HL + (has_halo ? hl % XH : 0), 0, w - 1);

    uint2 pend[G], hpend = make_uint2(0u, 0u);
    auto issue = [&](int g) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < G; u++) pend[u] = fr.fetch(fr.at(xc, row_of(g * G + u), BPP));
        if (has_halo) hpend = fr.fetch(fr.at(hxc, row_of(g * G + hrow), BPP));
    };
    auto convert = [&](int g, int b) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < G; u++) {
            const uint32_t off = fr.at(xc, row_of(g * G + u), BPP) & 3u;
            lum[b][u][tx] = luma_pv<BPP>(lut, __builtin_amdgcn_alignbyte(pend[u].y, pend[u].x, off));
        }
        if (has_halo) {
            const uint32_t off = fr.at(hxc, row_of(g * G + hrow), BPP) & 3u;
            lum[b][hrow][T + hl % XH] = luma_pv<BPP>(lut, __builtin_amdgcn_alignbyte(hpend.y, hpend.x, off));
        }
    };

    const double we = (double)p.edges, wt = (double)p.textures;
    float* const orow = p.out + (long long)(ys - p.y0) * p.out_stride + x;
    const bool inside = x < w;
    double ring[N][N];                                // ring[slot][k2], slot = input row mod N

    auto compute = [&](int g, int b) __attribute__((always_inline)) {
        sfor<G>([&](auto U) __attribute__((always_inline)) {
            constexpr int u = decltype(U)::value;
            const int i = g * G + u;
            if (i < n_in) {
                // the second index first (dx): window row = input row i
                double* r = ring[u % N];
#pragma unroll
                for (int k = 0; k < N; k++) r[k] = lum[b][u][tx + k];
                ddct_small<N>(ring[u % N], ct, wkr, wki);
                if (i >= N - 1) {
                    // then the first (dy) for each k2: line ii = input row i - N + 1 + ii
                    double a01 = 0.0, m0 = -1.0, a10 = 0.0, mp = 0.0;
#pragma unroll
                    for (int k2 = 0; k2 < N; k2++) {
                        double hv[N];
#pragma unroll
                        for (int j = 0; j < N; j++) hv[j] = ring[(u + 1 + j) % N][k2];
                        ddct_small<N>(hv, ct, wkr, wki);
                        // C[k1][k2] = hv[k1]
#pragma unroll
                        for (int k1 = 0; k1 < N; k1++) {
                            const double a = fabs(hv[k1]);
                            if (k1 == 0 && k2 == 0) continue;              // C00 is not scanned
                            if (k1 == 0 && k2 == 1) a01 = a;
                            else if (k1 == 0) m0 = fmax(m0, a);
                            else if (k1 == 1 && k2 == 0) a10 = a;
                            else mp = fmax(mp, a);
                        }
                    }
                    const double M = fmax(fmax(mp, a10), fmax(m0, a01));
                    const bool edge = !(mp == M) && (a10 == M || (!(m0 == M) && a01 == M));
                    if (inside) orow[(long long)(i - (N - 1)) * p.out_stride] = (float)(M * weight(edge, we, wt));
                }
            }
        });
    };

    issue(0);
    __syncthreads();                                  // lut
    for (int g = 0; g < ngroups; g++) {
        const int b = g & 1;
        convert(g, b);
        if (g + 1 < ngroups) issue(g + 1);
        __syncthreads();
        compute(g, b);
    }
}

template <int N, int BPP>
hipError_t launch_exact_pvs(const MapParams& p, hipStream_t s)
{
    dim3 grid((p.w + kEx8T - 1) / kEx8T, p.tiles_y);
    hipLaunchKernelGGL((dcte_exact_pvs<N, BPP>), grid, dim3(kEx8T), 0, s, p);
    return hipGetLastError();
}

template <int BPP>
hipError_t launch_preview_exact(int n, const MapParams& p, hipStream_t s)
{
    if (n == 8) return launch_exact_pv8t<BPP>(p, s);
    if (n == 16) return launch_exact_pv16t<BPP>(p, s);
    if (n == 4) return launch_exact_pvs<4, BPP>(p, s);
    if (n == 2) return launch_exact_pvs<2, BPP>(p, s);
    return hipErrorInvalidValue;
}

template <int BPP>
int preview_blocks_per_cu(int n)
{
    int v = 0;
    hipError_t e = hipErrorInvalidValue;
    if (n == 8) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact_pv8t<BPP>, kExPTT, 0);
    else if (n == 16) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact_pv16t<BPP>, kEx16T, 0);
    else if (n == 4) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact_pvs<4, BPP>, kEx8T, 0);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact_pvs<2, BPP>, kEx8T, 0);
    return e == hipSuccess ? v : 0;
}

}  // namespace

// workgroups of the exact kernel for (n, bpp, sem) one CU holds at once; cached
int exact_blocks_per_cu(int n, int bpp, int sem)
{
    static std::atomic<int> cache[2][4][3];
    const int ni = n == 2 ? 0 : (n == 4 ? 1 : (n == 8 ? 2 : 3)), bi = bpp == 1 ? 0 : (bpp == 3 ? 1 : 2);
    const int si = sem == kSemLqr ? 0 : 1;
    int v = cache[si][ni][bi].load(std::memory_order_relaxed);
    if (v) return v;
    hipError_t e = hipErrorInvalidValue;
    if (si == 1) {
        v = bpp == 1 ? preview_blocks_per_cu<1>(n) : (bpp == 3 ? preview_blocks_per_cu<3>(n) : preview_blocks_per_cu<4>(n));
        e = v > 0 ? hipSuccess : hipErrorInvalidValue;
    } else if (n == 8) e = bpp == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact8<1>, kEx8T, 0)
                                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact8<3>, kEx8T, 0);
    else if (n == 16) e = bpp == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact16<1>, kEx16T, 0)
                                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact16<3>, kEx16T, 0);
    else if (n == 4) e = bpp == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact_small<4, 1>, kExST, 0)
                                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact_small<4, 3>, kExST, 0);
    else e = bpp == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact_small<2, 1>, kExST, 0)
                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, dcte_exact_small<2, 3>, kExST, 0);
    if (e != hipSuccess || v <= 0) v = 1;
    cache[si][ni][bi].store(v, std::memory_order_relaxed);
    return v;
}

bool exact_supported(int n, int sem)
{
    return (sem == kSemLqr || sem == kSemPreview) && (n == 2 || n == 4 || n == 8 || n == 16);
}
int exact_tile_w(int n, int sem)
{
    if (sem != kSemLqr) return n == 8 ? kExPTW : (n == 16 ? kExP16TW : kEx8T);
    return n == 8 ? kEx8T : (n == 16 ? 64 : (kExST / 64) * (64 - (n - 1)));
}
int exact_default_tile_h(int n, int sem)
{
    if (sem != kSemLqr && n == 16) return 64;
    return (sem != kSemLqr && n == 8) ? kExPTT : DCTE_EX_TILE_H;
}
int exact_max_tile_h(int n, int sem)
{
    if (sem != kSemLqr && n == 16) return 64;                  // a lane per output row
    return (sem != kSemLqr && n == 8) ? kExPTT : (1 << 30);
}

hipError_t launch_map_exact(int n, int bpp, int sem, const MapParams& p, hipStream_t s)
{
    if (p.tiles_y <= 0) return hipSuccess;
    if (sem == kSemPreview) {
        if (bpp == 1) return launch_preview_exact<1>(n, p, s);
        if (bpp == 3) return launch_preview_exact<3>(n, p, s);
        if (bpp == 4) return launch_preview_exact<4>(n, p, s);
        return hipErrorInvalidValue;
    }
    if (sem != kSemLqr) return hipErrorInvalidValue;
    if (n == 8) {
        if (bpp == 1) return launch_exact8<1>(p, s);
        if (bpp == 3) return launch_exact8<3>(p, s);
    } else if (n == 16) {
        if (bpp == 1) return launch_exact16<1>(p, s);
        if (bpp == 3) return launch_exact16<3>(p, s);
    } else if (n == 4) {
        if (bpp == 1) return launch_exact_small<4, 1>(p, s);
        if (bpp == 3) return launch_exact_small<4, 3>(p, s);
    } else if (n == 2) {
        if (bpp == 1) return launch_exact_small<2, 1>(p, s);
        if (bpp == 3) return launch_exact_small<2, 3>(p, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace dcte
