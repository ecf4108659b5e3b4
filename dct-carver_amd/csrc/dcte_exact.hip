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
#define DCTE_EX_MINW 2       // waves per SIMD the register budget is cut for (<= 256 VGPRs)
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

using r64::K8;

// Pass 2 of ddct8x8s on coefficient row k1 (shrtdct.c:90-117: a[k1][0..7] ->
// C_k1,0..7), folded into the scan's maxima.  v[j] = a[k1][j] after pass 1.
//   ROLE 0 (k1 = 0): a01 = |C01|, m0 = max |C0,2..7| (C00 is never scanned)
//   ROLE 1 (k1 = 1): a10 = |C10| (into a01's slot), mp = max(mp, |C1,1..7|)
//   ROLE 2 (k1 >= 2): mp = max(mp, |C_k1,0..7|)
template <int ROLE>
__device__ __forceinline__ void col8(double v0, double v1, double v2, double v3, double v4, double v5,
                                     double v6, double v7, double& a, double& m)
{
    const double x0r = v0 + v7, x1r = v0 - v7;
    const double x0i = v2 + v5, x1i = v2 - v5;
    const double x2r = v4 + v3, x3r = v4 - v3;
    const double x2i = v6 + v1, x3i = v6 - v1;
    double xr = x0r + x2r, xi = x0i + x2i;
    double acc;
    if constexpr (ROLE == 0) {
        acc = fabs(K8::c4 * (xr - xi));                       // C04
    } else if constexpr (ROLE == 1) {
        a = fabs(K8::c4 * (xr + xi));                          // C10
        acc = fmax(m, fabs(K8::c4 * (xr - xi)));               // C14
    } else {
        acc = fmax(m, K8::c4 * (fabs(xr) + fabs(xi)));         // max(|C_k1,0|, |C_k1,4|)
    }
    xr = x0r - x2r;
    xi = x0i - x2i;
    acc = fmax(acc, fabs(K8::c2 * xr - K8::s2 * xi));          // C_k1,2
    acc = fmax(acc, fabs(K8::c2 * xi + K8::s2 * xr));          // C_k1,6
    xr = K8::w4 * (x1i - x3i);
    const double y1i = K8::w4 * (x1i + x3i);
    const double y3i = y1i - x3r;
    const double z1i = y1i + x3r;
    const double y3r = x1r - xr;
    const double y1r = x1r + xr;
    const double c1 = K8::c1 * y1r - K8::s1 * z1i;             // C_k1,1
    if constexpr (ROLE == 0) {
        a = fabs(c1);
    } else {
        acc = fmax(acc, fabs(c1));
    }
    acc = fmax(acc, fabs(K8::c1 * z1i + K8::s1 * y1r));        // C_k1,7
    acc = fmax(acc, fabs(K8::c3 * y3r - K8::s3 * y3i));        // C_k1,3
    acc = fmax(acc, fabs(K8::c3 * y3i + K8::s3 * y3r));        // C_k1,5
    m = acc;
}

// Frame bytes through one bounds-checked buffer resource over the readable
// rows (a dword straddling the end reads as 0: the <= 3 tail bytes are fetched
// once by the workgroups that reach them and patched in).
struct Frame {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t base_off, nrec4, tail;
    bool tail_wg;

    __device__ __forceinline__ void init(const MapParams& p, int bpp, bool reaches_end)
    {
        const uintptr_t pbase = reinterpret_cast<uintptr_t>(p.px);
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
    __device__ __forceinline__ uint32_t at(const MapParams& p, int x, int y, int bpp) const
    {
        return base_off + (uint32_t)((long long)(y - p.in_row0) * p.rowstride) + (uint32_t)(x * bpp);
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
    const int ys = tile_row0(p, by), ye = tile_row1(p, by);
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
        for (int u = 0; u < G; u++) pend[u] = fr.fetch(fr.at(p, xc, row_of(g * G + u), BPP));
        if (has_halo) hpend = fr.fetch(fr.at(p, hxc, row_of(g * G + hrow), BPP));
    };
    auto convert = [&](int g, int b) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < G; u++) {
            const uint32_t off = fr.at(p, xc, row_of(g * G + u), BPP) & 3u;
            lum[b][u][tx] = luma_of<BPP>(lut, __builtin_amdgcn_alignbyte(pend[u].y, pend[u].x, off));
        }
        if (has_halo) {
            const uint32_t off = fr.at(p, hxc, row_of(g * G + hrow), BPP) & 3u;
            lum[b][hrow][T + hl % XH] = luma_of<BPP>(lut, __builtin_amdgcn_alignbyte(hpend.y, hpend.x, off));
        }
    };

    const double we = (double)p.edges, wt = (double)p.textures;
    float* const orow = p.out + (long long)(ys - p.y0) * p.out_stride + x;
    const bool inside = x < w;
    double ring[N][N];                                // ring[slot][k1], slot = input row mod 8

    auto compute = [&](int g, int b) __attribute__((always_inline)) {
        sfor<G>([&](auto U) {
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
                    const float e = (float)(M * (edge ? we : wt));
                    if (inside) orow[(long long)(i - (N - 1)) * p.out_stride] = e;
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

template <int BPP>
hipError_t launch_exact8(const MapParams& p, hipStream_t s)
{
    dim3 grid((p.w + kEx8T - 1) / kEx8T, p.tiles_y);
    hipLaunchKernelGGL((dcte_exact8<BPP>), grid, dim3(kEx8T), 0, s, p);
    return hipGetLastError();
}

}  // namespace

bool exact_supported(int n, int sem) { return sem == kSemLqr && n == 8; }
int exact_tile_w(int n) { return n == 8 ? kEx8T : 0; }
int exact_default_tile_h(int n) { return DCTE_EX_TILE_H; }

hipError_t launch_map_exact(int n, int bpp, int sem, const MapParams& p, hipStream_t s)
{
    if (p.tiles_y <= 0) return hipSuccess;
    if (sem != kSemLqr) return hipErrorInvalidValue;
    if (n == 8) {
        if (bpp == 1) return launch_exact8<1>(p, s);
        if (bpp == 3) return launch_exact8<3>(p, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace dcte
