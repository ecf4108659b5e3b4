// dcte_dp.hip -- minimum-energy seam on the device.
//
// The reference's carver is configured with delta_x = 1, rigidity 0
// (lqr_carver_init(carver, 1, 0), src/render.c:313), so liblqr's cumulative
// energy is the 3-neighbour recursion, in float [liblqr, unverified]:
//     M[0][x] = E[0][x],   M[y][x] = E[y][x] + min(M[y-1][x-1 .. x+1])
// candidates scanned left to right, replaced only on a strictly smaller
// value; the seam ends at the leftmost minimum of the last row and follows
// the parents up.  The oracle restates it (oracle/dcte_oracle.c
// orc_seam_find); results here are bit-identical (same float adds, same
// comparisons: min3 gives the same value as the strict-less scan, and the
// parent is the first candidate equal to it).
//
// Rows are sequential, so the DP is latency-bound: what matters is the
// instruction stream ONE wave issues per row (one wave per SIMD issues a VALU
// op every 4 cycles) and never stalling it on memory.
//   dcte_seam_dp     one wave per tile of kDpT = 32 C owned columns; lane l
//                    holds C adjacent columns of a 64 C-column span (the tile
//                    plus kDpR = 16 C halo columns per side) in registers and
//                    steps the recursion row by row; the two cross-lane
//                    neighbours come from DPP wave shifts.  Per row and lane:
//                    C map loads (buffer loads: scalar row offset + lane
//                    offset, prefetched 12 rows ahead through a ring of 4-row
//                    chunks inside a band's straight-line body, so the
//                    compiler's wait counts stay exact and under vmcnt's 6
//                    bits), no stores, and for each column one min3, two adds
//                    (energy + edge bias, then + min), and two compares + two
//                    selects carrying
//                    the column where the cell's parent chain entered the band
//                    (the per-band jump table, free of an extra pass).  Off the
//                    frame only M[-1] and M[w] matter (as the neighbours of
//                    columns 0 and w - 1): their energies get +inf added when
//                    they arrive, off the recursion's critical path, so those
//                    two columns stay +inf; other off-frame columns hold
//                    harmless finite values.
//                    After a band of kDpR rows the halo has decayed exactly to
//                    the tile.  The tile publishes its last-row M as 8-byte
//                    {value, epoch} words (write-through, no fences: each word
//                    carries its own validity) and the halo lanes of its two
//                    neighbours poll exactly the words they need.  Tiles are
//                    numbered so that neighbours share an XCD (blockIdx b runs
//                    on XCD b % 8).
//   dcte_seam_sjump  the jump table composed over kDpG = 16 bands.
//   dcte_seam_walk   one workgroup: argmin of the last row, then the chain's
//                    column at every band's last row, top-down in two levels
//                    (super-bands serially, then bands per super-band): ~h /
//                    (16 kDpR) + 16 dependent global loads instead of h.
//   dcte_seam_rows   one wave per band, all bands at once: the band's rows,
//                    re-derived from the band's top boundary in a window
//                    around the chain (nothing per row is kept by the DP).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dcte_kernels.h"

namespace dcte {

#ifndef DCTE_DP_C
#define DCTE_DP_C 2
#endif
constexpr int kDpLanes = 64;
constexpr int kDpC = DCTE_DP_C;                      // columns per lane (1, 2 or 4)
constexpr int kDpSpan = kDpLanes * kDpC;
#ifndef DCTE_DP_R
#define DCTE_DP_R (16 * DCTE_DP_C)
#endif
#ifndef DCTE_DP_Q
#define DCTE_DP_Q 4
#endif
constexpr int kDpR = DCTE_DP_R;                      // rows per band (= halo)
constexpr int kDpT = kDpSpan - 2 * kDpR;             // owned columns per wave
constexpr int kDpQ = DCTE_DP_Q;                      // rows per chunk
#ifndef DCTE_DP_NB
#define DCTE_DP_NB 4
#endif
constexpr int kDpNB = DCTE_DP_NB;                    // chunks in the prefetch ring
constexpr int kDpG = 16;                             // bands per super-band
constexpr int kXcds = 8;
constexpr unsigned kDpSpinLimit = 1u << 22;          // polls x s_sleep(1): ~0.5 s
static_assert(kDpC == 1 || kDpC == 2 || kDpC == 4, "C in {1, 2, 4}");
static_assert(kDpR % kDpQ == 0 && (kDpR / kDpQ) % kDpNB == 0,
              "a band is a whole number of chunks and of ring turns (static ring slots)");
static_assert(kDpT >= kDpR, "a halo lies inside one neighbour tile");
static_assert(kDpR % kDpC == 0, "the halo is a whole number of lanes");

int dp_tile_cols() { return kDpT; }
int dp_band_rows() { return kDpR; }
int dp_super_bands() { return kDpG; }

// lane i <- lane i - 1, lane i <- lane i + 1; the lane with no source reads 0
// (span-edge halo columns only: their values never reach the tile)
__device__ __forceinline__ int wave_shr1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int wave_shl1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x130, 0xF, 0xF, true); }

__global__ __launch_bounds__(kDpLanes) __attribute__((amdgpu_waves_per_eu(1, 1)))
void dcte_seam_dp(const DpParams p)
{
    constexpr int C = kDpC;
    const int per = (p.ntiles + kXcds - 1) / kXcds;
    const int k = (blockIdx.x % kXcds) * per + blockIdx.x / kXcds;
    if (k >= p.ntiles) return;
    const int lane = threadIdx.x;
    const int w = p.w, h = p.h;
    const long long pw = p.pw;
    const int c0 = k * kDpT;
    const int xa = c0 - kDpR + lane * C;             // first column of this lane
    const bool own = lane >= kDpR / C && lane < (kDpR + kDpT) / C;
    const float kInf = __builtin_inff();
    const bool left_edge = xa == 0;                  // column 0 is c = 0 of this lane
    unsigned xoff[C];                                // byte offset of the clamped column
    bool in[C];
    float bias[C];                                   // +inf on columns -1 and w, else 0
#pragma unroll
    for (int c = 0; c < C; c++) {
        const int x = xa + c;
        in[c] = x >= 0 && x < w;
        xoff[c] = (unsigned)min(max(x, 0), w - 1) * 4u;
        bias[c] = (x == -1 || x == w) ? kInf : 0.0f;
    }
    // map rows through a buffer resource based at the current band's first
    // row (row offsets stay 32-bit); rows past the frame read as 0 and are
    // never stepped
    const int rowb = (int)(p.stride * 4);
    __amdgpu_buffer_rsrc_t ers;
    auto set_map = [&](int y0) {
        const long long left = ((long long)(h - 1 - y0) * p.stride + w) * 4;
        ers = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.map) + (long long)y0 * p.stride,
                                                (short)0, (int)min(left, 0x7fffffffLL),
                                                (int)0x00020000);
    };
    auto load_row = [&](float (&e)[C], int r) {      // row r of the current map window
#pragma unroll
        for (int c = 0; c < C; c++)
            e[c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                 ers, (int)xoff[c], r * rowb, 0));
    };
    float m[C];
    int s[C];
    auto step = [&](const float (&e)[C]) {
        const float L = __int_as_float(wave_shr1(__float_as_int(m[C - 1])));
        const float R = __int_as_float(wave_shl1(__float_as_int(m[0])));
        const int sL = wave_shr1(s[C - 1]);
        const int sR = wave_shl1(s[0]);
        float nm[C];
        int ns[C];
#pragma unroll
        for (int c = 0; c < C; c++) {
            const float a = c == 0 ? L : m[c - 1];
            const float b = m[c];
            const float cc = c == C - 1 ? R : m[c + 1];
            const int sa = c == 0 ? sL : s[c - 1];
            const int sc = c == C - 1 ? sR : s[c + 1];
            const float best = fminf(fminf(a, b), cc);
            // leftmost minimum; the off-frame left neighbour of column 0 never
            // ties (an all-+inf row keeps the chain on the frame, as the
            // reference's in-frame scan does); on the right an off-frame +inf
            // can never be strictly smaller
            const bool isA = (a == best) & (c != 0 || !left_edge), isB = b == best;
            const int sbc = isB ? s[c] : sc;
            ns[c] = isA ? sa : sbc;
            nm[c] = (e[c] + bias[c]) + best;         // e + 0 is e: exact
        }
#pragma unroll
        for (int c = 0; c < C; c++) { m[c] = nm[c]; s[c] = ns[c]; }
    };

    auto publish = [&](int j) {                      // band j's last row (row 0 for h = 1)
        if (own) {
#pragma unroll
            for (int c = 0; c < C; c++) {
                const unsigned long long word =
                    ((unsigned long long)p.epoch << 32) | (unsigned)__float_as_int(m[c]);
                __hip_atomic_store(p.xch + (long long)j * pw + xa + c, word, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                p.jump[(long long)j * pw + xa + c] = s[c];
            }
        }
    };

    auto take_halo = [&](int j) -> bool {            // band j - 1's last row, halo columns
        const unsigned long long* xo = p.xch + (long long)(j - 1) * pw;
        bool need[C];
#pragma unroll
        for (int c = 0; c < C; c++) need[c] = in[c] && !own;
        const unsigned limit = p.spin_limit ? p.spin_limit : kDpSpinLimit;
        unsigned spins = 0;
        for (;;) {
            unsigned long long v[C];
#pragma unroll
            for (int c = 0; c < C; c++)
                v[c] = __hip_atomic_load(xo + (xoff[c] >> 2), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
            bool ok = true;
#pragma unroll
            for (int c = 0; c < C; c++) ok = ok && (!need[c] || (unsigned)(v[c] >> 32) == p.epoch);
            if (__all(ok)) {
#pragma unroll
                for (int c = 0; c < C; c++)
                    if (need[c]) m[c] = __int_as_float((int)(unsigned)v[c]);
                return true;
            }
            if (++spins >= limit) {
                __hip_atomic_fetch_or(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
            if ((spins & 255) == 0 &&
                __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                return false;
            __builtin_amdgcn_s_sleep(1);
        }
    };

    // row 0 seeds M; bands j = 0 .. nb - 1 cover rows [1 + j kDpR, 1 + (j + 1) kDpR).
    // A launch that starts at band j0 > 0 takes row 1 + j0 kDpR - 1 from band
    // j0 - 1's published words (every column: an earlier launch wrote them).
    const int jb = p.j0, je = p.j1;
    if (jb == 0) {
        float e0[C];
        set_map(0);
        load_row(e0, 0);
#pragma unroll
        for (int c = 0; c < C; c++) { m[c] = e0[c]; s[c] = xa + c; }
    } else {
        const unsigned long long* xo = p.xch + (long long)(jb - 1) * pw;
#pragma unroll
        for (int c = 0; c < C; c++) {
            m[c] = __int_as_float((int)(unsigned)__hip_atomic_load(xo + (xoff[c] >> 2), __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT));
            s[c] = xa + c;
        }
    }
    // ring of kDpNB chunks of kDpQ rows: chunk i + kDpNB - 1 is loaded while
    // chunk i runs.  A band's body is straight-line code, so the compiler
    // counts outstanding loads exactly (a loop-carried count would degrade
    // to waiting for everything).
    constexpr int kCh = kDpR / kDpQ;                 // chunks per band
    float ring[kDpNB][kDpQ][C];
    const int ystart = min(1 + jb * kDpR, h - 1);
    set_map(ystart);
#pragma unroll
    for (int i = 0; i < kDpNB - 1; i++)
#pragma unroll
        for (int r = 0; r < kDpQ; r++) load_row(ring[i][r], i * kDpQ + r);
    for (int j = jb; j < je; j++) {
        const int y0 = 1 + j * kDpR;
        if (j > jb) {
            publish(j - 1);
            if (!take_halo(j)) return;
#pragma unroll
            for (int c = 0; c < C; c++) s[c] = xa + c;   // chains enter band j at row y0 - 1
        }
        if (y0 + kDpR <= h) {
#pragma unroll
            for (int i = 0; i < kCh; i++) {
#pragma unroll
                for (int r = 0; r < kDpQ; r++)
                    load_row(ring[(i + kDpNB - 1) % kDpNB][r], (i + kDpNB - 1) * kDpQ + r);
#pragma unroll
                for (int r = 0; r < kDpQ; r++) step(ring[i % kDpNB][r]);
            }
        } else {                                     // the last, partial band
#pragma unroll
            for (int i = 0; i < kCh; i++) {
#pragma unroll
                for (int r = 0; r < kDpQ; r++)
                    load_row(ring[(i + kDpNB - 1) % kDpNB][r], (i + kDpNB - 1) * kDpQ + r);
#pragma unroll
                for (int r = 0; r < kDpQ; r++)
                    if (y0 + i * kDpQ + r < h) step(ring[i % kDpNB][r]);
            }
        }
        if (y0 + kDpR < h) set_map(y0 + kDpR);       // the ring already holds its first rows
    }
    // the last band's row: where the walk starts, or the next launch's seed
    publish(je - 1);
}

__global__ __launch_bounds__(256) void dcte_seam_sjump(const DpParams p)
{
    const int x = blockIdx.x * 256 + threadIdx.x, J = blockIdx.y;
    if (x >= p.w || *p.err) return;
    const int blo = J * kDpG, bhi = min(p.nb, blo + kDpG) - 1;
    int cur = x;
    for (int b = bhi; b >= blo; b--) cur = min(max(p.jump[(long long)b * p.pw + cur], 0), p.w - 1);
    p.sjump[(long long)J * p.pw + x] = cur;
}

constexpr int kWalkThreads = 1024;

__global__ __launch_bounds__(kWalkThreads) void dcte_seam_walk(const DpParams p)
{
    __shared__ float sv[kWalkThreads / 64];
    __shared__ int si[kWalkThreads / 64];
    __shared__ int xstar;
    const int tx = threadIdx.x, w = p.w, h = p.h;
    const long long pw = p.pw;
    if (*p.err) {
        for (int y = tx; y < h; y += kWalkThreads) p.seam[y] = -1;
        return;
    }
    // leftmost minimum of the last row (= the last band's published row)
    const unsigned long long* last = p.xch + (long long)(p.nb - 1) * pw;
    float bv = __builtin_inff();
    int bi = 0x7fffffff;
    int stale = 0;
    for (int x = tx; x < w; x += kWalkThreads) {
        const unsigned long long word = last[x];
        const float v = __int_as_float((int)(unsigned)word);
        stale |= (unsigned)(word >> 32) != p.epoch;  // every column published by this call
        if (v < bv) { bv = v; bi = x; }             // increasing x: strict < keeps the first
    }
    if (__syncthreads_or(stale)) {
        for (int y = tx; y < h; y += kWalkThreads) p.seam[y] = -1;
        if (tx == 0) *p.err = 2u;                    // dcte_seam_rows stands down
        return;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o);
        const int oi = __shfl_xor(bi, o);
        if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if ((tx & 63) == 0) { sv[tx >> 6] = bv; si[tx >> 6] = bi; }
    __syncthreads();
    if (tx == 0) {
        for (int i = 1; i < kWalkThreads / 64; i++)
            if (sv[i] < bv || (sv[i] == bv && si[i] < bi)) { bv = sv[i]; bi = si[i]; }
        // all-infinite last row (cannot happen for finite maps): column 0
        xstar = bi == 0x7fffffff ? 0 : bi;
        // super-bands, serially: sx[J] = column at the last row of super-band J
        const int ns = p.ns;
        int cur = xstar;
        p.sx[ns - 1] = cur;
        for (int J = ns - 1; J > 0; J--) {
            cur = min(max(p.sjump[(long long)J * pw + cur], 0), w - 1);
            p.sx[J - 1] = cur;
        }
    }
    __syncthreads();
    // bands per super-band: bx[b] = column at the last row of band b
    for (int J = tx; J < p.ns; J += kWalkThreads) {
        const int blo = J * kDpG, bhi = min(p.nb, blo + kDpG) - 1;
        int cur = p.sx[J];
        for (int b = bhi; b >= blo; b--) {
            p.bx[b] = cur;
            cur = min(max(p.jump[(long long)b * pw + cur], 0), w - 1);
        }
    }
}

// Rows of each band, one wave per band, all bands at once: the wave re-runs
// the recursion over its band in a 256-column window centred on bx[b] (the
// seam's column at the band's last row), from the exact M row above the band
// (row 0's energies, or band b - 1's published row), keeping every M row in
// LDS; the chain moves at most one column per row, so every value it reads is
// exact (the window's garbage edges decay inward one column per row: 128 >>
// kDpR), and the same floats and rule as dcte_seam_dp give the same parents.
// Lane 0 then walks the band bottom-up through LDS.
constexpr int kRwC = 4;                              // columns per lane
constexpr int kRwSpan = kDpLanes * kRwC;             // 256-column window
static_assert(kRwSpan / 2 > 2 * kDpR, "the window's exact core holds every chain of a band");

__global__ __launch_bounds__(kDpLanes) void dcte_seam_rows(const DpParams p)
{
    __shared__ float ml[kDpR][kRwSpan];              // M rows y0 - 1 .. y0 + kDpR - 2
    if (*p.err) return;
    const int b = blockIdx.x, lane = threadIdx.x;
    const int w = p.w, h = p.h;
    const int y0 = 1 + b * kDpR, y1 = min(h, y0 + kDpR);   // band b: rows [y0, y1)
    const int xb = p.bx[b];
    if (lane == 0) p.seam[max(y1, y0) - 1] = xb;     // h = 1: the one band is empty
    if (y1 <= y0) return;
    const float kInf = __builtin_inff();
    const int xw = xb - kRwSpan / 2;                 // window's first column
    const int xa = xw + lane * kRwC;
    long long xc[kRwC];
    float bias[kRwC], m[kRwC];
#pragma unroll
    for (int c = 0; c < kRwC; c++) {
        const int x = xa + c;
        xc[c] = min(max(x, 0), w - 1);
        bias[c] = (x == -1 || x == w) ? kInf : 0.0f;
    }
    if (b == 0) {
#pragma unroll
        for (int c = 0; c < kRwC; c++) m[c] = p.map[xc[c]];
    } else {
        const unsigned long long* xo = p.xch + (long long)(b - 1) * p.pw;
#pragma unroll
        for (int c = 0; c < kRwC; c++) m[c] = __int_as_float((int)(unsigned)xo[xc[c]]);
    }
#pragma unroll
    for (int c = 0; c < kRwC; c++) ml[0][lane * kRwC + c] = m[c];
    for (int y = y0; y < y1 - 1; y++) {              // rows whose M a parent lookup reads
        float e[kRwC];
#pragma unroll
        for (int c = 0; c < kRwC; c++) e[c] = p.map[(long long)y * p.stride + xc[c]];
        const float L = __int_as_float(wave_shr1(__float_as_int(m[kRwC - 1])));
        const float R = __int_as_float(wave_shl1(__float_as_int(m[0])));
        float nm[kRwC];
#pragma unroll
        for (int c = 0; c < kRwC; c++) {
            const float a = c == 0 ? L : m[c - 1];
            const float cc = c == kRwC - 1 ? R : m[c + 1];
            nm[c] = (e[c] + bias[c]) + fminf(fminf(a, m[c]), cc);
        }
#pragma unroll
        for (int c = 0; c < kRwC; c++) {
            m[c] = nm[c];
            ml[y - y0 + 1][lane * kRwC + c] = m[c];
        }
    }
    __syncthreads();
    if (lane != 0) return;
    // the parent of (y, x) is the leftmost minimum of M[y - 1][x - 1 .. x + 1],
    // off-frame columns never chosen (as in the DP)
    int cur = xb;
    for (int y = y1 - 1; y >= y0; y--) {
        const float* up = ml[y - y0];                // M row y - 1
        const int i = cur - xw;
        const float a = cur > 0 ? up[i - 1] : kInf;
        const float bb = up[i];
        const float c = cur < w - 1 ? up[i + 1] : kInf;
        const float best = fminf(fminf(a, bb), c);
        cur += (cur > 0 && a == best) ? -1 : (bb == best ? 0 : 1);
        cur = min(max(cur, 0), w - 1);               // NaN maps only: stay addressable
        p.seam[y - 1] = cur;
    }
}

hipError_t launch_seam_find(const DpParams& p, hipStream_t s, bool resident)
{
    if (p.w < 1 || p.h < 1 || p.pw < (long long)p.ntiles * kDpT) return hipErrorInvalidValue;
    const int per = (p.ntiles + kXcds - 1) / kXcds;
    if (resident) {
        // every tile resident at once: one launch, neighbours hand off in HBM
        DpParams q = p;
        q.j0 = 0;
        q.j1 = p.nb;
        hipLaunchKernelGGL(dcte_seam_dp, dim3(per * kXcds), dim3(kDpLanes), 0, s, q);
    } else {
        // one launch per band: a tile never waits for another in its launch
        // (the kernel boundary orders the hand-off), so no residency is assumed
        for (int j = 0; j < p.nb; j++) {
            DpParams q = p;
            q.j0 = j;
            q.j1 = j + 1;
            hipLaunchKernelGGL(dcte_seam_dp, dim3(per * kXcds), dim3(kDpLanes), 0, s, q);
        }
    }
    hipLaunchKernelGGL(dcte_seam_sjump, dim3((p.w + 255) / 256, p.ns), dim3(256), 0, s, p);
    hipLaunchKernelGGL(dcte_seam_walk, dim3(1), dim3(kWalkThreads), 0, s, p);
    hipLaunchKernelGGL(dcte_seam_rows, dim3(p.nb), dim3(kDpLanes), 0, s, p);
    return hipGetLastError();
}

// tiles the single-launch DP runs at once: every tile must be resident
// (tiles wait on their neighbours), and at most one per SIMD.  Two waves per
// SIMD are resident too, but their polls and steps share one issue port:
// measured 1.31 us/row at 100000 columns resident vs 0.35 us band-wise
// (profiles/r02/dp_width.jsonl), so wider frames go band-wise.
int dp_max_tiles(int device)
{
    constexpr int kSimdsPerCu = 4;
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dcte_seam_dp, kDpLanes, 0) !=
        hipSuccess)
        return 0;
    return cus * std::min(per_cu, kSimdsPerCu);
}

}  // namespace dcte
