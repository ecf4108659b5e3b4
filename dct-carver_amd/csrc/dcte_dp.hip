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
// comparisons).
//
// Rows are sequential, so the DP is latency-bound, not bandwidth-bound.
// Layout of the work:
//   dcte_seam_dp     one wave per tile of kDpT = 64 owned columns; each lane
//                    holds kDpC = 2 columns of a 128-column span (the tile
//                    plus kDpR = 32 halo columns per side) in registers and
//                    steps the recursion row by row with two lane shuffles;
//                    after a band of kDpR rows the halo has decayed exactly
//                    to the tile, whose last-row M is published to HBM with a
//                    release flag.  Neighbour tiles wait only on their two
//                    neighbours' flags (bounded spin; a timeout marks the
//                    result invalid instead of hanging).  Parent offsets
//                    (-1/0/+1) of owned cells go to an h x w byte plane.
//   dcte_seam_jump   per band and column: where the parent chain from the
//                    band's last row leaves the band (fully parallel).
//   dcte_seam_sjump  the same over kDpG = 16 bands.
//   dcte_seam_walk   one workgroup: argmin of the last row, then the chain is
//                    resolved top-down in three levels (super-bands serially,
//                    bands per super-band, rows per band), so the dependent
//                    global loads on the critical path are ~h/512 + 16 + 32
//                    instead of h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dcte_kernels.h"

namespace dcte {

constexpr int kDpLanes = 64;
constexpr int kDpC = 2;                              // columns per lane
constexpr int kDpSpan = kDpLanes * kDpC;             // 128
constexpr int kDpR = 32;                             // rows per band (= halo)
constexpr int kDpT = kDpSpan - 2 * kDpR;             // 64 owned columns per wave
constexpr int kDpG = 16;                             // bands per super-band
constexpr unsigned kDpSpinLimit = 1u << 24;          // x s_sleep(2): ~1 s

int dp_tile_cols() { return kDpT; }
int dp_band_rows() { return kDpR; }
int dp_super_bands() { return kDpG; }

__global__ __launch_bounds__(kDpLanes) void dcte_seam_dp(const DpParams p)
{
    const int k = blockIdx.x, lane = threadIdx.x;
    const int w = p.w, h = p.h;
    const int c0 = k * kDpT;
    const int xa = c0 - kDpR + lane * kDpC;          // first column of this lane
    const float kInf = __builtin_inff();
    bool in[kDpC], own[kDpC];
#pragma unroll
    for (int c = 0; c < kDpC; c++) {
        const int x = xa + c;
        in[c] = x >= 0 && x < w;
        own[c] = in[c] && x >= c0 && x < c0 + kDpT;
    }
    float m[kDpC];
    for (int j = 0; j < p.nb; j++) {
        const int y0 = j * kDpR, y1 = min(h, y0 + kDpR);
        int ys;
        if (j == 0) {
#pragma unroll
            for (int c = 0; c < kDpC; c++) m[c] = in[c] ? p.map[xa + c] : kInf;
            ys = 1;
        } else {
            if (lane == 0) {
                unsigned spins = 0;
                for (;;) {
                    bool ready = true;
                    if (k > 0 && __hip_atomic_load(&p.flags[k - 1], __ATOMIC_ACQUIRE,
                                                   __HIP_MEMORY_SCOPE_AGENT) < (unsigned)j)
                        ready = false;
                    if (k + 1 < p.ntiles && __hip_atomic_load(&p.flags[k + 1], __ATOMIC_ACQUIRE,
                                                              __HIP_MEMORY_SCOPE_AGENT) < (unsigned)j)
                        ready = false;
                    if (ready) break;
                    if (++spins > kDpSpinLimit ||
                        __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        __hip_atomic_fetch_or(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
            const float* b = p.bound + (long long)(j - 1) * w;
#pragma unroll
            for (int c = 0; c < kDpC; c++) m[c] = in[c] ? b[xa + c] : kInf;
            ys = y0;
        }
        // the band's energies, loaded up front (independent of the recursion)
        float e[kDpR][kDpC];
#pragma unroll
        for (int r = 0; r < kDpR; r++) {
            const int y = y0 + r;
#pragma unroll
            for (int c = 0; c < kDpC; c++)
                e[r][c] = (y >= ys && y < y1 && in[c]) ? p.map[(long long)y * p.stride + xa + c] : 0.0f;
        }
#pragma unroll
        for (int r = 0; r < kDpR; r++) {
            const int y = y0 + r;
            if (y < ys || y >= y1) continue;         // uniform
            float left = __shfl_up(m[kDpC - 1], 1);
            float right = __shfl_down(m[0], 1);
            if (lane == 0) left = kInf;
            if (lane == kDpLanes - 1) right = kInf;
            float nm[kDpC];
            int d[kDpC];
#pragma unroll
            for (int c = 0; c < kDpC; c++) {
                const float a = c == 0 ? left : m[c - 1];
                const float b = m[c];
                const float cc = c == kDpC - 1 ? right : m[c + 1];
                float best = a;                       // leftmost minimum
                int dd = -1;
                if (b < best) { best = b; dd = 0; }
                if (cc < best) { best = cc; dd = 1; }
                nm[c] = in[c] ? e[r][c] + best : kInf;
                d[c] = dd;
            }
#pragma unroll
            for (int c = 0; c < kDpC; c++) m[c] = nm[c];
            int8_t* prow = p.par + (long long)y * w + xa;
#pragma unroll
            for (int c = 0; c < kDpC; c++)
                if (own[c]) prow[c] = (int8_t)d[c];
        }
        float* bo = p.bound + (long long)j * w;
#pragma unroll
        for (int c = 0; c < kDpC; c++)
            if (own[c]) bo[xa + c] = m[c];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (lane == 0) __hip_atomic_store(&p.flags[k], (unsigned)(j + 1), __ATOMIC_RELEASE,
                                          __HIP_MEMORY_SCOPE_AGENT);
    }
}

// column where the parent chain from (band j's last row, x) leaves band j:
// the column in row y0 - 1 (row 0 for band 0)
__global__ __launch_bounds__(256) void dcte_seam_jump(const DpParams p)
{
    const int x = blockIdx.x * 256 + threadIdx.x, j = blockIdx.y;
    if (x >= p.w || *p.err) return;
    const int y0 = j * kDpR, y1 = min(p.h, y0 + kDpR);
    int cur = x;
    for (int y = y1 - 1; y >= max(y0, 1); y--) cur += p.par[(long long)y * p.w + cur];
    p.jump[(long long)j * p.w + x] = cur;
}

__global__ __launch_bounds__(256) void dcte_seam_sjump(const DpParams p)
{
    const int x = blockIdx.x * 256 + threadIdx.x, J = blockIdx.y;
    if (x >= p.w || *p.err) return;
    const int blo = J * kDpG, bhi = min(p.nb, blo + kDpG) - 1;
    int cur = x;
    for (int b = bhi; b >= blo; b--) cur = p.jump[(long long)b * p.w + cur];
    p.sjump[(long long)J * p.w + x] = cur;
}

constexpr int kWalkThreads = 1024;

__global__ __launch_bounds__(kWalkThreads) void dcte_seam_walk(const DpParams p)
{
    __shared__ float sv[kWalkThreads / 64];
    __shared__ int si[kWalkThreads / 64];
    __shared__ int xstar;
    const int tx = threadIdx.x, w = p.w, h = p.h;
    if (*p.err) {
        for (int y = tx; y < h; y += kWalkThreads) p.seam[y] = -1;
        return;
    }
    // leftmost minimum of the last row (= the last band's published row)
    const float* last = p.bound + (long long)(p.nb - 1) * w;
    float bv = __builtin_inff();
    int bi = 0x7fffffff;
    for (int x = tx; x < w; x += kWalkThreads) {
        const float v = last[x];
        if (v < bv) { bv = v; bi = x; }             // increasing x: strict < keeps the first
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
            cur = p.sjump[(long long)J * w + cur];
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
            cur = p.jump[(long long)b * w + cur];
        }
    }
    __syncthreads();
    // rows per band
    for (int b = tx; b < p.nb; b += kWalkThreads) {
        const int y0 = b * kDpR, y1 = min(h, y0 + kDpR);
        int cur = p.bx[b];
        p.seam[y1 - 1] = cur;
        for (int y = y1 - 1; y > y0; y--) {
            cur += p.par[(long long)y * w + cur];
            p.seam[y - 1] = cur;
        }
    }
}

hipError_t launch_seam_find(const DpParams& p, hipStream_t s)
{
    if (p.w < 1 || p.h < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(dcte_seam_dp, dim3(p.ntiles), dim3(kDpLanes), 0, s, p);
    hipLaunchKernelGGL(dcte_seam_jump, dim3((p.w + 255) / 256, p.nb), dim3(256), 0, s, p);
    hipLaunchKernelGGL(dcte_seam_sjump, dim3((p.w + 255) / 256, p.ns), dim3(256), 0, s, p);
    hipLaunchKernelGGL(dcte_seam_walk, dim3(1), dim3(kWalkThreads), 0, s, p);
    return hipGetLastError();
}

}  // namespace dcte
