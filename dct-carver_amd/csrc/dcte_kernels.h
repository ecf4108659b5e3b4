// dcte_kernels.h -- launch-side view of the energy-map kernels (no HIP types
// leak into the public C ABI; this header is internal to libdctenergy_hip).
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

namespace dcte {

// One launch computes output rows [y0, y1) of a w x h image -- and, when
// yb0 < yb1, rows [yb0, yb1) too (y1 <= yb0): a strong-scaling rank's two
// halo-dependent edge ranges in ONE launch.  Tile rows 0 .. tiles_a - 1 cover
// the first range, the rest the second (tile_row0 / tile_row1 below), so no
// workgroup straddles the gap.  The input pointer addresses global row
// `in_row0`; rows [in_row0, in_row0 + in_rows) are readable.  Every row the
// window clamp can touch for the output rows (clamp(y0 - N/2 + 1) ..
// clamp(last - 1 + N/2)) must be readable: a row band plus its halo, or the
// whole frame.
// N = 8 map launches below this many output pixels refine their sparse strips
// themselves (MapParams::epi)
#ifndef DCTE_EPI_MAX_PX
#define DCTE_EPI_MAX_PX 25000000LL
#endif
constexpr long long kEpiMaxPx = DCTE_EPI_MAX_PX;

struct MapParams {
    const uint8_t* px;
    long long rowstride;     // bytes
    int w, h;                // global image size
    int in_row0, in_rows;    // readable input rows (global)
    int y0, y1;              // output rows (global)
    int yb0, yb1;            // second output range (global; empty: yb0 = yb1)
    int tile_h;              // output rows per workgroup
    int tiles_a, tiles_y;    // tile rows of [y0, y1); of the launch
    int fair;                // > 0: priority levels a workgroup steps down through its tile
    int epi;                 // N = 8: the launch refines its own sparse strips (small launches)
    float* out;              // row y at out + (y - y0) * out_stride
    long long out_stride;    // floats
    float we, wt;            // edges / textures weights, pre-scaled to luma units
    float tie_tau;           // relative edge/texture margin sent to refinement
    float edges, textures;   // raw weights (refinement path)
    double ct[4];            // makect twiddles (N = 2, 4: the exact kernels)
    // Refinement lists, per 64-column strip s = (by * tiles_x + bx) * SPT +
    // strip in the tile (SPT = TW / 64 at N <= 8, 1 at N = 16): the pixels it
    // flags, as (y - ys) * 64 + (x - strip x0), at fix_list[s * 64 * tile_h ...];
    // their number in tile_count[s]; the strips with any in dirty_list[0 ..
    // *dirty_count) (dcte_fix_strips walks those).
    unsigned* fix_list;
    unsigned* tile_count;
    unsigned* dirty_list;
    unsigned* dirty_count;   // zero when the launch starts
    unsigned* dirty_next;    // zeroed by this launch: the next launch's dirty_count
    unsigned* fix_total;     // pixels refined (N = 8: the map's own sparse strips; null: none)
    // N = 8 (and N = 16 liblqr): the DENSE strips (more than kFixDirect flags)
    // once more, as one flat work list for the dense refinement walks
    // (fix_dense16_flat): *dense_ctr = {strips << 32 | entries}
    // (zero when the launch starts; dense_next zeroed by it), and per dense
    // strip dense_list[slot] = {strip, offset of its first entry in the
    // concatenation} -- the offsets ascend with the slot (one 64-bit atomic
    // hands out both)
    unsigned long long* dense_ctr;
    unsigned long long* dense_next;
    uint2* dense_list;
    // and (written by dcte_dense_index, between the map launch and its
    // refinement) per refinement batch b (16 entries of the flat list, N = 16
    // liblqr) the dense strip holding its first entry:
    // {its first column, its tile's first output row, strip, offset of its
    // first entry in the flat list}
    uint4* dense_batch;
    // timing-probe builds only (DCTE_TSTAMP): 3 words per workgroup {start,
    // end, HW_ID}, a buffer nothing else reads (null: no stamps)
    unsigned long long* stamps;
};

// first / one-past-last output row of the launch's tile row `by`
__host__ __device__ inline int tile_row0(const MapParams& p, int by)
{
    return by < p.tiles_a ? p.y0 + by * p.tile_h : p.yb0 + (by - p.tiles_a) * p.tile_h;
}
__host__ __device__ inline int tile_row1(const MapParams& p, int by)
{
    const int r = tile_row0(p, by) + p.tile_h, e = by < p.tiles_a ? p.y1 : p.yb1;
    return r < e ? r : e;
}

// dcte_fix_strips: the map launch's own parameters plus the fp64 pieces
struct TileFixParams {
    MapParams m;
    double ct[4];            // makect twiddles (N = 2, 4)
    unsigned* fix_total;     // += pixels refined (host-path diagnostic), or null
    int tiles_x;             // map grid width in tiles
    int tile_w;              // map tile width in columns (map_tile_w)
    int sparse_blocks;       // N = 8: blocks of the launch that walk sparse strips (the rest: dense)
};

struct FixParams {
    const uint8_t* px;
    long long rowstride;
    int w, h, in_row0, bpp, n, y0;
    int sem;                 // kSemLqr / kSemPreview
    float* out;
    long long out_stride;
    float edges, textures;
    double ct[4];            // makect twiddles (N = 2, 4)
    unsigned* fix_count;     // pixels flagged by the map kernel
    unsigned* fix_list;
    unsigned fix_cap;
    unsigned* fix_total;     // += pixels refined (host-path diagnostic), or null
    const int* pts;          // points mode: entry k is point k = (pts[2k], pts[2k+1]) -> out[k]
    unsigned max_items;      // most entries the list can hold for this launch (grid size)
};

// Seam removal + energy update (dcte_seam.hip) and energies at points.
struct SeamParams {
    const uint8_t* px;       // source frame, w x h, row 0 .. h - 1 readable
    long long rowstride;
    int w, h, bpp, n, sem;
    int in_row0;             // points: global row addressed by px
    const int* seam;         // h column indices (carve)
    const float* map;        // energies of the source frame (carve)
    long long map_stride;
    uint8_t* px_out;         // (w - 1) x h carved frame (carve)
    long long out_rowstride;
    float* map_out;          // carve: (w - 1) x h energies; points: count energies
    long long map_out_stride;
    const int* pts;          // points: (x, y) pairs
    int count;
    float we, wt, tie_tau;   // as MapParams
    unsigned* fix_count;
    unsigned* fix_list;
    unsigned fix_cap;
};

// Band of a carver step (dcte_band_gather, dcte_seam.hip)
struct BandParams {
    const int* seam;         // h columns just removed (frame coordinates before the step)
    int w, h, r, bw, bpp;    // carved width, rows, update radius, band width
    const float* map;        // carved frame's energies
    long long map_stride;
    const uint8_t* px;       // carved frame
    long long rowstride;
    int* x0;                 // h: first band column per row
    float* e;                // h x bw energies
    uint8_t* pxb;            // h x bw x bpp pixels
};

// Energies of given windows (dcte_windows): count windows of N x N doubles,
// the reference's data[i][j] layout, in the reference's arithmetic.
struct WinParams {
    const double* win;
    int count, n;
    double ct[4];            // makect twiddles (N = 2, 4)
    float edges, textures;
    float* out;
};

// Minimum-energy seam (dcte_dp.hip): scratch sized by the launcher.
struct DpParams {
    const float* map;        // w x h energies
    long long stride;        // floats
    int w, h;
    int nb, ns, ntiles;      // bands (dp_band_rows rows), super-bands, column tiles
    long long pw;            // padded row length of xch / par / jump / sjump (>= ntiles * tile)
    unsigned epoch;          // tag of this call's hand-off words (never 0)
    unsigned long long* xch; // nb x pw: {M at the band's last row (f32 bits), epoch << 32}
    int* jump;               // nb x pw: column where the chain from (band's last row, x)
                             // leaves the band (row y0 - 1; row 0 for band 0)
    int* sjump;              // ns x pw
    int* sx;                 // ns
    int* bx;                 // nb
    unsigned* err;           // 1, zeroed before the launch
    int* seam;               // h: column removed per row (-1 everywhere on failure)
    unsigned spin_limit;     // polls before a waiting tile gives up (0: the default)
    int j0, j1;              // dcte_seam_dp: bands [j0, j1) in this launch; j0 > 0 starts
                             // from band j0 - 1's published row (launched one band at a
                             // time when not every tile can be resident)
};

// host-side launchers (dcte_kernels.hip)
// ev_a / ev_b (or null): events the launch records at the kernel's start / end
hipError_t launch_map(int n, int bpp, int sem, const MapParams& p, hipStream_t s, hipEvent_t ev_a = nullptr,
                      hipEvent_t ev_b = nullptr);
hipError_t launch_fix(const FixParams& p, hipStream_t s);
hipError_t launch_fix_tiles(int n, int bpp, int sem, const TileFixParams& p, hipStream_t s);
hipError_t launch_seam_carve(const SeamParams& p, hipStream_t s);
hipError_t launch_points(const SeamParams& p, hipStream_t s);
hipError_t launch_band_gather(const BandParams& p, hipStream_t s);
hipError_t launch_windows(const WinParams& p, hipStream_t s);
hipError_t launch_seam_find(const DpParams& p, hipStream_t s, bool resident);
int dp_tile_cols();
int dp_band_rows();
int dp_super_bands();
int dp_max_tiles(int device);

// geometry the launcher uses (exported for tests / bench)
int map_tile_w(int n);
int map_default_tile_h(int n);
int map_tiles_x(int n, int w);   // map grid (tiles) of a launch
int map_tiles_y(int n, int rows, int tile_h);
int map_strips_per_tile(int n);
int map_blocks_per_cu(int n, int bpp, int sem);   // resident map workgroups per CU (occupancy)
int dense_batch_entries(int n, int sem);   // entries per dense refinement batch (0: no flat list)

// the exact map (dcte_exact.hip, DCTE_OPT_EXACT): the reference's fp64
// arithmetic in a sliding window, no refinement launch
hipError_t launch_map_exact(int n, int bpp, int sem, const MapParams& p, hipStream_t s);
bool exact_supported(int n, int sem);   // (every N, both semantics since r05)
int exact_tile_w(int n, int sem);       // output columns per workgroup
int exact_default_tile_h(int n, int sem);
int exact_max_tile_h(int n, int sem);     // rows one workgroup can take (preview N = 8: its lanes)
int exact_blocks_per_cu(int n, int bpp, int sem);

}  // namespace dcte
