// dcte_capi.cpp -- C ABI of libdctenergy_hip.so (declared in include/dctenergy.h).
//
// Context = a set of devices; per device: lazily created stream, staging
// buffers for the host entry point, and per-stream refinement scratch
// (counter + list) so calls on different streams never share it.
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <new>
#include <mutex>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/dctenergy.h"
#include "dcte_kernels.h"
#include "dcte_luma.h"
#include "dcte_host.h"
#include "dcte_norm.h"
#include "dcte_ref64.h"

namespace {

// Default refinement margins per N (DCTE_OPT_TIE_TAU unset): at least twice
// the DERIVED worst-case relative error of m_e and m_t together against the
// reference (fp32 rounding of the committed operation sequence, the fp32
// constants, the reference's own fp64 and luma rounding) -- tests/emu/
// tau_bound.cpp, asserted by tests/test_tau_bound.py, DESIGN.md §5:
// N = 2: 0.49e-6, 4: 1.74e-6, 8: 7.9e-6, 16: 2.31e-5.  (r02-r05 used 4e-6 for
// every N, set from an adversarial search; its worst find is 7.7e-7.)
double default_tie_tau(int n) { return n == 16 ? 5e-5 : n == 8 ? 2e-5 : 4e-6; }
constexpr int kMaxGridY = 65535;   // launch grid limit in y (map tiles of a band)
constexpr int kCountWords = 8;     // FixScratch::d_count

struct FixScratch {
    // [0] list length (points / seam), [1] refined, [2 + phase] dirty strips of
    // the map launches (two, alternating: each map launch zeroes the other one
    // for the next launch, so no memset is needed between launches), [4 + 2
    // phase] the same for the 64-bit dense-strip counter (N = 8)
    unsigned* d_count = nullptr;
    unsigned phase = 0;
    unsigned* d_list = nullptr;    // flagged pixels (map: per-tile regions)
    size_t cap = 0;
    unsigned* d_tiles = nullptr;   // map: per-strip counts | dirty-strip list | dense-strip pairs
    size_t tcap = 0;               // tiles
    void* d_batch = nullptr;       // map: the dense refinement batches' strips (uint4 each)
    size_t bcap = 0;               // bytes
};

struct DpScratch {                 // seam DP (dcte_dp.hip), per stream
    void* buf = nullptr;
    size_t cap = 0;
    // hand-off words live in a buffer of their own that never holds anything
    // else: every word in it is zero or tagged with an earlier call's epoch
    void* xbuf = nullptr;
    size_t xcap = 0;
    unsigned epoch = 0;            // hand-off tag of the last call
    int max_tiles = -1;            // co-resident DP tiles on this device
};

struct Device {
    int id = -1;
    int cus = 0;                   // compute units (queried on first map launch)
    hipStream_t stream = nullptr;  // used by the host entry point
    uint8_t* d_in = nullptr;
    size_t in_cap = 0;
    float* d_out = nullptr;
    size_t out_cap = 0;
    std::map<hipStream_t, FixScratch> fix;
    std::map<hipStream_t, DpScratch> dp;
    unsigned* d_keys = nullptr;    // min/max scratch (per device; stream-ordered)
    float* d_minmax = nullptr;
    uint8_t* d_u8 = nullptr;       // u8 staging for the host entry points
    size_t u8_cap = 0;
    uint8_t* d_tr = nullptr;       // transposed band (transposed maps)
    size_t tr_cap = 0;
    float* d_out2 = nullptr;       // the transposed frame's map (dcte_energy_map2)
    size_t out2_cap = 0;
    hipStream_t up = nullptr;      // host path: H2D copies
    hipStream_t down = nullptr;    // host path: D2H copies
    std::vector<hipEvent_t> ev;    // host path: chunk hand-offs
};

// Restores the calling thread's current device on every return path of a
// public entry point: the library switches devices internally (hipSetDevice),
// and a caller such as PyTorch allocates on whatever device is current.
struct DeviceGuard {
    int prev = -1;
    DeviceGuard()
    {
        if (hipGetDevice(&prev) != hipSuccess) {
            prev = -1;
            (void)hipGetLastError();
        }
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// one buffer resource addresses a frame's readable bytes: they must span < 4 GiB
bool span_ok(int h, long long rowstride, int w, int bpp)
{
    return (long long)(h - 1) * rowstride + (long long)w * bpp + 6 < (1LL << 32);
}

}  // namespace

struct ProfEvent {
    int dev;
    hipEvent_t a, b;
};

struct dcte_ctx {
    std::vector<Device> devs;
    double tie_tau = -1;            // DCTE_OPT_TIE_TAU; < 0: default_tie_tau(N)
    bool profile = false;
    double pin_mib = 1.0;           // DCTE_OPT_PIN_HOST (64 before r05: 4096^2 2.44 -> 1.67 ms at 1)
    int tile_h = 0;                 // DCTE_OPT_TILE_H (0: the kernel's default)
    bool dp_bandwise = false;       // DCTE_OPT_DP_BANDWISE
    unsigned dp_spin_limit = 0;     // DCTE_OPT_DP_SPIN_LIMIT (0: the kernel's default)
    unsigned long long* stamps = nullptr;   // DCTE_OPT_TSTAMP_BUF (timing-probe builds)
    int fail_inject = 0;            // DCTE_OPT_FAIL_INJECT (tests of the error paths)
    bool exact = false;             // DCTE_OPT_EXACT
    bool d2h_kernel = true;         // DCTE_OPT_D2H_KERNEL
    // page-locked staging of the host-call bytes no registration covers
    // (HostPin), per role: 0 the frame, 1 the map / layer, 2 map2's second map
    struct Stage {
        uint8_t* p = nullptr;
        size_t cap = 0;
    } stage[3];
    std::vector<ProfEvent> prof;
    long long last_refined = 0;
    std::string last_error;
};

namespace {

int hip_fail(dcte_ctx* ctx, hipError_t e, const char* where)
{
    ctx->last_error = std::string(where) + ": " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? DCTE_ENOMEM : DCTE_EHIP;
}

// argument errors carry the failed check in dcte_last_error
int bad_arg(dcte_ctx* ctx, const char* what)
{
    if (ctx) ctx->last_error = std::string("invalid argument: ") + what;
    return DCTE_EINVAL;
}
#define DCTE_ARG(ctx, cond)                                 \
    do {                                                    \
        if (!(cond)) return bad_arg((ctx), #cond);          \
    } while (0)

#define DCTE_HIP(ctx, expr)                                              \
    do {                                                                 \
        hipError_t e_ = (expr);                                          \
        if (e_ != hipSuccess) return hip_fail((ctx), e_, #expr);         \
    } while (0)

bool valid_n(int n) { return n == 2 || n == 4 || n == 8 || n == 16; }

// the refinement margin a call uses: the exact mode refines every pixel it
// does not compute in fp64 outright (seam bands and points; every map call
// goes to dcte_exact.hip's sliding kernels)
double eff_tau(const dcte_ctx* ctx, int n)
{
    return ctx->exact ? 1.0 : ctx->tie_tau >= 0 ? ctx->tie_tau : default_tie_tau(n);
}

// Runs a block of calls in a given arithmetic mode and restores the
// context's own afterwards: a dcte_carver carries the mode it was created in
// (DCTE_OPT_EXACT, DCTE_OPT_TIE_TAU), whatever the context was set to since.
struct ModeScope {
    dcte_ctx* ctx;
    bool exact;
    double tau;
    ModeScope(dcte_ctx* c, bool e, double t) : ctx(c), exact(c->exact), tau(c->tie_tau)
    {
        c->exact = e;
        c->tie_tau = t;
    }
    ~ModeScope()
    {
        ctx->exact = exact;
        ctx->tie_tau = tau;
    }
    ModeScope(const ModeScope&) = delete;
    ModeScope& operator=(const ModeScope&) = delete;
};

// window offsets -hl .. +hr of a semantics
void halo(int n, int sem, int& hl, int& hr)
{
    hl = sem == DCTE_LQR ? n / 2 - 1 : (n - 1) / 2 - 1;
    hr = n - 1 - hl;
}

// rows the clamp can touch for output rows [y0, y1)
void needed_rows(int n, int sem, int h, int y0, int y1, int& lo, int& hi)
{
    int hl, hr;
    halo(n, sem, hl, hr);
    lo = y0 - hl < 0 ? 0 : (y0 - hl > h - 1 ? h - 1 : y0 - hl);
    hi = y1 - 1 + hr > h - 1 ? h - 1 : (y1 - 1 + hr < 0 ? 0 : y1 - 1 + hr);
}

bool valid_sem_bpp(int sem, int bpp)
{
    if (sem == DCTE_LQR) return bpp == 1 || bpp == 3;
    if (sem == DCTE_PREVIEW) return bpp == 1 || bpp == 3 || bpp == 4;
    return false;
}

int ensure_fix(dcte_ctx* ctx, Device& d, hipStream_t s, size_t npix, FixScratch** out)
{
    FixScratch& f = d.fix[s];
    if (!f.d_count) {
        DCTE_HIP(ctx, hipMalloc(&f.d_count, kCountWords * sizeof(unsigned)));
        // on the scratch's own stream: a plain hipMemset is not ordered with
        // the (non-blocking) streams the kernels run on, and a map launch that
        // started before it landed would count from whatever the allocation held
        DCTE_HIP(ctx, hipMemsetAsync(f.d_count, 0, kCountWords * sizeof(unsigned), s));
    }
    if (f.cap < npix) {
        if (f.d_list) DCTE_HIP(ctx, hipFree(f.d_list));
        f.d_list = nullptr;
        f.cap = 0;
        DCTE_HIP(ctx, hipMalloc(&f.d_list, npix * sizeof(unsigned)));
        f.cap = npix;
    }
    *out = &f;
    return DCTE_OK;
}

int ensure_tiles(dcte_ctx* ctx, FixScratch* f, size_t ntiles)
{
    if (f->tcap >= ntiles) return DCTE_OK;
    if (f->d_tiles) DCTE_HIP(ctx, hipFree(f->d_tiles));
    f->d_tiles = nullptr;
    f->tcap = 0;
    // per-strip counts | dirty-strip list | dense-strip pairs (N = 8)
    DCTE_HIP(ctx, hipMalloc(&f->d_tiles, 4 * ntiles * sizeof(unsigned)));
    f->tcap = ntiles;
    return DCTE_OK;
}

using dcte::small_twiddles;

// kernel weights divide by this: hat units of dcte_math.h (C * N for N = 8, 16;
// C for the unnormalised N = 2, 4) times the luma unit (1/1275000 for liblqr,
// 1 for the preview's u8 luma)
double weight_scale(int n, int sem)
{
    return (sem == DCTE_LQR ? dcte::kLumaScale : 1.0) * (n >= 8 ? (double)n : 1.0);
}

dcte::FixParams fix_params(const uint8_t* px, long long rowstride, int w, int h, int in_row0,
                           int bpp, int n, int y0, int sem, float* out, long long out_stride,
                           float edges, float textures, const FixScratch* f)
{
    dcte::FixParams q{};
    q.px = px;
    q.rowstride = rowstride;
    q.w = w;
    q.h = h;
    q.in_row0 = in_row0;
    q.bpp = bpp;
    q.n = n;
    q.y0 = y0;
    q.sem = sem;
    q.out = out;
    q.out_stride = out_stride;
    q.edges = edges;
    q.textures = textures;
    small_twiddles(n, q.ct);
    q.fix_count = f->d_count;
    q.fix_list = f->d_list;
    q.fix_cap = (unsigned)f->cap;
    q.fix_total = f->d_count + 1;
    q.pts = nullptr;
    q.max_items = (unsigned)f->cap;
    return q;
}

int ensure_buf(dcte_ctx* ctx, void** p, size_t* cap, size_t bytes);

int device_cus(Device& d)
{
    if (d.cus <= 0 && hipDeviceGetAttribute(&d.cus, hipDeviceAttributeMultiprocessorCount, d.id) != hipSuccess)
        d.cus = 256;
    return d.cus;
}

// Output rows per map workgroup when DCTE_OPT_TILE_H does not fix them: the
// shape that finishes first under a rounds model.  A launch of nwg workgroups
// on `resident` slots takes ceil(nwg / resident) rounds, each as long as one
// tile: its rows plus a fixed prologue (the N - 1 warm-up rows and the group
// loop's setup, ~N + 3 rows).  Large frames keep th_max (128 rows: 8 full
// rounds at 16384^2, N = 8); a 4096^2 frame, whose 128-row tiles filled only
// half of the slots, gets 64 (one full round); 6000 x 4000 gets 96.  Ties go
// to the taller tile.
int pick_tile_h(int n, int rows_a, int rows_b, int tiles_x, long long resident, int th_max)
{
    const int w0 = n + 3;
    int best = th_max;
    double best_cost = 0.0;
    for (int th = th_max; th >= 16; th--) {
        const long long nwg = (long long)tiles_x * ((rows_a + th - 1) / th + (rows_b + th - 1) / th);
        const long long rounds = (nwg + resident - 1) / resident;
        const double cost = (double)rounds * (double)(th + w0);
        if (th == th_max || cost < best_cost * (1.0 - 1e-9)) {
            best = th;
            best_cost = cost;
        }
    }
    return best;
}

// The exact map (DCTE_OPT_EXACT, dcte_exact.hip): one launch of the fp64
// sliding-window kernel over the same row ranges, no refinement lists.  The
// arguments were checked by run_device.
int run_exact(dcte_ctx* ctx, Device& d, const void* d_px, long long rowstride, int w, int h, int bpp,
              int in_row0, int in_rows, int y0, int y1, int yb0, int yb1, int n, float edges,
              float textures, int sem, float* d_out, long long out_stride, hipStream_t s)
{
    const int rows_a = y1 - y0, rows_b = yb1 - yb0;
    DCTE_HIP(ctx, hipSetDevice(d.id));
    int tile_h = ctx->tile_h;
    if (tile_h <= 0) {
        const int tw = dcte::exact_tile_w(n, sem);
        tile_h = pick_tile_h(n, rows_a, rows_b, (w + tw - 1) / tw,
                             (long long)device_cus(d) * dcte::exact_blocks_per_cu(n, bpp, sem),
                             dcte::exact_default_tile_h(n, sem));
    }
    if (tile_h > dcte::exact_max_tile_h(n, sem)) tile_h = dcte::exact_max_tile_h(n, sem);
    if (tile_h > (rows_a > rows_b ? rows_a : rows_b)) tile_h = rows_a > rows_b ? rows_a : rows_b;
    const int tiles_a = (rows_a + tile_h - 1) / tile_h;
    const int tiles_y = tiles_a + (rows_b + tile_h - 1) / tile_h;
    if (tiles_y > kMaxGridY) {
        ctx->last_error = "tile rows exceed the launch grid (raise DCTE_OPT_TILE_H)";
        return DCTE_ERANGE;
    }
    dcte::MapParams p{};
    p.px = static_cast<const uint8_t*>(d_px);
    p.rowstride = rowstride;
    p.w = w;
    p.h = h;
    p.in_row0 = in_row0;
    p.in_rows = in_rows;
    p.y0 = y0;
    p.y1 = y1;
    p.yb0 = yb0;
    p.yb1 = yb1;
    p.tile_h = tile_h;
    p.tiles_a = tiles_a;
    p.tiles_y = tiles_y;
    p.out = d_out;
    p.out_stride = out_stride;
    p.edges = edges;
    p.textures = textures;
    small_twiddles(n, p.ct);
    hipError_t e = hipSuccess;
    if (ctx->profile) {
        ProfEvent ev{d.id, nullptr, nullptr};
        DCTE_HIP(ctx, hipEventCreate(&ev.a));
        if ((e = hipEventCreate(&ev.b)) != hipSuccess) {
            (void)hipEventDestroy(ev.a);
            return hip_fail(ctx, e, "hipEventCreate");
        }
        ctx->prof.push_back(ev);      // dcte_profile_read destroys them
        DCTE_HIP(ctx, hipEventRecord(ev.a, s));
        DCTE_HIP(ctx, dcte::launch_map_exact(n, bpp, sem, p, s));
        DCTE_HIP(ctx, hipEventRecord(ev.b, s));
    } else {
        DCTE_HIP(ctx, dcte::launch_map_exact(n, bpp, sem, p, s));
    }
    if (ctx->fail_inject == 1) {      // testing: the launch was queued, report it failed
        ctx->fail_inject = 0;
        return hip_fail(ctx, hipErrorLaunchFailure, "launch_map_exact (injected)");
    }
    // an armed refinement-launch failure (2) is consumed here: this call has no
    // refinement launch, and it must not fire in a later fast-mode call
    if (ctx->fail_inject == 2) ctx->fail_inject = 0;
    return DCTE_OK;
}

// Output rows [y0, y1) -- plus [yb0, yb1) when yb0 < yb1 (y1 <= yb0: one
// launch for both, the out row of y at d_out + (y - y0) * out_stride).
int run_device(dcte_ctx* ctx, Device& d, const void* d_px, long long rowstride, int w, int h,
               int bpp, int in_row0, int in_rows, int y0, int y1, int n, float edges,
               float textures, int sem, float* d_out, long long out_stride, hipStream_t s,
               int yb0 = 0, int yb1 = 0)
{
    DCTE_ARG(ctx, valid_n(n) && valid_sem_bpp(sem, bpp) && w > 0 && h > 0);
    DCTE_ARG(ctx, y0 >= 0 && y1 <= h && y0 <= y1 && d_px && d_out && out_stride >= w);
    DCTE_ARG(ctx, rowstride >= (long long)w * bpp);
    const bool two = yb0 < yb1;
    DCTE_ARG(ctx, !two || (yb0 >= y1 && yb1 <= h));
    if (!two) yb0 = yb1 = y1;
    if (y1 == y0 && !two) return DCTE_OK;
    // every row the clamp reaches for each range must be readable (the rows
    // between two ranges are never read)
    int lo, hi;
    if (y1 > y0) {
        needed_rows(n, sem, h, y0, y1, lo, hi);
        DCTE_ARG(ctx, lo >= in_row0 && hi < in_row0 + in_rows);
    }
    if (two) {
        needed_rows(n, sem, h, yb0, yb1, lo, hi);
        DCTE_ARG(ctx, lo >= in_row0 && hi < in_row0 + in_rows);
    }
    // one buffer resource addresses the readable rows: < 4 GiB
    long long span = (long long)(in_rows - 1) * rowstride + (long long)w * bpp + 3;
    if (span >= (1LL << 32)) return DCTE_ERANGE;
    size_t npix = (size_t)((two ? yb1 : y1) - y0) * (size_t)w;
    if (npix >= (1ULL << 32)) return DCTE_ERANGE;
    // one workgroup's output rows go through one buffer resource; a band
    // shorter than a tile is one tile of exactly its rows (same results, and
    // the refinement list below is sized for the rows that exist)
    const int rows_a = y1 - y0, rows_b = yb1 - yb0;
    const bool exact = ctx->exact && dcte::exact_supported(n, sem);
    if (exact) return run_exact(ctx, d, d_px, rowstride, w, h, bpp, in_row0, in_rows, y0, y1, yb0, yb1, n,
                                edges, textures, sem, d_out, out_stride, s);
    DCTE_HIP(ctx, hipSetDevice(d.id));
    int tile_h = ctx->tile_h;
    if (tile_h <= 0)
        tile_h = pick_tile_h(n, rows_a, rows_b, dcte::map_tiles_x(n, w),
                             (long long)device_cus(d) * dcte::map_blocks_per_cu(n, bpp, sem),
                             dcte::map_default_tile_h(n));
    if (tile_h > (rows_a > rows_b ? rows_a : rows_b)) tile_h = rows_a > rows_b ? rows_a : rows_b;
    if ((long long)tile_h * out_stride * 4 >= (1LL << 31)) return DCTE_ERANGE;
    const int tiles_a = dcte::map_tiles_y(n, rows_a, tile_h);

    // N = 8 launches of at most two rounds of workgroups (a strong-scaling
    // rank's 2048- or 4096-row band): the waves step their priority down
    // through the tile so the workgroups sharing a CU finish together
    // (dcte_map's set_prio: 2048-row band -6 %, 4096 rows -2.5 %,
    // profiles/r02/map_fair_ab.jsonl); longer launches even out by themselves.
    // (1024-thread lockstep tiles kept every CU busy to the end, 97 % slot-busy
    // vs 87 %, but ran each tile 20 % slower: profiles/r03/band_wide_ab.jsonl.)
    int fair = 0;
    if (n == 8) {
        device_cus(d);
        const long long nwg = (long long)dcte::map_tiles_x(n, w) *
                              (tiles_a + dcte::map_tiles_y(n, rows_b, tile_h));
        if (nwg <= 2LL * 4 * d.cus) fair = 3;
    }
    // refinement lists: one region of 64 * tile_h entries per 64-column strip
    const int tiles_x = dcte::map_tiles_x(n, w), tiles_y = tiles_a + dcte::map_tiles_y(n, rows_b, tile_h);
    if (tiles_y > kMaxGridY) {
        ctx->last_error = "tile rows exceed the launch grid (raise DCTE_OPT_TILE_H)";
        return DCTE_ERANGE;
    }
    const size_t ntiles = (size_t)tiles_x * (size_t)tiles_y * (size_t)dcte::map_strips_per_tile(n);
    const size_t list_len = ntiles * 64 * (size_t)tile_h;
    if (list_len >= (1ULL << 32)) return DCTE_ERANGE;
    FixScratch* f = nullptr;
    int rc = ensure_fix(ctx, d, s, list_len, &f);
    if (rc) return rc;
    rc = ensure_tiles(ctx, f, ntiles);
    if (rc) return rc;
    // the dense refinement's batch map (N = 16 liblqr): one uint4 per batch
    // the lists can hold
    if (const int epb = dcte::dense_batch_entries(n, sem)) {
        rc = ensure_buf(ctx, &f->d_batch, &f->bcap, (list_len / (size_t)epb + 1) * 16);
        if (rc) return rc;
    }

    const double scale = weight_scale(n, sem);
    dcte::MapParams p{};
    p.px = static_cast<const uint8_t*>(d_px);
    p.rowstride = rowstride;
    p.w = w;
    p.h = h;
    p.in_row0 = in_row0;
    p.in_rows = in_rows;
    p.y0 = y0;
    p.y1 = y1;
    p.yb0 = yb0;
    p.yb1 = yb1;
    p.tile_h = tile_h;
    p.tiles_a = tiles_a;
    p.tiles_y = tiles_y;
    p.fair = fair;
    // N = 8 launches of fewer than DCTE_EPI_MAX_PX output pixels refine their
    // sparse strips inside the map launch (dcte_map's epilogue): on a natural
    // 1024^2 / 2048^2 / 4096^2 frame the call is 8 / 5 / 2-3 % shorter (the
    // separate launch's sparse walk, a chain of dependent loads, is most of
    // that launch's cost); 6144^2 and 8192^2 even; at 16384^2 the tiles holding
    // a wave for their epilogue cost the map 1.2 % more than that walk
    // (profiles/r06/map_epi_ab.jsonl)
    p.epi = (long long)w * (rows_a + rows_b) < dcte::kEpiMaxPx ? 1 : 0;
    p.out = d_out;
    p.out_stride = out_stride;
    p.we = (float)((double)edges / scale);
    p.wt = (float)((double)textures / scale);
    p.tie_tau = (float)eff_tau(ctx, n);
    p.edges = edges;
    p.textures = textures;
    p.fix_list = f->d_list;
    p.tile_count = f->d_tiles;
    p.dirty_list = f->d_tiles + ntiles;
    p.dirty_count = f->d_count + 2 + f->phase;
    p.dirty_next = f->d_count + 2 + (f->phase ^ 1u);
    p.fix_total = f->d_count + 1;
    p.dense_ctr = reinterpret_cast<unsigned long long*>(f->d_count + 4) + f->phase;
    p.dense_next = reinterpret_cast<unsigned long long*>(f->d_count + 4) + (f->phase ^ 1u);
    p.dense_list = reinterpret_cast<uint2*>(f->d_tiles + 2 * ntiles);
    p.dense_batch = static_cast<uint4*>(f->d_batch);
    p.stamps = ctx->stamps;

    dcte::TileFixParams q{};
    q.m = p;
    small_twiddles(n, q.ct);
    q.fix_total = f->d_count + 1;
    q.tiles_x = tiles_x;
    q.tile_w = dcte::map_tile_w(n);

    // Any failure from here on leaves both dirty counters zeroed on the
    // stream: a map launch that never ran did not zero its successor's counter,
    // and a later call must not walk an older launch's dirty list.
    auto fail = [&](hipError_t e, const char* where) {
        (void)hipMemsetAsync(f->d_count + 2, 0, (kCountWords - 2) * sizeof(unsigned), s);
        return hip_fail(ctx, e, where);
    };
    hipError_t e = hipSuccess;
    if (ctx->profile) {
        ProfEvent ev{d.id, nullptr, nullptr};
        if ((e = hipEventCreate(&ev.a)) != hipSuccess) return fail(e, "hipEventCreate");
        if ((e = hipEventCreate(&ev.b)) != hipSuccess) {
            (void)hipEventDestroy(ev.a);
            return fail(e, "hipEventCreate");
        }
        ctx->prof.push_back(ev);      // dcte_profile_read destroys them
        if ((e = dcte::launch_map(n, bpp, sem, p, s, ev.a, ev.b)) != hipSuccess) return fail(e, "launch_map");
    } else if ((e = dcte::launch_map(n, bpp, sem, p, s)) != hipSuccess) {
        return fail(e, "launch_map");
    }
    // testing (DCTE_OPT_FAIL_INJECT): the launch was queued, report it failed
    auto injected = [&](int which) {
        if (ctx->fail_inject != which) return false;
        ctx->fail_inject = 0;
        return true;
    };
    if (injected(1)) return fail(hipErrorLaunchFailure, "launch_map (injected)");
    f->phase ^= 1u;   // the launch ran: the next one uses the counter it zeroed
    if ((p.we != p.wt && eff_tau(ctx, n) > 0) || eff_tau(ctx, n) >= 1.0) {
        if ((e = dcte::launch_fix_tiles(n, bpp, sem, q, s)) != hipSuccess) return fail(e, "launch_fix_tiles");
        if (injected(2)) return fail(hipErrorLaunchFailure, "launch_fix_tiles (injected)");
    }
    return DCTE_OK;
}

int ensure_buf(dcte_ctx* ctx, void** p, size_t* cap, size_t bytes)
{
    if (*cap >= bytes) return DCTE_OK;
    if (*p) DCTE_HIP(ctx, hipFree(*p));
    *p = nullptr;
    *cap = 0;
    DCTE_HIP(ctx, hipMalloc(p, bytes));
    *cap = bytes;
    return DCTE_OK;
}

int ensure_stream(dcte_ctx* ctx, Device& d)
{
    DCTE_HIP(ctx, hipSetDevice(d.id));
    if (!d.stream) DCTE_HIP(ctx, hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    if (!d.d_keys) {
        DCTE_HIP(ctx, hipMalloc(&d.d_keys, 2 * sizeof(unsigned) + 2 * sizeof(float)));
        d.d_minmax = reinterpret_cast<float*>(d.d_keys + 2);
    }
    return DCTE_OK;
}

bool valid_norm(int mode, int channels)
{
    return (mode == DCTE_NORM_LQR || mode == DCTE_NORM_PREVIEW) && channels >= 1 && channels <= 4;
}

// Page-locks a caller buffer for the duration of a host call (RAII), so that
// no copy of the call goes through the runtime's pageable path.  Only the
// WHOLE pages inside the caller's bytes are registered, [lo, hi), and only for
// buffers of at least DCTE_OPT_PIN_HOST MiB: a page the buffer shares with a
// neighbour is never locked by us.  (r05 registered exactly the caller's
// bytes, after a page-rounded range had made the runtime refuse copies into a
// neighbour -- tools/pin_probe.cpp; but the runtime locks whole pages, and a
// pageable copy of a neighbour sharing the first or last page -- the runtime
// pins such copies on the fly and unpins them afterwards -- then left the
// download into our buffer faulting: hipErrorIllegalAddress at the sync of
// test_extreme_aspect_ratios, a 3 x 100003 grey frame whose 300 KB frame copy
// was pageable and whose 1.2 MB map was registered.)  The bytes outside
// [lo, hi) -- the partial pages at either end, or the whole of a small buffer
// -- are staged through the context's page-locked arena for the role
// (dcte_ctx::stage): an input's are copied there when the pin is made, an
// output's are copied back by commit() after the call's streams are drained.
// (r06: pageable copies of one frame on several streams at once -- the band
// uploads of a multi-device context, whose halo rows share pages, or the
// transposed strips, which all read every row -- faulted the same way,
// test_exact_multi_device_host_path, profiles/r06/multi_device_pageable_fault.log.)
// With `mapped`, also the device address of lo (dev) for a copy kernel to
// write into; a caller-pinned buffer (hipHostMalloc, or registered by the
// caller) is used whole, with its own device address.  DCTE_OPT_PIN_HOST <= 0:
// no registration, every byte staged.  Only when the arena cannot be allocated
// do the outside bytes take the runtime's pageable path.
struct HostPin {
    void* base = nullptr;            // what we registered (unregistered at the end)
    uintptr_t p0 = 0, p1 = 0;        // the caller's bytes
    uintptr_t lo = 0, hi = 0;        // the pinned part (registered or caller-pinned)
    void* dev = nullptr;             // device address of lo (mapped), or null
    uint8_t* st = nullptr;           // staged [p0, lo) then [hi, p1), or null (pageable)
    bool output = false;
    HostPin(dcte_ctx* ctx, const void* p, size_t bytes, bool mapped, int role, bool is_output)
    {
        if (!p || bytes == 0) return;
        output = is_output;
        p0 = reinterpret_cast<uintptr_t>(p);
        p1 = p0 + bytes;
        void* v = const_cast<void*>(p);
        // a caller-pinned buffer first (registering part of it would fail)
        void* cdev = nullptr;
        if (hipHostGetDevicePointer(&cdev, v, 0) == hipSuccess && cdev) {
            lo = p0;
            hi = p1;
            dev = mapped ? cdev : nullptr;
            return;
        }
        (void)hipGetLastError();
        lo = hi = p1;                                  // nothing registered: all staged
        const uintptr_t a = (p0 + 4095u) & ~(uintptr_t)4095u, b = p1 & ~(uintptr_t)4095u;
        if (ctx->pin_mib > 0 && (double)bytes >= ctx->pin_mib * 1048576.0 && b > a) {
            void* va = reinterpret_cast<void*>(a);
            if (hipHostRegister(va, b - a, mapped ? hipHostRegisterMapped : hipHostRegisterDefault) ==
                hipSuccess) {
                base = va;
                lo = a;
                hi = b;
                if (mapped && hipHostGetDevicePointer(&dev, va, 0) != hipSuccess) {
                    dev = nullptr;
                    (void)hipGetLastError();
                }
            } else {
                (void)hipGetLastError();
            }
        }
        const size_t ns = (size_t)(lo - p0) + (size_t)(p1 - hi);
        if (!ns) return;
        auto& S = ctx->stage[role];
        if (S.cap < ns) {                              // no copy of an earlier call is in flight
            if (S.p) (void)hipHostFree(S.p);
            S.p = nullptr;
            S.cap = 0;
            if (hipHostMalloc(reinterpret_cast<void**>(&S.p), ns, hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                S.p = nullptr;                         // the pageable path, as before r06
                return;
            }
            S.cap = ns;
        }
        st = S.p;
        if (!output) {
            memcpy(st, reinterpret_cast<const void*>(p0), lo - p0);
            memcpy(st + (lo - p0), reinterpret_cast<const void*>(hi), p1 - hi);
        }
    }
    // the host address to copy caller bytes [a, ...) outside [lo, hi) to /
    // from: their staged copy (the piece must lie wholly before lo or wholly
    // at or after hi), or the caller's own bytes when nothing is staged
    uint8_t* outside(uintptr_t a) const
    {
        if (!st) return reinterpret_cast<uint8_t*>(a);
        return a < lo ? st + (a - p0) : st + (lo - p0) + (a - hi);
    }
    // an output's staged bytes into the caller's buffer (after the streams
    // are drained; a failed call leaves them untouched)
    void commit() const
    {
        if (!output || !st) return;
        memcpy(reinterpret_cast<void*>(p0), st, lo - p0);
        memcpy(reinterpret_cast<void*>(hi), st + (lo - p0), p1 - hi);
    }
    ~HostPin()
    {
        if (base) (void)hipHostUnregister(base);
    }
    HostPin(const HostPin&) = delete;
    HostPin& operator=(const HostPin&) = delete;
};

// Device -> host bytes of a host call: the part inside the pinned range by a
// copy kernel into its device address (the GPU's own stores over PCIe, so it
// runs beside the SDMA upload) or else the runtime's copy engine; the parts
// outside it (partial pages at the buffer's ends, a small buffer, or no pin)
// into their staged copies (HostPin::outside).
hipError_t download(const HostPin* pin, void* host, const void* dev, size_t bytes, hipStream_t s)
{
    const uintptr_t h0 = reinterpret_cast<uintptr_t>(host), h1 = h0 + bytes;
    const bool reg = pin && pin->hi > pin->lo;
    const uintptr_t m0 = reg ? std::max(h0, pin->lo) : h1;
    const uintptr_t m1 = reg ? std::min(h1, pin->hi) : h1;
    const uint8_t* d = static_cast<const uint8_t*>(dev);
    hipError_t e = hipSuccess;
    auto copy = [&](uintptr_t a, uintptr_t b, bool inside) {
        if (b > a && e == hipSuccess)
            e = hipMemcpyAsync(inside || !pin ? reinterpret_cast<void*>(a) : pin->outside(a), d + (a - h0), b - a,
                               hipMemcpyDeviceToHost, s);
    };
    if (m1 <= m0) {                                    // wholly before lo, or at / after hi
        copy(h0, h1, false);
        return e;
    }
    copy(h0, m0, false);
    if (e == hipSuccess) {
        const uint8_t* src = d + (m0 - h0);
        uint8_t* hd = pin->dev ? static_cast<uint8_t*>(pin->dev) + (m0 - pin->lo) : nullptr;
        if (hd && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(hd)) & 3u) == 0)
            e = dcte::launch_copy_to_host(src, hd, m1 - m0, s);
        else
            copy(m0, m1, true);
    }
    copy(m1, h1, false);
    return e;
}

// Host -> device rows (a 2-D copy: `rows` rows of `width` bytes, host row
// pitch spitch, device pitch dpitch), split so that every copy lies either
// inside the pinned range [lo, hi) or outside it: the rows inside go as one
// 2-D copy, the rows before / after it as 2-D copies from their staged bytes,
// a row that straddles lo or hi as 1-D pieces.
hipError_t upload_rows(const HostPin* pin, uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch,
                       size_t width, size_t rows, hipStream_t s)
{
    if (rows == 0 || width == 0) return hipSuccess;
    const uintptr_t s0 = reinterpret_cast<uintptr_t>(src);
    auto start = [&](size_t r) { return s0 + r * spitch; };
    // rows [r0, r1) as one 2-D copy, from the caller's bytes (inside) or their staged copy
    auto copy2d = [&](size_t r0, size_t r1, bool inside) -> hipError_t {
        if (r1 <= r0) return hipSuccess;
        const uint8_t* from = inside || !pin ? src + r0 * spitch : pin->outside(start(r0));
        return hipMemcpy2DAsync(dst + r0 * dpitch, dpitch, from, spitch, width, r1 - r0, hipMemcpyHostToDevice, s);
    };
    if (!pin || pin->hi <= pin->lo) return copy2d(0, rows, false);
    // first row starting at or after lo, first row ending after hi
    size_t r1 = pin->lo <= s0 ? 0 : (size_t)((pin->lo - s0 + spitch - 1) / spitch);
    size_t r2 = pin->hi < s0 + width ? 0 : (size_t)((pin->hi - s0 - width) / spitch) + 1;
    r1 = std::min(r1, rows);
    r2 = std::min(std::max(r2, r1), rows);
    hipError_t e = hipSuccess;
    auto piece = [&](size_t r, uintptr_t a, uintptr_t b) {   // bytes [a, b) of host row r, split at lo, hi
        const uintptr_t cuts[4] = {a, std::min(std::max(pin->lo, a), b), std::min(std::max(pin->hi, a), b), b};
        for (int k = 0; k < 3 && e == hipSuccess; k++)
            if (cuts[k + 1] > cuts[k])
                e = hipMemcpyAsync(dst + r * dpitch + (cuts[k] - start(r)),
                                   k == 1 ? reinterpret_cast<const uint8_t*>(cuts[k]) : pin->outside(cuts[k]),
                                   cuts[k + 1] - cuts[k], hipMemcpyHostToDevice, s);
    };
    auto outside_rows = [&](size_t a, size_t b, uintptr_t cut) {   // rows [a, b); one may straddle cut
        for (size_t r = a; r < b && e == hipSuccess;) {
            const uintptr_t r_lo = start(r), r_hi = r_lo + width;
            if (r_lo < cut && r_hi > cut) {
                piece(r, r_lo, r_hi);
                r++;
            } else {
                size_t q = r + 1;   // a run of rows that do not straddle
                while (q < b && !(start(q) < cut && start(q) + width > cut)) q++;
                e = copy2d(r, q, false);
                r = q;
            }
        }
    };
    outside_rows(0, r1, pin->lo);
    if (e == hipSuccess) e = copy2d(r1, r2, true);
    if (e == hipSuccess) outside_rows(r2, rows, pin->hi);
    return e;
}

#ifndef DCTE_CHUNK_ROWS
#define DCTE_CHUNK_ROWS 1024   // A/B: 22.4 ms per 16384^2 RGB frame vs 23.1 at 2048 (profiles/r02/host_chunks.jsonl)
#endif
#ifndef DCTE_MAX_CHUNKS
#define DCTE_MAX_CHUNKS 16
#endif
#ifndef DCTE_CHUNK_SPLIT
#define DCTE_CHUNK_SPLIT 8      // at least this many chunks per band ...
#endif
#ifndef DCTE_CHUNK_MIN_ROWS
#define DCTE_CHUNK_MIN_ROWS 256 // ... of at least this many rows
#endif
constexpr int kChunkRows = DCTE_CHUNK_ROWS;   // host path: output rows per pipeline chunk
constexpr int kMaxChunks = DCTE_MAX_CHUNKS;

// rows per chunk of a host-path band of `rows` rows: at least DCTE_CHUNK_SPLIT
// chunks where the band allows (a shorter first upload and last download: the
// pipeline's ramp), at least DCTE_CHUNK_MIN_ROWS rows, at most kChunkRows
int chunk_rows(int rows)
{
    int crows = rows / DCTE_CHUNK_SPLIT;
    return crows < DCTE_CHUNK_MIN_ROWS ? DCTE_CHUNK_MIN_ROWS : (crows > kChunkRows ? kChunkRows : crows);
}

int ensure_pipe(dcte_ctx* ctx, Device& d, size_t nev)
{
    DCTE_HIP(ctx, hipSetDevice(d.id));
    if (!d.up) DCTE_HIP(ctx, hipStreamCreateWithFlags(&d.up, hipStreamNonBlocking));
    if (!d.down) DCTE_HIP(ctx, hipStreamCreateWithFlags(&d.down, hipStreamNonBlocking));
    while (d.ev.size() < nev) {
        hipEvent_t e;
        DCTE_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        d.ev.push_back(e);
    }
    return DCTE_OK;
}

// Zeroes the refined-pixel counter of the host path's stream before a band's
// launches (sync_bands reads it).  The exact mode has no refinement lists, so
// only a fast-mode call grows them to the band's size.
int reset_refined(dcte_ctx* ctx, Device& d, int w, int rows, int n, int sem)
{
    FixScratch* f = nullptr;
    if (!(ctx->exact && dcte::exact_supported(n, sem))) {
        int rc = ensure_fix(ctx, d, d.stream, (size_t)w * (size_t)rows, &f);
        if (rc) return rc;
    } else {
        auto it = d.fix.find(d.stream);
        if (it == d.fix.end()) return DCTE_OK;
        f = &it->second;
    }
    DCTE_HIP(ctx, hipMemsetAsync(f->d_count + 1, 0, sizeof(unsigned), d.stream));
    return DCTE_OK;
}

// host frame -> device band maps (rows split over the context's devices),
// left on the devices in d.d_out; returns the number of devices used.
// Each band runs as a pipeline of row chunks on three streams -- H2D of the
// rows chunk c needs (up), its map (d.stream), D2H of its output rows into
// host_out when given (down) -- so the PCIe copies of neighbouring chunks
// overlap each other and the kernels.
// transposed: the map of the transposed frame (w x h -> h x w); device k
// takes a strip of source COLUMNS (= transposed rows) plus halo, transposes
// it in HBM and maps it (one chunk).
int map_bands(dcte_ctx* ctx, const uint8_t* px, int w, int h, int bpp, size_t rowstride, int n,
              float edges, float textures, int sem, int transposed, float* host_out, int* used,
              const HostPin* pin_in = nullptr, const HostPin* pin_out = nullptr)
{
    const int W = transposed ? h : w, H = transposed ? w : h;   // mapped frame
    const int G = (int)ctx->devs.size() < H ? (int)ctx->devs.size() : H;
    *used = G;                         // even on error: the caller drains these streams
    int hl, hr;
    halo(n, sem, hl, hr);
    for (int k = 0; k < G; k++) {
        Device& d = ctx->devs[k];
        int y0 = (int)((long long)H * k / G), y1 = (int)((long long)H * (k + 1) / G);
        int lo, hi;
        needed_rows(n, sem, H, y0, y1, lo, hi);
        const size_t pitch = (size_t)W * bpp;                   // mapped-frame row
        size_t in_bytes = pitch * (size_t)(hi - lo + 1);
        size_t out_bytes = sizeof(float) * (size_t)W * (size_t)(y1 - y0);
        int rc = ensure_stream(ctx, d);
        if (rc) return rc;
        rc = ensure_buf(ctx, (void**)&d.d_in, &d.in_cap, in_bytes);
        if (rc) return rc;
        rc = ensure_buf(ctx, (void**)&d.d_out, &d.out_cap, out_bytes);
        if (rc) return rc;
        rc = reset_refined(ctx, d, W, y1 - y0, n, sem);
        if (rc) return rc;
        if (transposed) {
            // source columns [lo, hi] of all h rows -> (h x cols) strip -> transpose
            const size_t sw = (size_t)(hi - lo + 1) * bpp;
            DCTE_HIP(ctx, upload_rows(pin_in, d.d_in, sw, px + (size_t)lo * bpp, rowstride, sw, h, d.stream));
            rc = ensure_buf(ctx, (void**)&d.d_tr, &d.tr_cap, in_bytes);
            if (rc) return rc;
            DCTE_HIP(ctx, dcte::launch_transpose_u8(d.d_in, (long long)sw, h, hi - lo + 1, bpp,
                                                    d.d_tr, (long long)pitch, d.stream));
            rc = run_device(ctx, d, d.d_tr, (long long)pitch, W, H, bpp, lo, hi - lo + 1, y0, y1,
                            n, edges, textures, sem, d.d_out, W, d.stream);
            if (rc) return rc;
            if (host_out)
                DCTE_HIP(ctx, download(pin_out, host_out + (size_t)y0 * W, d.d_out, out_bytes, d.stream));
            continue;
        }
        const int crows = chunk_rows(y1 - y0);
        int nch = (y1 - y0 + crows - 1) / crows;
        nch = nch < 1 ? 1 : (nch > kMaxChunks ? kMaxChunks : nch);
        rc = ensure_pipe(ctx, d, 2 * (size_t)nch);
        if (rc) return rc;
        int loaded = lo - 1;                                    // last uploaded row
        for (int c = 0; c < nch; c++) {
            const int a = y0 + (int)((long long)(y1 - y0) * c / nch);
            const int b = y0 + (int)((long long)(y1 - y0) * (c + 1) / nch);
            if (a == b) continue;
            const int need = b - 1 + hr < H - 1 ? b - 1 + hr : H - 1;
            hipEvent_t ev_up = d.ev[2 * c], ev_map = d.ev[2 * c + 1];
            if (need > loaded) {
                DCTE_HIP(ctx, upload_rows(pin_in, d.d_in + (size_t)(loaded + 1 - lo) * pitch, pitch,
                                          px + (size_t)(loaded + 1) * rowstride, rowstride, pitch,
                                          (size_t)(need - loaded), d.up));
                loaded = need;
            }
            DCTE_HIP(ctx, hipEventRecord(ev_up, d.up));
            DCTE_HIP(ctx, hipStreamWaitEvent(d.stream, ev_up, 0));
            rc = run_device(ctx, d, d.d_in, (long long)pitch, W, H, bpp, lo, loaded - lo + 1, a, b,
                            n, edges, textures, sem, d.d_out + (size_t)(a - y0) * W, W, d.stream);
            if (rc) return rc;
            if (host_out) {
                DCTE_HIP(ctx, hipEventRecord(ev_map, d.stream));
                DCTE_HIP(ctx, hipStreamWaitEvent(d.down, ev_map, 0));
                DCTE_HIP(ctx, download(pin_out, host_out + (size_t)a * W, d.d_out + (size_t)(a - y0) * W,
                                       sizeof(float) * (size_t)W * (size_t)(b - a), d.down));
            }
        }
    }
    return DCTE_OK;
}

// Host path on ONE device with the whole frame resident (the
// plug-in's build for a vertical resize needs the maps of both orientations,
// src/render.c:358-364): row chunks of the frame go up on d.up; with `out`,
// each chunk is mapped on d.stream as soon as its rows and halo are in and its
// map goes down on d.down; with `out_t`, the resident frame is then
// transposed in HBM and the transposed frame mapped in row chunks (= source
// column strips), each downloaded as soon as it is mapped -- one upload for
// both orientations, and the downloads of both maps back to back on d.down.
int map_pipeline_one(dcte_ctx* ctx, const uint8_t* px, int w, int h, int bpp, size_t rowstride,
                     int n, float edges, float textures, int sem, float* out, float* out_t,
                     const HostPin* pin_in, const HostPin* pin_out, const HostPin* pin_out_t)
{
    Device& d = ctx->devs[0];
    int hl, hr;
    halo(n, sem, hl, hr);
    const size_t pitch = (size_t)w * bpp, pitch_t = (size_t)h * bpp;
    const size_t fbytes = pitch * (size_t)h, mbytes = sizeof(float) * (size_t)w * (size_t)h;
    int rc = ensure_stream(ctx, d);
    if (rc) return rc;
    if ((rc = ensure_buf(ctx, (void**)&d.d_in, &d.in_cap, fbytes))) return rc;
    if (out && (rc = ensure_buf(ctx, (void**)&d.d_out, &d.out_cap, mbytes))) return rc;
    if (out_t) {
        if ((rc = ensure_buf(ctx, (void**)&d.d_tr, &d.tr_cap, fbytes))) return rc;
        if ((rc = ensure_buf(ctx, (void**)&d.d_out2, &d.out2_cap, mbytes))) return rc;
    }
    if ((rc = reset_refined(ctx, d, w, h, n, sem))) return rc;
    // at least 8 chunks of >= 256 rows where the frame allows (map_bands)
    auto chunks = [](int rows) {
        const int crows = chunk_rows(rows);
        int nch = (rows + crows - 1) / crows;
        return nch < 1 ? 1 : (nch > kMaxChunks ? kMaxChunks : nch);
    };
    const int nch0 = chunks(h), nch1 = out_t ? chunks(w) : 0;
    if ((rc = ensure_pipe(ctx, d, 2 * (size_t)nch0 + (size_t)nch1))) return rc;
    int loaded = -1;                                            // last uploaded row
    for (int c = 0; c < nch0; c++) {
        const int a = (int)((long long)h * c / nch0), b = (int)((long long)h * (c + 1) / nch0);
        if (a == b) continue;
        const int need = out ? (b - 1 + hr < h - 1 ? b - 1 + hr : h - 1) : b - 1;
        hipEvent_t ev_up = d.ev[2 * c], ev_map = d.ev[2 * c + 1];
        if (need > loaded) {
            DCTE_HIP(ctx, upload_rows(pin_in, d.d_in + (size_t)(loaded + 1) * pitch, pitch,
                                      px + (size_t)(loaded + 1) * rowstride, rowstride, pitch,
                                      (size_t)(need - loaded), d.up));
            loaded = need;
        }
        DCTE_HIP(ctx, hipEventRecord(ev_up, d.up));
        if (!out) continue;
        DCTE_HIP(ctx, hipStreamWaitEvent(d.stream, ev_up, 0));
        rc = run_device(ctx, d, d.d_in, (long long)pitch, w, h, bpp, 0, loaded + 1, a, b, n, edges,
                        textures, sem, d.d_out + (size_t)a * w, w, d.stream);
        if (rc) return rc;
        DCTE_HIP(ctx, hipEventRecord(ev_map, d.stream));
        DCTE_HIP(ctx, hipStreamWaitEvent(d.down, ev_map, 0));
        DCTE_HIP(ctx, download(pin_out, out + (size_t)a * w, d.d_out + (size_t)a * w,
                               sizeof(float) * (size_t)w * (size_t)(b - a), d.down));
    }
    if (!out_t) return DCTE_OK;
    // the whole frame is in once the last upload is (ordered after every copy on d.up)
    DCTE_HIP(ctx, hipEventRecord(d.ev[2 * nch0 - 2], d.up));
    DCTE_HIP(ctx, hipStreamWaitEvent(d.stream, d.ev[2 * nch0 - 2], 0));
    DCTE_HIP(ctx, dcte::launch_transpose_u8(d.d_in, (long long)pitch, h, w, bpp, d.d_tr,
                                            (long long)pitch_t, d.stream));
    for (int c = 0; c < nch1; c++) {
        const int a = (int)((long long)w * c / nch1), b = (int)((long long)w * (c + 1) / nch1);
        if (a == b) continue;
        rc = run_device(ctx, d, d.d_tr, (long long)pitch_t, h, w, bpp, 0, w, a, b, n, edges, textures,
                        sem, d.d_out2 + (size_t)a * h, h, d.stream);
        if (rc) return rc;
        hipEvent_t ev_map = d.ev[2 * nch0 + c];
        DCTE_HIP(ctx, hipEventRecord(ev_map, d.stream));
        DCTE_HIP(ctx, hipStreamWaitEvent(d.down, ev_map, 0));
        DCTE_HIP(ctx, download(pin_out_t, out_t + (size_t)a * h, d.d_out2 + (size_t)a * h,
                               sizeof(float) * (size_t)h * (size_t)(b - a), d.down));
    }
    return DCTE_OK;
}

// error path: wait for every stream of the first G devices, keep last_error
void drain(dcte_ctx* ctx, int G)
{
    for (int k = 0; k < G; k++) {
        Device& d = ctx->devs[k];
        if (hipSetDevice(d.id) != hipSuccess) continue;
        if (d.up) (void)hipStreamSynchronize(d.up);
        if (d.stream) (void)hipStreamSynchronize(d.stream);
        if (d.down) (void)hipStreamSynchronize(d.down);
    }
}

struct HostPin;
int normalize_bands(dcte_ctx* ctx, int w, int h, int mode, int channels, uint8_t* out, int G,
                    const HostPin* pin_out);

int sync_bands(dcte_ctx* ctx, int G)
{
    for (int k = 0; k < G; k++) {
        Device& d = ctx->devs[k];
        hipError_t e = hipSetDevice(d.id);
        if (e == hipSuccess && d.up) e = hipStreamSynchronize(d.up);
        if (e == hipSuccess) e = hipStreamSynchronize(d.stream);
        if (e == hipSuccess && d.down) e = hipStreamSynchronize(d.down);
        if (e != hipSuccess) {
            // the caller's buffers are unpinned on return: nothing of this
            // call may still be in flight on any device
            const int rc = hip_fail(ctx, e, "sync_bands");
            drain(ctx, G);
            return rc;
        }
        auto it = d.fix.find(d.stream);
        if (it != d.fix.end()) {
            unsigned cnt = 0;
            DCTE_HIP(ctx, hipMemcpy(&cnt, it->second.d_count + 1, sizeof(unsigned), hipMemcpyDeviceToHost));
            ctx->last_refined += cnt;
        }
    }
    return DCTE_OK;
}

}  // namespace

extern "C" {

int dcte_abi_version(void) { return DCTE_ABI_VERSION; }

int dcte_device_count(void)
{
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

int dcte_create(dcte_ctx** out, int ngpus, unsigned flags)
{
    if (!out || ngpus < 0 || (flags & ~DCTE_CREATE_SAME_DEVICE)) return DCTE_EINVAL;
    *out = nullptr;
    int count = dcte_device_count();
    if (count <= 0) return DCTE_ENODEV;
    const bool same = (flags & DCTE_CREATE_SAME_DEVICE) != 0;
    if (ngpus == 0) ngpus = same ? 1 : count;
    if (!same && ngpus > count) ngpus = count;
    dcte_ctx* ctx = new (std::nothrow) dcte_ctx;
    if (!ctx) return DCTE_ENOMEM;
    ctx->devs.resize(ngpus);
    for (int i = 0; i < ngpus; i++) ctx->devs[i].id = same ? 0 : i;
    const char* tau = getenv("DCTE_TIE_TAU");
    if (tau && *tau) ctx->tie_tau = atof(tau);
    const char* pin = getenv("DCTE_PIN_HOST");       // DCTE_OPT_PIN_HOST's initial value (diagnostics)
    if (pin && *pin) ctx->pin_mib = atof(pin);
    *out = ctx;
    return DCTE_OK;
}

void dcte_destroy(dcte_ctx* ctx)
{
    DeviceGuard guard_;
    if (!ctx) return;
    for (Device& d : ctx->devs) {
        if (d.id < 0) continue;
        if (hipSetDevice(d.id) != hipSuccess) continue;
        if (d.stream) (void)hipStreamSynchronize(d.stream);
        for (auto& kv : d.fix) {
            (void)hipStreamSynchronize(kv.first);
            if (kv.second.d_count) (void)hipFree(kv.second.d_count);
            if (kv.second.d_list) (void)hipFree(kv.second.d_list);
            if (kv.second.d_tiles) (void)hipFree(kv.second.d_tiles);
            if (kv.second.d_batch) (void)hipFree(kv.second.d_batch);
        }
        for (auto& kv : d.dp) {
            (void)hipStreamSynchronize(kv.first);
            if (kv.second.buf) (void)hipFree(kv.second.buf);
            if (kv.second.xbuf) (void)hipFree(kv.second.xbuf);
        }
        if (d.d_in) (void)hipFree(d.d_in);
        if (d.d_out) (void)hipFree(d.d_out);
        if (d.d_keys) (void)hipFree(d.d_keys);
        if (d.d_u8) (void)hipFree(d.d_u8);
        if (d.d_tr) (void)hipFree(d.d_tr);
        if (d.d_out2) (void)hipFree(d.d_out2);
        if (d.up) (void)hipStreamSynchronize(d.up);
        if (d.down) (void)hipStreamSynchronize(d.down);
        for (hipEvent_t e : d.ev) (void)hipEventDestroy(e);
        if (d.up) (void)hipStreamDestroy(d.up);
        if (d.down) (void)hipStreamDestroy(d.down);
        if (d.stream) (void)hipStreamDestroy(d.stream);
    }
    for (auto& st : ctx->stage)
        if (st.p) (void)hipHostFree(st.p);
    delete ctx;
}

int dcte_ctx_devices(const dcte_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int dcte_set_option(dcte_ctx* ctx, int option, double value)
{
    if (!ctx) return DCTE_EINVAL;
    switch (option) {
    case DCTE_OPT_TIE_TAU:
        if (value != value) return DCTE_EINVAL;
        ctx->tie_tau = value < 0 ? -1 : value;   // < 0: the per-N defaults again
        return DCTE_OK;
    case DCTE_OPT_PROFILE:
        ctx->profile = value != 0;
        return DCTE_OK;
    case DCTE_OPT_PIN_HOST:
        if (!(value >= 0)) return DCTE_EINVAL;
        ctx->pin_mib = value;
        return DCTE_OK;
    case DCTE_OPT_TILE_H:
        if (!(value >= 0 && value <= 4096)) return DCTE_EINVAL;
        ctx->tile_h = (int)value;
        return DCTE_OK;
    case DCTE_OPT_DP_BANDWISE:
        ctx->dp_bandwise = value != 0;
        return DCTE_OK;
    case DCTE_OPT_DP_SPIN_LIMIT:
        if (!(value >= 0 && value <= 4294967295.0)) return DCTE_EINVAL;
        ctx->dp_spin_limit = (unsigned)value;
        // re-enables the single-launch search on streams a timeout moved to
        // band-wise launches
        for (Device& d : ctx->devs)
            for (auto& kv : d.dp) kv.second.max_tiles = -1;
        return DCTE_OK;
    case DCTE_OPT_TSTAMP_BUF:
        // a device address (exact in a double below 2^53); 0 = none
        if (!(value >= 0 && value < 9007199254740992.0)) return DCTE_EINVAL;
        ctx->stamps = reinterpret_cast<unsigned long long*>((uintptr_t)value);
        return DCTE_OK;
    case DCTE_OPT_FAIL_INJECT:
        if (!(value == 0 || value == 1 || value == 2)) return DCTE_EINVAL;
        ctx->fail_inject = (int)value;
        return DCTE_OK;
    case DCTE_OPT_LEGACY_8:
        // DCTE_OPT_WIDE_BANDS of the first release (removed; results never
        // depended on it): still accepted, ignored
        return DCTE_OK;
    case DCTE_OPT_EXACT:
        ctx->exact = value != 0;
        return DCTE_OK;
    case DCTE_OPT_D2H_KERNEL:
        ctx->d2h_kernel = value != 0;
        return DCTE_OK;
    default: return DCTE_EINVAL;
    }
}

int dcte_energy_map_device(dcte_ctx* ctx, int device, const void* d_px, long long rowstride,
                           int w, int h, int bpp, int in_row0, int in_rows, int y0, int y1,
                           int n, float edges, float textures, int semantics, float* d_out,
                           long long out_stride, void* stream)
{
    DeviceGuard guard_;
    if (!ctx || device < 0 || device >= (int)ctx->devs.size()) return DCTE_EINVAL;
    return run_device(ctx, ctx->devs[device], d_px, rowstride, w, h, bpp, in_row0, in_rows, y0,
                      y1, n, edges, textures, semantics, d_out, out_stride, (hipStream_t)stream);
}

int dcte_energy_map_device2(dcte_ctx* ctx, int device, const void* d_px, long long rowstride,
                            int w, int h, int bpp, int in_row0, int in_rows, int y0, int y1,
                            int yb0, int yb1, int n, float edges, float textures, int semantics,
                            float* d_out, long long out_stride, void* stream)
{
    DeviceGuard guard_;
    if (!ctx || device < 0 || device >= (int)ctx->devs.size()) return DCTE_EINVAL;
    DCTE_ARG(ctx, yb0 <= yb1);
    return run_device(ctx, ctx->devs[device], d_px, rowstride, w, h, bpp, in_row0, in_rows, y0,
                      y1, n, edges, textures, semantics, d_out, out_stride, (hipStream_t)stream,
                      yb0, yb1);
}

int dcte_seam_carve_device(dcte_ctx* ctx, int device, const void* d_px, long long rowstride, int w,
                           int h, int bpp, const int* d_seam, const float* d_map,
                           long long map_stride, void* d_px_out, long long out_rowstride,
                           float* d_map_out, long long map_out_stride, int n, float edges,
                           float textures, int semantics, void* stream)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, device >= 0 && device < (int)ctx->devs.size());
    DCTE_ARG(ctx, valid_n(n) && valid_sem_bpp(semantics, bpp) && w >= 2 && h >= 1);
    DCTE_ARG(ctx, d_px && d_seam && d_map && d_px_out && d_map_out);
    DCTE_ARG(ctx, rowstride >= (long long)w * bpp && out_rowstride >= (long long)(w - 1) * bpp);
    DCTE_ARG(ctx, map_stride >= w && map_out_stride >= w - 1);
    Device& d = ctx->devs[device];
    hipStream_t s = (hipStream_t)stream;
    DCTE_HIP(ctx, hipSetDevice(d.id));
    FixScratch* f = nullptr;
    const size_t npix = (size_t)(w - 1) * (size_t)h;
    if (npix >= (1ULL << 32)) return DCTE_ERANGE;
    // the shift and band kernels address both frames through 32-bit buffer offsets
    if (!span_ok(h, rowstride, w, bpp) || !span_ok(h, out_rowstride, w - 1, bpp)) {
        ctx->last_error = "frame spans 4 GiB or more";
        return DCTE_ERANGE;
    }
    int rc = ensure_fix(ctx, d, s, npix, &f);
    if (rc) return rc;
    const double scale = weight_scale(n, semantics);
    dcte::SeamParams p{};
    p.px = static_cast<const uint8_t*>(d_px);
    p.rowstride = rowstride;
    p.w = w;
    p.h = h;
    p.bpp = bpp;
    p.n = n;
    p.sem = semantics;
    p.seam = d_seam;
    p.map = d_map;
    p.map_stride = map_stride;
    p.px_out = static_cast<uint8_t*>(d_px_out);
    p.out_rowstride = out_rowstride;
    p.map_out = d_map_out;
    p.map_out_stride = map_out_stride;
    p.we = (float)((double)edges / scale);
    p.wt = (float)((double)textures / scale);
    p.tie_tau = (float)eff_tau(ctx, n);
    p.fix_count = f->d_count;
    p.fix_list = f->d_list;
    p.fix_cap = (unsigned)f->cap;
    DCTE_HIP(ctx, hipMemsetAsync(f->d_count, 0, sizeof(unsigned), s));
    DCTE_HIP(ctx, dcte::launch_seam_carve(p, s));
    if ((p.we != p.wt && eff_tau(ctx, n) > 0) || eff_tau(ctx, n) >= 1.0) {
        dcte::FixParams q = fix_params(p.px_out, out_rowstride, w - 1, h, 0, bpp, n, 0, semantics,
                                       d_map_out, map_out_stride, edges, textures, f);
        DCTE_HIP(ctx, dcte::launch_fix(q, s));
    }
    return DCTE_OK;
}

int dcte_energy_points_device(dcte_ctx* ctx, int device, const void* d_px, long long rowstride,
                              int w, int h, int bpp, const int* d_xy, int count, int n,
                              float edges, float textures, int semantics, float* d_out,
                              void* stream)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, device >= 0 && device < (int)ctx->devs.size());
    DCTE_ARG(ctx, valid_n(n) && valid_sem_bpp(semantics, bpp) && w >= 1 && h >= 1 && count >= 0);
    DCTE_ARG(ctx, rowstride >= (long long)w * bpp);
    if (count == 0) return DCTE_OK;
    DCTE_ARG(ctx, d_px && d_xy && d_out);
    Device& d = ctx->devs[device];
    hipStream_t s = (hipStream_t)stream;
    DCTE_HIP(ctx, hipSetDevice(d.id));
    FixScratch* f = nullptr;
    int rc = ensure_fix(ctx, d, s, (size_t)count, &f);
    if (rc) return rc;
    const double scale = weight_scale(n, semantics);
    dcte::SeamParams p{};
    p.px = static_cast<const uint8_t*>(d_px);
    p.rowstride = rowstride;
    p.w = w;
    p.h = h;
    p.bpp = bpp;
    p.n = n;
    p.sem = semantics;
    p.in_row0 = 0;
    p.pts = d_xy;
    p.count = count;
    p.map_out = d_out;
    p.we = (float)((double)edges / scale);
    p.wt = (float)((double)textures / scale);
    p.tie_tau = (float)eff_tau(ctx, n);
    p.fix_count = f->d_count;
    p.fix_list = f->d_list;
    p.fix_cap = (unsigned)f->cap;
    DCTE_HIP(ctx, hipMemsetAsync(f->d_count, 0, sizeof(unsigned), s));
    DCTE_HIP(ctx, dcte::launch_points(p, s));
    if ((p.we != p.wt && eff_tau(ctx, n) > 0) || eff_tau(ctx, n) >= 1.0) {
        dcte::FixParams q = fix_params(p.px, rowstride, w, h, 0, bpp, n, 0, semantics, d_out, 0,
                                       edges, textures, f);
        q.pts = d_xy;
        q.max_items = (unsigned)count;
        DCTE_HIP(ctx, dcte::launch_fix(q, s));
    }
    return DCTE_OK;
}

int dcte_energy_points(dcte_ctx* ctx, const uint8_t* px, int w, int h, int bpp, size_t rowstride,
                       const int* xy, int count, int n, float edges, float textures, int semantics,
                       float* out)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, valid_n(n) && valid_sem_bpp(semantics, bpp) && w >= 1 && h >= 1 && count >= 0);
    DCTE_ARG(ctx, rowstride >= (size_t)w * bpp);
    if (count == 0) return DCTE_OK;
    DCTE_ARG(ctx, px && xy && out);
    for (int k = 0; k < count; k++)
        DCTE_ARG(ctx, xy[2 * k] >= 0 && xy[2 * k] < w && xy[2 * k + 1] >= 0 && xy[2 * k + 1] < h);
    ctx->last_refined = 0;
    Device& d = ctx->devs[0];
    int rc = ensure_stream(ctx, d);
    if (rc) return rc;
    // frame rows packed, then the points (4-byte aligned)
    const size_t frame = (size_t)w * bpp * (size_t)h, pts = sizeof(int) * 2 * (size_t)count;
    const size_t pts_off = (frame + 3) & ~(size_t)3;
    rc = ensure_buf(ctx, (void**)&d.d_in, &d.in_cap, pts_off + pts);
    if (rc) return rc;
    rc = ensure_buf(ctx, (void**)&d.d_out, &d.out_cap, sizeof(float) * (size_t)count);
    if (rc) return rc;
    DCTE_HIP(ctx, hipMemcpy2DAsync(d.d_in, (size_t)w * bpp, px, rowstride, (size_t)w * bpp, h,
                                   hipMemcpyHostToDevice, d.stream));
    int* d_xy = reinterpret_cast<int*>(d.d_in + pts_off);
    DCTE_HIP(ctx, hipMemcpyAsync(d_xy, xy, pts, hipMemcpyHostToDevice, d.stream));
    FixScratch* f = nullptr;
    rc = ensure_fix(ctx, d, d.stream, (size_t)count, &f);
    if (rc) return rc;
    DCTE_HIP(ctx, hipMemsetAsync(f->d_count + 1, 0, sizeof(unsigned), d.stream));
    rc = dcte_energy_points_device(ctx, 0, d.d_in, (long long)w * bpp, w, h, bpp, d_xy, count, n,
                                   edges, textures, semantics, d.d_out, d.stream);
    if (rc) return rc;
    DCTE_HIP(ctx, hipMemcpyAsync(out, d.d_out, sizeof(float) * (size_t)count,
                                 hipMemcpyDeviceToHost, d.stream));
    return sync_bands(ctx, 1);
}

int dcte_energy_windows_device(dcte_ctx* ctx, int device, const double* d_win, int count, int n,
                               float edges, float textures, float* d_out, void* stream)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, device >= 0 && device < (int)ctx->devs.size());
    DCTE_ARG(ctx, valid_n(n) && count >= 0);
    if (count == 0) return DCTE_OK;
    DCTE_ARG(ctx, d_win && d_out);
    DCTE_HIP(ctx, hipSetDevice(ctx->devs[device].id));
    dcte::WinParams p{};
    p.win = d_win;
    p.count = count;
    p.n = n;
    small_twiddles(n, p.ct);
    p.edges = edges;
    p.textures = textures;
    p.out = d_out;
    DCTE_HIP(ctx, dcte::launch_windows(p, (hipStream_t)stream));
    return DCTE_OK;
}

int dcte_energy_windows(dcte_ctx* ctx, const double* win, int count, int n, float edges,
                        float textures, float* out)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, valid_n(n) && count >= 0);
    if (count == 0) return DCTE_OK;
    DCTE_ARG(ctx, win && out);
    Device& d = ctx->devs[0];
    int rc = ensure_stream(ctx, d);
    if (rc) return rc;
    const size_t wbytes = sizeof(double) * (size_t)n * n * (size_t)count;
    rc = ensure_buf(ctx, (void**)&d.d_in, &d.in_cap, wbytes);
    if (rc) return rc;
    rc = ensure_buf(ctx, (void**)&d.d_out, &d.out_cap, sizeof(float) * (size_t)count);
    if (rc) return rc;
    DCTE_HIP(ctx, hipMemcpyAsync(d.d_in, win, wbytes, hipMemcpyHostToDevice, d.stream));
    rc = dcte_energy_windows_device(ctx, 0, reinterpret_cast<const double*>(d.d_in), count, n, edges,
                                    textures, d.d_out, d.stream);
    if (rc) {
        drain(ctx, 1);
        return rc;
    }
    DCTE_HIP(ctx, hipMemcpyAsync(out, d.d_out, sizeof(float) * (size_t)count, hipMemcpyDeviceToHost,
                                 d.stream));
    DCTE_HIP(ctx, hipStreamSynchronize(d.stream));
    return DCTE_OK;
}

// A resident-mode seam search that timed out (tiles of the launch were not all
// scheduled: other work held the CUs) switches this stream to one launch per
// band for good; true if that is a change, i.e. worth running again.
static bool dp_fall_back(Device& d, hipStream_t s)
{
    auto it = d.dp.find(s);
    if (it == d.dp.end() || it->second.max_tiles == 0) return false;
    it->second.max_tiles = 0;
    return true;
}

int dcte_seam_find_device(dcte_ctx* ctx, int device, const float* d_map, long long map_stride,
                          int w, int h, int* d_seam, void* stream)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, device >= 0 && device < (int)ctx->devs.size());
    DCTE_ARG(ctx, d_map && d_seam && w >= 1 && h >= 1 && map_stride >= w);
    Device& d = ctx->devs[device];
    hipStream_t s = (hipStream_t)stream;
    DCTE_HIP(ctx, hipSetDevice(d.id));
    const int R = dcte::dp_band_rows(), G = dcte::dp_super_bands(), T = dcte::dp_tile_cols();
    dcte::DpParams p{};
    p.map = d_map;
    p.stride = map_stride;
    p.w = w;
    p.h = h;
    p.nb = h > 1 ? (h - 1 + R - 1) / R : 1;  // bands of R rows from row 1 (row 0 seeds M)
    p.ns = (p.nb + G - 1) / G;
    p.ntiles = (w + T - 1) / T;
    p.pw = (long long)p.ntiles * T;
    DpScratch& sc = d.dp[s];
    if (sc.max_tiles < 0) sc.max_tiles = dcte::dp_max_tiles(d.id);
    // all tiles resident: one launch; otherwise (a frame wider than the chip
    // holds tiles, or DCTE_OPT_DP_BANDWISE) one launch per band of rows
    const bool resident = p.ntiles <= sc.max_tiles && !ctx->dp_bandwise;
    // scratch: jump | sjump | sx | bx | err; xch apart
    const size_t PW = (size_t)p.pw;
    const size_t n_x = (size_t)p.nb * PW, n_jump = (size_t)p.nb * PW, n_sj = (size_t)p.ns * PW;
    const size_t words = n_jump + n_sj + p.ns + p.nb + 1;
    const size_t bytes = words * 4;
    if (sc.cap < bytes) {
        if (sc.buf) DCTE_HIP(ctx, hipFree(sc.buf));
        sc.buf = nullptr;
        sc.cap = 0;
        DCTE_HIP(ctx, hipMalloc(&sc.buf, bytes));
        sc.cap = bytes;
    }
    if (sc.xcap < n_x * 8) {
        if (sc.xbuf) DCTE_HIP(ctx, hipFree(sc.xbuf));
        sc.xbuf = nullptr;
        sc.xcap = 0;
        DCTE_HIP(ctx, hipMalloc(&sc.xbuf, n_x * 8));
        sc.xcap = n_x * 8;
        DCTE_HIP(ctx, hipMemsetAsync(sc.xbuf, 0, sc.xcap, s));
        sc.epoch = 0;
    }
    if (++sc.epoch == 0) {                   // wrapped: clear stale tags
        DCTE_HIP(ctx, hipMemsetAsync(sc.xbuf, 0, sc.xcap, s));
        sc.epoch = 1;
    }
    p.epoch = sc.epoch;
    p.xch = static_cast<unsigned long long*>(sc.xbuf);
    uint32_t* wbase = static_cast<uint32_t*>(sc.buf);
    p.jump = reinterpret_cast<int*>(wbase);
    p.sjump = p.jump + n_jump;
    p.sx = p.sjump + n_sj;
    p.bx = p.sx + p.ns;
    p.err = reinterpret_cast<unsigned*>(p.bx + p.nb);
    p.seam = d_seam;
    p.spin_limit = ctx->dp_spin_limit;
    DCTE_HIP(ctx, hipMemsetAsync(p.err, 0, sizeof(unsigned), s));
    DCTE_HIP(ctx, dcte::launch_seam_find(p, s, resident));
    return DCTE_OK;
}

int dcte_seam_find(dcte_ctx* ctx, const float* map, int w, int h, int* seam)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, map && seam && w >= 1 && h >= 1);
    Device& d = ctx->devs[0];
    int rc = ensure_stream(ctx, d);
    if (rc) return rc;
    const size_t mbytes = sizeof(float) * (size_t)w * (size_t)h;
    rc = ensure_buf(ctx, (void**)&d.d_out, &d.out_cap, mbytes + sizeof(int) * (size_t)h);
    if (rc) return rc;
    int* d_seam = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(d.d_out) + mbytes);
    DCTE_HIP(ctx, hipMemcpyAsync(d.d_out, map, mbytes, hipMemcpyHostToDevice, d.stream));
    rc = dcte_seam_find_device(ctx, 0, d.d_out, w, w, h, d_seam, d.stream);
    if (rc) {
        drain(ctx, 1);
        return rc;
    }
    DCTE_HIP(ctx, hipMemcpyAsync(seam, d_seam, sizeof(int) * (size_t)h, hipMemcpyDeviceToHost,
                                 d.stream));
    DCTE_HIP(ctx, hipStreamSynchronize(d.stream));
    if (h > 0 && seam[0] < 0) {
        if (dp_fall_back(d, d.stream)) return dcte_seam_find(ctx, map, w, h, seam);
        ctx->last_error = "seam search timed out waiting for a neighbour tile";
        return DCTE_EHIP;
    }
    return DCTE_OK;
}

int dcte_carve(dcte_ctx* ctx, const uint8_t* px, int w, int h, int bpp, size_t rowstride, int n,
               float edges, float textures, int semantics, int seams, int transposed,
               uint8_t* out, int* seam_cols)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, px && out && valid_n(n) && valid_sem_bpp(semantics, bpp) && w > 0 && h > 0);
    DCTE_ARG(ctx, rowstride >= (size_t)w * bpp);
    const int W = transposed ? h : w, H = transposed ? w : h;   // the frame that is carved
    DCTE_ARG(ctx, seams >= 0 && seams < W);
    ctx->last_refined = 0;
    Device& d = ctx->devs[0];
    int rc = ensure_stream(ctx, d);
    if (rc) return rc;
    hipStream_t s = d.stream;
    auto align = [](size_t v) { return (v + 255) & ~(size_t)255; };
    // one allocation: carved frame | its map | seams | (transposed) staging frame
    const size_t pitch = (size_t)W * bpp;
    const size_t fbytes = align(pitch * (size_t)H);
    const size_t mbytes = align(sizeof(float) * (size_t)W * (size_t)H);
    const size_t sbytes = sizeof(int) * (size_t)H * (size_t)(seams > 0 ? seams : 1);
    rc = ensure_buf(ctx, (void**)&d.d_in, &d.in_cap,
                    fbytes + mbytes + align(sbytes) + (transposed ? fbytes : 0));
    if (rc) return rc;
    uint8_t* d_px = d.d_in;
    float* d_map = reinterpret_cast<float*>(d.d_in + fbytes);
    int* d_seams = reinterpret_cast<int*>(d.d_in + fbytes + mbytes);
    uint8_t* d_tmp = d.d_in + fbytes + mbytes + align(sbytes);
    FixScratch* f = nullptr;
    rc = ensure_fix(ctx, d, s, (size_t)W * (size_t)H, &f);
    if (rc) return rc;
    DCTE_HIP(ctx, hipMemsetAsync(f->d_count + 1, 0, sizeof(unsigned), s));
    const size_t spitch = (size_t)w * bpp;                       // source row
    if (transposed) {
        DCTE_HIP(ctx, hipMemcpy2DAsync(d_tmp, spitch, px, rowstride, spitch, h,
                                       hipMemcpyHostToDevice, s));
        DCTE_HIP(ctx, dcte::launch_transpose_u8(d_tmp, (long long)spitch, h, w, bpp, d_px,
                                                (long long)pitch, s));
    } else {
        DCTE_HIP(ctx, hipMemcpy2DAsync(d_px, pitch, px, rowstride, pitch, h,
                                       hipMemcpyHostToDevice, s));
    }
    // map, then (seam -> carve in place + energy update) per step, all in HBM
    rc = run_device(ctx, d, d_px, (long long)pitch, W, H, bpp, 0, H, 0, H, n, edges, textures,
                    semantics, d_map, W, s);
    for (int k = 0; rc == DCTE_OK && k < seams; k++) {
        int* sk = d_seams + (size_t)k * H;
        rc = dcte_seam_find_device(ctx, 0, d_map, W, W - k, H, sk, s);
        if (rc == DCTE_OK)
            rc = dcte_seam_carve_device(ctx, 0, d_px, (long long)pitch, W - k, H, bpp, sk, d_map, W,
                                        d_px, (long long)pitch, d_map, W, n, edges, textures,
                                        semantics, s);
    }
    if (rc) {
        drain(ctx, 1);
        return rc;
    }
    // the seams first: a search that timed out is re-run from the caller's px
    // before anything is written to out (which may overlap px)
    std::vector<int> own;
    int* hs = seam_cols;
    if (seams > 0 && !hs) {
        own.resize((size_t)seams * H);
        hs = own.data();
    }
    if (seams > 0) {
        DCTE_HIP(ctx, hipMemcpyAsync(hs, d_seams, sizeof(int) * (size_t)seams * H,
                                     hipMemcpyDeviceToHost, s));
        DCTE_HIP(ctx, hipStreamSynchronize(s));
    }
    for (int k = 0; k < seams; k++)
        if (hs[(size_t)k * H] < 0) {
            if (dp_fall_back(d, s))   // out is untouched: carve again band-wise
                return dcte_carve(ctx, px, w, h, bpp, rowstride, n, edges, textures, semantics,
                                  seams, transposed, out, seam_cols);
            ctx->last_error = "seam search timed out waiting for a neighbour tile";
            return DCTE_EHIP;
        }
    const int Wo = W - seams;
    if (transposed) {   // H x Wo carved frame -> Wo x H = (h - seams) x w
        DCTE_HIP(ctx, dcte::launch_transpose_u8(d_px, (long long)pitch, H, Wo, bpp, d_tmp,
                                                (long long)H * bpp, s));
        DCTE_HIP(ctx, hipMemcpyAsync(out, d_tmp, (size_t)Wo * (size_t)H * bpp,
                                     hipMemcpyDeviceToHost, s));
    } else {
        DCTE_HIP(ctx, hipMemcpy2DAsync(out, (size_t)Wo * bpp, d_px, pitch, (size_t)Wo * bpp, H,
                                       hipMemcpyDeviceToHost, s));
    }
    return sync_bands(ctx, 1);
}

}  // extern "C"

// ---- device mirror of a liblqr carver (the update_emap hook) ----
struct dcte_carver {
    dcte_ctx* ctx = nullptr;
    int W0 = 0, H = 0, w = 0, bpp = 0, n = 0, r = 0, bw = 0;
    float edges = 0, textures = 0;
    bool exact = false;        // DCTE_OPT_EXACT when the carver was created
    double tie_tau = 0;        // DCTE_OPT_TIE_TAU likewise
    size_t pitch = 0;
    uint8_t* d_px = nullptr;   // carved frame (row pitch W0 * bpp)
    float* d_map = nullptr;    // its energies (row pitch W0)
    int* d_seam = nullptr;     // H
    int* d_x0 = nullptr;       // H
    float* d_be = nullptr;     // H x bw
    uint8_t* d_bpx = nullptr;  // H x bw x bpp
    std::vector<int> seam;     // host copy of the last seam
};

namespace {

void carver_free(dcte_carver* c)
{
    if (!c) return;
    if (!c->ctx->devs.empty() && hipSetDevice(c->ctx->devs[0].id) == hipSuccess) {
        if (c->ctx->devs[0].stream) (void)hipStreamSynchronize(c->ctx->devs[0].stream);
        for (void* p : {(void*)c->d_px, (void*)c->d_map, (void*)c->d_seam, (void*)c->d_x0,
                        (void*)c->d_be, (void*)c->d_bpx})
            if (p) (void)hipFree(p);
    }
    delete c;
}

}  // namespace

extern "C" {

int dcte_carver_create2(dcte_ctx* ctx, const uint8_t* px, int w, int h, int bpp, size_t rowstride,
                        int n, float edges, float textures, int transposed, float* map_out,
                        float* map_other_out, dcte_carver** out)
{
    DeviceGuard guard_;
    if (!ctx || !out) return DCTE_EINVAL;
    *out = nullptr;
    DCTE_ARG(ctx, px && valid_n(n) && valid_sem_bpp(DCTE_LQR, bpp) && w > 0 && h > 0);
    DCTE_ARG(ctx, rowstride >= (size_t)w * bpp);
    Device& d = ctx->devs[0];
    int rc = ensure_stream(ctx, d);
    if (rc) return rc;
    hipStream_t s = d.stream;
    dcte_carver* c = new (std::nothrow) dcte_carver;
    if (!c) return DCTE_ENOMEM;
    c->ctx = ctx;
    c->W0 = transposed ? h : w;
    c->H = transposed ? w : h;
    c->w = c->W0;
    c->bpp = bpp;
    c->n = n;
    c->r = n / 2;                    // the radius the plug-in registers (src/render.c:314-315)
    c->bw = 8 * c->r + 4;            // reading windows of the update band too (dcte_band_gather)
    c->edges = edges;
    c->textures = textures;
    c->exact = ctx->exact;           // the carver keeps this mode for every step
    c->tie_tau = ctx->tie_tau;
    c->pitch = (size_t)c->W0 * bpp;
    c->seam.assign(c->H, 0);
    const size_t fbytes = c->pitch * (size_t)c->H;
    const size_t mbytes = sizeof(float) * (size_t)w * (size_t)h;
    uint8_t* d_tmp = nullptr;        // the other orientation's frame
    float* d_other = nullptr;        // its map
    auto release_tmp = [&]() {
        if (d_tmp || d_other) (void)hipStreamSynchronize(s);
        if (d_tmp) (void)hipFree(d_tmp);
        if (d_other) (void)hipFree(d_other);
        d_tmp = nullptr;
        d_other = nullptr;
    };
    auto fail = [&](hipError_t e, const char* where) {
        int code = hip_fail(ctx, e, where);
        release_tmp();
        carver_free(c);
        return code;
    };
    hipError_t e;
    if ((e = hipMalloc(&c->d_px, fbytes)) != hipSuccess) return fail(e, "hipMalloc frame");
    if ((e = hipMalloc(&c->d_map, mbytes)) != hipSuccess) return fail(e, "hipMalloc map");
    if ((e = hipMalloc(&c->d_seam, sizeof(int) * (size_t)c->H)) != hipSuccess) return fail(e, "hipMalloc seam");
    if ((e = hipMalloc(&c->d_x0, sizeof(int) * (size_t)c->H)) != hipSuccess) return fail(e, "hipMalloc x0");
    if ((e = hipMalloc(&c->d_be, sizeof(float) * (size_t)c->H * c->bw)) != hipSuccess) return fail(e, "hipMalloc band");
    if ((e = hipMalloc(&c->d_bpx, (size_t)c->H * c->bw * bpp)) != hipSuccess) return fail(e, "hipMalloc band px");
    const size_t spitch = (size_t)w * bpp;
    if (transposed || map_other_out)
        if ((e = hipMalloc(&d_tmp, fbytes)) != hipSuccess) return fail(e, "hipMalloc staging");
    if (map_other_out && (e = hipMalloc(&d_other, mbytes)) != hipSuccess) return fail(e, "hipMalloc other map");
    // one upload: the frame as given, or (transposed) into the staging buffer
    // and transposed from there; the other orientation is the staging frame
    // (transposed) or the frame transposed into it
    if (transposed) {
        e = hipMemcpy2DAsync(d_tmp, spitch, px, rowstride, spitch, h, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = dcte::launch_transpose_u8(d_tmp, (long long)spitch, h, w, bpp, c->d_px, (long long)c->pitch, s);
        if (e != hipSuccess) return fail(e, "upload (transposed)");
    } else {
        e = hipMemcpy2DAsync(c->d_px, c->pitch, px, rowstride, spitch, h, hipMemcpyHostToDevice, s);
        if (e == hipSuccess && map_other_out)
            e = dcte::launch_transpose_u8(c->d_px, (long long)c->pitch, h, w, bpp, d_tmp, (long long)h * bpp, s);
        if (e != hipSuccess) return fail(e, "upload");
    }
    rc = run_device(ctx, d, c->d_px, (long long)c->pitch, c->W0, c->H, bpp, 0, c->H, 0, c->H, n,
                    edges, textures, DCTE_LQR, c->d_map, c->W0, s);
    if (rc == DCTE_OK && map_out &&
        (e = hipMemcpyAsync(map_out, c->d_map, mbytes, hipMemcpyDeviceToHost, s)) != hipSuccess)
        rc = hip_fail(ctx, e, "map download");
    if (rc == DCTE_OK && map_other_out) {
        const int ow = c->H, oh = c->W0;      // the other orientation's frame: ow x oh
        rc = run_device(ctx, d, d_tmp, (long long)ow * bpp, ow, oh, bpp, 0, oh, 0, oh, n, edges,
                        textures, DCTE_LQR, d_other, ow, s);
        if (rc == DCTE_OK &&
            (e = hipMemcpyAsync(map_other_out, d_other, mbytes, hipMemcpyDeviceToHost, s)) != hipSuccess)
            rc = hip_fail(ctx, e, "other map download");
    }
    if (rc == DCTE_OK && (e = hipStreamSynchronize(s)) != hipSuccess) rc = hip_fail(ctx, e, "sync");
    release_tmp();
    if (rc) {
        carver_free(c);
        return rc;
    }
    *out = c;
    return DCTE_OK;
}

int dcte_carver_create(dcte_ctx* ctx, const uint8_t* px, int w, int h, int bpp, size_t rowstride,
                       int n, float edges, float textures, int transposed, float* map_out,
                       dcte_carver** out)
{
    return dcte_carver_create2(ctx, px, w, h, bpp, rowstride, n, edges, textures, transposed,
                               map_out, nullptr, out);
}

int dcte_carver_width(const dcte_carver* c) { return c ? c->w : 0; }
int dcte_carver_height(const dcte_carver* c) { return c ? c->H : 0; }
int dcte_carver_band_width(const dcte_carver* c) { return c ? c->bw : 0; }

int dcte_carver_step(dcte_carver* c, int* seam, int* band_x0, float* band_e, uint8_t* band_px)
{
    DeviceGuard guard_;
    if (!c) return DCTE_EINVAL;
    dcte_ctx* ctx = c->ctx;
    DCTE_ARG(ctx, c->w >= 2);
    Device& d = ctx->devs[0];
    int rc = ensure_stream(ctx, d);
    if (rc) return rc;
    hipStream_t s = d.stream;
    ModeScope mode(ctx, c->exact, c->tie_tau);   // the carver's mode, not the context's now
    // the seam first, checked on the host before anything moves (a search
    // that timed out is re-run band-wise, as dcte_seam_find does)
    for (;;) {
        rc = dcte_seam_find_device(ctx, 0, c->d_map, c->W0, c->w, c->H, c->d_seam, s);
        if (rc) return rc;
        DCTE_HIP(ctx, hipMemcpyAsync(c->seam.data(), c->d_seam, sizeof(int) * (size_t)c->H,
                                     hipMemcpyDeviceToHost, s));
        DCTE_HIP(ctx, hipStreamSynchronize(s));
        if (c->seam[0] >= 0) break;
        if (!dp_fall_back(d, s)) {
            ctx->last_error = "seam search timed out waiting for a neighbour tile";
            return DCTE_EHIP;
        }
    }
    rc = dcte_seam_carve_device(ctx, 0, c->d_px, (long long)c->pitch, c->w, c->H, c->bpp, c->d_seam,
                                c->d_map, c->W0, c->d_px, (long long)c->pitch, c->d_map, c->W0,
                                c->n, c->edges, c->textures, DCTE_LQR, s);
    if (rc) {
        drain(ctx, 1);
        return rc;
    }
    c->w--;
    dcte::BandParams b{};
    b.seam = c->d_seam;
    b.w = c->w;
    b.h = c->H;
    b.r = c->r;
    b.bw = c->bw;
    b.bpp = c->bpp;
    b.map = c->d_map;
    b.map_stride = c->W0;
    b.px = c->d_px;
    b.rowstride = (long long)c->pitch;
    b.x0 = c->d_x0;
    b.e = c->d_be;
    b.pxb = c->d_bpx;
    DCTE_HIP(ctx, dcte::launch_band_gather(b, s));
    if (seam) memcpy(seam, c->seam.data(), sizeof(int) * (size_t)c->H);
    if (band_x0)
        DCTE_HIP(ctx, hipMemcpyAsync(band_x0, c->d_x0, sizeof(int) * (size_t)c->H, hipMemcpyDeviceToHost, s));
    if (band_e)
        DCTE_HIP(ctx, hipMemcpyAsync(band_e, c->d_be, sizeof(float) * (size_t)c->H * c->bw,
                                     hipMemcpyDeviceToHost, s));
    if (band_px)
        DCTE_HIP(ctx, hipMemcpyAsync(band_px, c->d_bpx, (size_t)c->H * c->bw * c->bpp,
                                     hipMemcpyDeviceToHost, s));
    DCTE_HIP(ctx, hipStreamSynchronize(s));
    return DCTE_OK;
}

void dcte_carver_destroy(dcte_carver* c)
{
    DeviceGuard guard_;
    carver_free(c);
}

int dcte_energy_map(dcte_ctx* ctx, const uint8_t* px, int w, int h, int bpp, size_t rowstride,
                    int n, float edges, float textures, int semantics, int transposed, float* out)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, px && out && valid_n(n) && valid_sem_bpp(semantics, bpp) && w > 0 && h > 0);
    DCTE_ARG(ctx, rowstride >= (size_t)w * bpp);
    ctx->last_refined = 0;
    const bool one = ctx->devs.size() == 1;
    HostPin pin_in(ctx, px, (size_t)(h - 1) * rowstride + (size_t)w * bpp, false, 0, false);
    HostPin pin_out(ctx, out, sizeof(float) * (size_t)w * (size_t)h, one && ctx->d2h_kernel, 1, true);
    int G = 0;
    int rc;
    if (transposed && one) {   // chunked: the map's download overlaps its launches
        G = 1;
        rc = map_pipeline_one(ctx, px, w, h, bpp, rowstride, n, edges, textures, semantics, nullptr, out,
                              &pin_in, nullptr, &pin_out);
    } else {
        rc = map_bands(ctx, px, w, h, bpp, rowstride, n, edges, textures, semantics, transposed, out, &G,
                       &pin_in, &pin_out);
    }
    if (rc) {
        drain(ctx, G);              // nothing in flight may still use px / out
        return rc;
    }
    rc = sync_bands(ctx, G);
    if (rc == DCTE_OK) pin_out.commit();
    return rc;
}

int dcte_energy_map2(dcte_ctx* ctx, const uint8_t* px, int w, int h, int bpp, size_t rowstride,
                     int n, float edges, float textures, int semantics, float* out, float* out_t)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, px && (out || out_t) && valid_n(n) && valid_sem_bpp(semantics, bpp) && w > 0 && h > 0);
    DCTE_ARG(ctx, rowstride >= (size_t)w * bpp);
    if (ctx->devs.size() > 1) {     // row bands per device: one call per orientation
        int rc = out ? dcte_energy_map(ctx, px, w, h, bpp, rowstride, n, edges, textures, semantics, 0, out)
                     : DCTE_OK;
        long long refined = ctx->last_refined;
        if (rc == DCTE_OK && out_t)
            rc = dcte_energy_map(ctx, px, w, h, bpp, rowstride, n, edges, textures, semantics, 1, out_t);
        ctx->last_refined += refined;
        return rc;
    }
    ctx->last_refined = 0;
    HostPin pin_in(ctx, px, (size_t)(h - 1) * rowstride + (size_t)w * bpp, false, 0, false);
    HostPin pin_out(ctx, out, out ? sizeof(float) * (size_t)w * (size_t)h : 0, ctx->d2h_kernel, 1, true);
    HostPin pin_out_t(ctx, out_t, out_t ? sizeof(float) * (size_t)w * (size_t)h : 0, ctx->d2h_kernel, 2, true);
    int rc = map_pipeline_one(ctx, px, w, h, bpp, rowstride, n, edges, textures, semantics, out, out_t,
                              &pin_in, &pin_out, &pin_out_t);
    if (rc) {
        drain(ctx, 1);              // nothing in flight may still use px / out / out_t
        return rc;
    }
    rc = sync_bands(ctx, 1);
    if (rc == DCTE_OK) {
        pin_out.commit();
        pin_out_t.commit();
    }
    return rc;
}

int dcte_energy_image_u8(dcte_ctx* ctx, const uint8_t* px, int w, int h, int bpp,
                         size_t rowstride, int n, float edges, float textures, int semantics,
                         int mode, int channels, uint8_t* out)
{
    DeviceGuard guard_;
    if (!ctx) return DCTE_EINVAL;
    DCTE_ARG(ctx, px && out && valid_n(n) && valid_sem_bpp(semantics, bpp) && w > 0 && h > 0);
    DCTE_ARG(ctx, rowstride >= (size_t)w * bpp && valid_norm(mode, channels));
    ctx->last_refined = 0;
    int G = 0;
    HostPin pin_in(ctx, px, (size_t)(h - 1) * rowstride + (size_t)w * bpp, false, 0, false);
    HostPin pin_out(ctx, out, (size_t)w * (size_t)h * (size_t)channels,
                    ctx->devs.size() == 1 && ctx->d2h_kernel, 1, true);
    int rc = map_bands(ctx, px, w, h, bpp, rowstride, n, edges, textures, semantics, 0, nullptr,
                       &G, &pin_in);
    if (rc == DCTE_OK) rc = normalize_bands(ctx, w, h, mode, channels, out, G, &pin_out);
    if (rc) {
        drain(ctx, G);              // nothing in flight may still use px / out
        return rc;
    }
    rc = sync_bands(ctx, G);
    if (rc == DCTE_OK) pin_out.commit();
    return rc;
}

}  // extern "C"

namespace {

// energy_image_u8, second half: global min/max over the band maps, then u8
int normalize_bands(dcte_ctx* ctx, int w, int h, int mode, int channels, uint8_t* out, int G,
                    const HostPin* pin_out)
{
    int rc;
    // per-band min/max, reduced on the host (2 floats per device)
    float gmin = 0, gmax = 0;
    for (int k = 0; k < G; k++) {
        Device& d = ctx->devs[k];
        int y0 = (int)((long long)h * k / G), y1 = (int)((long long)h * (k + 1) / G);
        DCTE_HIP(ctx, hipSetDevice(d.id));
        DCTE_HIP(ctx, dcte::launch_minmax(d.d_out, (long long)w * (y1 - y0), d.d_keys, d.d_minmax, d.stream));
        float mm[2];
        DCTE_HIP(ctx, hipMemcpyAsync(mm, d.d_minmax, sizeof(mm), hipMemcpyDeviceToHost, d.stream));
        DCTE_HIP(ctx, hipStreamSynchronize(d.stream));
        gmin = k == 0 ? mm[0] : (mm[0] < gmin ? mm[0] : gmin);
        gmax = k == 0 ? mm[1] : (mm[1] > gmax ? mm[1] : gmax);
    }
    for (int k = 0; k < G; k++) {
        Device& d = ctx->devs[k];
        int y0 = (int)((long long)h * k / G), y1 = (int)((long long)h * (k + 1) / G);
        size_t npx = (size_t)w * (size_t)(y1 - y0);
        DCTE_HIP(ctx, hipSetDevice(d.id));
        float mm[2] = {gmin, gmax};
        DCTE_HIP(ctx, hipMemcpyAsync(d.d_minmax, mm, sizeof(mm), hipMemcpyHostToDevice, d.stream));
        rc = ensure_buf(ctx, (void**)&d.d_u8, &d.u8_cap, npx * channels);
        if (rc) return rc;
        DCTE_HIP(ctx, dcte::launch_to_u8(d.d_out, (long long)npx, d.d_minmax, mode, channels, d.d_u8, d.stream));
        DCTE_HIP(ctx, download(pin_out, out + (size_t)y0 * w * channels, d.d_u8, npx * channels, d.stream));
    }
    return DCTE_OK;
}

}  // namespace

extern "C" {

int dcte_normalize_u8(dcte_ctx* ctx, const float* E, size_t n, int mode, int channels, uint8_t* out)
{
    DeviceGuard guard_;
    if (!ctx || !E || !out || n == 0 || !valid_norm(mode, channels)) return DCTE_EINVAL;
    Device& d = ctx->devs[0];
    int rc = ensure_stream(ctx, d);
    if (rc) return rc;
    rc = ensure_buf(ctx, (void**)&d.d_out, &d.out_cap, n * sizeof(float));
    if (rc) return rc;
    rc = ensure_buf(ctx, (void**)&d.d_u8, &d.u8_cap, n * channels);
    if (rc) return rc;
    DCTE_HIP(ctx, hipMemcpyAsync(d.d_out, E, n * sizeof(float), hipMemcpyHostToDevice, d.stream));
    DCTE_HIP(ctx, dcte::launch_minmax(d.d_out, (long long)n, d.d_keys, d.d_minmax, d.stream));
    DCTE_HIP(ctx, dcte::launch_to_u8(d.d_out, (long long)n, d.d_minmax, mode, channels, d.d_u8, d.stream));
    DCTE_HIP(ctx, hipMemcpyAsync(out, d.d_u8, n * channels, hipMemcpyDeviceToHost, d.stream));
    DCTE_HIP(ctx, hipStreamSynchronize(d.stream));
    return DCTE_OK;
}

int dcte_minmax_device(dcte_ctx* ctx, int device, const float* d_E, long long n, float* d_minmax,
                       void* stream)
{
    DeviceGuard guard_;
    if (!ctx || device < 0 || device >= (int)ctx->devs.size() || !d_E || !d_minmax || n <= 0)
        return DCTE_EINVAL;
    Device& d = ctx->devs[device];
    int rc = ensure_stream(ctx, d);
    if (rc) return rc;
    // per-stream key scratch would be needed for concurrent calls on several
    // streams of one device; min/max calls are stream-ordered per device
    DCTE_HIP(ctx, dcte::launch_minmax(d_E, n, d.d_keys, d_minmax, (hipStream_t)stream));
    return DCTE_OK;
}

int dcte_normalize_u8_device(dcte_ctx* ctx, int device, const float* d_E, long long n,
                             const float* d_minmax, int mode, int channels, uint8_t* d_out,
                             void* stream)
{
    DeviceGuard guard_;
    if (!ctx || device < 0 || device >= (int)ctx->devs.size() || !d_E || !d_minmax || !d_out ||
        n <= 0 || !valid_norm(mode, channels))
        return DCTE_EINVAL;
    DCTE_HIP(ctx, hipSetDevice(ctx->devs[device].id));
    DCTE_HIP(ctx, dcte::launch_to_u8(d_E, n, d_minmax, mode, channels, d_out, (hipStream_t)stream));
    return DCTE_OK;
}

int dcte_profile_read(dcte_ctx* ctx, long long* launches, double* kernel_ms)
{
    DeviceGuard guard_;
    if (!ctx || !launches || !kernel_ms) return DCTE_EINVAL;
    double total = 0.0;
    int rc = DCTE_OK;
    for (ProfEvent& ev : ctx->prof) {
        if (rc == DCTE_OK) {
            float ms = 0.0f;
            hipError_t e = hipSetDevice(ev.dev);
            if (e == hipSuccess) e = hipEventSynchronize(ev.b);
            if (e == hipSuccess) e = hipEventElapsedTime(&ms, ev.a, ev.b);
            if (e != hipSuccess) rc = hip_fail(ctx, e, "dcte_profile_read");
            total += ms;
        }
        (void)hipEventDestroy(ev.a);
        (void)hipEventDestroy(ev.b);
    }
    *launches = (long long)ctx->prof.size();
    *kernel_ms = total;
    ctx->prof.clear();
    return rc;
}

// ---- context-free CPU entries --------------------------------
// The per-window callback body for a caller that keeps its own reading
// windows on the CPU (a carver after seams shrank it): dctNxN
// (src/dct.c:77-94) + weighted_max_dct_correlation (src/dct.c:96-110) in
// fp64 in the reference's operation order (dcte_ref64.h, the same functions
// the device refinement runs).  No device, no context, no fallback role:
// the GPU entry points never call these.
long long dcte_last_refined(const dcte_ctx* ctx) { return ctx ? ctx->last_refined : 0; }

const char* dcte_strerror(int code)
{
    switch (code) {
    case DCTE_OK: return "success";
    case DCTE_EINVAL: return "invalid argument";
    case DCTE_ENODEV: return "no HIP device";
    case DCTE_ENOMEM: return "out of memory";
    case DCTE_EHIP: return "HIP runtime error";
    case DCTE_ERANGE: return "frame too large for one launch";
    case DCTE_ENOTSUP: return "not supported by this build";
    default: return "unknown error";
    }
}

const char* dcte_last_error(const dcte_ctx* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

}  // extern "C"
