"""Bench: DCT energy map of a 16384^2 RGB frame, N = 8 (BASELINE.json configs[2..3]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 8] [--size 16384] [--weak]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU.  With --gpus N > 1 and no launcher around it (WORLD_SIZE
unset), bench.py starts its N rank processes itself before anything touches a
GPU, then exits with their status.

A "step" is one pass of the hot path over the frame: every rank maps its row
band of ONE size x size frame (strong scaling, BASELINE configs[3]) -- the
halo rows exchanged with the neighbour ranks (RCCL point-to-point over xGMI)
while the interior rows run, then the halo-dependent rows.  Input resident in
HBM, output left in HBM.  --weak gives every rank its own size x size band of
a (N * size) x size frame instead.

Prints ONE JSON line (rank 0).  `value` = Mpx/s over all ranks.  `roofline`
prices the map kernel (dcte_map<N,RGB>) against the 8 TB/s HBM roof with the
algorithmic 7 B/px (3 B in + 4 B out), timed by HIP events around each launch
on the launch stream (dcte_profile_read); the binding roof is the VALU,
reported in `valu`.  `cpu_baseline` times the reference's own transforms
(oracle/_ref, src/fft2d compiled unmodified) on this host's cores over a
bounded sample of the frame; `host_path` times the plug-in's real call
(host frame -> dcte_energy_map -> host map, PCIe-inclusive).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

METRIC = "Mpixels/sec DCT-energy-map on 16384² RGB; % MI355X HBM roofline at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0
# gfx950: 256 CU x 4 SIMD, a wave64 VALU instruction every 2 cycles per SIMD
VALU_PEAK_LANE_OPS = 256 * 4 * 64 / 2 * 2.4e9


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--edges", type=float, default=0.3)
    ap.add_argument("--textures", type=float, default=0.7)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=0,
                    help="output rows of the CPU-baseline sample (0: sized to ~15 s of CPU work)")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--no-stress", action="store_true",
                    help="skip the tie-dense (line-art) frame timed after the headline")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the configs[1] / configs[4] timings after the headline")
    ap.add_argument("--no-exact", action="store_true",
                    help="skip the DCTE_OPT_EXACT (bit-identical fp64) map timed after the headline")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: stage halos through host memory (rehearsal of the N>1 path "
                         "on a box with fewer GPUs than ranks)")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling: every rank owns its own size x size band of a "
                         "(N * size) x size frame")
    ap.add_argument("--check", action="store_true",
                    help="after timing, recompute every band from regenerated rows (no "
                         "exchange) and require bit-equality (default on for --gpus > 1)")
    ap.add_argument("--no-check", action="store_true", help="skip that check for --gpus > 1")
    ap.add_argument("--no-e2e", action="store_true",
                    help="--gpus > 1: skip the end-to-end figure (step + band gather to rank 0)")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="RCCL rehearsal on a box with fewer GPUs than ranks: the self-launched "
                         "ranks get distinct NCCL_HOSTIDs so RCCL accepts several ranks on one "
                         "device (halos then travel over its socket transport on loopback "
                         "instead of xGMI; the RCCL code path itself is the one measured runs use)")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="no GPU: launch the ranks, split a --size frame into bands and "
                         "exchange the halos over gloo on CPU tensors, check them against "
                         "the global frame (tests/test_bench_launch.py)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher
def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(r, n, port, shared_gpu=False):
    """Environment of rank r of n.  shared_gpu: RCCL refuses two ranks on one
    device of one host ("Duplicate GPU detected"); a distinct NCCL_HOSTID per
    rank makes each rank its own host, so RCCL connects them through its net
    transport (sockets on loopback, no InfiniBand)."""
    env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
               LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if shared_gpu:
        env.update(NCCL_HOSTID=f"dcte-rehearsal-rank{r}", NCCL_SOCKET_IFNAME="lo",
                   NCCL_IB_DISABLE="1")
    return env


def launch_ranks(n, argv, shared_gpu=False):
    """Start n rank processes of this script (RANK/LOCAL_RANK/WORLD_SIZE and a
    127.0.0.1 rendezvous in their environment) and wait for them.  Runs before
    this process touches a GPU; children are started, never exec'd into.
    Returns the first non-zero exit status (the others are then stopped)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = rank_env(r, n, port, shared_gpu)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc if rc >= 0 else 128 - rc


# ------------------------------------------------------------------ baselines
def cpu_threads():
    """Host threads this process may use: the CPUs it is allowed to run on,
    capped by OMP_NUM_THREADS when the environment sets it (the GPU box gives
    one GPU's job a 16-CPU share of the host)."""
    allowed = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(allowed, int(env))) if env and env.isdigit() else max(1, allowed)


def cpu_baseline(frame_rows_host, W, n, e, t, sample_rows):
    """The reference path on the host cores over the first `sample_rows`
    output rows of the bench frame: the reference's own transforms
    (oracle/_ref = src/fft2d compiled unmodified + the restated dct.c /
    render.c glue, OpenMP over rows), and the port (oracle/dcte_oracle.c,
    bit-identical to them) beside it."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    threads = cpu_threads()
    img = frame_rows_host
    res = None
    if O.ref_available():
        L = np.ascontiguousarray(O.luma_plane(img))          # liblqr's rcache: luma once
        t0 = time.perf_counter()
        O.ref_energy_map_luma_rows(L, n, e, t, y0=0, y1=sample_rows, h=L.shape[0],
                                   nthreads=threads)
        dt = time.perf_counter() - t0
        res = {"value": round(sample_rows * W / dt / 1e6, 3), "unit": "Mpx/s", "cores": threads,
               "kind": "reference",
               "sample": f"output rows 0..{sample_rows - 1} x {W} cols of the bench frame "
                         f"(N={n}, e={e}, t={t}): the reference's own src/fft2d transforms "
                         f"(oracle/_ref) per pixel in liblqr build order, luma precomputed, "
                         f"OpenMP over rows on {threads} threads, {dt:.2f} s wall = "
                         f"{dt * threads:.1f} thread-s"}
        # the reference as it runs in the plug-in: one thread (liblqr calls
        # the callback serially, src/render.c:314-315)
        rows1 = min(64, sample_rows)
        t0 = time.perf_counter()
        O.ref_energy_map_luma_rows(L, n, e, t, y0=0, y1=rows1, h=L.shape[0], nthreads=1)
        d1 = time.perf_counter() - t0
        res["single_thread"] = {"value": round(rows1 * W / d1 / 1e6, 3), "unit": "Mpx/s",
                                "cores": 1, "sample": f"output rows 0..{rows1 - 1}, {d1:.2f} s"}
    t0 = time.perf_counter()
    O.energy_map(img, n, e, t, y0=0, y1=sample_rows, nthreads=threads)
    dp = time.perf_counter() - t0
    port = {"value": round(sample_rows * W / dp / 1e6, 3), "unit": "Mpx/s", "cores": threads,
            "kind": "port",
            "sample": f"same rows; oracle/dcte_oracle.c (bit-identical restatement incl. the "
                      f"luma), {dp:.2f} s wall"}
    if res is None:
        res = port
    else:
        res["port"] = port
    res["host_cpus"] = os.cpu_count()
    res["cpus_allowed"] = (len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
                           else os.cpu_count())
    return res


def link_floor(px_pin, d_px, downs, dev, iters):
    """-> (floor_s, up_s, down_s, both_s): median times of the frame's H2D
    alone, the maps' D2H alone and both at once on two streams, pinned
    buffers.  floor = max(up, down): no call can move these bytes faster,
    whatever engines it uses (r06: on some boxes the runtime serialises an
    SDMA upload with an SDMA download, so `both` is not a floor -- the library
    downloads through a copy kernel and beats it)."""
    import torch
    s_up, s_down = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def med(up, down):
        ts = []
        for _ in range(iters + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if up:
                with torch.cuda.stream(s_up):
                    d_px.copy_(px_pin, non_blocking=True)
            if down:
                with torch.cuda.stream(s_down):
                    for dst, src in downs:
                        dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts = sorted(ts[1:])
        return ts[len(ts) // 2]

    up, down, both = med(True, False), med(False, True), med(True, True)
    return max(up, down), up, down, both


def host_path(ctx, frame_dev, n, e, t, iters=3):
    """The plug-in's own call: a pageable host frame (GIMP's rgb buffer,
    src/render.c:159-173) -> dcte_energy_map -> a pageable host map; the library
    page-locks both for the call and pipelines H2D / map / D2H in row chunks."""
    import numpy as np
    px = frame_dev.cpu().numpy()
    H, W = px.shape[:2]
    out = np.empty((H, W), np.float32)
    ctx.energy_map(px, n, e, t, out=out)
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        ctx.energy_map(px, n, e, t, out=out)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    med = ts[len(ts) // 2]
    # the floor: each direction alone from pinned buffers, full duplex assumed
    import torch
    px_pin = torch.empty(tuple(px.shape), dtype=torch.uint8, pin_memory=True)
    out_pin = torch.empty((H, W), dtype=torch.float32, pin_memory=True)
    d_px = torch.empty(tuple(px.shape), dtype=torch.uint8, device=frame_dev.device)
    d_out = torch.empty((H, W), dtype=torch.float32, device=frame_dev.device)
    floor, up, down, both = link_floor(px_pin, d_px, [(out_pin, d_out)], frame_dev.device, iters)
    del px_pin, out_pin, d_px, d_out
    return {"value": round(H * W / med / 1e9, 2), "unit": "Gpx/s", "ms": round(med * 1e3, 2),
            "best_ms": round(ts[0] * 1e3, 2), "iters": iters,
            "bytes_h2d": int(px.nbytes), "bytes_d2h": int(out.nbytes),
            "duplex_floor_ms": round(floor * 1e3, 2), "frac_of_floor": round(floor / med, 3),
            "h2d_alone_ms": round(up * 1e3, 2), "d2h_alone_ms": round(down * 1e3, 2),
            "sdma_both_ms": round(both * 1e3, 2),
            "what": f"{H}x{W} RGB pageable host frame -> dcte_energy_map -> host map "
                    f"(PCIe-inclusive; page-locked per call, chunk pipeline); floor = max(the frame's "
                    f"H2D alone, the map's D2H alone) from pinned buffers; sdma_both = both copies at "
                    f"once on two streams (torch, copy engines)"}


def host_path_vertical(ctx, frame_dev, n, e, t, iters=3):
    """The plug-in's build for a VERTICAL resize (vals->vertically,
    src/render.c:358-364, src/main.h:21): both orientations' maps of the
    pageable host frame -- dcte_energy_map2, one upload, the transposed map
    chunked so its download overlaps the launches.  Floor = the frame's H2D
    and the two maps' D2H at once on two streams from pinned buffers."""
    import numpy as np
    import torch
    px = frame_dev.cpu().numpy()
    H, W = px.shape[:2]
    out = np.empty((H, W), np.float32)
    out_t = np.empty((W, H), np.float32)
    ctx.energy_map2(px, n, e, t, out=out, out_t=out_t)
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        ctx.energy_map2(px, n, e, t, out=out, out_t=out_t)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    med = ts[len(ts) // 2]
    # the two separate calls the glue made before (r05), for comparison
    t0 = time.perf_counter()
    ctx.energy_map(px, n, e, t, out=out)
    ctx.energy_map(px, n, e, t, transposed=True, out=out_t)
    two_calls = time.perf_counter() - t0
    px_pin = torch.empty(tuple(px.shape), dtype=torch.uint8, pin_memory=True)
    out_pin = torch.empty((H, W), dtype=torch.float32, pin_memory=True)
    out_pin2 = torch.empty((W, H), dtype=torch.float32, pin_memory=True)
    d_px = torch.empty(tuple(px.shape), dtype=torch.uint8, device=frame_dev.device)
    d_out = torch.empty((H, W), dtype=torch.float32, device=frame_dev.device)
    floor, up, down, both = link_floor(px_pin, d_px, [(out_pin, d_out), (out_pin2.view(H, W), d_out)],
                                       frame_dev.device, iters)
    del px_pin, out_pin, out_pin2, d_px, d_out
    return {"value": round(H * W / med / 1e9, 2), "unit": "Gpx/s (frame pixels, both maps)",
            "ms": round(med * 1e3, 2), "best_ms": round(ts[0] * 1e3, 2), "iters": iters,
            "two_calls_ms": round(two_calls * 1e3, 2),
            "bytes_h2d": int(px.nbytes), "bytes_d2h": int(2 * out.nbytes),
            "duplex_floor_ms": round(floor * 1e3, 2), "ratio_to_floor": round(med / floor, 3),
            "h2d_alone_ms": round(up * 1e3, 2), "d2h_alone_ms": round(down * 1e3, 2),
            "sdma_both_ms": round(both * 1e3, 2),
            "what": f"{H}x{W} RGB pageable host frame -> dcte_energy_map2 -> both maps on the host "
                    f"(one upload; PCIe-inclusive); floor = max(one H2D alone, two D2H alone) from "
                    f"pinned buffers; sdma_both = all three copies at once on two streams (torch); "
                    f"two_calls = the r05 glue's two dcte_energy_map calls"}


def time_calls(ctx, call, st, iters, rounds):
    """-> (call_ms, map_ms, call_ms_with_events): the stream time per call in
    rounds WITHOUT the profiling events (r06: the two events DCTE_OPT_PROFILE
    records around each map launch cost a 4096^2 call ~6 us of its ~0.1 ms,
    which r05 counted as refinement), the map launches alone from rounds WITH
    them (HIP events around each), and those rounds' call time; best of
    `rounds` interleaved rounds of `iters` calls each."""
    import torch
    import dctenergy
    best_call, best_map, best_ev = 1e9, 1e9, 1e9
    for _ in range(rounds):
        for prof in (0, 1):
            ctx.profile_read()
            ctx.set_option(dctenergy.DCTE_OPT_PROFILE, prof)
            a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a0.record(st)
            for _ in range(iters):
                call()
            a1.record(st)
            torch.cuda.synchronize()
            ctx.set_option(dctenergy.DCTE_OPT_PROFILE, 0)
            launches, kms = ctx.profile_read()
            ms = a0.elapsed_time(a1) / iters
            if prof:
                best_ev = min(best_ev, ms)
                best_map = min(best_map, kms / max(1, launches))
            else:
                best_call = min(best_call, ms)
    return best_call, best_map, best_ev


def stress(ctx, n, S, e, t, dev, stream, iters=10, rounds=3):
    """The worst realistic frame for the fp64 tie refinement, timed like the
    headline after it: line-art RGB (black lines on white every 23 rows, every
    31 columns and along x + 2y = 0 mod 97, tools/fix_study.py's "lineart_rgb").
    Its edge/texture ties are exact in real arithmetic (src/dct.c:100-109), so
    the reference's rounding decides them and ~2.7 % of the pixels go through
    the fp64 refinement.  map_ms: the map launches alone (HIP events around
    each); call_ms: map + refinement (HIP events on the stream, rounds without
    the per-launch events: time_calls); best of `rounds` rounds of `iters`
    calls."""
    import torch
    import dctenergy
    yy = torch.arange(S, device=dev).view(-1, 1)
    xx = torch.arange(S, device=dev).view(1, -1)
    line = (yy % 23 == 0) | (xx % 31 == 0) | ((xx + 2 * yy) % 97 == 0)
    fr = torch.where(line, 0, 255).to(torch.uint8).unsqueeze(-1).expand(S, S, 3).contiguous()
    del line
    out = torch.empty((S, S), dtype=torch.float32, device=dev)

    def call():
        ctx.energy_map_device(fr.data_ptr(), fr.stride(0), S, S, 3, 0, S, 0, S, n, e, t,
                              out.data_ptr(), out.stride(0), stream)
    for _ in range(2):
        call()
    torch.cuda.synchronize()
    best_call, best_map, _ = time_calls(ctx, call, torch.cuda.current_stream(dev), iters, rounds)
    # flagged count: the host entry point reports it (same kernels)
    host = fr.cpu().numpy()
    ctx.energy_map(host, n, e, t)
    flagged = int(ctx.last_refined)
    del fr, out, host
    return {"frame": f"line-art RGB {S}x{S} (lines every 23 rows / 31 cols / x+2y=0 mod 97), N={n}, "
                     f"e={e}, t={t}",
            "map_ms": round(best_map, 4), "refinement_ms": round(best_call - best_map, 4),
            "call_ms": round(best_call, 4), "flagged": flagged,
            "flagged_frac": round(flagged / (S * S), 5),
            "value": round(S * S / best_call / 1e3, 1), "unit": "Mpx/s",
            "what": "after the timed region; map + fp64 tie refinement of the tie-dense frame, "
                    f"best of {rounds} rounds of {iters} device calls (HIP events)"}


# timed steps between two whose map launches record their start / end (main)
PROF_EVERY = 5

# fp64 VALU operations per output pixel of the exact kernels (dcte_exact.hip):
# the reference's own ops (ddct8x8s / ddct16x16s / ddct2d, no FMA), the scan's
# maxima and the decision per output pixel (idle halo lanes included), counted
# from the kernels (DESIGN.md §3 "exact map"); the N = 16 figure includes the
# pass-1 work the eight waves of a column repeat (246 instead of 114 per pixel)
EXACT_FP64_OPS = {2: 21, 4: 105, 8: 425, 16: 2270}
def other_configs(ctx, e, t, dev, stream, iters=20, rounds=3):
    """BASELINE configs[1] (4096^2 RGB, N = 8) and configs[4] (8192^2 RGB,
    N = 16) on this GPU, timed like the headline after it, on the same kind of
    synthetic natural-like frame: call_ms = map + refinement per call (HIP
    events on the stream; the headline's step), map_ms = the map launches
    alone (HIP events around each), call_ms_with_events = the call in the
    rounds that record those events (time_calls); best of `rounds` rounds of
    `iters`."""
    import torch
    import dctenergy
    from dctenergy import synth
    res = {}
    st = torch.cuda.current_stream(dev)
    # (plus a 2048^2 layer, the size GIMP users carve most: the per-call costs
    # weigh most there)
    for S, n, key in ((4096, 8, "config2_4096_rgb_n8"), (8192, 16, "config5_8192_rgb_n16"),
                      (2048, 8, "layer_2048_rgb_n8")):
        fr = synth.natural_rows(0, S, S, 3, seed=0, device=dev)
        out = torch.empty((S, S), dtype=torch.float32, device=dev)

        def call():
            ctx.energy_map_device(fr.data_ptr(), fr.stride(0), S, S, 3, 0, S, 0, S, n, e, t,
                                  out.data_ptr(), out.stride(0), stream)
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        best_call, best_map, best_ev = time_calls(ctx, call, st, iters, rounds)
        # the same call with the refinement off (tie_tau = 0: the map launch
        # alone) -- what one launch costs beyond its kernel, so call_ms minus
        # this is the refinement launch's own cost
        ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, 0.0)
        one_call, _, _ = time_calls(ctx, call, st, iters, rounds)
        ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, -1.0)
        res[key] = {"frame": f"{S}x{S} RGB natural-like, N={n}, e={e}, t={t}",
                    "call_ms": round(best_call, 4), "map_ms": round(best_map, 4),
                    "call_ms_with_events": round(best_ev, 4), "call_over_map": round(best_call / best_map, 4),
                    "one_launch_call_ms": round(one_call, 4),
                    "one_launch_over_map": round(one_call / best_map, 4),
                    "refinement_launch_ms": round(best_call - one_call, 4),
                    "value": round(S * S / best_call / 1e3, 1), "unit": "Mpx/s",
                    "hbm_frac_of_map": round(S * S * 7 / (best_map * 1e-3) / 8.0e12, 4)}
        del fr, out
        if n == 16:                    # the N = 16 tie-dense worst case beside it
            res[key]["stress"] = stress(ctx, 16, S, e, t, dev, stream)
    torch.cuda.empty_cache()
    res["what"] = ("BASELINE configs[1] and configs[4] (and a 2048^2 layer) after the timed region "
                   "(the headline is configs[2]); call = map + tie refinement, as the headline's step")
    return res


# gfx950 fp64 VALU: 16 lanes / clk / SIMD x 1024 SIMDs x 2.4 GHz
FP64_PEAK_OPS = 256 * 4 * 16 * 2.4e9


def exact(n, S, e, t, dev, frame, iters=10, rounds=3):
    """DCTE_OPT_EXACT on the headline frame, timed after the headline: the map
    bit-identical to the reference (its fp64 operation order, dcte_exact.hip),
    HIP events around each launch; best of `rounds` rounds of `iters`."""
    import torch
    import dctenergy
    out = torch.empty((S, S), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    with dctenergy.Context(ngpus=0, exact=True) as cx:
        def call():
            cx.energy_map_device(frame.data_ptr(), frame.stride(0), S, S, 3, 0, S, 0, S, n, e, t,
                                 out.data_ptr(), out.stride(0), stream)
        for _ in range(2):
            call()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(rounds):
            cx.profile_read()
            cx.set_option(dctenergy.DCTE_OPT_PROFILE, 1)
            for _ in range(iters):
                call()
            torch.cuda.synchronize()
            cx.set_option(dctenergy.DCTE_OPT_PROFILE, 0)
            launches, kms = cx.profile_read()
            best = min(best, kms / launches)
    del out
    ops = EXACT_FP64_OPS[n]
    rate = S * S * ops / (best * 1e-3)
    return {"ms": round(best, 4), "value": round(S * S / best / 1e3, 1), "unit": "Mpx/s",
            "kernel": f"dcte_exact{n if n >= 8 else '_small'}",
            "fp64": {"ops_per_px": ops, "achieved_tops": round(rate / 1e12, 2),
                     "peak_tops": round(FP64_PEAK_OPS / 1e12, 2),
                     "frac": round(rate / FP64_PEAK_OPS, 4)},
            "what": "DCTE_OPT_EXACT (every pixel bit-identical to the reference's fp64 "
                    "arithmetic) on the same frame after the timed region; map launches alone, "
                    f"HIP events, best of {rounds} rounds of {iters}"}


def pmc_figures(n, W, px_per_rank):
    """Counter figures for dcte_map<n,RGB> from the committed rocprofv3 --pmc
    summary (profiles/pmc_summary.json, tools/pmc_summary.py), per pixel, so a
    rank is charged for ITS band: HBM bytes (FETCH_SIZE x 2 on gfx950 +
    WRITE_SIZE, MI355X_MICROARCH.md §HBM) and VALU lane-ops (SQ_INSTS_VALU x 64)."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            allsum = json.load(f)
    except (OSError, ValueError):
        return {}
    best = None
    for key, v in allsum.items():
        if not key.startswith(f"dcte_map<{n},3>@"):
            continue
        if best is None or abs(v["frame"][1] - W) < abs(best["frame"][1] - W):
            best = v
    if best is None:
        return {}
    px = best["pixels"]
    out = {"valu_lane_ops_per_px": best.get("valu_lane_ops_per_px"),
           "pmc_frame": best["frame"], "pmc_round": best.get("round")}
    if best.get("hbm_bytes_per_launch"):
        out["hbm_bytes_per_px"] = best["hbm_bytes_per_launch"] / px
        out["traffic"] = round(out["hbm_bytes_per_px"] * px_per_rank)
    return out


def cpu_rehearsal(args):
    """The rank/band/halo plumbing of a step without a GPU: every rank holds
    its band of the global frame with the halo rows zeroed, exchanges halos
    over gloo, and checks that its buffer equals the global frame's rows."""
    import torch
    import torch.distributed as dist
    from dctenergy import dist as D
    from dctenergy import synth
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    n, S = args.n, args.size
    H, W = (world * S, S) if args.weak else (S, S)
    band = (D.make_band(H, rank, world, n, rows_per_rank=S) if args.weak
            else D.make_band(H, rank, world, n))
    buf = torch.zeros((band.rows, W, 3), dtype=torch.uint8)
    buf[band.top:band.top + band.own] = synth.natural_rows(band.Y0, band.own, W, 3, device="cpu")
    for r in (D.exchange_halos(buf, band) if world > 1 else []):
        r.wait()
    ok = torch.tensor([int(torch.equal(buf, synth.natural_rows(band.row0, band.rows, W, 3,
                                                               device="cpu")))])
    rows = torch.tensor([band.own])
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        everyone = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(everyone, rows)
        rows_all = [int(v) for v in everyone]
    else:
        rows_all = [band.own]
    if rank == 0:
        print(json.dumps({"rehearsal": "cpu", "n_gpus": world,
                          "scaling": "weak" if args.weak else "strong",
                          "global_frame": [H, W], "rows_per_rank": rows_all,
                          "check_halo_exact": bool(ok.item())}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if ok.item() else 1


# ------------------------------------------------------------------ bench
def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.shared_gpu))

    sys.path.insert(0, os.path.join(ROOT, "dct-carver_amd"))
    if args.cpu_rehearsal:
        sys.exit(cpu_rehearsal(args))
    # stdout carries exactly the one JSON line: whatever the runtime libraries
    # print there (RCCL's version banner at communicator init) goes to stderr
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    import dctenergy
    from dctenergy import dist as D
    from dctenergy import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev)          # == local on a full node
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    gloo = args.dist_backend == "gloo"
    rccl_log = D.rccl_log_setup("dcte-bench") if world > 1 and not gloo else None
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    n, S = args.n, args.size
    strong = not args.weak
    if strong:
        H, W = S, S
        band = D.make_band(H, rank, world, n)
    else:
        H, W = world * S, S
        band = D.make_band(H, rank, world, n, rows_per_rank=S)
    buf = torch.zeros((band.rows, W, 3), dtype=torch.uint8, device=dev)
    # own rows of the global frame (generated per global row index); halos
    # arrive through the exchange, never regenerated
    chunk = 2048
    for a in range(0, band.own, chunk):
        b = min(band.own, a + chunk)
        buf[band.top + a:band.top + b] = synth.natural_rows(band.Y0 + a, b - a, W, 3, seed=0, device=dev)
    out = torch.empty((band.own, W), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()

    ctx = dctenergy.Context(ngpus=0)
    dev_index = gpu
    stream = torch.cuda.current_stream(dev).cuda_stream
    e, t = args.edges, args.textures
    i0, i1 = band.interior()
    row0 = band.row0

    def run_rows(y0, y1, st=stream):
        if y1 <= y0:
            return
        ctx.energy_map_device(buf.data_ptr(), buf.stride(0), W, H, 3, row0, band.rows, y0, y1,
                              n, e, t, out[y0 - band.Y0:].data_ptr(), out.stride(0), st,
                              dev_index)

    def run_edges(st=stream):
        """the band's halo-dependent rows: both edge ranges in ONE map launch
        and one refinement launch (dcte_energy_map_device2)"""
        eds = band.edges()
        if len(eds) == 2:
            (a0, a1), (b0, b1) = eds
            ctx.energy_map_device2(buf.data_ptr(), buf.stride(0), W, H, 3, row0, band.rows, a0, a1,
                                   b0, b1, n, e, t, out[a0 - band.Y0:].data_ptr(), out.stride(0), st,
                                   dev_index)
        for a, b in (eds if len(eds) == 1 else []):
            run_rows(a, b, st)

    # The halo-dependent edge rows go AFTER the interior on the same stream,
    # which waits for the halos only then (they have long landed: the
    # exchange overlaps the 2041-row interior).  A stream of their own, beside
    # the interior, was the r02-r04 choice; with the edges in ONE two-range
    # launch the sequential order costs less: 1.034x vs 1.052x the one-launch
    # band at N = 8, 1.023x vs 1.037x at N = 16 (tools/band_bench.py,
    # profiles/r05/band_split_ab.jsonl)
    rccl_path = world > 1 and not gloo

    host_buf = torch.empty(buf.shape, dtype=torch.uint8, pin_memory=True) if world > 1 and gloo else None

    def step():
        if host_buf is not None:
            # rehearsal path: halo rows via host memory and gloo
            run_rows(i0, i1)
            t0_, o_ = band.top, band.own
            host_buf[t0_:t0_ + band.hr].copy_(buf[t0_:t0_ + band.hr])          # to rank-1
            if band.hl:
                host_buf[t0_ + o_ - band.hl:t0_ + o_].copy_(buf[t0_ + o_ - band.hl:t0_ + o_])
            for r in D.exchange_halos(host_buf, band):
                r.wait()
            if band.top:
                buf[:band.top].copy_(host_buf[:band.top], non_blocking=True)
            if band.bot:
                buf[band.rows - band.bot:].copy_(host_buf[band.rows - band.bot:], non_blocking=True)
            run_edges()
        elif rccl_path:
            reqs = D.exchange_halos(buf, band)   # after this rank's previous step (incl. its edges)
            run_rows(i0, i1)                     # overlaps the exchange
            for r in reqs:
                r.wait()                         # the stream waits for the halos, then the edges
            run_edges()
        else:
            run_rows(i0, i1)
            run_edges()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.profile_read()
    # the map launches of every PROF_EVERY-th timed step record their start /
    # end (DCTE_OPT_PROFILE): those events cost a step 2.8 us at 16384^2 but
    # 6.9 us (3.9 %) on a 2048-row band (interior + edge launch), which would
    # bend the scaling curve (tools/prof_overhead.py, profiles/r06/prof_overhead.jsonl)
    profiled = 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        prof = i % PROF_EVERY == 0
        ctx.set_option(dctenergy.DCTE_OPT_PROFILE, 1 if prof else 0)
        profiled += prof
        step()
    enqueued = time.perf_counter() - t0       # host time to issue the K steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_option(dctenergy.DCTE_OPT_PROFILE, 0)
    launches, kern_ms = ctx.profile_read()
    kern_ms = kern_ms / max(1, profiled) * args.steps   # per-step average x K
    stats = torch.tensor([elapsed, kern_ms / args.steps, enqueued], dtype=torch.float64,
                         device="cpu" if gloo else dev)
    per_rank_kernel_ms = [kern_ms / args.steps]
    if world > 1:
        everyone = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(everyone, stats)
        per_rank_kernel_ms = [round(float(v[1]), 4) for v in everyone]
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    elapsed = float(stats[0])
    kernel_ms_max_rank = float(stats[1])
    host_ms_per_step = float(stats[2]) * 1e3 / args.steps

    px_per_rank = band.own * W
    total_px = H * W if strong else px_per_rank * world
    value = total_px * args.steps / elapsed / 1e6
    ms_per_step = elapsed * 1e3 / args.steps

    # roofline of the map kernel on this rank: algorithmic bytes per step over
    # the summed launch time of its map launches per step (interior + edges)
    kernel_ms_per_step = kern_ms / args.steps
    bytes_per_step = px_per_rank * (3 + 4)
    achieved_gbs = bytes_per_step / (kernel_ms_per_step * 1e-3) / 1e9
    pmc = pmc_figures(n, W, px_per_rank)
    valu_per_px = pmc.get("valu_lane_ops_per_px")
    valu_rate = (px_per_rank * valu_per_px / (kernel_ms_per_step * 1e-3)) if valu_per_px else None

    check = None
    if args.check or (world > 1 and not args.no_check):
        # regenerate this band's rows INCLUDING the halo rows straight from the
        # global frame definition and recompute without any exchange
        ref_in = synth.natural_rows(band.row0, band.rows, W, 3, seed=0, device=dev)
        ref_out = torch.empty_like(out)
        ctx.energy_map_device(ref_in.data_ptr(), ref_in.stride(0), W, H, 3, band.row0, band.rows,
                              band.Y0, band.Y1, n, e, t, ref_out.data_ptr(), ref_out.stride(0),
                              stream, dev_index)
        torch.cuda.synchronize()
        ok = torch.tensor([1 if (torch.equal(ref_out, out) and torch.equal(ref_in, buf)) else 0],
                          dtype=torch.int64, device="cpu" if gloo else dev)
        if world > 1:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        check = bool(ok.item())
        del ref_in, ref_out

    # the halo exchange alone (after the metric's region): one exchange per
    # step, timed over `reps` exchanges on their own, max over ranks; and which
    # RCCL transport carried them (the ranks' RCCL INFO logs)
    exchange = None
    if world > 1 and not gloo:
        reps = 20
        for r in D.exchange_halos(buf, band):
            r.wait()
        torch.cuda.synchronize()
        dist.barrier()
        x0 = time.perf_counter()
        for _ in range(reps):
            for r in D.exchange_halos(buf, band):
                r.wait()
        torch.cuda.synchronize()
        xms = torch.tensor([(time.perf_counter() - x0) * 1e3 / reps], dtype=torch.float64, device=dev)
        dist.all_reduce(xms, op=dist.ReduceOp.MAX)
        summ = (D.transport_summary(rccl_log, rank) if rccl_log
                else {"error": "RCCL's log routed by the caller (NCCL_DEBUG_FILE / INFO or TRACE)"})
        gathered = [None] * world
        dist.all_gather_object(gathered, summ)
        halo_bytes = (band.hl + band.hr) * W * 3
        exchange = {"ms_per_exchange": round(float(xms.item()), 4),
                    "halo_bytes_per_rank": halo_bytes,
                    "transport_per_rank": [g.get("transports") for g in gathered],
                    "transport_errors": sorted({g["error"] for g in gathered if g.get("error")}) or None,
                    "rccl_version": gathered[0].get("version"),
                    "connections_rank0": gathered[0].get("connections"),
                    "what": f"{reps} halo exchanges alone (batch_isend_irecv of N/2-1 + N/2 rows "
                            "each way), after the timed region, max over ranks; transports "
                            "parsed from each rank's RCCL INFO log (NCCL_DEBUG_FILE)"}

    # end to end: the step plus the gather of every band's
    # map to rank 0 over RCCL, reported beside the kernel-only metric
    e2e = None
    if world > 1 and not gloo and not args.no_e2e:
        reps = 3
        D.gather_bands(out, band)                     # warm
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        for _ in range(reps):
            whole = D.gather_bands(out, band)
        torch.cuda.synchronize()
        dist.barrier()
        gms = torch.tensor([(time.perf_counter() - g0) * 1e3 / reps], dtype=torch.float64, device=dev)
        dist.all_reduce(gms, op=dist.ReduceOp.MAX)
        gather_ms = float(gms.item())
        del whole
        e2e = {"gather_ms": round(gather_ms, 4),
               "step_plus_gather_ms": round(ms_per_step + gather_ms, 4),
               "value": round(total_px / ((ms_per_step + gather_ms) * 1e-3) / 1e6, 1),
               "unit": "Mpx/s",
               "what": "one step, then every band's f32 map gathered to rank 0 "
                       "(dctenergy.dist.gather_bands, RCCL); kernel-only scaling is `value`"}

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "Mpx/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            # host time to ISSUE one step (max over ranks): near ms_per_step
            # means the launches, not the GPU, set the pace
            "host_ms_per_step": round(host_ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic natural-like RGB (counter-hash noise), generated on device",
            "config": {
                "workload": (f"{H}x{W} RGB frame split into {world} row band(s)" if strong
                             else f"{S}x{S} RGB per GPU (global {H}x{W} frame, row bands)")
                            + f", N={n}, edges={e}, textures={t}, liblqr-callback semantics",
                "rows_per_gpu": band.own, "global_frame": [H, W], "block": n,
                "parallelism": f"row-band x{world}" + (", RCCL P2P halo exchange overlapped"
                                                        " with interior rows" if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": pmc.get("traffic"),
                "traffic_source": (f"rocprofv3 PMC of dcte_map<{n},3> at {pmc['pmc_frame'][0]}x"
                                   f"{pmc['pmc_frame'][1]} ({pmc['pmc_round']}), HBM bytes per "
                                   f"pixel x this rank's {px_per_rank} px") if "traffic" in pmc
                else None,
                "kernel": f"dcte_map<{n},3>",
                "kernel_ms": round(kernel_ms_per_step, 4),
                "kernel_ms_max_rank": round(kernel_ms_max_rank, 4),
                "algorithmic_bytes_per_px": 7,
                "px_per_rank": px_per_rank,
                "launches_timed": launches,
                "steps_profiled": f"{profiled} of {args.steps} (every {PROF_EVERY}th timed step)",
                "note": "rank 0's map launches; binding roof is VALU (see valu) -- the HBM "
                        "fraction this computation can reach is bounded by its VALU op count "
                        "(N=8: ~24 %; DESIGN.md §4)",
            },
            "valu": {
                "lane_ops_per_px": valu_per_px,
                "achieved_tops": round(valu_rate / 1e12, 2) if valu_rate else None,
                "peak_tops": round(VALU_PEAK_LANE_OPS / 1e12, 2),
                "frac": round(valu_rate / VALU_PEAK_LANE_OPS, 4) if valu_rate else None,
                "source": "SQ_INSTS_VALU x 64 / pixels from profiles/pmc_summary.json; "
                          "peak = 256 CU x 4 SIMD x 64 lanes / 2 cyc x 2.4 GHz",
            },
        }
        if check is not None:
            res["check_bands_bit_exact"] = check
        if e2e is not None:
            res["end_to_end"] = e2e
        if world > 1:
            res["per_rank_kernel_ms"] = per_rank_kernel_ms
        if exchange is not None:
            res["halo_exchange"] = exchange
        if world > 1 and gloo:
            res["config"]["parallelism"] += " (halo via gloo rehearsal)"
        if world > 1 and not gloo and args.shared_gpu:
            res["config"]["parallelism"] += (" (RCCL rehearsal: distinct NCCL_HOSTID per rank, "
                                             "halos over RCCL's socket transport on loopback)")
        if world > 1 and (gloo or args.shared_gpu) and ndev < world:
            res["config"]["parallelism"] += f"; {world} ranks share {ndev} GPU(s)"
        if world == 1 and not args.no_stress:
            res["stress"] = stress(ctx, n, S, e, t, dev, stream)
        if world == 1 and not args.no_exact:
            res["exact"] = exact(n, S, e, t, dev, buf)
        if world == 1 and not args.no_configs and S == 16384 and n == 8:
            res["configs_1gpu"] = other_configs(ctx, e, t, dev, stream)
        # (r05 timed the host path before configs_1gpu: after other device
        # work its SDMA download and upload were serialised by the runtime, 38
        # instead of 22.4 ms; since r06 the download is a copy kernel, and
        # the order no longer matters -- tools/host_diag.py)
        if world == 1 and not args.no_host_path:
            res["host_path"] = host_path(ctx, buf, n, e, t)
            res["host_path_vertical"] = host_path_vertical(ctx, buf, n, e, t)
            if S > 4096:                       # BASELINE configs[1]'s frame size, a 4096^2 crop
                res["host_path_4096"] = host_path(ctx, buf[:4096, :4096].contiguous(), n, e, t, iters=7)
        if world == 1 and not args.no_cpu_baseline:
            rows = args.cpu_rows or max(64, S // 2)
            rows = min(rows, H)
            host = buf[:min(H, rows + n)].cpu().numpy()
            res["cpu_baseline"] = cpu_baseline(host, W, n, e, t, rows)
        print(json.dumps(res), file=result_out, flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
