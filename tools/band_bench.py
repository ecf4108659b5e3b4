"""Per-rank cost of a strong-scaling step on one GPU (no exchange): a band of
`--rows` output rows of a 16384-wide frame, launched as bench.py does at
world > 1 (interior rows, then the N/2-1 top and N/2 bottom halo-dependent
rows in ONE two-range launch, dcte_energy_map_device2: 2 map + 2 refinement
launches) vs one launch over the band, and vs r03's three map launches.  HIP-event timing on the
launch stream; prints one JSON line per pattern.

    python tools/band_bench.py [--rows 2048] [--n 8] [--iters 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2048)
    ap.add_argument("--width", type=int, default=16384)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--tile-h", type=int, default=0)
    ap.add_argument("--lib", default=None, help="libdctenergy_hip.so to load (A/B)")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    if a.lib:
        os.environ["DCTE_LIB"] = os.path.abspath(a.lib)
    import torch
    import dctenergy
    from dctenergy import synth
    n, W, R = a.n, a.width, a.rows
    hl, hr = n // 2 - 1, n // 2
    H = 8 * R                                   # a middle band of an 8-band frame
    Y0, Y1 = 3 * R, 4 * R
    buf = synth.natural_rows(Y0 - hl, R + hl + hr, W, 3, seed=0, device="cuda")
    out = torch.empty((R, W), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    with dctenergy.Context(ngpus=1) as ctx:
        ctx.set_option(dctenergy.DCTE_OPT_TILE_H, a.tile_h)

        def run(y0, y1):
            ctx.energy_map_device(buf.data_ptr(), buf.stride(0), W, H, 3, Y0 - hl, buf.shape[0], y0, y1,
                                  n, 0.3, 0.7, out[y0 - Y0:].data_ptr(), out.stride(0), s.cuda_stream)
        def run2(a0, a1, b0, b1):
            ctx.energy_map_device2(buf.data_ptr(), buf.stride(0), W, H, 3, Y0 - hl, buf.shape[0], a0, a1,
                                   b0, b1, n, 0.3, 0.7, out[a0 - Y0:].data_ptr(), out.stride(0), s.cuda_stream)
        s2 = torch.cuda.Stream()

        def run2_side(i0, i1, a0, a1, b0, b1):
            # bench.py world > 1: the interior on the launch stream, the two
            # edge ranges on a stream of their own beside it (there they wait
            # for the halo exchange, here for the start of the step), joined
            ev = torch.cuda.Event()
            ev.record(s)
            s2.wait_event(ev)
            run(i0, i1)
            ctx.energy_map_device2(buf.data_ptr(), buf.stride(0), W, H, 3, Y0 - hl, buf.shape[0], a0, a1,
                                   b0, b1, n, 0.3, 0.7, out[a0 - Y0:].data_ptr(), out.stride(0), s2.cuda_stream)
            s.wait_stream(s2)
        pats = {"one launch": [(Y0, Y1)],
                "interior + two-range edge launch on a second stream (as bench.py)":
                    [("side", Y0 + hl, Y1 - hr, Y0, Y0 + hl, Y1 - hr, Y1)],
                "interior + one two-range edge launch (bench.py world > 1)":
                    [(Y0 + hl, Y1 - hr), (Y0, Y0 + hl, Y1 - hr, Y1)],
                "interior + 2 edge launches (r03)": [(Y0 + hl, Y1 - hr), (Y0, Y0 + hl), (Y1 - hr, Y1)]}
        res = {}
        for rnd in range(a.rounds):
            if True:
                for name, ranges in pats.items():
                    for _ in range(5):
                        for r in ranges:
                            (run2_side(*r[1:]) if r[0] == "side" else (run2 if len(r) == 4 else run)(*r))
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record(s)
                    h0 = time.perf_counter()
                    for _ in range(a.iters):
                        for r in ranges:
                            (run2_side(*r[1:]) if r[0] == "side" else (run2 if len(r) == 4 else run)(*r))
                    host_ms = (time.perf_counter() - h0) * 1e3 / a.iters
                    e1.record(s)
                    torch.cuda.synchronize()
                    res.setdefault(name, []).append((e0.elapsed_time(e1) / a.iters, host_ms))
        for name, v in res.items():
            ms = sorted(t for t, _ in v)[len(v) // 2]
            print(json.dumps({"pattern": name, "lib": os.path.basename(a.lib or "default"),
                              "rows": R, "width": W, "n": n, "tile_h": a.tile_h,
                              "ms_per_step": round(ms, 4),
                              "host_ms_per_step": round(sorted(h for _, h in v)[len(v) // 2], 4),
                              "mpx_s": round(R * W / ms / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
