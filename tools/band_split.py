"""Cost of the N > 1 step shape on one GPU, without any exchange: a rank's
band (default 2048 x 16384 RGB, N = 8: strong scaling at 8 GPUs) mapped as
the bench's ranks do it -- interior rows, then the two halo-dependent edge
strips -- against the same rows in ONE call.  HIP events on the stream.

    python tools/band_split.py [--rows 2048] [--width 16384] [--reps 50]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2048)
    ap.add_argument("--width", type=int, default=16384)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import torch
    import dctenergy
    from dctenergy import dist as D
    from dctenergy import synth
    n, W = a.n, a.width
    H = a.rows * 8
    band = D.make_band(H, 3, 8, n)                  # a middle rank of 8
    buf = synth.natural_rows(band.row0, band.rows, W, 3, seed=0, device="cuda")
    out = torch.empty((band.own, W), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    i0, i1 = band.interior()
    side = torch.cuda.Stream()
    with dctenergy.Context(ngpus=0) as ctx:
        def rows(y0, y1, st=stream):
            ctx.energy_map_device(buf.data_ptr(), buf.stride(0), W, H, 3, band.row0, band.rows, y0, y1,
                                  n, 0.3, 0.7, out[y0 - band.Y0:].data_ptr(), out.stride(0), st, 0)

        def split():
            rows(i0, i1)
            for y0, y1 in band.edges():
                rows(y0, y1)

        def overlap():
            # edges on a second stream that waits only for what the halos
            # would wait for (here: the step's start), so they run beside
            # the interior; the main stream joins them at the end
            ev = torch.cuda.Event()
            ev.record()
            side.wait_event(ev)
            rows(i0, i1)
            for y0, y1 in band.edges():
                rows(y0, y1, side.cuda_stream)
            torch.cuda.current_stream().wait_stream(side)

        def whole():
            rows(band.Y0, band.Y1)

        res = {}
        for name, fn in (("whole", whole), ("split", split), ("overlap", overlap),
                         ("whole", whole), ("split", split), ("overlap", overlap)):
            for _ in range(5):
                fn()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(a.reps):
                fn()
            t1.record()
            torch.cuda.synchronize()
            ms = t0.elapsed_time(t1) / a.reps
            res[name] = min(res.get(name, 1e9), ms)
    print(json.dumps({"tool": "band_split", "band": [band.own, W], "n": n,
                      "whole_ms": round(res["whole"], 4), "split_ms": round(res["split"], 4),
                      "overlap_ms": round(res["overlap"], 4),
                      "split_overhead_ms": round(res["split"] - res["whole"], 4),
                      "overlap_overhead_ms": round(res["overlap"] - res["whole"], 4)}), flush=True)


if __name__ == "__main__":
    main()
