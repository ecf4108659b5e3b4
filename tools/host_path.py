"""Host-buffer (PCIe-inclusive) rate of dcte_energy_map / dcte_energy_image_u8.

The plug-in boundary hands over host buffers (src/render.c:312): this times the
whole call -- H2D of the frame, the map kernel, D2H of the map -- for pageable
numpy frames and for page-locked (torch pin_memory) frames, next to the bare
copy rates of the same bytes.  Prints one JSON line per case.

    python tools/host_path.py --size 16384 --n 8
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


DEFAULT_PIN_MIB = 1.0     # DCTE_OPT_PIN_HOST's default (dcte_capi.cpp)


def timed(fn, iters):
    fn()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--lib", default=None, help="libdctenergy_hip.so to load (A/B)")
    ap.add_argument("--quick", action="store_true", help="only the default host->host case")
    a = ap.parse_args()
    if a.lib:
        os.environ["DCTE_LIB"] = os.path.abspath(a.lib)
    import numpy as np
    import torch
    import dctenergy
    from dctenergy import synth
    S = a.size
    dev = synth.natural_rows(0, S, S, 3, seed=0, device="cuda")
    px_pin = torch.empty((S, S, 3), dtype=torch.uint8, pin_memory=True)
    px_pin.copy_(dev)
    px_np = px_pin.numpy().copy()                       # pageable
    out_pin = torch.empty((S, S), dtype=torch.float32, pin_memory=True)
    out_np = np.empty((S, S), np.float32)
    d_out = torch.empty((S, S), dtype=torch.float32, device="cuda")
    mpx = S * S / 1e6
    res = []
    with dctenergy.Context(ngpus=1) as ctx:
        cases = (("pageable, DCTE_OPT_PIN_HOST=0 (runtime-staged copies)", px_np, out_np, 0),
                 ("pageable, page-locked per call (default)", px_np, out_np, -1),
                 ("pageable, page-locked per call from 1 MiB", px_np, out_np, 1),
                 ("pageable, page-locked per call from 64 MiB", px_np, out_np, 64),
                 ("caller-pinned buffers", px_pin.numpy(), out_pin.numpy(), 64))
        if a.quick:
            cases = cases[1:2]
        for name, src, dst, pin in cases:
            # pin < 0: the library's default threshold (a fresh context)
            ctx.set_option(dctenergy.DCTE_OPT_PIN_HOST, pin if pin >= 0 else DEFAULT_PIN_MIB)
            med, best = timed(lambda: ctx.energy_map(src, a.n, 0.3, 0.7, out=dst), a.iters)
            res.append({"case": f"dcte_energy_map host->host ({name})", "lib": os.path.basename(dctenergy.LIB_PATH),
                        "ms": round(med * 1e3, 2),
                        "best_ms": round(best * 1e3, 2), "mpx_s": round(mpx / med, 1)})
        ctx.set_option(dctenergy.DCTE_OPT_PIN_HOST, DEFAULT_PIN_MIB)
        if a.quick:
            for r in res:
                r.update({"size": S, "n": a.n})
                print(json.dumps(r), flush=True)
            return
        med, best = timed(lambda: ctx.energy_image_u8(px_np, a.n, 0.3, 0.7), a.iters)
        res.append({"case": "dcte_energy_image_u8 host->host (pageable, fresh output array per call)",
                    "ms": round(med * 1e3, 2),
                    "mpx_s": round(mpx / med, 1)})
        u8 = np.empty((S, S), np.uint8)
        med, best = timed(lambda: ctx.energy_image_u8(px_np, a.n, 0.3, 0.7, out=u8), a.iters)
        res.append({"case": "dcte_energy_image_u8 host->host (pageable, output array reused)",
                    "ms": round(med * 1e3, 2),
                    "mpx_s": round(mpx / med, 1)})
    # bare copy rates of the same bytes (torch, same stream semantics)
    for name, fn, nbytes in (
            ("H2D pageable frame", lambda: dev.copy_(torch.from_numpy(px_np)), px_np.nbytes),
            ("H2D pinned frame", lambda: dev.copy_(px_pin), px_np.nbytes),
            ("D2H map pageable", lambda: torch.from_numpy(out_np).copy_(d_out), out_np.nbytes),
            ("D2H map pinned", lambda: out_pin.copy_(d_out), out_np.nbytes)):
        def run(f=fn):
            f()
            torch.cuda.synchronize()
        med, _ = timed(run, a.iters)
        res.append({"case": name, "ms": round(med * 1e3, 2), "GB_s": round(nbytes / med / 1e9, 2)})
    # the host path's floor: the frame's H2D and the map's D2H at the same
    # time on two streams (pinned buffers) -- what the chunk pipeline overlaps
    s_up, s_down = torch.cuda.Stream(), torch.cuda.Stream()
    d_px = torch.empty_like(dev)

    def duplex():
        with torch.cuda.stream(s_up):
            d_px.copy_(px_pin, non_blocking=True)
        with torch.cuda.stream(s_down):
            out_pin.copy_(d_out, non_blocking=True)
        torch.cuda.synchronize()
    med, _ = timed(duplex, a.iters)
    res.append({"case": "H2D frame + D2H map concurrently (pinned, two streams)", "ms": round(med * 1e3, 2),
                "GB_s": round((px_np.nbytes + out_np.nbytes) / med / 1e9, 2)})
    for r in res:
        r.update({"size": S, "n": a.n})
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
