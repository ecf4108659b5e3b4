"""A/B of the host path's download engine (DCTE_OPT_D2H_KERNEL): the copy
kernel into the mapped page-locked output (1, default) against the runtime's
SDMA copies (0), at frame sizes from 1024^2 to 16384^2 (RGB, N = 8, pageable
numpy frame and map, page-locked per call), interleaved in one process.
One JSON line per (size, engine): median / best ms over `iters` calls, and
the same bytes' duplex floor (pinned buffers, H2D and D2H at once).

    python tools/d2h_ab.py [sizes...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def main():
    import numpy as np
    import torch
    import dctenergy
    from dctenergy import synth
    sizes = [int(a) for a in sys.argv[1:]] or [1024, 2048, 4096, 8192, 16384]
    with dctenergy.Context(ngpus=1) as ctx:
        for S in sizes:
            iters = 9 if S <= 4096 else 3
            px = synth.natural_rows(0, S, S, 3, seed=0, device="cuda").cpu().numpy()
            out = np.empty((S, S), np.float32)
            res = {}
            for rnd in range(2):
                for kern in (1, 0):
                    ctx.set_option(dctenergy.DCTE_OPT_D2H_KERNEL, kern)
                    ctx.energy_map(px, 8, 0.3, 0.7, out=out)
                    ts = []
                    for _ in range(iters):
                        t0 = time.perf_counter()
                        ctx.energy_map(px, 8, 0.3, 0.7, out=out)
                        ts.append((time.perf_counter() - t0) * 1e3)
                    res.setdefault(kern, []).extend(ts)
            ctx.set_option(dctenergy.DCTE_OPT_D2H_KERNEL, 1)
            p_pin = torch.empty(tuple(px.shape), dtype=torch.uint8, pin_memory=True)
            o_pin = torch.empty((S, S), dtype=torch.float32, pin_memory=True)
            d_px = torch.empty(tuple(px.shape), dtype=torch.uint8, device="cuda")
            d_o = torch.empty((S, S), dtype=torch.float32, device="cuda")
            su, sd = torch.cuda.Stream(), torch.cuda.Stream()
            fl = []
            for _ in range(iters + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                with torch.cuda.stream(su):
                    d_px.copy_(p_pin, non_blocking=True)
                with torch.cuda.stream(sd):
                    o_pin.copy_(d_o, non_blocking=True)
                torch.cuda.synchronize()
                fl.append((time.perf_counter() - t0) * 1e3)
            floor = sorted(fl[1:])[len(fl[1:]) // 2]
            for kern, ts in res.items():
                ts.sort()
                print(json.dumps({"size": S, "d2h_kernel": kern, "median_ms": round(ts[len(ts) // 2], 3),
                                  "best_ms": round(ts[0], 3), "floor_ms": round(floor, 3)}), flush=True)
            del px, out, p_pin, o_pin, d_px, d_o
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
