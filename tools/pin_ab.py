"""A/B of the host path's page-locking threshold at plug-in frame sizes
(DCTE_OPT_PIN_HOST moved from 64 MiB to 1 MiB in r05; the A/B
then covered only 2048^2 and 4096^2).  For 1-8 MiB frames -- 1024x768 up to
1920x1080 RGB, what GIMP layers usually are -- times dcte_energy_map with the
threshold at 0 (never page-lock: r05 the runtime staged the copies; since
r06 the library stages every byte through its page-locked arena), 1 MiB (the
default) and 64 MiB (r04), with the SAME numpy buffers reused across calls
and with FRESH buffers every call (a new rgb buffer per carver build, as
init_carver_from_vals allocates, src/render.c:159-173).  One JSON line per
(size, threshold, buffers): median / best ms over `iters` calls.

    python tools/pin_ab.py [HxW ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def main():
    import numpy as np
    import dctenergy
    iters = 15
    rng = np.random.default_rng(0)
    sizes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]] or \
        [(768, 1024), (1024, 1280), (1080, 1920), (1536, 2048)]
    with dctenergy.Context(ngpus=1) as ctx:
        for h, w in sizes:
            base = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
            for pin in (0, 1, 64):
                ctx.set_option(dctenergy.DCTE_OPT_PIN_HOST, pin)
                for mode in ("reused", "fresh"):
                    px = base.copy()
                    out = np.empty((h, w), np.float32)
                    ctx.energy_map(px, 8, 0.3, 0.7, out=out)
                    ts = []
                    for _ in range(iters):
                        if mode == "fresh":
                            px = base.copy()
                            out = np.empty((h, w), np.float32)
                        t0 = time.perf_counter()
                        ctx.energy_map(px, 8, 0.3, 0.7, out=out)
                        ts.append((time.perf_counter() - t0) * 1e3)
                    ts.sort()
                    print(json.dumps({"h": h, "w": w, "frame_mib": round(px.nbytes / 2**20, 2),
                                      "map_mib": round(out.nbytes / 2**20, 2), "pin_mib": pin,
                                      "buffers": mode, "median_ms": round(ts[len(ts) // 2], 3),
                                      "best_ms": round(ts[0], 3)}), flush=True)
            ctx.set_option(dctenergy.DCTE_OPT_PIN_HOST, 1)


if __name__ == "__main__":
    main()
