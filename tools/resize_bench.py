"""liblqr resize loop through the patched callback, with and without the
update_emap hook: served fractions and the time spent in
the update callbacks per seam.

    python tools/resize_bench.py [--size 1024x768] [--seams 16] [--n 8] [--exact]

--exact sets DCTE_PLUGIN_EXACT: the maps and the hook's
band updates in the reference's fp64 arithmetic.

Uses the fake liblqr of tests/fake_lqr (energy build + per seam: DP, carve,
update_emap over the band liblqr re-evaluates [liblqr, unverified]); the
original per-window code is played by the oracle's window transform.  One
JSON line per mode.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="1024x768")
    ap.add_argument("--seams", type=int, default=16)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--transposed", action="store_true")
    ap.add_argument("--exact", action="store_true", help="DCTE_PLUGIN_EXACT")
    ap.add_argument("--verify", action="store_true",
                    help="re-run the original body on every hook-served callback (not timed fairly)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from dctenergy import synth
    from test_plugin_shim import fake, resize
    fake().fake_set_plugin_flags(2 if a.exact else 0)
    w, h = (int(v) for v in a.size.split("x"))
    img = synth.natural_rows(0, h, w, 3, seed=0, device="cuda").cpu().numpy()
    for hook in (False, True):
        r = resize(img, a.n, 0.3, 0.7, a.seams, use_gpu=True, hook=hook, transposed=a.transposed,
                   verify=a.verify)
        upd = r["callbacks"] - r["initial"]
        print(json.dumps({
            "frame": f"{w}x{h} RGB", "n": a.n, "seams": a.seams, "transposed": a.transposed,
            "exact": a.exact,
            "hook": hook, "callbacks": r["callbacks"], "build_callbacks": r["initial"],
            "update_callbacks": upd, "update_callbacks_per_seam": round(upd / a.seams, 1),
            "served_gpu": r["callbacks"] - r["fallback"],
            "served_frac": round((r["callbacks"] - r["fallback"]) / r["callbacks"], 4),
            "fallback": r["fallback"], "mirror_steps": r["steps"], "hook_misses": r["missed"],
            "hook_on_at_end": r["hook_on"], "verified": r["verified"], "verified_off_tol": r["bad"],
            "hook_reads_per_update_callback": round(r["reads"] / max(upd, 1), 2),
            "update_ms_per_seam": round(r["update_ns"] / 1e6 / a.seams, 3)}), flush=True)


if __name__ == "__main__":
    main()
