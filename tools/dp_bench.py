"""Seam-search timing on the device (dcte_seam_find_device: DP + jump
composition + walk), map resident in HBM; checks the seam against the CPU
restatement on a sampled case.

    python tools/dp_bench.py --size 16384 --reps 10 [--lib path.so] [--bandwise]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default="")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--bandwise", action="store_true", help="DCTE_OPT_DP_BANDWISE: one launch per band")
    a = ap.parse_args()
    if a.lib:
        os.environ["DCTE_LIB"] = a.lib
    sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd"), os.path.join(ROOT, "tests")]
    import torch
    import dctenergy
    H, W = a.size, a.width or a.size
    g = torch.Generator(device="cuda").manual_seed(0)
    emap = torch.rand((H, W), generator=g, device="cuda", dtype=torch.float32)
    seam = torch.empty(H, dtype=torch.int32, device="cuda")
    with dctenergy.Context(ngpus=1) as ctx:
        if a.bandwise:
            ctx.set_option(dctenergy.DCTE_OPT_DP_BANDWISE, 1)
        for _ in range(2):
            ctx.seam_find_tensor(emap, seam)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.reps):
            ctx.seam_find_tensor(emap, seam)
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / a.reps
        ok = None
        if a.check:
            import oracle_py as O
            ok = bool((seam.cpu().numpy() == O.seam_find(emap.cpu().numpy())).all())
    print(json.dumps({"tool": "dp_bench", "lib": os.path.basename(a.lib) or "default", "h": H, "w": W, "bandwise": a.bandwise,
                      "ms_per_seam_search": round(ms, 4), "ns_per_row": round(ms * 1e6 / H, 1),
                      "matches_oracle": ok}), flush=True)


if __name__ == "__main__":
    main()
