"""Why does the page-locked host path slow down after other device work?
  One scenario per process, so every scenario starts
from a fresh HIP runtime:

  fresh          the plug-in's call (16384^2 RGB, N = 8, pageable numpy frame
                 -> dcte_energy_map -> numpy map) in a new process
  torch_churn    torch allocates and frees ~2.7 GB of device frames (what
                 bench.py's configs_1gpu does) + empty_cache, then the call
  torch_keep     the same churn without empty_cache (torch keeps the blocks)
  pre_churn      the call once first (the library's buffers exist), then the
                 churn, then the call again
  lib_growth     the library's OWN buffer growth: a host call at 8192^2 N = 16,
                 then the 16384^2 call (ensure_buf frees and re-allocates)
  big_free       one 8 GiB hipMalloc + hipFree through torch, then the call

Prints one JSON line: the scenario, the call's median / best ms over `iters`.
Run under rocprofv3 --memory-copy-trace --kernel-trace to see the copies.

    python tools/host_diag.py torch_churn
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def main():
    scen = sys.argv[1]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    import numpy as np
    import torch
    import dctenergy
    from dctenergy import synth
    S = 16384
    px = synth.natural_rows(0, S, S, 3, seed=0, device="cuda").cpu().numpy()
    torch.cuda.empty_cache()
    out = np.empty((S, S), np.float32)

    def churn(empty=True):
        for s, n in ((4096, 8), (8192, 16)):
            fr = synth.natural_rows(0, s, s, 3, seed=0, device="cuda")
            o = torch.empty((s, s), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            del fr, o
        if empty:
            torch.cuda.empty_cache()

    def call_times(ctx):
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            ctx.energy_map(px, 8, 0.3, 0.7, out=out)
            ts.append((time.perf_counter() - t0) * 1e3)
        return ts

    res = {"scenario": scen}
    with dctenergy.Context(ngpus=1) as ctx:
        if scen == "torch_churn":
            churn(True)
        elif scen == "torch_keep":
            churn(False)
        elif scen == "pre_churn":
            res["before_ms"] = sorted(call_times(ctx))
            churn(True)
        elif scen == "lib_growth":
            small = synth.natural_rows(0, 8192, 8192, 3, seed=1, device="cuda").cpu().numpy()
            torch.cuda.empty_cache()
            ctx.energy_map(small, 16, 0.3, 0.7)
        elif scen == "big_free":
            b = torch.empty(8 << 30, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            del b
            torch.cuda.empty_cache()
        elif scen != "fresh":
            raise SystemExit(f"unknown scenario {scen}")
        ts = call_times(ctx)
    ts_sorted = sorted(ts)
    res.update({"ms": ts, "median_ms": round(ts_sorted[len(ts) // 2], 2),
                "best_ms": round(ts_sorted[0], 2)})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
