"""The long adversarial searches behind tests/test_tau_bound.py's committed
margin: for each case, tests/emu/tau_search.cpp hill-climbs over integer
pixel windows (restarts x iters evaluations of the map kernel's own fp32
code against the exact transform) and reports the largest relative error of
a candidate maximum.  One JSON line per case (with the worst window, so the
test can re-evaluate it).

    python tools/tau_long.py OUT.jsonl [--n 2,4,8,16] [--jobs 8]

The cases and budgets are r02's (profiles/r02/tau_search.jsonl); r05 re-ran
them after the N = 16 odd half moved to a scaled form (dcte_math.h
dct16_odd_sc), which changes that kernel's fp32 rounding.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

CASES = [(16, 0, 1, 400), (16, 0, 3, 400), (16, 1, 3, 300),
         (2, 0, 3, 4000), (4, 0, 1, 4000), (4, 0, 3, 4000),
         (8, 0, 1, 2000), (8, 0, 3, 2000), (8, 1, 3, 2000)]
ITERS, SEED = 5000, 7


def run(case):
    import emu_py as EM
    n, sem, bpp, restarts = case
    t0 = time.time()
    d, win, me, mt = EM.tau_search(n, sem, bpp, restarts, ITERS, SEED)
    return {"n": n, "sem": sem, "bpp": bpp, "restarts": restarts, "iters": ITERS, "seed": SEED,
            "evals": restarts * ITERS, "delta": d, "me": me, "mt": mt,
            "window": win.tolist(), "s": round(time.time() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--n", default="2,4,8,16")
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    ns = {int(v) for v in a.n.split(",")}
    cases = [c for c in CASES if c[0] in ns]
    with ProcessPoolExecutor(a.jobs) as ex, open(a.out, "w") as f:
        for r in ex.map(run, cases):
            f.write(json.dumps(r) + "\n")
            print({k: v for k, v in r.items() if k != "window"}, flush=True)


if __name__ == "__main__":
    main()
