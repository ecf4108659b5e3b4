"""Per-kernel durations of the default bench command from a rocprofv3
--kernel-trace run (run_kernel_trace.csv), restricted to the launches the
bench line times, so the average can be set beside the line's HIP-event
figures:
  * dcte_map<8,3,0> over the full frame (grid 64 x 128 at 16384^2): the first
    warmup + steps launches (10 + 50 by default), the last `steps` of them
    being the timed region;
  * dcte_exact8<3> (the `exact` object): the launches after its 2 warm-up calls.

    python tools/trace_summary.py gpurun_out/01_trace profiles/r05/bench_trace_summary.json \
        [--bench-json gpurun_out/bench.json] [--warmup 10] [--steps 50]
"""
import argparse
import csv
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("out")
    ap.add_argument("--bench-json", default=None)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(os.path.join(a.trace_dir, "run_kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))

    def durs(name_sub, grid=None):
        out = []
        for r in rows:
            if name_sub not in r["Kernel_Name"]:
                continue
            if grid and (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"])) != grid:
                continue
            out.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
        return out

    res = {}
    # full-frame launches: the grid of a 16384^2 frame (64 tiles of 256 columns
    # x 128 tile rows, 256 threads: Grid_Size_X counts threads)
    full = durs("dcte_map<8, 3, 0>", (64 * 256, 128))
    first = full[:a.warmup + a.steps]
    timed = first[a.warmup:]
    if first:
        res["dcte_map<8,3,0> full-frame launches of bench.py (warm-up + timed)"] = {
            "n": len(first), "avg_ms": round(sum(first) / len(first), 4),
            "avg_timed_ms": round(sum(timed) / max(1, len(timed)), 4), "n_timed": len(timed),
            "min_ms": round(min(first), 4), "max_ms": round(max(first), 4)}
    ex = durs("dcte_exact8<3>")
    if len(ex) > 2:
        t = ex[2:]
        res["dcte_exact8<3> launches of the exact object (after 2 warm-up)"] = {
            "n": len(t), "avg_ms": round(sum(t) / len(t), 4), "min_ms": round(min(t), 4),
            "max_ms": round(max(t), 4)}
    if a.bench_json and os.path.exists(a.bench_json):
        b = json.load(open(a.bench_json))
        res["bench_line_kernel_ms_hip_events"] = b["roofline"]["kernel_ms"]
        res["bench_line_exact_ms"] = b.get("exact", {}).get("ms")
        res["bench_value_mpx_s"] = b["value"]
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
