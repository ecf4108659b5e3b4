"""Per-workgroup timeline of one dcte_map launch (timing-probe build only).

    tools/variants.sh "tstamp -DDCTE_TSTAMP=1"
    python tools/tstamp.py --lib dct-carver_amd/build/variants/tstamp.so --rows 2048 [--tile-h 128]

The probe build writes each workgroup's start / end on the 100 MHz real-time
counter and its HW_ID into a stamp buffer of its own (DCTE_OPT_TSTAMP_BUF;
the map stays right); this prints, for a
band of --rows rows of a 16384-wide RGB frame (N = 8): the spread of start
times (dispatch ramp), the workgroup durations, the spread of end times
(tail), and the same split by co-residency slot on a CU.  One JSON line.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--rows", type=int, default=2048)
    ap.add_argument("--width", type=int, default=16384)
    ap.add_argument("--tile-h", type=int, default=128)
    ap.add_argument("--n", type=int, default=8)
    a = ap.parse_args()
    os.environ["DCTE_LIB"] = os.path.abspath(a.lib)
    import numpy as np
    import torch
    import dctenergy
    from dctenergy import synth
    n, W, R = a.n, a.width, a.rows
    hl, hr = n // 2 - 1, n // 2
    H = 8 * R
    Y0 = 3 * R
    buf = synth.natural_rows(Y0 - hl, R + hl + hr, W, 3, seed=0, device="cuda")
    out = torch.empty((R, W), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    tw = 256 if n != 16 else 64
    nwg = ((W + tw - 1) // tw) * ((R + a.tile_h - 1) // a.tile_h)
    slots = 4                                               # workgroups a CU holds at once
    stamps = torch.zeros(3 * nwg, dtype=torch.int64, device="cuda")
    with dctenergy.Context(ngpus=1) as ctx:
        ctx.set_option(dctenergy.DCTE_OPT_TILE_H, a.tile_h)
        ctx.set_option(dctenergy.DCTE_OPT_TSTAMP_BUF, stamps.data_ptr())
        ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, 0.0)     # the map launch alone
        for _ in range(6):
            ctx.energy_map_device(buf.data_ptr(), buf.stride(0), W, H, 3, Y0 - hl, buf.shape[0],
                                  Y0, Y0 + R, n, 0.3, 0.7, out.data_ptr(), out.stride(0), s.cuda_stream)
        torch.cuda.synchronize()
    ts = stamps.cpu().numpy().reshape(nwg, 3)
    if not ts[:, 1].any():
        raise SystemExit("no stamps written: --lib is not a DCTE_TSTAMP=1 build")
    start, end, hwid = ts[:, 0], ts[:, 1], ts[:, 2]
    t0 = start.min()
    us = lambda v: round(float(v) / 100.0, 2)        # 100 MHz ticks -> us
    dur = end - start
    cu = (hwid >> 8) & 15
    se = (hwid >> 13) & 7
    res = {"rows": R, "tile_h": a.tile_h, "workgroups": int(nwg),
           "launch_span_us": us(end.max() - t0),
           "start_spread_us": us(start.max() - t0),
           "start_p50_us": us(np.percentile(start - t0, 50)),
           "end_first_us": us(end.min() - t0), "end_p50_us": us(np.percentile(end - t0, 50)),
           "dur_min_us": us(dur.min()), "dur_p50_us": us(np.percentile(dur, 50)),
           "dur_max_us": us(dur.max()),
           "distinct_cu_se": int(len(set(zip(cu.tolist(), se.tolist()))))}
    # workgroups that started in the first 5 us (the first round) vs later
    first = (start - t0) < 500
    res["first_round"] = int(first.sum())
    res["first_round_dur_p50_us"] = us(np.percentile(dur[first], 50)) if first.any() else None
    res["later_dur_p50_us"] = us(np.percentile(dur[~first], 50)) if (~first).any() else None
    # per CU (XCD = dispatch order L % 8, the hardware deals workgroups
    # round-robin over the XCDs): how many of the launch's workgroups each
    # CU held, and how long they took
    xcd = np.arange(nwg) % 8
    key = xcd * 1024 + se * 64 + cu
    keys, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    res["cus"] = int(len(keys))
    res["wg_per_cu_hist"] = {int(k): int(v) for k, v in zip(*np.unique(cnt, return_counts=True))}
    for c in sorted(set(cnt.tolist())):
        sel = cnt[inv] == c
        res[f"dur_p50_us_on_cus_with_{c}"] = us(np.percentile(dur[sel], 50))
        res[f"dur_max_us_on_cus_with_{c}"] = us(dur[sel].max())
    # when each CU ran out of work: its last workgroup's end (the launch's
    # tail is the spread of these)
    last = np.zeros(len(keys), np.int64)
    np.maximum.at(last, inv, end - t0)
    res["cu_idle_from_us"] = {"min": us(last.min()), "p50": us(np.percentile(last, 50)),
                              "max": us(last.max())}
    # busy fraction: sum of workgroup durations / (slots x CUs x span)
    res["slot_busy_frac"] = round(float(dur.sum()) / (slots * len(keys) * float(end.max() - t0)), 4)
    # per XCD: median duration
    res["dur_p50_us_per_xcd"] = [us(np.percentile(dur[xcd == x], 50)) for x in range(8)]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
