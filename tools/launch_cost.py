"""What the refinement launch costs a small-frame call.

    python tools/launch_cost.py [--sizes 2048,4096] [--n 8]

For each frame (natural-like RGB, and a flat grey RGB frame that flags no
pixel) and size: the device call timed without profiling events (bench.py's
time_calls) with the per-N default tie margin, and the same call with
tie_tau = 0 (no refinement launch at all).  Their difference on the flat
frame is the cost of an EMPTY refinement launch (the dirty list is empty, every
wave exits after reading the counter); on the natural frame, of a launch that
refines its few hundred flagged pixels.  One JSON line per frame and size.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dct-carver_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="2048,4096")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    if a.lib:
        os.environ["DCTE_LIB"] = os.path.abspath(a.lib)
    import torch
    import dctenergy
    from dctenergy import synth
    from bench import time_calls
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, e, t = a.n, 0.3, 0.7
    with dctenergy.Context(ngpus=1) as ctx:
        for S in [int(v) for v in a.sizes.split(",")]:
            frames = {"natural_rgb": synth.natural_rows(0, S, S, 3, seed=0, device=dev),
                      "flat_rgb": torch.full((S, S, 3), 128, dtype=torch.uint8, device=dev)}
            out = torch.empty((S, S), dtype=torch.float32, device=dev)
            for name, fr in frames.items():
                def call():
                    ctx.energy_map_device(fr.data_ptr(), fr.stride(0), S, S, 3, 0, S, 0, S, n, e, t,
                                          out.data_ptr(), out.stride(0), st.cuda_stream)
                for _ in range(3):
                    call()
                torch.cuda.synchronize()
                ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, -1.0)
                c_ref, m_ref, _ = time_calls(ctx, call, st, a.iters, a.rounds)
                ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, 0.0)
                c_one, m_one, _ = time_calls(ctx, call, st, a.iters, a.rounds)
                ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, -1.0)
                host = fr.cpu().numpy()
                ctx.energy_map(host, n, e, t)
                print(json.dumps({"frame": name, "size": S, "n": n, "lib": os.path.basename(dctenergy.LIB_PATH),
                                  "flagged": int(ctx.last_refined),
                                  "call_ms": round(c_ref, 4), "one_launch_call_ms": round(c_one, 4),
                                  "refinement_launch_us": round((c_ref - c_one) * 1e3, 2),
                                  "map_ms": round(m_ref, 4), "map_ms_tau0": round(m_one, 4)}), flush=True)
            del frames, out


if __name__ == "__main__":
    main()
