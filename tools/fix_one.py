"""One frame kind of tools/fix_study.py, map + refinement `--iters` times on
the device (for rocprofv3 kernel traces and counter passes of dcte_fix_tiles).

    python tools/fix_one.py --frame lineart_rgb [--size 16384] [--n 8] [--iters 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd"), os.path.join(ROOT, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frame", default="lineart_rgb")
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tau", type=float, default=-1, help="DCTE_OPT_TIE_TAU (< 0: the per-N defaults)")
    a = ap.parse_args()
    if a.lib:
        os.environ["DCTE_LIB"] = os.path.abspath(a.lib)
    import torch
    import dctenergy
    import fix_study
    dev = torch.device("cuda", 0)
    fr = {k.split()[0]: v for k, v in fix_study.frames(a.size, torch, dev).items()}[a.frame]
    out = torch.empty((a.size, a.size), dtype=torch.float32, device=dev)
    with dctenergy.Context(ngpus=1) as ctx:
        ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, a.tau)
        for _ in range(a.iters):
            ctx.energy_map_tensor(fr, out, a.n, 0.3, 0.7)
        torch.cuda.synchronize()
    print("done", a.frame, a.size, a.n)


if __name__ == "__main__":
    main()
