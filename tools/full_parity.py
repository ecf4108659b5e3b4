"""Whole-frame parity sweep beyond the GPU tests' two full frames: every
pixel of the device map against the OpenMP oracle (bit-identical to the
reference transforms, tests/test_oracle.py) for each block size, both
semantics (liblqr callback, GTK preview) and every layer format they take.
One JSON line per configuration: off-tolerance pixels (|d| > 1e-5 |ref| +
ATOL), class flips, the largest relative error, and how many pixels are
bit-identical.

    python tools/full_parity.py [--size 16384] [--size16 8192] [--threads 16]
                                [--kind natural|lineart|dots|text|grid8] [--n 8,16] [--exact]

--exact runs the context in DCTE_OPT_EXACT (the sliding fp64 maps; preview
through the fp64 pass over every pixel), where bit_identical must equal pixels.

--kind other than natural takes the tie-dense frames of tools/fix_study.py
(binary line art, isolated dots, 4-px text blocks, 8-px grid: exact edge /
texture ties decided by the reference's rounding, so most of their flagged
pixels go through the fp64 refinement), replicated over the channels.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384, help="frame side for N = 2, 4, 8")
    ap.add_argument("--size16", type=int, default=8192, help="frame side for N = 16")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--edges", type=float, default=0.3)
    ap.add_argument("--textures", type=float, default=0.7)
    ap.add_argument("--kind", default="natural")
    ap.add_argument("--n", default="2,4,8,16", help="block sizes, comma-separated")
    ap.add_argument("--exact", action="store_true",
                    help="DCTE_OPT_EXACT: the bar is every pixel bit-identical")
    a = ap.parse_args()
    import torch
    import dctenergy
    import oracle_py as O
    from dctenergy import synth
    from golden_util import ATOL, RTOL
    e, t = a.edges, a.textures
    lo, hi = min(e, t) / max(e, t), max(e, t) / min(e, t)
    cases = [(dctenergy.DCTE_LQR, "liblqr", bpp) for bpp in (1, 3)] + \
            [(dctenergy.DCTE_PREVIEW, "preview", bpp) for bpp in (1, 3, 4)]
    with dctenergy.Context(ngpus=1, exact=a.exact) as ctx:
        def make(S, bpp):
            if a.kind == "natural":
                return synth.natural_rows(0, S, S, bpp, seed=1, device="cuda")
            g = torch.Generator(device="cuda")
            g.manual_seed(5)
            yy = torch.arange(S, device="cuda").view(-1, 1)
            xx = torch.arange(S, device="cuda").view(1, -1)
            if a.kind == "lineart":
                ink = (yy % 23 == 0) | (xx % 31 == 0) | ((xx + 2 * yy) % 97 == 0)
                grey = torch.where(ink, 0, 255)
            elif a.kind == "dots":
                grey = torch.where(torch.rand((S, S), generator=g, device="cuda") < 1 / 64, 255, 16)
            elif a.kind == "text":
                blk = torch.rand((S // 4 + 1, S // 4 + 1), generator=g, device="cuda") < 0.3
                ink = blk.repeat_interleave(4, 0).repeat_interleave(4, 1)[:S, :S]
                grey = torch.where(ink, 0, 255)
            elif a.kind == "grid8":
                grey = torch.where((yy % 8 == 0) | (xx % 8 == 0), 0, 255)
            else:
                raise SystemExit(f"unknown --kind {a.kind}")
            grey = grey.to(torch.uint8)
            return grey.unsqueeze(-1).expand(S, S, bpp).contiguous()

        for n in [int(v) for v in a.n.split(",")]:
            S = a.size16 if n == 16 else a.size
            for sem, sname, bpp in cases:
                frame = make(S, bpp)
                if bpp == 1:
                    frame = frame.reshape(S, S).contiguous()
                out = torch.empty((S, S), dtype=torch.float32, device="cuda")
                ctx.energy_map_tensor(frame, out, n, e, t, semantics=sem)
                torch.cuda.synchronize()
                host = frame.cpu().numpy()
                t0 = time.perf_counter()
                ref = (O.energy_map if sem == dctenergy.DCTE_LQR else O.preview_map)(
                    host, n, e, t, nthreads=a.threads)
                t_ref = time.perf_counter() - t0
                del host
                bad = flips = same = 0
                worst = 0.0
                for r0 in range(0, S, 2048):
                    r = torch.from_numpy(ref[r0:r0 + 2048]).cuda().to(torch.float64)
                    g = out[r0:r0 + 2048].to(torch.float64)
                    err = (g - r).abs()
                    off = err > RTOL * r.abs() + ATOL
                    bad += int(off.sum())
                    same += int((err == 0).sum())
                    worst = max(worst, float(torch.where(r.abs() > 0, err / r.abs(), err).max()))
                    if e != t and off.any():
                        ratio = g[off] / r[off]
                        flips += int((((ratio - lo).abs() < 1e-3 * lo) |
                                      ((ratio - hi).abs() < 1e-3 * hi)).sum())
                print(json.dumps({"kind": a.kind, "exact": a.exact, "n": n, "semantics": sname, "bpp": bpp, "frame": [S, S],
                                  "edges": e, "textures": t, "pixels": S * S,
                                  "off_tolerance": bad, "class_flips": flips,
                                  "bit_identical": same, "max_rel_err": worst,
                                  "oracle_s": round(t_ref, 2)}),
                      flush=True)
                del ref, out, frame
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
