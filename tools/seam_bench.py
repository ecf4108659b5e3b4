"""Seam-step timing on the device: dcte_seam_carve_device (frame compaction +
energy update + refinement) per removed seam, frame and map resident in HBM.

    python tools/seam_bench.py --size 16384 --n 8 --seams 20
Prints one JSON line: ms per seam and the HBM rate of the compaction
(algorithmic bytes per seam: (bpp + 4) B read + (bpp + 4) B written per pixel).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--seams", type=int, default=20)
    ap.add_argument("--bpp", type=int, default=3)
    ap.add_argument("--inplace", action="store_true")
    ap.add_argument("--find", action="store_true",
                    help="full carve loop: each seam found on the device (dcte_seam_find_device)")
    a = ap.parse_args()
    import torch
    import dctenergy
    from dctenergy import synth
    S, n = a.size, a.n
    frame = synth.natural_rows(0, S, S, a.bpp, seed=0, device="cuda")
    shape = lambda w: (S, w) + ((a.bpp,) if a.bpp > 1 else ())  # noqa: E731
    # ping-pong buffers at full width (row strides stay S * bpp / S floats),
    # or one buffer pair carved in place
    px = [frame, frame if a.inplace else torch.empty(shape(S), dtype=torch.uint8, device="cuda")]
    em0 = torch.empty((S, S), dtype=torch.float32, device="cuda")
    em = [em0, em0 if a.inplace else torch.empty((S, S), dtype=torch.float32, device="cuda")]
    g = torch.Generator(device="cpu").manual_seed(0)
    with dctenergy.Context(ngpus=1) as ctx:
        ctx.energy_map_tensor(px[0], em[0], n, 0.3, 0.7)
        seams = []
        for k in range(a.seams + 2):     # 8-connected random walks
            steps = torch.randint(-1, 2, (S,), generator=g)
            s = (S // 2 + torch.cumsum(steps, 0)).clamp(0, S - 2 - k).to(torch.int32)
            seams.append(s.cuda())
        w = S

        found = torch.empty(S, dtype=torch.int32, device="cuda")

        def step(k):
            nonlocal w
            i, o = k & 1, (k + 1) & 1
            src, dst = px[i][:, :w], px[o][:, :w - 1]
            seam = seams[k]
            if a.find:
                ctx.seam_find_tensor(em[i][:, :w], found)
                seam = found
            ctx.seam_carve_tensor(src, seam, em[i][:, :w], dst, em[o][:, :w - 1], n, 0.3, 0.7)
            w -= 1

        for k in range(2):                # warm-up
            step(k)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for k in range(2, a.seams + 2):
            step(k)
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / a.seams
    # copy: every pixel read + written; in place: the right part (half on average)
    bytes_per_seam = 2 * (a.bpp + 4) * S * S // (2 if a.inplace else 1)
    print(json.dumps({"tool": "seam_bench", "size": S, "n": n, "bpp": a.bpp, "seams": a.seams, "inplace": a.inplace, "find": a.find,
                      "ms_per_seam": round(ms, 4),
                      "compaction_GB_s": round(bytes_per_seam / ms / 1e6, 1),
                      "algorithmic_bytes_per_seam": bytes_per_seam}), flush=True)


if __name__ == "__main__":
    main()
