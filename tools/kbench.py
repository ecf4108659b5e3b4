"""Kernel A/B on the GPU: time dcte_map over a 16384^2 RGB frame for several
builds of libdctenergy_hip.so, interleaved rounds in ONE process per build
set (cdna_hip_programming.md rule 24).

    python tools/kbench.py --n 8 --size 16384 build/variants/a.so build/variants/b.so ...
Each .so is loaded under its own ctypes handle; prints one JSON line per build.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def load(path, exact=False, tile_h=0):
    L = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    L.dcte_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_uint]
    L.dcte_set_option.argtypes = [vp, ctypes.c_int, ctypes.c_double]
    L.dcte_energy_map_device.argtypes = [vp, ctypes.c_int, vp, ctypes.c_longlong, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                         ctypes.c_float, ctypes.c_int, vp, ctypes.c_longlong, vp]
    L.dcte_profile_read.argtypes = [vp, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]
    h = vp()
    assert L.dcte_create(ctypes.byref(h), 1, 0) == 0
    L.dcte_set_option(h, 2, 1.0)
    if exact:
        assert L.dcte_set_option(h, 10, 1.0) == 0          # DCTE_OPT_EXACT
    if tile_h:
        assert L.dcte_set_option(h, 4, float(tile_h)) == 0  # DCTE_OPT_TILE_H
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--bpp", type=int, default=3)
    ap.add_argument("--sem", type=int, default=0)
    ap.add_argument("--e2e", action="store_true",
                    help="time whole calls (map + refinement + launch gaps) with stream events "
                         "instead of the map launches alone")
    ap.add_argument("--check", type=int, default=0,
                    help="also map a CHECKxCHECK natural frame and a dots-on-flat frame with "
                         "every build and compare with the CPU oracle (tolerance, class flips)")
    ap.add_argument("--exact", action="store_true", help="DCTE_OPT_EXACT (the fp64 map)")
    ap.add_argument("--width", type=int, default=0, help="frame width (default --size)")
    ap.add_argument("--height", type=int, default=0, help="frame height (default --size)")
    ap.add_argument("--tile-h", default="0",
                    help="comma-separated DCTE_OPT_TILE_H values, each a separate entry per lib (0: the launcher's pick)")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    import torch
    from dctenergy import synth
    S = a.size
    W, H = a.width or S, a.height or S
    frame = synth.natural_rows(0, H, W, a.bpp, seed=0, device="cuda")
    out = torch.empty((H, W), dtype=torch.float32, device="cuda")
    ref = None
    ths = [int(v) for v in a.tile_h.split(",")]
    libs = [(f"{p}@th{th}" if len(ths) > 1 else p, *load(p, a.exact, th)) for p in a.libs for th in ths]
    stream = torch.cuda.current_stream().cuda_stream
    times = {p[0]: [] for p in libs}
    same = {}
    for r in range(a.rounds):
        for p, L, h in libs:
            def call():
                rc = L.dcte_energy_map_device(h, 0, frame.data_ptr(), frame.stride(0), W, H, a.bpp, 0, H,
                                              0, H, a.n, 0.3, 0.7, a.sem, out.data_ptr(), out.stride(0), stream)
                assert rc == 0, rc
            n = ctypes.c_longlong()
            ms = ctypes.c_double()
            if a.e2e:
                call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    call()
                e1.record()
                torch.cuda.synchronize()
                L.dcte_profile_read(h, ctypes.byref(n), ctypes.byref(ms))
                times[p].append(e0.elapsed_time(e1) / a.iters)
            else:
                for _ in range(a.iters + 1):
                    call()
                L.dcte_profile_read(h, ctypes.byref(n), ctypes.byref(ms))
                times[p].append(ms.value / n.value)
            if r == 0:
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                same[p] = bool(torch.equal(out, ref))
    checks = {}
    if a.check:
        import numpy as np
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_py as O
        from golden_util import within_tol
        C = a.check
        rng = np.random.default_rng(5)
        nat = synth.natural_rows(0, C, C, a.bpp, seed=1, device="cuda")
        dots = np.where(rng.random((C, C)) < 1 / 64, 255, 16).astype(np.uint8)
        dots = torch.from_numpy(np.repeat(dots[..., None], a.bpp, -1).copy()).cuda()
        frames = [(nat, O.energy_map(nat.cpu().numpy(), a.n, 0.3, 0.7)),
                  (dots, O.energy_map(dots.cpu().numpy(), a.n, 0.3, 0.7))]
        cout = torch.empty((C, C), dtype=torch.float32, device="cuda")
        for p, L, h in libs:
            bad = flips = 0
            worst = 0.0
            for fr, ref in frames:
                rc = L.dcte_energy_map_device(h, 0, fr.data_ptr(), fr.stride(0), C, C, a.bpp, 0, C,
                                              0, C, a.n, 0.3, 0.7, a.sem, cout.data_ptr(),
                                              cout.stride(0), stream)
                assert rc == 0, rc
                torch.cuda.synchronize()
                got = cout.cpu().numpy()
                bad += int((~within_tol(got, ref)).sum())
                rel = np.abs(got.astype(np.float64) - ref) / np.maximum(np.abs(ref), 1e-30)
                worst = max(worst, float(rel[np.abs(ref) > 1e-9].max()))
                # a class flip changes the weight: e = 0.3 vs t = 0.7 differ by > 2x
                flips += int((np.abs(got - ref) > 0.25 * np.abs(ref)).sum())
            checks[p] = {"check_off_tol": bad, "check_flips": flips, "check_max_rel": worst}
    for p, _, _ in libs:
        t = times[p]
        print(json.dumps({"lib": os.path.basename(p), "n": a.n, "size": S, "w": W, "h": H, "e2e": a.e2e, "exact": a.exact,
                          "median_ms": round(statistics.median(t), 4), "min_ms": round(min(t), 4),
                          "mpx_s": round(W * H / statistics.median(t) / 1e3, 1),
                          "bit_equal_first": same[p], **checks.get(p, {})}))


if __name__ == "__main__":
    main()
