"""Do the default-tau GPU maps lead liblqr's DP to the same seams as the
reference arithmetic -- and does the exact mode (DCTE_OPT_EXACT) always?  (VERDICT r03 "What's weak", parity caveat: at the
default tau most pixels of a natural frame differ from the reference by a few
ulp, within the 1e-5 bar; the DP compares sums of those floats.)

For each frame, block size and weight pair: the device carve loop
(dcte_carve: map, then per seam liblqr's DP [dcte_seam_find_device] + carve +
band update, src/render.c:313,377 [liblqr, unverified]) with the default tau
against the same loop in the exact mode (DCTE_OPT_EXACT: the map in the
reference's fp64 operation order, dcte_exact.hip, and every seam-band pixel
refined in fp64 -- bit-identical maps; tests/test_exact.py shows that loop
equals the CPU loop on the reference's arithmetic seam for seam).  With
--oracle the exact loop is also checked against the CPU loop on the oracle
(oracle/_ref's arithmetic) for every configuration: "exact_vs_cpu_identical".
Reports how many of the S seams agree before the first difference and in
total, and the fraction of map pixels that are bit-identical.

    python tools/seam_agreement.py [--seams 32] [--oracle] > profiles/r05/seam_agreement.jsonl
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd"), os.path.join(ROOT, "tests")]


def frames():
    import numpy as np
    import torch
    from dctenergy import synth
    from golden_util import load_input
    out = {}
    for name in ("natural_rgb_73x59.npy", "natural_rgb_97x41.npy", "natural_grey_200x120.npy",
                 "wilber_rgb_74x59.npy", "grey512.npy"):
        out["golden " + name[:-4]] = load_input(name)
    for seed in range(3):
        out[f"natural RGB 1024x768 seed {seed}"] = synth.natural_rows(0, 768, 1024, 3, seed=seed,
                                                                      device="cuda").cpu().numpy()
    yy, xx = np.mgrid[0:512, 0:512]
    line = (yy % 23 == 0) | (xx % 31 == 0) | ((xx + 2 * yy) % 97 == 0)
    out["line-art grey 512x512"] = np.where(line, 0, 255).astype(np.uint8)
    del torch
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seams", type=int, default=32)
    ap.add_argument("--oracle", action="store_true",
                    help="also run the CPU carve loop on the oracle and compare the exact loop with it")
    a = ap.parse_args()
    import numpy as np
    import dctenergy
    with dctenergy.Context(ngpus=1) as fast, dctenergy.Context(ngpus=1, exact=True) as exact:
        for name, img in frames().items():
            for n in (2, 4, 8, 16):
                for e, t in ((0.5, 0.5), (0.3, 0.7)):
                    S = min(a.seams, img.shape[1] // 4)
                    Ef = fast.energy_map(img, n, e, t)
                    Ex = exact.energy_map(img, n, e, t)
                    _, cf = fast.carve(img, S, n, e, t)
                    _, cx = exact.carve(img, S, n, e, t)
                    same = [bool(np.array_equal(cf[k], cx[k])) for k in range(S)]
                    cpu = None
                    if a.oracle:
                        import oracle_py as O
                        from seam_util import carve
                        host, cpu = img, True
                        for k in range(S):
                            rs = O.seam_find(O.energy_map(host, n, e, t, nthreads=16))
                            cpu = cpu and bool(np.array_equal(rs, cx[k]))
                            host = carve(host, rs)
                    prefix = next((k for k, s in enumerate(same) if not s), S)
                    print(json.dumps({
                        "frame": name, "shape": list(img.shape), "n": n, "edges": e, "textures": t,
                        "seams": S, "identical_prefix": prefix, "identical_total": int(sum(same)),
                        "first_seam_same": same[0] if S else None,
                        "map_bit_identical_frac": round(float(np.mean(Ef == Ex)), 4),
                        "exact_vs_cpu_identical": cpu,
                        "map_max_rel_diff": float(np.max(np.abs(Ef.astype(np.float64) - Ex) /
                                                         np.maximum(np.abs(Ex), 1e-30))),
                    }), flush=True)


if __name__ == "__main__":
    main()
