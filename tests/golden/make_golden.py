"""Generate the golden fixtures in tests/golden/ (run in the build container).

Expected outputs come from the REFERENCE's own transforms (oracle/_ref,
i.e. /root/reference/src/fft2d/*.c compiled unmodified, driven by
oracle/ref_harness.c which restates the dctNxN dispatch, the weighted max of
src/dct.c and the window gather of src/render.c:122-157).  Inputs are seeded
synthetic images plus the reference's one real image (help/images/wilber.png).
The luma plane handed to the reference is liblqr's LQR_ER_LUMA formula
(0.2126 R + 0.7152 G + 0.0722 B on channel/255 in double; grey: v/255)
[liblqr, unverified -- liblqr is not in this image]; see manifest.json.

Every fixture is data only: .npy arrays (no pickles) and manifest.json.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_py as O  # noqa: E402

REF_PNG = "/root/reference/help/images/wilber.png"


def natural(h, w, c, seed):
    """'Natural-like' synthetic image."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    base = 128 + 60 * np.sin(x / 17) + 40 * np.cos(y / 11)
    if c == 1:
        img = base + rng.normal(0, 20, (h, w))
    else:
        img = base[..., None] + rng.normal(0, 20, (h, w, c))
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def special_images():
    imgs = {}
    imgs["const_rgb_40x33"] = np.full((33, 40, 3), 137, np.uint8)
    yy, xx = np.mgrid[0:48, 0:52]
    imgs["checker1_grey_48x52"] = (((xx + yy) & 1) * 255).astype(np.uint8)
    imgs["checker3_rgb_48x52"] = np.stack([(((xx // 3 + yy // 3) & 1) * 200 + 20)] * 3, -1).astype(np.uint8)
    imgs["vstripes_grey_37x45"] = ((np.mgrid[0:37, 0:45][1] % 5 < 2) * 180 + 30).astype(np.uint8)
    imgs["hstep_rgb_41x29"] = np.where(np.mgrid[0:41, 0:29][0][..., None] < 17,
                                       np.array([10, 200, 90], np.uint8),
                                       np.array([250, 20, 60], np.uint8)).astype(np.uint8)
    imgs["diag_grey_40x40"] = np.clip(np.mgrid[0:40, 0:40].sum(0) * 6, 0, 255).astype(np.uint8)
    imgs["gradient_grey_64x64"] = (np.mgrid[0:64, 0:64][1] * 4).astype(np.uint8)
    imgs["bright_smooth_grey_32x48"] = (np.full((32, 48), 250) - (np.mgrid[0:32, 0:48][0] > 15)).astype(np.uint8)
    rng = np.random.default_rng(7)
    imgs["binary_rgb_35x31"] = (rng.integers(0, 2, (35, 31, 3)) * 255).astype(np.uint8)
    imgs["uniform_rgb_57x63"] = rng.integers(0, 256, (57, 63, 3)).astype(np.uint8)
    # images smaller than the window
    imgs["tiny_rgb_1x1"] = np.array([[[12, 200, 99]]], np.uint8)
    imgs["tiny_grey_2x3"] = np.array([[0, 255, 7], [90, 91, 255]], np.uint8)
    imgs["tiny_rgb_5x1"] = rng.integers(0, 256, (5, 1, 3)).astype(np.uint8)
    imgs["tiny_grey_1x7"] = rng.integers(0, 256, (1, 7)).astype(np.uint8)
    imgs["thin_rgb_3x40"] = rng.integers(0, 256, (3, 40, 3)).astype(np.uint8)
    return imgs


def kat_windows():
    """Known-answer windows, reference layout [dx][dy]."""
    out = {}
    for n in (2, 4, 8, 16):
        k = np.arange(n)
        # orthonormal (n=8,16) or unnormalised (n=2,4) DCT-II basis images
        def atom(k1, k2):
            b1 = np.cos(np.pi * (k + 0.5) * k1 / n)
            b2 = np.cos(np.pi * (k + 0.5) * k2 / n)
            return np.outer(b1, b2)
        out[f"const_n{n}"] = np.full((n, n), 0.42)
        out[f"atom01_n{n}"] = 0.3 * atom(0, 1)
        out[f"atom10_n{n}"] = -0.2 * atom(1, 0)
        if n >= 4:
            out[f"atom23_n{n}"] = 0.25 * atom(2, 3)
        out[f"atom11_n{n}"] = 0.1 * atom(1, 1)
        # equal-magnitude edge/texture tie: the texture atom wins (last max)
        out[f"tie_n{n}"] = 0.5 * atom(0, 1) / np.abs(O.ref_dct(atom(0, 1))[0, 1]) + \
            0.5 * atom(1, 1) / np.abs(O.ref_dct(atom(1, 1))[1, 1])
    return out


def main():
    if not O.ref_available():
        O.build_oracle()
        import subprocess
        subprocess.run(["make", "-s", "-C", O.ORACLE_DIR, "ref"], check=True)
    manifest = {
        "generator": "tests/golden/make_golden.py",
        "expected_outputs": "oracle/_ref (reference src/fft2d transforms, unmodified)",
        "luma": "LQR_ER_LUMA: bpp=3 -> 0.2126*(R/255.) + 0.7152*(G/255.) + 0.0722*(B/255.) "
                "(double, that association); bpp=1 -> v/255. [liblqr, unverified]",
        "window": "dct_pixel_energy: d[i][j] = L(clamp(x+i-(r-1)), clamp(y+j-(r-1))), r=N/2",
        "output_dtype": "float32 (gfloat returned by weighted_max_dct_correlation)",
        "maps": [],
        "kat": [],
    }

    def add_map(name, img, n, e, t):
        L = O.luma_plane(img)
        E = O.ref_energy_map_luma(L, n, e, t)
        ofile = f"{name}__n{n}_e{e}_t{t}.npy"
        np.save(os.path.join(HERE, "maps", ofile), E)
        manifest["maps"].append({"input": f"{name}.npy", "output": ofile, "N": n,
                                 "edges": e, "textures": t,
                                 "shape": list(img.shape)})

    os.makedirs(os.path.join(HERE, "inputs"), exist_ok=True)
    os.makedirs(os.path.join(HERE, "maps"), exist_ok=True)

    inputs = {}
    inputs["grey512"] = natural(512, 512, 1, 0)          # BASELINE config 1
    inputs["natural_rgb_73x59"] = natural(59, 73, 3, 1)  # odd sizes
    inputs["natural_rgb_97x41"] = natural(41, 97, 3, 2)
    inputs["natural_grey_200x120"] = natural(120, 200, 1, 3)
    try:
        from PIL import Image
        inputs["wilber_rgb_74x59"] = np.asarray(Image.open(REF_PNG).convert("RGB"), np.uint8)
    except Exception as exc:  # pragma: no cover
        print("wilber.png not used:", exc)
    inputs.update(special_images())
    for name, img in inputs.items():
        np.save(os.path.join(HERE, "inputs", name + ".npy"), np.ascontiguousarray(img))

    # BASELINE config 1: 512^2 grey, 8x8, defaults e=t=0.5 and e!=t
    add_map("grey512", inputs["grey512"], 8, 0.5, 0.5)
    add_map("grey512", inputs["grey512"], 8, 0.3, 0.7)
    for n in (2, 4, 16):
        add_map("natural_grey_200x120", inputs["natural_grey_200x120"], n, 0.5, 0.5)
    for name in inputs:
        if name == "grey512":
            continue
        for n in (2, 4, 8, 16):
            add_map(name, inputs[name], n, 0.15, 0.85)

    # preview semantics (src/render.c:31-109): float energies from the
    # reference transforms over the restated row streaming, plus the u8
    # image normalize_image would draw (numpy restatement, tests/oracle_py.py)
    manifest["preview"] = []
    rng = np.random.default_rng(21)
    prev_inputs = {
        "natural_rgb_73x59": inputs["natural_rgb_73x59"],
        "natural_grey_200x120": inputs["natural_grey_200x120"],
        "rgba_45x38": np.concatenate([natural(38, 45, 3, 5), rng.integers(0, 256, (38, 45, 1), dtype=np.uint8)], -1),
        "uniform_rgb_57x63": inputs["uniform_rgb_57x63"],
        "tiny_grey_2x3": inputs["tiny_grey_2x3"],
        "tiny_rgb_1x1": inputs["tiny_rgb_1x1"],
    }
    if "wilber_rgb_74x59" in inputs:
        prev_inputs["wilber_rgb_74x59"] = inputs["wilber_rgb_74x59"]
    np.save(os.path.join(HERE, "inputs", "rgba_45x38.npy"), prev_inputs["rgba_45x38"])
    for name, img in prev_inputs.items():
        for n in (2, 4, 8, 16):
            for e, t in ((0.5, 0.5), (0.15, 0.85)):
                E = O.ref_preview_map(img, n, e, t)
                ofile = f"preview__{name}__n{n}_e{e}_t{t}.npy"
                np.save(os.path.join(HERE, "maps", ofile), E)
                ch = 1 if img.ndim == 2 else img.shape[2]
                u8file = ofile.replace(".npy", "_u8.npy")
                np.save(os.path.join(HERE, "maps", u8file), O.normalize_preview(E, ch))
                manifest["preview"].append({"input": f"{name}.npy", "output": ofile,
                                            "output_u8": u8file, "N": n, "edges": e,
                                            "textures": t, "channels": ch})

    kats = kat_windows()
    os.makedirs(os.path.join(HERE, "kat"), exist_ok=True)
    for name, win in kats.items():
        np.save(os.path.join(HERE, "kat", name + ".npy"), win)
        for e, t in ((0.5, 0.5), (0.15, 0.85), (1.0, 0.0), (0.0, 1.0)):
            manifest["kat"].append({"window": name + ".npy", "edges": e, "textures": t,
                                    "energy": O.ref_window_energy(win, e, t)})

    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(len(manifest["maps"]), "maps,", len(manifest["preview"]), "preview maps,",
          len(manifest["kat"]), "KAT entries")


if __name__ == "__main__":
    main()
