"""The CPU oracle is pinned to the reference before anything is checked against it.

* bit-exact against every golden map / KAT produced by the reference's own
  transforms (tests/golden/make_golden.py, oracle/_ref);
* bit-exact against oracle/_ref itself on random windows, where it was built.
"""
import numpy as np
import pytest

import oracle_py as O
from golden_util import load_input, load_kat, load_map, manifest


@pytest.mark.parametrize("entry", manifest()["maps"], ids=lambda e: e["output"])
def test_oracle_matches_golden_map(entry):
    img = load_input(entry["input"])
    ref = load_map(entry["output"])
    got = O.energy_map(img, entry["N"], entry["edges"], entry["textures"])
    assert got.dtype == np.float32 and got.shape == ref.shape
    assert np.array_equal(got, ref)


def test_oracle_matches_kat():
    for k in manifest()["kat"]:
        win = load_kat(k["window"])
        assert O.window_energy(win, k["edges"], k["textures"]) == np.float32(k["energy"]), k


def test_kat_semantics():
    """Known answers that follow from src/dct.c:96-110 directly."""
    for n in (2, 4, 8, 16):
        assert O.window_energy(np.full((n, n), 0.42), 0.3, 0.7) == 0.0
        # a pure (0,1) atom -> edge class
        k = np.arange(n)
        atom = np.outer(np.ones(n), np.cos(np.pi * (k + 0.5) / n))
        e = O.window_energy(atom, 0.25, 0.75)
        c01 = abs(O.dct(atom)[0, 1])
        assert e == np.float32(c01 * np.float32(0.25))


def test_row_range_composes():
    img = load_input("natural_rgb_97x41.npy")
    for n in (2, 4, 8, 16):
        full = O.energy_map(img, n, 0.15, 0.85)
        parts = [O.energy_map(img, n, 0.15, 0.85, y0=a, y1=b) for a, b in ((0, 7), (7, 30), (30, 41))]
        assert np.array_equal(np.concatenate(parts), full)


def test_bad_n_rejected():
    img = np.zeros((8, 8), np.uint8)
    for n in (0, 1, 3, 6, 32):
        with pytest.raises(ValueError):
            O.energy_map(img, n, 0.5, 0.5)


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (no /root/reference)")
def test_oracle_bit_exact_vs_reference_transforms():
    rng = np.random.default_rng(123)
    for n in (2, 4, 8, 16):
        for scale in (1e-4, 1.0, 300.0):
            for _ in range(300):
                w = rng.standard_normal((n, n)) * scale
                assert np.array_equal(O.dct(w), O.ref_dct(w))
                e, t = rng.random(2).astype(np.float32)
                assert O.window_energy(w, e, t) == O.ref_window_energy(w, e, t)


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (no /root/reference)")
def test_oracle_map_vs_reference_random_images():
    rng = np.random.default_rng(5)
    for n in (2, 4, 8, 16):
        img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
        L = O.luma_plane(img)
        assert np.array_equal(O.energy_map(img, n, 0.2, 0.8), O.ref_energy_map_luma(L, n, 0.2, 0.8))


@pytest.mark.parametrize("entry", manifest()["preview"], ids=lambda e: e["output"])
def test_oracle_preview_matches_golden(entry):
    img = load_input(entry["input"])
    got = O.preview_map(img, entry["N"], entry["edges"], entry["textures"])
    assert np.array_equal(got, load_map(entry["output"]))
    assert np.array_equal(O.normalize_preview(got, entry["channels"]), load_map(entry["output_u8"]))


def test_preview_luma_is_the_macro():
    """RGB2LUMINANCE (src/render.h:5) evaluated in double, truncated."""
    for rgb in ((0, 0, 0), (255, 255, 255), (10, 200, 30), (255, 0, 128)):
        px = np.array(rgb, np.uint8)
        want = int(16.0 + rgb[0] * 0.2568 + rgb[1] * 0.5041 + rgb[2] * 0.0979)
        assert O.lib().orc_preview_luma(px.ctypes.data_as(O._u8p), 3) == want
