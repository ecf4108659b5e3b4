"""Drop-in check: the patched liblqr callback, driven by a fake
liblqr energy build (tests/fake_lqr), served from libdctenergy_hip.so.

CPU: without a device the plug-in glue reports the error and every callback
runs the original per-window code -- the map equals the reference exactly.
GPU: at the carver's original size every callback is answered from the GPU
map (no per-window work) within the parity tolerance; once seams change the
carver size the original code takes over again.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import dctenergy
import oracle_py as O
from golden_util import load_input, load_map, manifest, within_tol

HERE = os.path.dirname(os.path.abspath(__file__))
FAKE_DIR = os.path.join(HERE, "fake_lqr")
_lib = None


def fake():
    global _lib
    if _lib is None:
        dctenergy.lib()
        O.lib()
        subprocess.run(["make", "-s", "-C", FAKE_DIR], check=True)
        L = ctypes.CDLL(os.path.join(FAKE_DIR, "build", "libfake_lqr.so"))
        L.fake_build_emap.restype = ctypes.c_int
        L.fake_build_emap.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.c_longlong),
                                      ctypes.POINTER(ctypes.c_int)]
        L.fake_resize.restype = ctypes.c_int
        L.fake_resize.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_int)]
        L.fake_set_plugin_flags.restype = None
        L.fake_set_plugin_flags.argtypes = [ctypes.c_uint]
        L.fake_set_interleave.restype = None
        L.fake_set_interleave.argtypes = [ctypes.c_int]
        L.fake_preview.restype = ctypes.c_int
        L.fake_preview.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_uint,
                                   ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.fake_window_check_selftest.restype = ctypes.c_int
        L.fake_window_check_selftest.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint]
        _lib = L
    return _lib


def build_emap(img, n, e, t, use_gpu, removed=0, transposed=False):
    img = np.ascontiguousarray(img)
    h, w = img.shape[:2]
    bpp = 1 if img.ndim == 2 else img.shape[2]
    out = np.empty((w - removed, h) if transposed else (h, w - removed), np.float32)
    calls = ctypes.c_longlong()
    status = ctypes.c_int()
    rc = fake().fake_build_emap(img.ctypes.data, w, h, bpp, n, e, t, int(use_gpu), removed,
                                int(transposed), out.ctypes.data, ctypes.byref(calls),
                                ctypes.byref(status))
    assert rc == 0
    return out, calls.value, status.value


DIVERGE = {"none": 0, "perturb": 1, "shift_row": 2, "rightmost_ties": 3, "repass": 4}


def resize(img, n, e, t, seams, use_gpu, hook, transposed=False, diverge="none", verify=False):
    """fake liblqr resize loop (tests/fake_lqr: energy build, then per seam DP,
    carve, update_emap through the patched callback) -> dict.  diverge: how
    the fake liblqr departs from the mirror (fake_resize's doc); verify: the
    original body re-run on every hook-served callback ("verified", "bad")."""
    img = np.ascontiguousarray(img)
    h, w = img.shape[:2]
    bpp = 1 if img.ndim == 2 else img.shape[2]
    fw, fh = (h, w) if transposed else (w, h)
    emap = np.empty((fh, fw - seams), np.float32)
    px = np.empty((fh, fw - seams) + img.shape[2:], np.uint8)
    seam_cols = np.empty((max(seams, 1), fh), np.int32)
    counts = (ctypes.c_longlong * 12)()
    status = ctypes.c_int()
    rc = fake().fake_resize(img.ctypes.data, w, h, bpp, n, e, t, int(use_gpu), int(hook), seams,
                            int(transposed), DIVERGE[diverge], int(verify), emap.ctypes.data,
                            px.ctypes.data, seam_cols.ctypes.data, counts, ctypes.byref(status))
    assert rc == 0
    c = list(counts)
    return {"emap": emap, "px": px, "seams": seam_cols[:seams], "callbacks": c[0],
            "fallback": c[1], "served_map": c[2], "served_band": c[3], "steps": c[4], "update_ns": c[5],
            "verified": c[6], "bad": c[7], "missed": c[8], "hook_on": c[9], "reads": c[10],
            "interleaved": c[11], "status": status.value, "initial": fw * fh}


def preview(drawable, n, e, t, flags=0, rect=None):
    """The patched dct_energy_preview of tests/fake_lqr
    on an HxW(xC) drawable; rect = (x1, y1, w, h), default the whole
    drawable -> (drawn u8 layer h x w (x C), the glue's status)."""
    d = np.ascontiguousarray(drawable)
    dh, dw = d.shape[:2]
    ch = 1 if d.ndim == 2 else d.shape[2]
    x1, y1, w, h = rect or (0, 0, dw, dh)
    out = np.empty((h, w) + ((ch,) if ch > 1 else ()), np.uint8)
    status = ctypes.c_int()
    rc = fake().fake_preview(d.ctypes.data, dw, dh, ch, x1, y1, w, h, n, e, t, flags,
                             out.ctypes.data, ctypes.byref(status))
    assert rc == 0
    return out, status.value


@pytest.mark.parametrize("n", [2, 4, 8, 16])
@pytest.mark.parametrize("bpp", [1, 3])
def test_hook_window_check(n, bpp):
    """The hook's window test on the host (no device): over a synthetic band
    around a wandering seam, every update pixel's gathered window matches the
    band, the same window with any one element moved by one 8-bit luma step
    is rejected, and a window past the band misses."""
    for seed in (1, 2, 3):
        assert fake().fake_window_check_selftest(n, bpp, seed) == 0


def test_resize_loop_without_gpu_is_the_reference():
    """CPU: no device -> every callback of the build and of every update_emap
    runs the original per-window code, and the final energies equal the
    reference map of the carved image exactly (the update band liblqr
    re-evaluates covers every pixel whose window the seam touched)."""
    if dctenergy.device_count() > 0:
        pytest.skip("device visible; covered by the GPU test")
    img = load_input("natural_rgb_73x59.npy")
    for n, transposed in ((8, False), (4, True), (16, False)):
        r = resize(img, n, 0.15, 0.85, 6, use_gpu=True, hook=True, transposed=transposed,
                   verify=True)
        assert r["status"] == dctenergy.DCTE_ENODEV
        assert r["fallback"] == r["callbacks"] > r["initial"]
        assert r["served_map"] == r["served_band"] == r["steps"] == 0
        assert np.array_equal(r["emap"], O.energy_map(r["px"], n, 0.15, 0.85))


@pytest.mark.gpu
@pytest.mark.parametrize("n,transposed", [(8, False), (8, True), (4, False), (16, False), (2, True)])
def test_seam_hook_serves_update_emap(n, transposed):
    """The update_emap hook: with it every callback of a
    liblqr resize -- the build and every seam's update band -- is answered by
    the GPU (no per-window transform), every served value equals what the
    original body returns for the same window (re-run on each), and the
    energies liblqr ends with are bit-identical to the GPU map of the carved
    image; without it only the build is served."""
    img = load_input("natural_rgb_97x41.npy")
    seams = 9
    plain = resize(img, n, 0.15, 0.85, seams, use_gpu=True, hook=False, transposed=transposed)
    hooked = resize(img, n, 0.15, 0.85, seams, use_gpu=True, hook=True, transposed=transposed,
                    verify=True)
    for r in (plain, hooked):
        assert r["status"] == dctenergy.DCTE_OK
        assert within_tol(r["emap"], O.energy_map(r["px"], n, 0.15, 0.85)).all()
    # without the hook the plug-in's counters stay untouched: served = the rest
    assert plain["fallback"] == plain["callbacks"] - plain["initial"] > 0
    assert hooked["fallback"] == 0 and hooked["steps"] == seams and hooked["hook_on"] == 1
    assert hooked["served_map"] + hooked["served_band"] == hooked["callbacks"]
    assert hooked["verified"] == hooked["served_band"] > 0 and hooked["bad"] == 0
    # each band pixel read once per seam: about two reads per update callback
    assert hooked["reads"] < 4 * (hooked["callbacks"] - hooked["initial"])
    with dctenergy.Context(ngpus=1) as ctx:
        assert np.array_equal(hooked["emap"], ctx.energy_map(hooked["px"], n, 0.15, 0.85))
    print(n, transposed, "served without hook",
          (plain["callbacks"] - plain["fallback"]) / plain["callbacks"], "with hook", 1.0)


def two_flat_stripes():
    """natural frame with two flat vertical stripes of different grey: both
    interiors have E = 0, so the DP's last row ties between them, and a
    leftmost and a rightmost tie rule carve seams 40 columns apart"""
    img = load_input("natural_rgb_97x41.npy").copy()
    img[:, 14:30] = 60
    img[:, 62:78] = 200
    return img


@pytest.mark.gpu
def test_seam_hook_follows_liblqr():
    """The fake liblqr's seams are the ones the GPU search finds on the GPU
    maps of the successively carved frames: the mirror carves the same
    pixels, and the hook stays on."""
    img = load_input("natural_rgb_97x41.npy")
    r = resize(img, 8, 0.3, 0.7, 5, use_gpu=True, hook=True, verify=True)
    with dctenergy.Context(ngpus=1) as ctx:
        px = np.ascontiguousarray(img)
        for k in range(5):
            s = ctx.seam_find(ctx.energy_map(px, 8, 0.3, 0.7))
            assert np.array_equal(s, r["seams"][k])
            px = np.ascontiguousarray(np.stack([np.delete(px[y], s[y], axis=0)
                                                for y in range(px.shape[0])]))
    assert np.array_equal(px, r["px"])
    assert r["hook_on"] == 1 and r["bad"] == 0 and r["fallback"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 8, 16])
@pytest.mark.parametrize("diverge", ["perturb", "shift_row", "rightmost_ties", "repass"])
def test_seam_hook_never_serves_a_foreign_window(n, diverge):
    """liblqr departs from the mirror: its image is perturbed after the build,
    or every seam it carves differs from the mirror's by one column in one
    row, or its DP breaks ties to the right (two flat stripes tie the last
    row 40 columns apart), or its image changes after the first seam's update
    and it runs that pass again at the same width (every window of the second
    pass was checked in the first: the hook must check them again).  The hook checks each callback's whole reading
    window against the mirror's pixels before it serves, so every value it
    serves equals the original body's for that window (re-run on each: 0 off
    tolerance), the first mismatch switches it off, and the original body
    answers from there: liblqr's final energies are the reference map of its
    carved image."""
    img = two_flat_stripes() if diverge == "rightmost_ties" else load_input("natural_rgb_97x41.npy")
    seams = 6
    ref_seams = resize(img, n, 0.3, 0.7, seams, use_gpu=True, hook=True)["seams"]
    d = resize(img, n, 0.3, 0.7, seams, use_gpu=True, hook=True, diverge=diverge, verify=True)
    assert d["status"] == dctenergy.DCTE_OK
    if diverge not in ("perturb", "repass"):   # (the same seams over a different image)
        assert not np.array_equal(d["seams"], ref_seams), "the fake liblqr did not diverge"
    assert d["bad"] == 0 and d["verified"] == d["served_band"]
    assert d["hook_on"] == 0 and d["fallback"] > 0
    assert d["served_map"] + d["served_band"] + d["fallback"] == d["callbacks"]
    if diverge != "repass":    # (repass: liblqr's luma no longer comes from its bytes)
        assert within_tol(d["emap"], O.energy_map(d["px"], n, 0.3, 0.7)).all()
    if diverge == "perturb":
        assert d["steps"] == 1 and d["served_band"] == 0
    print(n, diverge, "served before the switch-off:", d["served_band"], "misses:", d["missed"])


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_original_path_without_gpu(n):
    if dctenergy.device_count() > 0:
        pytest.skip("device visible; covered by the GPU test")
    img = load_input("natural_rgb_73x59.npy")
    out, calls, status = build_emap(img, n, 0.15, 0.85, use_gpu=True)
    assert status == dctenergy.DCTE_ENODEV
    assert calls == img.shape[0] * img.shape[1]
    assert np.array_equal(out, O.energy_map(img, n, 0.15, 0.85))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_gpu_map_serves_callbacks(n):
    img = load_input("natural_rgb_97x41.npy")
    out, calls, status = build_emap(img, n, 0.15, 0.85, use_gpu=True)
    assert status == dctenergy.DCTE_OK
    assert calls == 0
    assert within_tol(out, O.energy_map(img, n, 0.15, 0.85)).all()
    # after 3 "seams": carver is narrower -> original code, exact
    out2, calls2, _ = build_emap(img, n, 0.15, 0.85, use_gpu=True, removed=3)
    assert calls2 == img.shape[0] * (img.shape[1] - 3)
    assert np.array_equal(out2, O.energy_map(np.ascontiguousarray(img[:, :-3]), n, 0.15, 0.85))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 8, 16])
def test_gpu_map_serves_transposed_carver(n):
    """Vertical resize: liblqr evaluates the energy on the transposed carver;
    the transposed map answers those callbacks."""
    img = load_input("natural_rgb_73x59.npy")
    out, calls, status = build_emap(img, n, 0.15, 0.85, use_gpu=True, transposed=True)
    assert status == dctenergy.DCTE_OK
    assert calls == 0
    ref = O.energy_map(np.ascontiguousarray(np.swapaxes(img, 0, 1)), n, 0.15, 0.85)
    assert within_tol(out, ref).all()


@pytest.mark.gpu
@pytest.mark.parametrize("n,transposed", [(8, False), (8, True), (16, False), (4, True)])
def test_carver_mirror_band_is_the_map_of_the_carved_frame(n, transposed):
    """dcte_carver (the hook's device mirror): its first map is dcte_energy_map
    of the (transposed) frame; each step removes the seam dcte_seam_find picks
    on the current map, and the band it returns holds exactly the pixels and
    the dcte_energy_map energies of the carved frame at those columns."""
    img = load_input("natural_rgb_97x41.npy")
    px = np.ascontiguousarray(np.swapaxes(img, 0, 1)) if transposed else img.copy()
    with dctenergy.Context(ngpus=1) as ctx:
        c, first = ctx.carver(img, n, 0.3, 0.7, transposed)
        assert np.array_equal(first, ctx.energy_map(px, n, 0.3, 0.7))
        H = px.shape[0]
        assert c.height == H and c.width == px.shape[1] and c.band_width == 4 * n + 4
        for _ in range(6):
            want = ctx.seam_find(ctx.energy_map(px, n, 0.3, 0.7))
            seam, x0, e, bpx = c.step()
            assert np.array_equal(seam, want)
            px = np.ascontiguousarray(np.stack([np.delete(px[y], seam[y], axis=0) for y in range(H)]))
            E = ctx.energy_map(px, n, 0.3, 0.7)
            W = px.shape[1]
            assert c.width == W
            for y in range(H):
                cols = np.minimum(x0[y] + np.arange(c.band_width), W - 1)
                assert np.array_equal(e[y], E[y, cols])
                assert np.array_equal(bpx[y], px[y, cols])
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,transposed", [(8, False), (16, False), (4, True)])
def test_exact_plugin_resize_is_the_reference(n, transposed):
    """DCTE_PLUGIN_EXACT: every value liblqr receives --
    the build from the exact map, each update from the hook's exact band --
    is the reference's own; the resize loop then carves the CPU reference
    loop's seams and ends with exactly the reference map of its image."""
    img = load_input("wilber_rgb_74x59.npy")
    fake().fake_set_plugin_flags(2)               # DCTE_PLUGIN_EXACT
    try:
        d = resize(img, n, 0.3, 0.7, 8, use_gpu=True, hook=True, transposed=transposed)
    finally:
        fake().fake_set_plugin_flags(0)
    assert d["status"] == dctenergy.DCTE_OK
    assert d["served_map"] + d["served_band"] > 0.9 * d["callbacks"]
    host = np.ascontiguousarray(np.swapaxes(img, 0, 1)) if transposed else img
    for k in range(8):
        ref_seam = O.seam_find(O.energy_map(host, n, 0.3, 0.7))
        assert np.array_equal(d["seams"][k], ref_seam), f"seam {k}"
        host = np.stack([np.delete(host[y], ref_seam[y], axis=0) for y in range(host.shape[0])])
    assert np.array_equal(d["emap"], O.energy_map(d["px"], n, 0.3, 0.7))


def _reference_resize(img, n, e, t, seams, transposed):
    """The CPU reference loop: per seam the oracle's map, its seam, the carve."""
    host = np.ascontiguousarray(np.swapaxes(img, 0, 1)) if transposed else img
    out = []
    for _ in range(seams):
        s = O.seam_find(O.energy_map(host, n, e, t))
        out.append(s)
        host = np.stack([np.delete(host[y], s[y], axis=0) for y in range(host.shape[0])])
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("n,transposed", [(8, False), (16, False), (4, True)])
def test_exact_carver_keeps_its_mode_through_fast_dialog_calls(n, transposed):
    """The mode belongs to the carver: an exact carver
    built first, then -- after its build and after every seam -- the dialog
    redraws the preview and sets up another carver in the fast mode on the
    same shared context.  The exact carver's resize loop still cuts the CPU
    reference loop's seams and ends with exactly the reference map of its
    image."""
    img = load_input("wilber_rgb_74x59.npy")
    fake().fake_set_plugin_flags(2)               # DCTE_PLUGIN_EXACT
    fake().fake_set_interleave(1)
    try:
        d = resize(img, n, 0.3, 0.7, 8, use_gpu=True, hook=True, transposed=transposed)
    finally:
        fake().fake_set_plugin_flags(0)
        fake().fake_set_interleave(0)
    assert d["status"] == dctenergy.DCTE_OK
    assert d["interleaved"] == 2 * (8 + 1)       # a fast build and a fast preview each time
    assert d["steps"] == 8 and d["hook_on"] == 1 and d["fallback"] == 0
    for k, ref_seam in enumerate(_reference_resize(img, n, 0.3, 0.7, 8, transposed)):
        assert np.array_equal(d["seams"][k], ref_seam), f"seam {k}"
    assert np.array_equal(d["emap"], O.energy_map(d["px"], n, 0.3, 0.7))


@pytest.mark.gpu
def test_carver_mode_is_captured_at_create():
    """ABI level: a dcte_carver created in the exact mode keeps computing its
    band energies in it after the context is switched to the fast mode (and
    a fast carver stays fast after the context is switched to exact)."""
    img = load_input("wilber_rgb_74x59.npy")
    with dctenergy.Context(ngpus=1, exact=True) as ctx:
        c, first = ctx.carver(img, 8, 0.3, 0.7)
        ctx.set_option(dctenergy.DCTE_OPT_EXACT, 0)
        fast_map = ctx.energy_map(img, 8, 0.3, 0.7)     # a fast call in between
        assert np.array_equal(first, O.energy_map(img, 8, 0.3, 0.7))
        px = img.copy()
        for _ in range(5):
            seam, x0, e, bpx = c.step()
            px = np.ascontiguousarray(np.stack([np.delete(px[y], seam[y], axis=0)
                                                for y in range(px.shape[0])]))
            ref = O.energy_map(px, 8, 0.3, 0.7)
            W = px.shape[1]
            for y in range(px.shape[0]):
                cols = np.minimum(x0[y] + np.arange(c.band_width), W - 1)
                assert np.array_equal(e[y], ref[y, cols])
        c.close()
        assert within_tol(fast_map, O.energy_map(img, 8, 0.3, 0.7)).all()


@pytest.mark.gpu
def test_plugin_preview_is_the_golden_layer():
    """dcte_plugin_preview_u8 through the patched dct_energy_preview: every
    golden preview layer (tests/golden, from the reference's transforms) --
    bit-identical with DCTE_PLUGIN_EXACT, within +-1 in the fast mode."""
    entries = manifest()["preview"]
    assert entries
    for entry in entries:
        img = load_input(entry["input"])
        want = load_map(entry["output_u8"])
        if entry["channels"] != (1 if img.ndim == 2 else img.shape[2]):
            continue
        got, st = preview(img, entry["N"], entry["edges"], entry["textures"], flags=2)
        assert st == dctenergy.DCTE_OK
        assert np.array_equal(got, want), entry["output_u8"]
        got, st = preview(img, entry["N"], entry["edges"], entry["textures"], flags=0)
        assert st == dctenergy.DCTE_OK
        assert np.abs(got.astype(int) - want.astype(int)).max() <= 1, entry["output_u8"]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_plugin_preview_rectangle(n):
    """A preview rectangle inside a larger drawable: the region-relative
    clamp of src/render.c:456-468 (the rectangle's own rows and columns)."""
    img = load_input("natural_rgb_97x41.npy")
    rect = (13, 7, 61, 29)
    x1, y1, w, h = rect
    region = np.ascontiguousarray(img[y1:y1 + h, x1:x1 + w])
    want = O.normalize_preview(O.preview_map(region, n, 0.3, 0.7), channels=3)
    got, st = preview(img, n, 0.3, 0.7, flags=2, rect=rect)
    assert st == dctenergy.DCTE_OK
    assert np.array_equal(got, want)


def test_plugin_preview_without_gpu():
    """CPU: no device -> the glue reports it and the original loop draws the
    layer: the golden preview layers exactly."""
    if dctenergy.device_count() > 0:
        pytest.skip("device visible; covered by the GPU test")
    for entry in manifest()["preview"]:
        img = load_input(entry["input"])
        if entry["channels"] != (1 if img.ndim == 2 else img.shape[2]):
            continue
        got, st = preview(img, entry["N"], entry["edges"], entry["textures"], flags=2)
        assert st == dctenergy.DCTE_ENODEV
        assert np.array_equal(got, load_map(entry["output_u8"])), entry["output_u8"]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 8])
def test_seam_hook_repass_on_one_row(n):
    """A re-pass that starts on the previous callback's row: on a
    1-row frame every pass is one row, so only the column order tells a new
    pass; the hook must re-check and, liblqr's image having changed, switch
    itself off without serving a foreign value."""
    img = np.ascontiguousarray(load_input("natural_rgb_97x41.npy")[20:21])
    d = resize(img, n, 0.3, 0.7, 4, use_gpu=True, hook=True, diverge="repass", verify=True)
    assert d["status"] == dctenergy.DCTE_OK
    assert d["bad"] == 0 and d["verified"] == d["served_band"]
    assert d["hook_on"] == 0 and d["fallback"] > 0
