"""DCTE_OPT_EXACT: the map bit-identical to the reference for every pixel.

The exact mode computes the reference's own fp64 arithmetic (ddct8x8s /
ddct16x16s / ddct2d in their operation order, src/fft2d/shrtdct.c,
src/fft2d/fftsg2d.c; the last-maximum scan, src/dct.c:96-110) in a sliding
window (dcte_exact.hip), so the bar here is np.array_equal against the oracle
(itself pinned bit-exactly to oracle/_ref, the reference's own transforms) --
not a tolerance.  Covered: every golden map, borders and odd shapes, strided
rows, row bands and two-range launches, BASELINE configs 2, 3 and 5 over every
pixel, tie-dense frames (line art, dots, an 8-px grid: exact edge/texture ties
decided only by the reference's rounding), and the carve loop (liblqr's DP on
the exact map cuts the reference's seams); the preview semantics through
their own kernels (golden maps and u8 layers, shapes, strides, tile heights,
bands, tie-dense and 4096^2 frames); the multi-device host path.
"""
import os

import numpy as np
import pytest

import dctenergy
import oracle_py as O
from golden_util import load_input, load_map, manifest
from seam_util import carve

pytestmark = pytest.mark.gpu

NTHREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def ex():
    if dctenergy.device_count() == 0:
        pytest.skip("no device")
    with dctenergy.Context(ngpus=1, exact=True) as c:
        yield c


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no device")
    return torch


def _equal_dev(got_dev, ref, what):
    """every pixel bit-identical (compared on the device in row chunks)"""
    torch = _torch()
    bad = 0
    first = None
    for a in range(0, ref.shape[0], 2048):
        r = torch.from_numpy(np.ascontiguousarray(ref[a:a + 2048])).to(got_dev.device)
        g = got_dev[a:a + 2048]
        ne = g.view(torch.int32) != r.view(torch.int32)
        k = int(ne.sum())
        if k and first is None:
            yx = torch.nonzero(ne)[0].tolist()
            first = (a + yx[0], yx[1], float(g[yx[0], yx[1]]), float(r[yx[0], yx[1]]))
        bad += k
    print({"frame": what, "pixels": int(ref.size), "not_bit_identical": bad})
    assert bad == 0, f"{what}: {bad} pixels differ, first {first}"


def test_exact_golden_maps(ex):
    for entry in manifest()["maps"]:
        img = load_input(entry["input"])
        got = ex.energy_map(img, entry["N"], entry["edges"], entry["textures"])
        assert np.array_equal(got, load_map(entry["output"])), entry["output"]


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_exact_shapes_and_borders(ex, n):
    shapes = [(1, 1), (1, 300), (300, 1), (2, 3), (5, 7), (8, 8), (17, 255), (33, 256),
              (9, 257), (130, 129), (129, 513), (260, 700)]
    for shape in shapes:
        rng = np.random.default_rng(hash((n,) + shape) & 0xFFFF)
        for bpp in (1, 3):
            img = rng.integers(0, 256, shape + ((bpp,) if bpp == 3 else ()), dtype=np.uint8)
            for e, t in ((0.15, 0.85), (0.5, 0.5)):
                ref = O.energy_map(img, n, e, t, nthreads=NTHREADS)
                got = ex.energy_map(img, n, e, t)
                assert np.array_equal(got, ref), (shape, bpp, e, t)


def test_exact_strided_rows(ex):
    big = load_input("natural_rgb_73x59.npy")
    pad = np.zeros((59, 80, 3), np.uint8)
    pad[:, :73] = big
    for n in (2, 4, 8, 16):
        assert np.array_equal(ex.energy_map(pad[:, :73], n, 0.15, 0.85),
                              O.energy_map(big, n, 0.15, 0.85)), n


def test_exact_tile_heights(ex):
    """DCTE_OPT_TILE_H only re-partitions the work."""
    img = load_input("natural_rgb_97x41.npy")
    ref = {n: O.energy_map(img, n, 0.3, 0.7) for n in (2, 4, 8, 16)}
    try:
        for th in (1, 2, 7, 8, 9, 33, 64):
            ex.set_option(dctenergy.DCTE_OPT_TILE_H, th)
            for n in (2, 4, 8, 16):
                assert np.array_equal(ex.energy_map(img, n, 0.3, 0.7), ref[n]), (th, n)
    finally:
        ex.set_option(dctenergy.DCTE_OPT_TILE_H, 0)


def _tie_frames(S, rng):
    yy, xx = np.mgrid[0:S, 0:S]
    line = np.where((yy % 23 == 0) | (xx % 31 == 0) | ((xx + 2 * yy) % 97 == 0), 0, 255).astype(np.uint8)
    grid = np.where((yy % 8 == 0) | (xx % 8 == 0), 0, 255).astype(np.uint8)
    ink = np.array([[20, 40, 200], [200, 30, 30], [0, 0, 0]], np.uint8)
    strokes = np.full((S, S, 3), 255, np.uint8)
    for k in range(3):
        m = ((xx + (k + 1) * yy) % (41 + 6 * k)) == 0
        strokes[m] = ink[k]
    return {
        "lineart_grey": line,
        "lineart_rgb": np.repeat(line[..., None], 3, -1),
        "strokes_rgb": strokes,
        "grid8_grey": grid,
        "dots_rgb": np.repeat(np.where(rng.random((S, S)) < 1 / 64, 255, 16).astype(np.uint8)[..., None], 3, -1),
        "uniform_rgb": rng.integers(0, 256, (S, S, 3), dtype=np.uint8),
    }


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_exact_tie_dense_frames(ex, n):
    """Frames full of exact edge/texture ties: every pixel bit-identical."""
    torch = _torch()
    S = 2048 if n == 8 else 1024
    rng = np.random.default_rng(40 + n)
    for name, img in _tie_frames(S, rng).items():
        got = torch.from_numpy(ex.energy_map(img, n, 0.3, 0.7)).cuda()
        _equal_dev(got, O.energy_map(img, n, 0.3, 0.7, nthreads=NTHREADS), f"{name} {S}^2 N={n}")


def test_exact_bands_and_two_range_launch(ex):
    """Row bands with halos and the two-range launch == the full exact map."""
    torch = _torch()
    from dctenergy import synth
    H, W = 700, 517
    frame = synth.natural_rows(0, H, W, 3, seed=9, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for n in (2, 4, 8, 16):
        full = torch.empty((H, W), dtype=torch.float32, device="cuda")
        ex.energy_map_tensor(frame, full, n, 0.3, 0.7)
        torch.cuda.synchronize()
        assert np.array_equal(full.cpu().numpy(), O.energy_map(frame.cpu().numpy(), n, 0.3, 0.7,
                                                                nthreads=NTHREADS)), n
        parts = torch.full((H, W), -1.0, dtype=torch.float32, device="cuda")
        r = n // 2
        cuts = [0, 1, 2, 130, 131, 512, 699, 700]
        for a, b in zip(cuts[:-1], cuts[1:]):
            lo, hi = max(0, a - (r - 1)), min(H - 1, b - 1 + r)
            band = frame[lo:hi + 1].clone()
            ex.energy_map_tensor(band, parts[a:b], n, 0.3, 0.7, h=H, in_row0=lo, y0=a, y1=b)
        torch.cuda.synchronize()
        assert torch.equal(full, parts), n
        for a0, a1, b0, b1 in [(0, 3, 696, 700), (100, 104, 300, 303), (10, 150, 200, 480), (5, 9, 9, 9)]:
            got = torch.full((H, W), -1.0, dtype=torch.float32, device="cuda")
            ex.energy_map_device2(frame.data_ptr(), frame.stride(0), W, H, 3, 0, H, a0, a1, b0, b1, n,
                                  0.3, 0.7, got[a0:].data_ptr(), got.stride(0), st)
            torch.cuda.synchronize()
            want = torch.full((H, W), -1.0, dtype=torch.float32, device="cuda")
            want[a0:a1] = full[a0:a1]
            want[b0:b1] = full[b0:b1]
            assert torch.equal(got, want), (n, (a0, a1, b0, b1))


def _full_frame(ex, S, n, seed):
    torch = _torch()
    from dctenergy import synth
    frame = synth.natural_rows(0, S, S, 3, seed=seed, device="cuda")
    out = torch.empty((S, S), dtype=torch.float32, device="cuda")
    ex.energy_map_tensor(frame, out, n, 0.3, 0.7)
    torch.cuda.synchronize()
    host = frame.cpu().numpy()
    del frame
    ref = O.energy_map(host, n, 0.3, 0.7, nthreads=NTHREADS)
    del host
    _equal_dev(out, ref, f"{S}^2 RGB N={n}")
    del out, ref
    torch.cuda.empty_cache()


def test_exact_config2_4096_rgb_n8(ex):
    _full_frame(ex, 4096, 8, 1)


def test_exact_config3_16384_rgb_n8(ex):
    _full_frame(ex, 16384, 8, 0)


def test_exact_config5_8192_rgb_n16(ex):
    _full_frame(ex, 8192, 16, 5)


@pytest.mark.parametrize("n", [4, 8, 16])
def test_exact_carve_equals_cpu_reference_loop(ex, n):
    """liblqr's DP on exact maps (the map, then every seam-band update) cuts
    the CPU loop's seams on the reference's arithmetic, step for step."""
    img = load_input("wilber_rgb_74x59.npy")
    out, cols = ex.carve(img, 10, n, 0.3, 0.7)
    host = img
    for k in range(10):
        ref_seam = O.seam_find(O.energy_map(host, n, 0.3, 0.7))
        assert np.array_equal(cols[k], ref_seam), f"seam {k}"
        host = carve(host, ref_seam)
    assert np.array_equal(out, host)


def test_exact_profile_and_injected_failure(ex):
    """Profiling events bracket the exact launch; a launch reported failed
    after it was queued leaves the context usable."""
    img = load_input("natural_rgb_97x41.npy")
    ref = O.energy_map(img, 8, 0.3, 0.7)
    ex.set_option(dctenergy.DCTE_OPT_PROFILE, 1)
    try:
        ex.profile_read()
        assert np.array_equal(ex.energy_map(img, 8, 0.3, 0.7), ref)
        launches, ms = ex.profile_read()
        assert launches >= 1 and ms > 0
    finally:
        ex.set_option(dctenergy.DCTE_OPT_PROFILE, 0)
    ex.set_option(dctenergy.DCTE_OPT_FAIL_INJECT, 1)
    with pytest.raises(dctenergy.DcteError) as ei:
        ex.energy_map(img, 8, 0.3, 0.7)
    assert ei.value.code == dctenergy.DCTE_EHIP
    assert np.array_equal(ex.energy_map(img, 8, 0.3, 0.7), ref)


def test_exact_off_again_is_the_fast_map(ex):
    """The option switches back: exact off gives the fp32 map (within 1e-5)."""
    img = load_input("natural_rgb_97x41.npy")
    with dctenergy.Context(ngpus=1) as fast:
        f = fast.energy_map(img, 8, 0.3, 0.7)
    ex.set_option(dctenergy.DCTE_OPT_EXACT, 0)
    try:
        assert np.array_equal(ex.energy_map(img, 8, 0.3, 0.7), f)
    finally:
        ex.set_option(dctenergy.DCTE_OPT_EXACT, 1)


def test_exact_preview_maps_and_u8_layers(ex):
    """Preview semantics in the exact mode (dcte_exact_pv / dcte_exact_pvs):
    the maps AND the drawn u8 layers equal the reference's golden ones
    exactly (the fast mode's u8 layer is within +-1)."""
    for entry in manifest()["preview"]:
        img = load_input(entry["input"])
        E = ex.energy_map(img, entry["N"], entry["edges"], entry["textures"],
                          semantics=dctenergy.DCTE_PREVIEW)
        assert np.array_equal(E, load_map(entry["output"])), entry["output"]
        u8 = ex.energy_image_u8(img, entry["N"], entry["edges"], entry["textures"],
                                dctenergy.DCTE_NORM_PREVIEW, entry["channels"],
                                semantics=dctenergy.DCTE_PREVIEW)
        assert np.array_equal(u8, load_map(entry["output_u8"])), entry["output_u8"]


def test_exact_energy_layer_and_points(ex):
    """The u8 energy layer (display_carver_energy) and point energies in the
    exact mode are the reference's: the layer is normalize_lqr of the oracle
    map, the points its values."""
    img = load_input("natural_rgb_97x41.npy")
    for n in (2, 4, 8, 16):
        ref = O.energy_map(img, n, 0.3, 0.7)
        u8 = ex.energy_image_u8(img, n, 0.3, 0.7, dctenergy.DCTE_NORM_LQR, 1)
        assert np.array_equal(u8, O.normalize_lqr(ref)), n
        rng = np.random.default_rng(n)
        xy = np.stack([rng.integers(0, img.shape[1], 200), rng.integers(0, img.shape[0], 200)], 1)
        got = ex.energy_points(img, xy.astype(np.int32), n, 0.3, 0.7)
        assert np.array_equal(got, ref[xy[:, 1], xy[:, 0]]), n


PV = dctenergy.DCTE_PREVIEW


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_exact_preview_shapes_and_borders(ex, n):
    """The preview window (offsets -(c - 1) .. N - c, data[dy][dx], u8 luma)
    through the preview's sliding kernels: ragged shapes from 1 x 1 up, grey,
    RGB and RGBA, both weightings -- every pixel bit-identical."""
    shapes = [(1, 1), (1, 300), (300, 1), (2, 3), (5, 7), (8, 8), (17, 255), (33, 256),
              (9, 257), (130, 129), (129, 513), (260, 700)]
    for shape in shapes:
        rng = np.random.default_rng(hash((n, 7) + shape) & 0xFFFF)
        for bpp in (1, 3, 4):
            img = rng.integers(0, 256, shape + ((bpp,) if bpp > 1 else ()), dtype=np.uint8)
            for e, t in ((0.15, 0.85), (0.5, 0.5)):
                ref = O.preview_map(img, n, e, t, nthreads=NTHREADS)
                got = ex.energy_map(img, n, e, t, semantics=PV)
                assert np.array_equal(got, ref), (shape, bpp, e, t)


def test_exact_preview_tile_heights_and_strides(ex):
    img = load_input("natural_rgb_97x41.npy")
    pad = np.zeros((41, 110, 3), np.uint8)
    pad[:, :97] = img
    ref = {n: O.preview_map(img, n, 0.3, 0.7) for n in (2, 4, 8, 16)}
    for n in (2, 4, 8, 16):
        assert np.array_equal(ex.energy_map(pad[:, :97], n, 0.3, 0.7, semantics=PV), ref[n]), n
    try:
        for th in (1, 2, 7, 8, 9, 33, 64):
            ex.set_option(dctenergy.DCTE_OPT_TILE_H, th)
            for n in (2, 4, 8, 16):
                assert np.array_equal(ex.energy_map(img, n, 0.3, 0.7, semantics=PV), ref[n]), (th, n)
    finally:
        ex.set_option(dctenergy.DCTE_OPT_TILE_H, 0)


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_exact_preview_tie_dense_frames(ex, n):
    torch = _torch()
    S = 1024
    rng = np.random.default_rng(50 + n)
    for name, img in _tie_frames(S, rng).items():
        got = torch.from_numpy(ex.energy_map(img, n, 0.3, 0.7, semantics=PV)).cuda()
        _equal_dev(got, O.preview_map(img, n, 0.3, 0.7, nthreads=NTHREADS), f"preview {name} {S}^2 N={n}")


def test_exact_preview_bands(ex):
    """Preview row bands (the preview's own halo: c - 1 rows above, N - c
    below) and a two-range launch == the full preview map."""
    torch = _torch()
    from dctenergy import synth
    H, W = 300, 517
    frame = synth.natural_rows(0, H, W, 4, seed=4, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for n in (2, 4, 8, 16):
        full = torch.empty((H, W), dtype=torch.float32, device="cuda")
        ex.energy_map_tensor(frame, full, n, 0.3, 0.7, semantics=PV)
        torch.cuda.synchronize()
        assert np.array_equal(full.cpu().numpy(), O.preview_map(frame.cpu().numpy(), n, 0.3, 0.7,
                                                                 nthreads=NTHREADS)), n
        c = (n - 1) // 2
        up, down = max(0, c - 1), max(0, n - c)
        parts = torch.full((H, W), -1.0, dtype=torch.float32, device="cuda")
        cuts = [0, 1, 2, 130, 131, 299, 300]
        for a, b in zip(cuts[:-1], cuts[1:]):
            lo, hi = max(0, a - up), min(H - 1, b - 1 + down)
            band = frame[lo:hi + 1].clone()
            ex.energy_map_tensor(band, parts[a:b], n, 0.3, 0.7, h=H, in_row0=lo, y0=a, y1=b, semantics=PV)
        torch.cuda.synchronize()
        assert torch.equal(full, parts), n
        got = torch.full((H, W), -1.0, dtype=torch.float32, device="cuda")
        ex.energy_map_device2(frame.data_ptr(), frame.stride(0), W, H, 4, 0, H, 0, 3, 296, 300, n,
                              0.3, 0.7, got.data_ptr(), got.stride(0), st, semantics=PV)
        torch.cuda.synchronize()
        want = torch.full((H, W), -1.0, dtype=torch.float32, device="cuda")
        want[0:3] = full[0:3]
        want[296:300] = full[296:300]
        assert torch.equal(got, want), n


@pytest.mark.parametrize("n,S", [(8, 4096), (16, 4096), (4, 4096), (2, 4096)])
def test_exact_preview_full_frames(ex, n, S):
    torch = _torch()
    from dctenergy import synth
    frame = synth.natural_rows(0, S, S, 3, seed=n, device="cuda")
    out = torch.empty((S, S), dtype=torch.float32, device="cuda")
    ex.energy_map_tensor(frame, out, n, 0.3, 0.7, semantics=PV)
    torch.cuda.synchronize()
    ref = O.preview_map(frame.cpu().numpy(), n, 0.3, 0.7, nthreads=NTHREADS)
    _equal_dev(out, ref, f"preview {S}^2 RGB N={n}")


@pytest.mark.parametrize("G", [2, 3])
def test_exact_multi_device_host_path(G):
    """The single-process multi-device host path (band split, halo rows, the
    per-device chunk pipelines, transposed strips) in the exact mode: every
    pixel the reference's, for both semantics."""
    if dctenergy.device_count() == 0:
        pytest.skip("no device")
    rng = np.random.default_rng(G)
    img = rng.integers(0, 256, (2100, 301, 3), dtype=np.uint8)
    img[:, 100:200] //= 7
    with dctenergy.Context(ngpus=G, same_device=True, exact=True) as many:
        for n in (2, 8, 16):
            assert np.array_equal(many.energy_map(img, n, 0.3, 0.7),
                                  O.energy_map(img, n, 0.3, 0.7, nthreads=NTHREADS)), n
            assert np.array_equal(many.energy_map(img[:700], n, 0.3, 0.7, transposed=True),
                                  O.energy_map(np.ascontiguousarray(np.swapaxes(img[:700], 0, 1)), n, 0.3, 0.7,
                                               nthreads=NTHREADS)), n
            assert np.array_equal(many.energy_map(img, n, 0.3, 0.7, semantics=PV),
                                  O.preview_map(img, n, 0.3, 0.7, nthreads=NTHREADS)), n
