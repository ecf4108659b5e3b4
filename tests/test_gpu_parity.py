"""GPU parity: libdctenergy_hip.so (through its C ABI) against the oracle.

Bar (BASELINE.json north_star): |E_gpu - E_ref| <= 1e-5 |E_ref| + 1e-9 for
every pixel, on the committed golden fixtures (the reference's own
transforms), on BASELINE configs 2 (4096^2 RGB, N=8) and 5 (8192^2 RGB,
N=16, sampled rows), and at 16384^2 through size-independent properties
(row-band composition is bit-exact, sampled rows match the oracle).
"""
import os

import numpy as np
import pytest

import dctenergy
import emu_py as EM
import oracle_py as O
from golden_util import ATOL, RTOL, load_input, load_map, manifest, within_tol

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)


def _assert_tol(got, ref, what=""):
    ok = within_tol(got, ref)
    if not ok.all():
        bad = np.argwhere(~ok)[:5]
        raise AssertionError(f"{what}: {int((~ok).sum())} pixels off tolerance; first "
                             f"{[(tuple(b), float(got[tuple(b)]), float(ref[tuple(b)])) for b in bad]}")


@pytest.mark.parametrize("entry", manifest()["maps"], ids=lambda e: e["output"])
def test_golden_maps(ctx, entry):
    img = load_input(entry["input"])
    ref = load_map(entry["output"])
    got = ctx.energy_map(img, entry["N"], entry["edges"], entry["textures"])
    _assert_tol(got, ref, entry["output"])


def test_refine_everything_is_bit_exact():
    """tie_tau >= 1 routes every pixel through the fp64 path, which follows the
    reference's operation order: the result must be bit-identical."""
    with dctenergy.Context(ngpus=1, tie_tau=1.0) as c:
        for entry in manifest()["maps"]:
            img = load_input(entry["input"])
            got = c.energy_map(img, entry["N"], entry["edges"], entry["textures"])
            assert np.array_equal(got, load_map(entry["output"])), entry["output"]
            assert c.last_refined == img.shape[0] * img.shape[1]


def test_fast_path_equals_host_emulation():
    """With refinement off, the device result is bit-identical to the host
    emulation of the same fp32 arithmetic (tests/emu)."""
    rng = np.random.default_rng(2)
    imgs = [load_input("natural_rgb_97x41.npy"), load_input("grey512.npy")[:200, :300],
            rng.integers(0, 256, (70, 301, 3), dtype=np.uint8)]
    with dctenergy.Context(ngpus=1, tie_tau=0.0) as c:
        for img in imgs:
            for n in (2, 4, 8, 16):
                got = c.energy_map(img, n, 0.3, 0.7)
                E, _, _ = EM.energy_map(img, n, 0.3, 0.7)
                assert np.array_equal(got, E), (img.shape, n)


@pytest.mark.parametrize("n", [2, 4, 8, 16])
@pytest.mark.parametrize("shape", [(1, 1), (1, 300), (300, 1), (2, 3), (5, 7), (17, 255),
                                   (33, 256), (9, 257), (130, 129), (129, 513), (260, 700)])
def test_shapes_and_borders(ctx, n, shape):
    rng = np.random.default_rng(hash((n,) + shape) & 0xFFFF)
    for bpp in (1, 3):
        img = rng.integers(0, 256, shape + ((bpp,) if bpp == 3 else ()), dtype=np.uint8)
        ref = O.energy_map(img, n, 0.15, 0.85, nthreads=NTHREADS)
        _assert_tol(ctx.energy_map(img, n, 0.15, 0.85), ref, f"{shape} bpp={bpp}")


def test_strided_rows(ctx):
    """rowstride > w*bpp (a sub-rectangle of a larger buffer)."""
    big = load_input("natural_rgb_73x59.npy")
    pad = np.zeros((59, 80, 3), np.uint8)
    pad[:, :73] = big
    view = pad[:, :73]
    assert view.strides[0] == 240
    got = ctx.energy_map(view, 8, 0.15, 0.85)
    _assert_tol(got, O.energy_map(big, 8, 0.15, 0.85), "strided")


def test_bad_arguments(ctx):
    img = np.zeros((16, 16, 3), np.uint8)
    for n in (0, 3, 5, 32):
        with pytest.raises(dctenergy.DcteError) as ei:
            ctx.energy_map(img, n)
        assert ei.value.code == dctenergy.DCTE_EINVAL
    with pytest.raises(dctenergy.DcteError) as ei:
        ctx.energy_map(np.zeros((16, 16, 2), np.uint8), 8)
    assert ei.value.code == dctenergy.DCTE_EINVAL
    with pytest.raises(dctenergy.DcteError) as ei:
        ctx.energy_map(img, 8, semantics=7)
    assert ei.value.code == dctenergy.DCTE_EINVAL


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no device")
    return torch


def test_config2_4096_rgb_n8(ctx):
    """BASELINE config 2: 4096^2 RGB, 8x8, full-frame tolerance vs the oracle."""
    torch = _torch()
    from dctenergy import synth
    frame = synth.natural_rows(0, 4096, 4096, 3, seed=1, device="cuda")
    out = torch.empty((4096, 4096), dtype=torch.float32, device="cuda")
    for e, t in ((0.5, 0.5), (0.3, 0.7)):
        ctx.energy_map_tensor(frame, out, 8, e, t)
        torch.cuda.synchronize()
        ref = O.energy_map(frame.cpu().numpy(), 8, e, t, nthreads=NTHREADS)
        _assert_tol(out.cpu().numpy(), ref, f"4096^2 e={e} t={t}")


def test_device_bands_compose_bit_exact(ctx):
    """Row bands with halos (the multi-GPU decomposition) == the full frame."""
    torch = _torch()
    from dctenergy import synth
    H, W = 1000, 777
    frame = synth.natural_rows(0, H, W, 3, seed=4, device="cuda")
    for n in (2, 4, 8, 16):
        full = torch.empty((H, W), dtype=torch.float32, device="cuda")
        ctx.energy_map_tensor(frame, full, n, 0.3, 0.7)
        parts = torch.full((H, W), -1.0, dtype=torch.float32, device="cuda")
        r = n // 2
        cuts = [0, 1, 2, 130, 131, 512, 999, 1000]
        for a, b in zip(cuts[:-1], cuts[1:]):
            lo, hi = max(0, a - (r - 1)), min(H - 1, b - 1 + r)
            band = frame[lo:hi + 1].clone()       # only band + halo is readable
            ctx.energy_map_tensor(band, parts[a:b], n, 0.3, 0.7, h=H, in_row0=lo, y0=a, y1=b)
        torch.cuda.synchronize()
        assert torch.equal(full, parts), n


def test_16384_rgb_properties(ctx):
    """BASELINE config 3 (16384^2 RGB, N=8) at full size: sampled rows equal the
    oracle within tolerance and four row bands reproduce the full frame."""
    torch = _torch()
    from dctenergy import synth
    H = W = 16384
    frame = synth.natural_rows(0, H, W, 3, seed=0, device="cuda")
    out = torch.empty((H, W), dtype=torch.float32, device="cuda")
    ctx.energy_map_tensor(frame, out, 8, 0.3, 0.7)
    torch.cuda.synchronize()
    rows = [0, 1, 2, 3, 4, 5000, 8191, 8192, 12345, H - 5, H - 4, H - 3, H - 2, H - 1]
    host = {}
    for y in rows:
        lo, hi = max(0, y - 3), min(H - 1, y + 4)
        host[y] = frame[lo:hi + 1].cpu().numpy()
    for y in rows:
        lo = max(0, y - 3)
        sub = host[y]
        # oracle on the clamped strip: pad the strip so row y keeps its window
        ref = _oracle_row(sub, lo, y, H, 8, 0.3, 0.7)
        _assert_tol(out[y].cpu().numpy()[None], ref[None], f"row {y}")
    parts = torch.empty_like(out)
    for k in range(4):
        a, b = H * k // 4, H * (k + 1) // 4
        lo, hi = max(0, a - 3), min(H - 1, b + 3)
        ctx.energy_map_tensor(frame[lo:hi + 1], parts[a:b], 8, 0.3, 0.7, h=H, in_row0=lo, y0=a, y1=b)
    torch.cuda.synchronize()
    assert torch.equal(out, parts)
    del frame, out, parts
    torch.cuda.empty_cache()


def _oracle_row(strip, lo, y, H, n, e, t):
    """Oracle value of global row y from the rows [lo, lo + len(strip)) around it:
    rebuild the exact clamped window rows as a small image."""
    r = n // 2
    rows = [min(max(y + j, 0), H - 1) - lo for j in range(-(r - 1), r + 1)]
    img = np.stack([strip[i] for i in rows])       # N rows, window row order
    # in a frame of exactly these N rows, row r-1 sees the same window rows
    return O.energy_map(img, n, e, t, y0=r - 1, y1=r, nthreads=1)[0]


def test_config5_8192_rgb_n16_sampled(ctx):
    """BASELINE config 5 (8192^2 RGB, N=16): sampled rows vs the oracle."""
    torch = _torch()
    from dctenergy import synth
    H = W = 8192
    frame = synth.natural_rows(0, H, W, 3, seed=5, device="cuda")
    out = torch.empty((H, W), dtype=torch.float32, device="cuda")
    ctx.energy_map_tensor(frame, out, 16, 0.3, 0.7)
    torch.cuda.synchronize()
    for y in (0, 3, 7, 8, 4097, H - 9, H - 8, H - 1):
        lo, hi = max(0, y - 7), min(H - 1, y + 8)
        ref = _oracle_row(frame[lo:hi + 1].cpu().numpy(), lo, y, H, 16, 0.3, 0.7)
        _assert_tol(out[y].cpu().numpy()[None], ref[None], f"row {y}")
    del frame, out
    torch.cuda.empty_cache()


def test_ties_are_refined_to_reference(ctx):
    """Images full of exact edge/texture ties (isolated pixels on flat ground)
    match the reference bit-exactly where the class is decided by rounding."""
    rng = np.random.default_rng(9)
    for img in ((np.full((64, 64), 254) + (rng.random((64, 64)) < 0.03)).astype(np.uint8),
                (rng.random((64, 64)) < 0.03).astype(np.uint8)):
        for n in (4, 8, 16):
            ref = O.energy_map(img, n, 0.3, 0.7)
            got = ctx.energy_map(img, n, 0.3, 0.7)
            _assert_tol(got, ref, f"ties n={n}")
            # the device flags exactly the pixels the emulated fp32 path puts
            # inside the refinement band
            _, me, mt = EM.energy_map(img, n, 0.3, 0.7)
            assert ctx.last_refined == int(EM.refine_mask(me, mt, 0.3, 0.7).sum())
            if n < 16:
                assert ctx.last_refined > 0


@pytest.mark.parametrize("channels", [1, 3])
def test_normalize_u8(ctx, channels):
    """energy map -> 8-bit image, both modes, vs numpy restatements."""
    for entry in manifest()["maps"][:12]:
        E = load_map(entry["output"])
        got = ctx.normalize_u8(E, dctenergy.DCTE_NORM_PREVIEW, channels)
        assert np.array_equal(got, O.normalize_preview(E, channels)), entry["output"]
        got = ctx.normalize_u8(E, dctenergy.DCTE_NORM_LQR, channels)
        assert np.array_equal(got, O.normalize_lqr(E, channels)), entry["output"]
    flat = np.full((7, 9), 0.25, np.float32)
    assert not ctx.normalize_u8(flat, dctenergy.DCTE_NORM_PREVIEW).any()


def test_energy_image_u8_fused(ctx):
    img = load_input("natural_rgb_97x41.npy")
    E = ctx.energy_map(img, 8, 0.3, 0.7)
    u8 = ctx.energy_image_u8(img, 8, 0.3, 0.7, dctenergy.DCTE_NORM_LQR, 1)
    assert np.array_equal(u8, O.normalize_lqr(E))
    u8p = ctx.energy_image_u8(img, 8, 0.3, 0.7, dctenergy.DCTE_NORM_PREVIEW, 3)
    assert np.array_equal(u8p, O.normalize_preview(E, 3))


@pytest.mark.parametrize("entry", manifest()["preview"], ids=lambda e: e["output"])
def test_preview_golden(ctx, entry):
    """Preview semantics (src/render.c:31-109) on the GPU: float energies within
    tolerance, the u8 image equal to normalize_image of them."""
    img = load_input(entry["input"])
    E = ctx.energy_map(img, entry["N"], entry["edges"], entry["textures"],
                       semantics=dctenergy.DCTE_PREVIEW)
    _assert_tol(E, load_map(entry["output"]), entry["output"])
    u8 = ctx.energy_image_u8(img, entry["N"], entry["edges"], entry["textures"],
                             dctenergy.DCTE_NORM_PREVIEW, entry["channels"],
                             semantics=dctenergy.DCTE_PREVIEW)
    assert np.array_equal(u8, O.normalize_preview(E, entry["channels"]))
    gold = load_map(entry["output_u8"]).astype(np.int16)
    assert np.abs(u8.astype(np.int16) - gold).max() <= 1


def test_preview_refine_everything_is_bit_exact():
    with dctenergy.Context(ngpus=1, tie_tau=1.0) as c:
        for entry in manifest()["preview"]:
            img = load_input(entry["input"])
            got = c.energy_map(img, entry["N"], entry["edges"], entry["textures"],
                               semantics=dctenergy.DCTE_PREVIEW)
            assert np.array_equal(got, load_map(entry["output"])), entry["output"]


def test_preview_fast_path_equals_emulation():
    rng = np.random.default_rng(8)
    imgs = [load_input("rgba_45x38.npy"), rng.integers(0, 256, (70, 301, 3), dtype=np.uint8),
            rng.integers(0, 256, (33, 257), dtype=np.uint8)]
    with dctenergy.Context(ngpus=1, tie_tau=0.0) as c:
        for img in imgs:
            for n in (2, 4, 8, 16):
                got = c.energy_map(img, n, 0.3, 0.7, semantics=dctenergy.DCTE_PREVIEW)
                E, _, _ = EM.energy_map(img, n, 0.3, 0.7, sem=1)
                assert np.array_equal(got, E), (img.shape, n)


def test_preview_rejects_two_channels(ctx):
    with pytest.raises(dctenergy.DcteError) as ei:
        ctx.energy_map(np.zeros((8, 8, 2), np.uint8), 8, semantics=dctenergy.DCTE_PREVIEW)
    assert ei.value.code == dctenergy.DCTE_EINVAL


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_transposed_map(ctx, n):
    """transposed=1 is the map of the transposed frame (vertical carving)."""
    for name in ("natural_rgb_73x59.npy", "natural_grey_200x120.npy", "tiny_rgb_5x1.npy"):
        img = load_input(name)
        tr = np.ascontiguousarray(np.swapaxes(img, 0, 1))
        h, w = img.shape[:2]
        out = np.empty((w, h), np.float32)
        got = ctx.energy_map(img, n, 0.15, 0.85, transposed=True, out=out)
        assert np.array_equal(got, ctx.energy_map(tr, n, 0.15, 0.85)), name
        _assert_tol(got, O.energy_map(tr, n, 0.15, 0.85), name)


def test_sharded_energy_image_u8_single_rank(ctx):
    """dist.energy_image_u8 (band min/max -> all-reduce -> normalise) on one
    rank equals the fused host entry point; the multi-rank reduction and the
    band gather are covered with gloo in test_dist_gloo.py."""
    torch = _torch()
    from dctenergy import dist as D
    img = load_input("natural_rgb_97x41.npy")
    frame = torch.from_numpy(img).cuda()
    E = torch.empty(img.shape[:2], dtype=torch.float32, device="cuda")
    ctx.energy_map_tensor(frame, E, 8, 0.3, 0.7)
    for mode, ch in ((dctenergy.DCTE_NORM_LQR, 1), (dctenergy.DCTE_NORM_PREVIEW, 3)):
        out = torch.empty(img.shape[:2] + ((ch,) if ch > 1 else ()), dtype=torch.uint8,
                          device="cuda")
        D.energy_image_u8(ctx, E, out, mode, ch)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ctx.energy_image_u8(img, 8, 0.3, 0.7, mode, ch))
