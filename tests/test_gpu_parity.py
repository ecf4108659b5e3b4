"""GPU parity: libdctenergy_hip.so (through its C ABI) against the oracle.

Bar (BASELINE.json north_star): |E_gpu - E_ref| <= 1e-5 |E_ref| + 1e-9 for
every pixel, on the committed golden fixtures (the reference's own
transforms), on BASELINE configs 2 (4096^2 RGB, N=8), 3 (16384^2 RGB,
N=8) and 5 (8192^2 RGB, N=16), through size-independent properties
(row-band composition is bit-exact) and at configs 3 and 5 over every
pixel against the OpenMP oracle, plus tie-prone stress frames.
"""
import os

import numpy as np
import pytest

import dctenergy
import emu_py as EM
import oracle_py as O
from golden_util import ATOL, RTOL, load_input, load_map, manifest, within_tol

pytestmark = pytest.mark.gpu

NTHREADS = max(1, min(16, len(os.sched_getaffinity(0))))   # the GPU box's CPU share


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


def test_two_range_launch_equals_full_map(ctx):
    """dcte_energy_map_device2 (a band's two halo-dependent edge ranges in ONE
    map launch + ONE refinement launch) writes exactly the full map's rows of
    both ranges and nothing else: natural and tie-dense (line-art, RGB and
    grey) frames, every N, both semantics, ranges from one row to more than a
    tile."""
    torch = _torch()
    from dctenergy import synth
    H, W = 600, 517
    nat = synth.natural_rows(0, H, W, 3, seed=6, device="cuda")
    yy = torch.arange(H, device="cuda").view(-1, 1)
    xx = torch.arange(W, device="cuda").view(1, -1)
    line = torch.where((yy % 23 == 0) | (xx % 31 == 0) | ((xx + 2 * yy) % 97 == 0), 0, 255)
    art = line.to(torch.uint8).unsqueeze(-1).expand(H, W, 3).contiguous()
    grey = line.to(torch.uint8).contiguous()       # grey: the N = 8 dense walk's window memo
    cases = [(0, 3, 596, 600), (100, 104, 300, 303), (0, 1, 599, 600), (10, 150, 200, 480),
             (50, 60, 60, 70), (5, 9, 9, 9)]
    for frame in (nat, art, grey):
        bpp = 1 if frame.dim() == 2 else 3
        for sem in (dctenergy.DCTE_LQR, dctenergy.DCTE_PREVIEW):
            for n in (2, 4, 8, 16):
                full = torch.empty((H, W), dtype=torch.float32, device="cuda")
                ctx.energy_map_tensor(frame, full, n, 0.3, 0.7, semantics=sem)
                for a0, a1, b0, b1 in cases:
                    got = torch.full((H, W), -1.0, dtype=torch.float32, device="cuda")
                    ctx.energy_map_device2(frame.data_ptr(), frame.stride(0), W, H, bpp, 0, H, a0, a1,
                                           b0, b1, n, 0.3, 0.7, got[a0:].data_ptr(), got.stride(0),
                                           torch.cuda.current_stream().cuda_stream, semantics=sem)
                    torch.cuda.synchronize()
                    want = torch.full((H, W), -1.0, dtype=torch.float32, device="cuda")
                    want[a0:a1] = full[a0:a1]
                    want[b0:b1] = full[b0:b1]
                    assert torch.equal(got, want), (n, sem, (a0, a1, b0, b1))


def test_two_range_launch_band_buffer(ctx):
    """The same from a band buffer holding only the rows the clamp reaches
    (what a rank holds after the halo exchange), and the error for a second
    range that overlaps the first."""
    torch = _torch()
    from dctenergy import synth
    H, W = 2048, 1031
    frame = synth.natural_rows(0, H, W, 3, seed=7, device="cuda")
    for n in (8, 16):
        r = n // 2
        full = torch.empty((H, W), dtype=torch.float32, device="cuda")
        ctx.energy_map_tensor(frame, full, n, 0.3, 0.7)
        Y0, Y1 = 512, 1024
        lo, hi = Y0 - (r - 1), Y1 - 1 + r
        band = frame[lo:hi + 1].clone()
        out = torch.full((Y1 - Y0, W), -1.0, dtype=torch.float32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        ctx.energy_map_device(band.data_ptr(), band.stride(0), W, H, 3, lo, band.shape[0],
                              Y0 + r - 1, Y1 - r, n, 0.3, 0.7, out[r - 1:].data_ptr(), out.stride(0), st)
        ctx.energy_map_device2(band.data_ptr(), band.stride(0), W, H, 3, lo, band.shape[0],
                               Y0, Y0 + r - 1, Y1 - r, Y1, n, 0.3, 0.7, out.data_ptr(), out.stride(0), st)
        torch.cuda.synchronize()
        assert torch.equal(out, full[Y0:Y1]), n
        with pytest.raises(dctenergy.DcteError) as ei:
            ctx.energy_map_device2(band.data_ptr(), band.stride(0), W, H, 3, lo, band.shape[0],
                                   Y0, Y0 + 10, Y0 + 5, Y0 + 20, n, 0.3, 0.7, out.data_ptr(),
                                   out.stride(0), st)
        assert ei.value.code == dctenergy.DCTE_EINVAL


def _compare_full(got_dev, ref, e, t, what):
    """Whole-frame comparison on the device, in row chunks: every pixel within
    the tolerance, and the class flips (a pixel whose value is the OTHER
    class's weight times its maximum: ratio e/t or t/e) counted separately.
    Returns the stats it printed."""
    torch = _torch()
    H = ref.shape[0]
    bad = flips = 0
    worst = 0.0
    lo, hi = min(e, t) / max(e, t), max(e, t) / min(e, t)
    for a in range(0, H, 2048):
        r = torch.from_numpy(ref[a:a + 2048]).to(got_dev.device, torch.float64)
        g = got_dev[a:a + 2048].to(torch.float64)
        err = (g - r).abs()
        off = err > RTOL * r.abs() + ATOL
        bad += int(off.sum())
        rel = torch.where(r.abs() > 0, err / r.abs(), err)
        worst = max(worst, float(rel.max()))
        if e != t and off.any():
            ratio = g[off] / r[off]
            flips += int((((ratio - lo).abs() < 1e-3 * lo) | ((ratio - hi).abs() < 1e-3 * hi)).sum())
    stats = {"frame": what, "pixels": int(ref.size), "off_tolerance": bad, "class_flips": flips,
             "max_rel_err": worst}
    print(stats)
    assert bad == 0 and flips == 0, stats
    return stats


def test_config3_16384_rgb_full_frame(ctx):
    """BASELINE config 3 (16384^2 RGB, N=8, e=0.3 t=0.7): EVERY pixel against
    the OpenMP oracle (bit-identical to the reference transforms), 0 class
    flips; four row bands with halos reproduce the full frame bit-exactly."""
    torch = _torch()
    from dctenergy import synth
    H = W = 16384
    frame = synth.natural_rows(0, H, W, 3, seed=0, device="cuda")
    out = torch.empty((H, W), dtype=torch.float32, device="cuda")
    ctx.energy_map_tensor(frame, out, 8, 0.3, 0.7)
    torch.cuda.synchronize()
    host = frame.cpu().numpy()
    ref = O.energy_map(host, 8, 0.3, 0.7, nthreads=NTHREADS)
    del host
    _compare_full(out, ref, 0.3, 0.7, "16384^2 RGB N=8")
    del ref
    parts = torch.empty_like(out)
    for k in range(4):
        a, b = H * k // 4, H * (k + 1) // 4
        lo, hi = max(0, a - 3), min(H - 1, b + 3)
        ctx.energy_map_tensor(frame[lo:hi + 1], parts[a:b], 8, 0.3, 0.7, h=H, in_row0=lo, y0=a, y1=b)
    torch.cuda.synchronize()
    assert torch.equal(out, parts)
    del frame, out, parts
    torch.cuda.empty_cache()


def test_config5_8192_rgb_n16_full_frame(ctx):
    """BASELINE config 5 (8192^2 RGB, N=16): every pixel against the oracle."""
    torch = _torch()
    from dctenergy import synth
    H = W = 8192
    frame = synth.natural_rows(0, H, W, 3, seed=5, device="cuda")
    out = torch.empty((H, W), dtype=torch.float32, device="cuda")
    ctx.energy_map_tensor(frame, out, 16, 0.3, 0.7)
    torch.cuda.synchronize()
    ref = O.energy_map(frame.cpu().numpy(), 16, 0.3, 0.7, nthreads=NTHREADS)
    _compare_full(out, ref, 0.3, 0.7, "8192^2 RGB N=16")
    del frame, out, ref
    torch.cuda.empty_cache()


def _stress_frames(S, rng):
    """Inputs that stress the class decision (SURVEY §8d "stress" frame and
    the tie-prone kinds): uniform random RGB; binary random dots on flat
    ground; line art (1-px lines on white); a 1-px checkerboard."""
    yy, xx = np.mgrid[0:S, 0:S]
    line = np.full((S, S), 255, np.uint8)
    line[(yy % 23 == 0) | (xx % 31 == 0) | ((xx + 2 * yy) % 97 == 0)] = 0
    return {
        "uniform_rgb": rng.integers(0, 256, (S, S, 3), dtype=np.uint8),
        "dots_grey": np.where(rng.random((S, S)) < 1 / 64, 255, 16).astype(np.uint8),
        "lineart_grey": line,
        "checker_rgb": np.repeat(((xx + yy) % 2 * 255).astype(np.uint8)[..., None], 3, -1),
    }


@pytest.mark.parametrize("n", [4, 8, 16])
def test_stress_frames_full(ctx, n):
    """2048^2 stress frames (4096^2 for N=8) at e=0.3 t=0.7: every pixel
    within tolerance, 0 class flips."""
    torch = _torch()
    S = 4096 if n == 8 else 2048
    rng = np.random.default_rng(11 + n)
    for name, img in _stress_frames(S, rng).items():
        out = torch.from_numpy(ctx.energy_map(img, n, 0.3, 0.7)).cuda()
        refined = ctx.last_refined
        ref = O.energy_map(img, n, 0.3, 0.7, nthreads=NTHREADS)
        st = _compare_full(out, ref, 0.3, 0.7, f"{name} {S}^2 N={n}")
        print(name, n, "refined", refined, st)


def test_tie_dense_full_size(ctx):
    """The worst realistic inputs for the fp64 refinement at the metric's
    size (16384^2, N=8, e=0.3 t=0.7): line art as RGB (2.7 % of the pixels
    flagged, most strips dense) and dots on flat ground (0.37 %, sparse
    strips) -- every pixel against the oracle, 0 class flips."""
    torch = _torch()
    S = 16384
    yy, xx = np.ogrid[0:S, 0:S]
    ink = (yy % 23 == 0) | (xx % 31 == 0) | ((xx + 2 * yy) % 97 == 0)
    line = np.repeat(np.where(ink, 0, 255).astype(np.uint8)[..., None], 3, -1)
    del ink
    dots = np.where(np.random.default_rng(21).random((S, S), dtype=np.float32) < 1 / 64,
                    255, 16).astype(np.uint8)
    for name, img in (("lineart_rgb", line), ("dots_grey", dots)):
        out = torch.from_numpy(ctx.energy_map(img, 8, 0.3, 0.7)).cuda()
        refined = ctx.last_refined
        ref = O.energy_map(img, 8, 0.3, 0.7, nthreads=NTHREADS)
        st = _compare_full(out, ref, 0.3, 0.7, f"{name} {S}^2 N=8")
        print(name, "refined", refined, st)
        assert refined > 100000
        del out, ref
        torch.cuda.empty_cache()


def test_tie_dense_one_launch(ctx):
    """A whole 16384^2 frame in ONE device launch (the host entry point maps
    1024-row chunks): text-like blocks dirty almost every 64-column strip, more
    strips than the refinement launch's sparse walkers take in one stride,
    and hold sparse and dense strips side by side.  Every pixel against the
    oracle, at N = 8 and (8192^2) N = 16, 0 class flips."""
    torch = _torch()
    for S, n in ((16384, 8), (8192, 16)):
        rng = np.random.default_rng(31 + n)
        blk = rng.random((S // 4 + 1, S // 4 + 1)) < 0.3
        img = np.where(np.repeat(np.repeat(blk, 4, 0), 4, 1)[:S, :S], 0, 255).astype(np.uint8)
        del blk
        out = torch.empty((S, S), dtype=torch.float32, device="cuda")
        ctx.energy_map_tensor(torch.from_numpy(img).cuda(), out, n, 0.3, 0.7)
        torch.cuda.synchronize()
        ref = O.energy_map(img, n, 0.3, 0.7, nthreads=NTHREADS)
        st = _compare_full(out, ref, 0.3, 0.7, f"text {S}^2 N={n} one launch")
        print("text one launch", S, n, st)
        del out, ref
        torch.cuda.empty_cache()


def test_tie_dense_full_size_n4(ctx):
    """N = 4 on the frames whose ties it refines most (the lane walk with the
    grey memo since r04): line art as RGB (5.5 % flagged) and grey dots on
    flat ground (10 %) at 8192^2, each in one device launch -- every pixel
    against the oracle, 0 class flips."""
    torch = _torch()
    S = 8192
    yy, xx = np.ogrid[0:S, 0:S]
    ink = (yy % 23 == 0) | (xx % 31 == 0) | ((xx + 2 * yy) % 97 == 0)
    line = np.repeat(np.where(ink, 0, 255).astype(np.uint8)[..., None], 3, -1)
    del ink
    dots = np.where(np.random.default_rng(22).random((S, S), dtype=np.float32) < 1 / 64,
                    255, 16).astype(np.uint8)
    for name, img in (("lineart_rgb", line), ("dots_grey", dots)):
        out = torch.empty((S, S), dtype=torch.float32, device="cuda")
        ctx.energy_map_tensor(torch.from_numpy(img).cuda(), out, 4, 0.3, 0.7)
        torch.cuda.synchronize()
        ref = O.energy_map(img, 4, 0.3, 0.7, nthreads=NTHREADS)
        st = _compare_full(out, ref, 0.3, 0.7, f"{name} {S}^2 N=4 one launch")
        print(name, "N=4", st)
        del out, ref
        torch.cuda.empty_cache()


def test_tie_dense_full_size_n16(ctx):
    """N = 16 (configs[4]'s block size, 8192^2) on line art: 4.3 % of the
    pixels flagged, their dense strips refined four lanes per pixel with the
    window transposed across the wave's rows (fix_dense16_flat) -- RGB at the
    config's size and grey at 4096^2, every pixel against the oracle, 0 class
    flips."""
    torch = _torch()
    for S, rgb in ((8192, True), (4096, False)):
        yy, xx = np.ogrid[0:S, 0:S]
        ink = (yy % 23 == 0) | (xx % 31 == 0) | ((xx + 2 * yy) % 97 == 0)
        img = np.where(ink, 0, 255).astype(np.uint8)
        del ink
        if rgb:
            img = np.repeat(img[..., None], 3, -1)
        out = torch.from_numpy(ctx.energy_map(img, 16, 0.3, 0.7)).cuda()
        refined = ctx.last_refined
        ref = O.energy_map(img, 16, 0.3, 0.7, nthreads=NTHREADS)
        st = _compare_full(out, ref, 0.3, 0.7, f"lineart {'rgb' if rgb else 'grey'} {S}^2 N=16")
        print("lineart", S, "rgb" if rgb else "grey", "refined", refined, st)
        assert refined > 100000
        del out, ref
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
            assert ctx.last_refined == int(EM.refine_mask(me, mt, 0.3, 0.7, n).sum())
            if n < 16:
                assert ctx.last_refined > 0


def _border_dots(H, W, bpp):
    """Isolated bright pixels on flat ground only at the frame's corners and
    along its four edges (exact edge / texture ties right at the border):
    every flagged window is clamped at a frame edge, and the bottom-right ones
    read the last bytes of the frame."""
    g = np.full((H, W), 16, np.uint8)
    for y, x in ((0, 0), (0, W - 1), (H - 1, 0), (H - 1, W - 1), (H - 1, W - 2), (H - 2, W - 1)):
        g[y, x] = 255
    g[::7, 0] = g[3::7, 1] = g[::7, W - 1] = g[3::7, W - 2] = 255
    g[0, ::11] = g[1, 5::11] = g[H - 1, ::11] = g[H - 2, 5::11] = 255
    return g if bpp == 1 else np.repeat(g[..., None], bpp, -1).copy()


@pytest.mark.parametrize("n", [4, 8, 16])
def test_refinement_at_frame_borders(ctx, n):
    """Flagged pixels only in windows clamped at the frame borders (odd widths,
    so the frame's byte count is not a dword multiple): the refinement's
    per-pixel gathers at the left / right edges and its reads of the frame's
    last bytes agree with the reference, both semantics, every layer format."""
    cases = [(dctenergy.DCTE_LQR, bpp) for bpp in (1, 3)] + \
            [(dctenergy.DCTE_PREVIEW, bpp) for bpp in (1, 3, 4)]
    for H, W in ((37, 301), (41, 517)):
        for sem, bpp in cases:
            img = _border_dots(H, W, bpp)
            got = ctx.energy_map(img, n, 0.3, 0.7, semantics=sem)
            refined = ctx.last_refined
            ref = (O.energy_map if sem == dctenergy.DCTE_LQR else O.preview_map)(img, n, 0.3, 0.7)
            _assert_tol(got, ref, f"border dots {H}x{W} bpp={bpp} sem={sem} n={n}")
            assert refined > 0, (H, W, bpp, sem, n)


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


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_energy_map2_is_the_two_calls(ctx, n):
    """dcte_energy_map2 (the plug-in's vertical build,
    src/render.c:358-364): both orientations from one upload, bit-equal to
    the two dcte_energy_map calls -- every semantics, ragged and tall frames
    (several row chunks each way), either output alone."""
    rng = np.random.default_rng(n)
    tall = rng.integers(0, 256, (3001, 700, 3), dtype=np.uint8)
    tall[:, 200:420] //= 9                        # flat stretch: ties, refinement
    for img in (load_input("natural_rgb_73x59.npy"), load_input("natural_grey_200x120.npy"),
                load_input("tiny_rgb_5x1.npy"), tall):
        for sem in (dctenergy.DCTE_LQR, dctenergy.DCTE_PREVIEW):
            a = ctx.energy_map(img, n, 0.3, 0.7, semantics=sem)
            b = ctx.energy_map(img, n, 0.3, 0.7, semantics=sem, transposed=True)
            o, ot = ctx.energy_map2(img, n, 0.3, 0.7, semantics=sem)
            assert np.array_equal(o, a) and np.array_equal(ot, b), (img.shape, sem)
            o1, none = ctx.energy_map2(img, n, 0.3, 0.7, semantics=sem, want=(True, False))
            none2, ot1 = ctx.energy_map2(img, n, 0.3, 0.7, semantics=sem, want=(False, True))
            assert none is None and none2 is None
            assert np.array_equal(o1, a) and np.array_equal(ot1, b), (img.shape, sem)
        if img is not tall:
            tr = np.ascontiguousarray(np.swapaxes(img, 0, 1))
            _assert_tol(ot, O.preview_map(tr, n, 0.3, 0.7), img.shape)


def test_energy_map2_exact_and_multi_device(ctx):
    """The exact mode through dcte_energy_map2 is the reference's bits in both
    orientations; on G logical devices (the row-band host path) the same maps
    as on one."""
    img = load_input("wilber_rgb_74x59.npy")
    tr = np.ascontiguousarray(np.swapaxes(img, 0, 1))
    with dctenergy.Context(ngpus=1, exact=True) as ex:
        for n in (2, 4, 8, 16):
            o, ot = ex.energy_map2(img, n, 0.3, 0.7)
            assert np.array_equal(o, O.energy_map(img, n, 0.3, 0.7)), n
            assert np.array_equal(ot, O.energy_map(tr, n, 0.3, 0.7)), n
    big = np.random.default_rng(5).integers(0, 256, (1500, 333, 3), dtype=np.uint8)
    with dctenergy.Context(ngpus=3, same_device=True) as many:
        for n in (8, 16):
            o, ot = ctx.energy_map2(big, n, 0.3, 0.7)
            o3, ot3 = many.energy_map2(big, n, 0.3, 0.7)
            assert np.array_equal(o, o3) and np.array_equal(ot, ot3), n


@pytest.mark.parametrize("transposed", [False, True])
def test_carver_create2_other_orientation(ctx, transposed):
    """dcte_carver_create2: the mirror's first map and the OTHER orientation's
    map from the same upload == dcte_energy_map of each orientation."""
    img = load_input("natural_rgb_97x41.npy")
    for n in (4, 8, 16):
        c, first, second = ctx.carver(img, n, 0.3, 0.7, transposed, other=True)
        a = ctx.energy_map(img, n, 0.3, 0.7)
        b = ctx.energy_map(img, n, 0.3, 0.7, transposed=True)
        assert np.array_equal(first, b if transposed else a), n
        assert np.array_equal(second, a if transposed else b), n
        c.close()


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


@pytest.mark.parametrize("G", [2, 3, 8])
def test_multi_device_host_path_on_one_gpu(ctx, G):
    """The single-process multi-device host path (band split, halo rows,
    per-device chunk pipelines, transposed strips, the u8 min/max merge) on G
    logical devices that are all device 0: bit-identical to the 1-device map."""
    rng = np.random.default_rng(G)
    img = rng.integers(0, 256, (4500, 301, 3), dtype=np.uint8)
    img[:, 100:200] //= 7                          # smoother region: ties and refinement
    with dctenergy.Context(ngpus=G, same_device=True) as many:
        assert many.ndevices == G
        for n in (2, 8, 16):
            a = ctx.energy_map(img, n, 0.3, 0.7)
            assert np.array_equal(a, many.energy_map(img, n, 0.3, 0.7)), n
            assert np.array_equal(ctx.energy_map(img[:700], n, 0.3, 0.7, transposed=True),
                                  many.energy_map(img[:700], n, 0.3, 0.7, transposed=True)), n
            for mode, ch in ((dctenergy.DCTE_NORM_LQR, 1), (dctenergy.DCTE_NORM_PREVIEW, 3)):
                assert np.array_equal(ctx.energy_image_u8(img, n, 0.3, 0.7, mode, ch),
                                      many.energy_image_u8(img, n, 0.3, 0.7, mode, ch)), (n, mode)


def test_kernel_download_equals_copy_engine(ctx):
    """DCTE_OPT_D2H_KERNEL (default 1): the host entry points' maps come down
    through a copy kernel writing the page-locked output; bit-identical to
    the runtime's copies (0) -- aligned and 4-byte-offset outputs (the
    dword path), both orientations, dcte_energy_map2, frames above and below
    the 1 MiB page-locking threshold, and a caller-pinned output."""
    import torch
    rng = np.random.default_rng(11)
    for h, w in ((1003, 777), (100, 300), (2050, 129)):
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        want = {}
        for kern in (0, 1):
            ctx.set_option(dctenergy.DCTE_OPT_D2H_KERNEL, kern)
            a = ctx.energy_map(img, 8, 0.3, 0.7)
            b = ctx.energy_map(img, 16, 0.3, 0.7, transposed=True)
            o, ot = ctx.energy_map2(img, 4, 0.3, 0.7)
            raw = np.zeros(h * w * 4 + 8, np.uint8)        # a float map 4 bytes off 16-byte alignment
            off = raw[4:4 + h * w * 4].view(np.float32).reshape(h, w)
            ctx.energy_map(img, 8, 0.3, 0.7, out=off)
            pinned = torch.empty((h, w), dtype=torch.float32, pin_memory=True).numpy()
            ctx.energy_map(img, 8, 0.3, 0.7, out=pinned)
            want[kern] = (a, b, o, ot, off.copy(), pinned.copy())
        for x, y in zip(want[0], want[1]):
            assert np.array_equal(x, y), (h, w)
        assert np.array_equal(want[1][0], want[1][4]) and np.array_equal(want[1][0], want[1][5])
    ctx.set_option(dctenergy.DCTE_OPT_D2H_KERNEL, 1)


def test_host_path_split_at_pinned_pages(ctx):
    """The host path page-locks only the whole pages inside the caller's
    buffers and copies the partial pages at their ends through the runtime's
    pageable path (dcte_capi.cpp HostPin / upload_rows / download): frames at
    odd offsets with padded row strides (rows straddling the first and last
    locked page), grey layers whose pageable frame shares pages with a
    locked map (the 3 x 100003 case that faulted with exact-byte
    registration), u8 layers and both orientations -- all bit-equal to the
    same calls without page-locking."""
    rng = np.random.default_rng(3)
    cases = [(3, 100003, 1, 0, 0), (700, 511, 3, 13, 4093), (1031, 333, 3, 1, 7), (257, 4099, 1, 5, 1)]
    for h, w, bpp, pad, off in cases:
        rs = w * bpp + pad
        buf = np.zeros(off + h * rs + 64, np.uint8)
        frame = np.lib.stride_tricks.as_strided(buf[off:], (h, w, bpp), (rs, bpp, 1)) if bpp > 1 else \
            np.lib.stride_tricks.as_strided(buf[off:], (h, w), (rs, 1))
        frame[...] = rng.integers(0, 256, frame.shape, dtype=np.uint8)
        got = {}
        for pin in (0, 1):
            ctx.set_option(dctenergy.DCTE_OPT_PIN_HOST, pin)
            r = []
            for n in (8, 16):
                out = np.zeros(h * w + 3, np.float32)[1:1 + h * w].reshape(h, w)   # 4 bytes off 16
                r.append(ctx.energy_map(frame, n, 0.3, 0.7, out=out).copy())
                r.append(ctx.energy_map(frame, n, 0.3, 0.7, transposed=True))
                r.append(ctx.energy_image_u8(frame, n, 0.3, 0.7, dctenergy.DCTE_NORM_PREVIEW, 3))
            got[pin] = r
        ctx.set_option(dctenergy.DCTE_OPT_PIN_HOST, 1)
        for a, b in zip(got[0], got[1]):
            assert np.array_equal(a, b), (h, w, bpp, pad, off)


def test_host_buffers_sharing_pages(ctx):
    """Frame and output packed into one allocation, so they share a page at
    unaligned addresses (the page-locking of the host path registers exactly
    the caller's bytes; a page-rounded registration made the runtime refuse
    the copy into the neighbour, tools/pin_probe.cpp).  Both orders, outputs
    above and below the 1 MiB pinning threshold: identical to separately
    allocated buffers."""
    h, w = 1003, 520
    img = np.random.default_rng(7).integers(0, 256, (h, w, 3), dtype=np.uint8)
    ref = ctx.energy_map(img, 8, 0.3, 0.7)
    ref_u8 = ctx.energy_image_u8(img, 8, 0.3, 0.7, dctenergy.DCTE_NORM_LQR)
    A, Bf, Bu = img.nbytes, ref.nbytes, ref_u8.nbytes
    for out_first in (False, True):
        big = np.zeros(100 + A + Bf + 64, np.uint8)
        o_px, o_out = (100 + Bf, 100) if out_first else (100, 100 + A)
        px = big[o_px:o_px + A].reshape(h, w, 3)
        px[...] = img
        out = big[o_out:o_out + Bf].view(np.float32).reshape(h, w)
        assert np.array_equal(ctx.energy_map(px, 8, 0.3, 0.7, out=out), ref), out_first
        o_u8 = 100 + A + 4 if not out_first else 100 + Bf - Bu - 4
        u8 = big[o_u8:o_u8 + Bu].reshape(h, w)
        assert np.array_equal(ctx.energy_image_u8(px, 8, 0.3, 0.7, dctenergy.DCTE_NORM_LQR, out=u8),
                              ref_u8), out_first
        assert np.array_equal(px, img)


def test_host_staging_multi_device_shared_pages(ctx):
    """Several devices of one context (the same GPU here) on host frames that
    are small (staged whole through the context's page-locked arena) and large
    (whole pages registered, the partial end pages staged), the frame and the
    map carved from ONE allocation so they share a page, both orientations and
    u8 layers: equal to the single-device results.  No copy of these calls
    takes the runtime's pageable path -- r06's fault: the band uploads of a
    multi-device context, or its transposed strips, copied overlapping pageable
    pages on several streams at once (test_exact_multi_device_host_path,
    profiles/r06/multi_device_pageable_fault.log)."""
    rng = np.random.default_rng(11)
    with dctenergy.Context(ngpus=3, same_device=True) as many:
        for h, w in ((700, 301), (2100, 301), (1500, 1031)):
            img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
            img[:, ::5] //= 9
            fb, ob = img.nbytes, 4 * h * w
            buf = np.zeros(fb + ob + 3 * 4096, np.uint8)
            off = (-buf.ctypes.data) % 4096 + 100           # the frame starts mid-page ...
            o_out = off + fb + (-(off + fb + buf.ctypes.data)) % 4   # ... the map on its last page
            frame = buf[off:off + fb].reshape(h, w, 3)
            frame[...] = img
            out = buf[o_out:o_out + ob].view(np.float32).reshape(h, w)
            for n in (8, 16):
                ref = ctx.energy_map(img, n, 0.3, 0.7)
                for c in (ctx, many):
                    out[...] = -1
                    assert np.array_equal(c.energy_map(frame, n, 0.3, 0.7, out=out), ref), (h, w, n)
                    assert np.array_equal(c.energy_map(frame, n, 0.3, 0.7, transposed=True),
                                          ctx.energy_map(img, n, 0.3, 0.7, transposed=True)), (h, w, n)
                    assert np.array_equal(c.energy_image_u8(frame, n, 0.3, 0.7, dctenergy.DCTE_NORM_PREVIEW, 3),
                                          ctx.energy_image_u8(img, n, 0.3, 0.7, dctenergy.DCTE_NORM_PREVIEW, 3))
            assert np.array_equal(frame, img)


def test_caller_pinned_views(ctx):
    """A frame and a map that lie INSIDE the caller's page-locked allocations
    (torch pin_memory), at odd offsets: used as they are (their device
    addresses from hipHostGetDevicePointer at the view's offset, no
    registration, no staging), on one device and on three -- equal to the
    same calls on ordinary numpy arrays."""
    import torch
    rng = np.random.default_rng(12)
    h, w = 900, 1201
    img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    img[::3] //= 11
    big = torch.empty(img.nbytes + 1000, dtype=torch.uint8, pin_memory=True).numpy()
    frame = big[333:333 + img.nbytes].reshape(h, w, 3)
    frame[...] = img
    mbuf = torch.empty(2 * h * w + 7, dtype=torch.float32, pin_memory=True).numpy()
    with dctenergy.Context(ngpus=3, same_device=True) as many:
        for n in (8, 16):
            ref = ctx.energy_map(img, n, 0.3, 0.7)
            reft = ctx.energy_map(img, n, 0.3, 0.7, transposed=True)
            for c in (ctx, many):
                out = mbuf[3:3 + h * w].reshape(h, w)
                out[...] = -1
                assert np.array_equal(c.energy_map(frame, n, 0.3, 0.7, out=out), ref), n
                out_t = mbuf[5 + h * w:5 + 2 * h * w].reshape(w, h)
                assert np.array_equal(c.energy_map(frame, n, 0.3, 0.7, transposed=True, out=out_t), reft), n
    assert np.array_equal(frame, img)


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_tile_height_does_not_change_results(n):
    """DCTE_OPT_TILE_H only re-partitions the work: any tile height gives the
    bit-identical map, refinement included (tie-dense input, e != t)."""
    rng = np.random.default_rng(n)
    img = np.where(rng.random((301, 333)) < 1 / 40, 255, 16).astype(np.uint8)
    img3 = rng.integers(0, 256, (150, 257, 3), dtype=np.uint8)
    with dctenergy.Context(ngpus=1) as c:
        ref = [c.energy_map(x, n, 0.3, 0.7) for x in (img, img3)]
        for th in (1, 7, 32, 64, 200):
            c.set_option(dctenergy.DCTE_OPT_TILE_H, th)
            for x, r in zip((img, img3), ref):
                assert np.array_equal(c.energy_map(x, n, 0.3, 0.7), r), (n, th)


def test_energy_windows_kat(ctx):
    """dcte_energy_windows on the golden known-answer windows (the
    reference's own transforms produced the energies): bit-exact."""
    from golden_util import load_kat
    for k in manifest()["kat"]:
        win = load_kat(k["window"])
        got = ctx.energy_windows(win[None], k["edges"], k["textures"])[0]
        assert got == np.float32(k["energy"]), k


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_energy_windows_bit_exact(ctx, n):
    """Random, luma-quantised and tie-prone windows: bit-identical to the
    oracle (pinned bit-exactly to the reference transforms, test_oracle.py)."""
    rng = np.random.default_rng(40 + n)
    wins = [rng.random((200, n, n)),
            O.luma_plane(rng.integers(0, 256, (200, n, n, 3), dtype=np.uint8)),
            (rng.random((200, n, n)) < 0.05) * (254 / 255) + 1 / 255]
    for w in wins:
        got = ctx.energy_windows(w, 0.3, 0.7)
        ref = np.array([O.window_energy(x, 0.3, 0.7) for x in w], np.float32)
        assert np.array_equal(got, ref), n


@pytest.mark.parametrize("n", [4, 8, 16])
def test_grey_rgb_refinement_paths(n):
    """The dense refinement walks read liblqr RGB luma through one table when
    every pixel of a batch's windows is grey (R = G = B) and through three
    otherwise: grey line art, line art whose strokes alternate between grey
    and colour (batches mixing both kinds of lane), random RGB with a few
    grey pixels, and a near-grey frame (one channel off by one) -- every
    pixel refined (tie_tau = 1): bit-identical to the oracle, one and many
    tile heights."""
    rng = np.random.default_rng(90 + n)
    H, W = 203, 333
    yy, xx = np.ogrid[0:H, 0:W]
    ink = (yy % 11 == 0) | (xx % 13 == 0) | ((xx + 2 * yy) % 37 == 0)
    grey = np.repeat(np.where(ink, 0, 255).astype(np.uint8)[..., None], 3, -1)
    mixed = grey.copy()
    mixed[(xx % 26 == 0) & (yy >= 0)] = (200, 30, 30)
    rnd = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    rnd[rng.random((H, W)) < 0.2] = 77
    near = grey.copy()
    near[..., 2] ^= (rng.random((H, W)) < 0.01).astype(np.uint8)
    with dctenergy.Context(ngpus=1, tie_tau=1.0) as c:
        for th in (0, 16):
            c.set_option(dctenergy.DCTE_OPT_TILE_H, th)
            for name, img in (("grey", grey), ("mixed", mixed), ("random", rnd), ("near", near)):
                got = c.energy_map(img, n, 0.3, 0.7)
                assert np.array_equal(got, O.energy_map(img, n, 0.3, 0.7)), (n, th, name)
    with dctenergy.Context(ngpus=1) as c:           # the default tau: the tie-dense strips
        for name, img in (("grey", grey), ("mixed", mixed)):
            _assert_tol(c.energy_map(img, n, 0.3, 0.7), O.energy_map(img, n, 0.3, 0.7), name)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 8, 16])
def test_window_memo_near_duplicates(n):
    """The dense walks answer a window whose bytes equal an earlier refined
    window's from a per-wave memo.  Frames built to defeat a wrong key: strokes
    of three inks (0, 1, 2) on a ground of 255 with 1-in-300 pixels at 254, so
    most windows repeat and many differ from a repeated one in ONE byte; the
    same as grey-valued RGB, as RGB whose G or B is off by one at 1-in-200
    pixels (R alone would collide), and a frame whose strokes repeat exactly
    along every row (all hits).  Every pixel refined (tie_tau = 1): liblqr and
    preview maps bit-identical to the oracle, two tile heights."""
    rng = np.random.default_rng(300 + n)
    H, W = 257, 517
    yy, xx = np.ogrid[0:H, 0:W]
    ink = np.full((H, W), 255, np.uint8)
    ink[rng.random((H, W)) < 1 / 300] = 254
    for k, m in enumerate(((yy % 11 == 0) & (xx >= 0), (xx % 13 == 0) & (yy >= 0), (xx + 2 * yy) % 37 == 0)):
        ink[m] = k
    rgb = np.repeat(ink[..., None], 3, -1)
    off = rgb.copy()
    sel = rng.random((H, W)) < 1 / 200
    off[sel, 1 + (rng.random(int(sel.sum())) < 0.5)] ^= 1
    rows = np.repeat(np.where((yy % 7 == 0) | (yy % 7 == 3), 0, 255).astype(np.uint8), W, 1)
    frames = (("grey", ink), ("rgb", rgb), ("off", off), ("rows", rows))
    with dctenergy.Context(ngpus=1, tie_tau=1.0) as c:
        for th in (0, 16):
            c.set_option(dctenergy.DCTE_OPT_TILE_H, th)
            for name, img in frames:
                got = c.energy_map(img, n, 0.3, 0.7)
                assert np.array_equal(got, O.energy_map(img, n, 0.3, 0.7)), (n, th, name, "liblqr")
                got = c.energy_map(img, n, 0.3, 0.7, semantics=dctenergy.DCTE_PREVIEW)
                assert np.array_equal(got, O.preview_map(img, n, 0.3, 0.7)), (n, th, name, "preview")


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_refine_all_bit_exact_every_layout(n):
    """tie_tau >= 1 sends every pixel through dcte_fix_strips (dense strips:
    staged bands; the frame-border strips: clamped staging; small frames:
    direct gathers): the map must equal the oracle bit for bit -- liblqr
    grey/RGB and preview grey/RGB/RGBA, odd sizes, several tile heights."""
    rng = np.random.default_rng(70 + n)
    frames = [rng.integers(0, 256, (97, 131), dtype=np.uint8),
              rng.integers(0, 256, (70, 301, 3), dtype=np.uint8),
              rng.integers(0, 256, (41, 67, 4), dtype=np.uint8)]
    with dctenergy.Context(ngpus=1, tie_tau=1.0) as c:
        for th in (0, 16):
            c.set_option(dctenergy.DCTE_OPT_TILE_H, th)
            for img in frames:
                if img.ndim == 2 or img.shape[2] == 3:
                    got = c.energy_map(img, n, 0.3, 0.7)
                    assert np.array_equal(got, O.energy_map(img, n, 0.3, 0.7)), (n, th, img.shape)
                    assert c.last_refined == img.shape[0] * img.shape[1]
                got = c.energy_map(img, n, 0.3, 0.7, semantics=dctenergy.DCTE_PREVIEW)
                assert np.array_equal(got, O.preview_map(img, n, 0.3, 0.7)), (n, th, img.shape, "preview")


def test_failed_call_then_good_call(ctx):
    """A device call the library rejects (tile rows past the launch grid's y
    limit -> DCTE_ERANGE) between good calls on the same stream leaves
    nothing behind: the calls after it give the same bits as the call before
    it, within tolerance of the reference (a stale dirty-strip
    counter would make the refinement walk an older launch's list)."""
    torch = _torch()
    rng = np.random.default_rng(17)
    img = (rng.random((96, 160)) < 0.03).astype(np.uint8) * 255
    ref = O.energy_map(img, 8, 0.3, 0.7)
    frame = torch.from_numpy(img).cuda()
    before = torch.empty((96, 160), dtype=torch.float32, device="cuda")
    ctx.energy_map_tensor(frame, before, 8, 0.3, 0.7)
    torch.cuda.synchronize()
    _assert_tol(before.cpu().numpy(), ref, "before")
    tall = torch.zeros((70000, 2), dtype=torch.uint8, device="cuda")
    tall_out = torch.empty((70000, 2), dtype=torch.float32, device="cuda")
    try:
        ctx.set_option(dctenergy.DCTE_OPT_TILE_H, 1)
        with pytest.raises(dctenergy.DcteError) as e:
            ctx.energy_map_tensor(tall, tall_out, 8, 0.3, 0.7)
        assert e.value.code == dctenergy.DCTE_ERANGE
    finally:
        ctx.set_option(dctenergy.DCTE_OPT_TILE_H, 0)
    for _ in range(2):
        after = torch.full((96, 160), -1.0, dtype=torch.float32, device="cuda")
        ctx.energy_map_tensor(frame, after, 8, 0.3, 0.7)
        torch.cuda.synchronize()
        assert torch.equal(after, before)


@pytest.mark.parametrize("which", [1, 2])
@pytest.mark.parametrize("n", [8, 16])
def test_injected_launch_failure_then_good_call(ctx, which, n):
    """a launch that fails AFTER the profiling events and the map
    launch were queued (DCTE_OPT_FAIL_INJECT: 1 = reported after the map
    launch, 2 = after the refinement launch) takes the error path that zeroes
    both dirty counters on the stream and does not flip the counter phase;
    the next calls on the same stream give the same bits as before."""
    torch = _torch()
    rng = np.random.default_rng(18)
    img = (rng.random((200, 333)) < 0.03).astype(np.uint8) * 255      # tie-dense: refinement runs
    frame = torch.from_numpy(img).cuda()
    before = torch.empty((200, 333), dtype=torch.float32, device="cuda")
    ctx.energy_map_tensor(frame, before, n, 0.3, 0.7)
    torch.cuda.synchronize()
    _assert_tol(before.cpu().numpy(), O.energy_map(img, n, 0.3, 0.7), "before")
    for profile in (0, 1):
        ctx.set_option(dctenergy.DCTE_OPT_PROFILE, profile)
        try:
            ctx.set_option(dctenergy.DCTE_OPT_FAIL_INJECT, which)
            junk = torch.empty_like(before)
            with pytest.raises(dctenergy.DcteError) as e:
                ctx.energy_map_tensor(frame, junk, n, 0.3, 0.7)
            assert e.value.code == dctenergy.DCTE_EHIP
        finally:
            ctx.set_option(dctenergy.DCTE_OPT_FAIL_INJECT, 0)
            ctx.set_option(dctenergy.DCTE_OPT_PROFILE, 0)
            ctx.profile_read()
        for _ in range(2):
            after = torch.full_like(before, -1.0)
            ctx.energy_map_tensor(frame, after, n, 0.3, 0.7)
            torch.cuda.synchronize()
            assert torch.equal(after, before), (which, profile)


@pytest.mark.parametrize("shape", [(33, 65537), (65537, 19), (3, 100003)])
def test_extreme_aspect_ratios(ctx, shape):
    """Frames past 65 536 columns (or rows) and only a few rows (or columns)
    tall: more column tiles than any square config, tile heights far above
    the frame, the border clamp on both sides of every window -- every N,
    both semantics, grey and RGB: within tolerance of the oracle, and the
    exact mode bit-identical."""
    rng = np.random.default_rng(shape[1])
    NT = max(1, min(16, len(os.sched_getaffinity(0))))
    for bpp in (1, 3):
        img = rng.integers(0, 256, shape + ((bpp,) if bpp > 1 else ()), dtype=np.uint8)
        img[:, ::7] //= 5                               # some smooth stretches: ties, refinement
        with dctenergy.Context(ngpus=1, exact=True) as ex:
            for n in (2, 4, 8, 16):
                ref = O.energy_map(img, n, 0.3, 0.7, nthreads=NT)
                assert within_tol(ctx.energy_map(img, n, 0.3, 0.7), ref).all(), (shape, bpp, n)
                assert np.array_equal(ex.energy_map(img, n, 0.3, 0.7), ref), (shape, bpp, n)
                pv = O.preview_map(img, n, 0.3, 0.7, nthreads=NT)
                assert within_tol(ctx.energy_map(img, n, 0.3, 0.7, semantics=dctenergy.DCTE_PREVIEW), pv).all()
                assert np.array_equal(ex.energy_map(img, n, 0.3, 0.7, semantics=dctenergy.DCTE_PREVIEW), pv)


def test_frames_past_one_buffer_resource_are_refused(ctx):
    """A launch addresses its readable rows through one 32-bit buffer
    resource: a row span of 4 GiB or more is refused with DCTE_ERANGE before
    anything is read (here a huge rowstride over a small buffer), in both
    modes, and the context stays usable."""
    torch = _torch()
    small = torch.zeros((4, 64, 3), dtype=torch.uint8, device="cuda")
    out = torch.empty((4, 64), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    with dctenergy.Context(ngpus=1, exact=True) as ex:
        for c in (ctx, ex):
            with pytest.raises(dctenergy.DcteError) as e:
                c.energy_map_device(small.data_ptr(), 1 << 31, 64, 4, 3, 0, 4, 0, 4, 8, 0.3, 0.7,
                                    out.data_ptr(), out.stride(0), st)
            assert e.value.code == dctenergy.DCTE_ERANGE
            c.energy_map_tensor(small, out, 8, 0.3, 0.7)
            torch.cuda.synchronize()
            assert torch.equal(out, torch.zeros_like(out))
