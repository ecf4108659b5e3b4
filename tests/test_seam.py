"""GPU: seam removal with energy update and energies at points.

Bar: after every carve step the updated map is BIT-identical to the full map
dcte_energy_map computes for the carved frame (same fp32 passes, same fp64
refinement), the carved frame equals numpy's, and the final map is within
the north_star tolerance of the oracle (reference arithmetic); with
refinement forced everywhere it equals the oracle exactly.
"""
import numpy as np
import pytest

import dctenergy
import oracle_py as O
from golden_util import load_input, within_tol
from seam_util import carve, random_seams

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    return torch


def _oracle(img, n, e, t, sem):
    return O.energy_map(img, n, e, t) if sem == dctenergy.DCTE_LQR else O.preview_map(img, n, e, t)


def _seams(seed, steps):
    """steps seams, each drawn for the width it is applied at (kinds rotate:
    connected walk, arbitrary jumps, left border, right border)."""
    def gen(k, h, width):
        return random_seams(h, width, seed=seed + 7 * k, count=4)[k % 4]
    return [gen] * steps


def _carve_run(ctx, img, n, e, t, sem, seams, inplace=False):
    """Carve seams one by one on the device; check every step.  seams: arrays,
    or callables (k, h, width) -> array.  inplace: the carved frame and map
    stay in the original buffers (narrowing views, original row strides)."""
    torch = _torch()
    dev = torch.device("cuda")
    cur = torch.from_numpy(img).to(dev)
    h, w = img.shape[:2]
    emap = torch.empty((h, w), dtype=torch.float32, device=dev)
    ctx.energy_map_tensor(cur, emap, n, e, t, semantics=sem)
    host = img
    for k, s in enumerate(seams):
        if callable(s):
            s = s(k, h, cur.shape[1])
        s = np.clip(s, 0, cur.shape[1] - 1).astype(np.int32)
        if inplace:
            nxt, nmap = cur[:, :cur.shape[1] - 1], emap[:, :cur.shape[1] - 1]
        else:
            nxt = torch.empty((h, cur.shape[1] - 1) + tuple(cur.shape[2:]), dtype=torch.uint8,
                              device=dev)
            nmap = torch.full((h, cur.shape[1] - 1), np.nan, dtype=torch.float32, device=dev)
        ctx.seam_carve_tensor(cur, torch.from_numpy(s).to(dev), emap, nxt, nmap, n, e, t,
                              semantics=sem)
        host = carve(host, s)
        full = torch.empty_like(nmap)
        ctx.energy_map_tensor(nxt, full, n, e, t, semantics=sem)
        torch.cuda.synchronize()
        assert np.array_equal(nxt.cpu().numpy(), host), f"frame after seam {k}"
        got, want = nmap.cpu().numpy(), full.cpu().numpy()
        if not np.array_equal(got, want):
            bad = np.argwhere(got != want)[:5]
            raise AssertionError(f"seam {k}: {int((got != want).sum())} pixels differ from the "
                                 f"full map, first {bad.tolist()}")
        cur, emap = nxt, nmap
    return host, emap.cpu().numpy()


@pytest.mark.parametrize("inplace", [False, True], ids=["copy", "inplace"])
@pytest.mark.parametrize("n", [2, 4, 8, 16])
@pytest.mark.parametrize("sem,name", [(0, "natural_rgb_73x59.npy"), (0, "natural_grey_200x120.npy"),
                                      (1, "rgba_45x38.npy"), (1, "natural_rgb_73x59.npy")])
def test_carve_updates_equal_full_map(ctx, n, sem, name, inplace):
    img = load_input(name)
    host, E = _carve_run(ctx, img, n, 0.15, 0.85, sem, _seams(n, 12), inplace)
    ref = _oracle(host, n, 0.15, 0.85, sem)
    assert within_tol(E, ref).all()


@pytest.mark.parametrize("n", [2, 8, 16])
def test_carve_refine_all_is_reference_exact(ctx, n):
    img = load_input("wilber_rgb_74x59.npy")
    h, w = img.shape[:2]
    ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, 1.0)
    try:
        host, E = _carve_run(ctx, img, n, 0.15, 0.85, 0, _seams(3, 6))
    finally:
        ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, -1)   # the per-N defaults
    assert np.array_equal(E, O.energy_map(host, n, 0.15, 0.85))


def test_carve_to_narrow_frames(ctx):
    """Down to a 2-pixel-wide frame: every pixel's window clamps."""
    img = load_input("natural_rgb_97x41.npy")[:, :10]
    img = np.ascontiguousarray(img)
    h = img.shape[0]
    seams = [np.full(h, k % 3, np.int32) for k in range(8)]
    host, E = _carve_run(ctx, img, 8, 0.3, 0.7, 0, seams)
    assert host.shape[1] == 2
    host2, E2 = _carve_run(ctx, img, 8, 0.3, 0.7, 0, seams, inplace=True)
    assert np.array_equal(host2, host) and np.array_equal(E2, E)
    assert within_tol(E, O.energy_map(host, 8, 0.3, 0.7)).all()


def test_carve_on_ties(ctx):
    """Exact edge/texture ties go through the refinement in the update too."""
    yy, xx = np.mgrid[0:48, 0:52]
    img = (((xx // 2 + yy // 2) & 1) * 200 + 20).astype(np.uint8)
    host, E = _carve_run(ctx, img, 4, 0.3, 0.7, 0, _seams(5, 8))
    assert within_tol(E, O.energy_map(host, 4, 0.3, 0.7)).all()


def test_carve_bad_arguments(ctx):
    torch = _torch()
    px = torch.zeros((8, 1, 3), dtype=torch.uint8, device="cuda")
    seam = torch.zeros(8, dtype=torch.int32, device="cuda")
    m = torch.zeros((8, 1), dtype=torch.float32, device="cuda")
    with pytest.raises(ValueError):
        ctx.seam_carve_tensor(px, seam, m, px, m)
    L = dctenergy.lib()
    # a 1-pixel-wide frame has no seam to remove; N = 6 is not a block size
    for w, n in ((1, 8), (2, 6)):
        rc = L.dcte_seam_carve_device(ctx._h, 0, px.data_ptr(), 3 * w, w, 8, 3, seam.data_ptr(),
                                      m.data_ptr(), w, px.data_ptr(), 3 * w, m.data_ptr(), w,
                                      n, 0.5, 0.5, 0, None)
        assert rc == dctenergy.DCTE_EINVAL


@pytest.mark.parametrize("n", [2, 4, 8, 16])
@pytest.mark.parametrize("sem,name", [(0, "natural_rgb_73x59.npy"), (0, "wilber_rgb_74x59.npy"),
                                      (1, "rgba_45x38.npy"), (1, "natural_grey_200x120.npy")])
def test_points_equal_map(ctx, n, sem, name):
    img = load_input(name)
    h, w = img.shape[:2]
    rng = np.random.default_rng(n)
    xy = np.stack([rng.integers(0, w, 500), rng.integers(0, h, 500)], 1).astype(np.int32)
    xy[:4] = [[0, 0], [w - 1, 0], [0, h - 1], [w - 1, h - 1]]
    full = ctx.energy_map(img, n, 0.15, 0.85, semantics=sem)
    got = ctx.energy_points(img, xy, n, 0.15, 0.85, semantics=sem)
    assert np.array_equal(got, full[xy[:, 1], xy[:, 0]])


def test_points_device_and_errors(ctx):
    torch = _torch()
    img = load_input("natural_rgb_73x59.npy")
    h, w = img.shape[:2]
    xy = np.array([[3, 4], [72, 58], [10, 0]], np.int32)
    out = torch.empty(3, dtype=torch.float32, device="cuda")
    ctx.energy_points_tensor(torch.from_numpy(img).cuda(), torch.from_numpy(xy).cuda(), out, 8,
                             0.3, 0.7)
    torch.cuda.synchronize()
    full = ctx.energy_map(img, 8, 0.3, 0.7)
    assert np.array_equal(out.cpu().numpy(), full[xy[:, 1], xy[:, 0]])
    assert len(ctx.energy_points(img, np.zeros((0, 2), np.int32), 8)) == 0
    with pytest.raises(dctenergy.DcteError) as ei:
        ctx.energy_points(img, np.array([[w, 0]], np.int32), 8)
    assert ei.value.code == dctenergy.DCTE_EINVAL
