"""GPU: minimum-energy seam (dcte_seam_find[_device]) against
the oracle's restatement of liblqr's recursion (bit-identical: same float
adds, same leftmost-minimum rule) [liblqr, unverified], and the whole carve
loop map -> seam -> carve on the device against the CPU loop."""
import numpy as np
import pytest

import dctenergy
import oracle_py as O
from golden_util import load_input
from seam_util import carve

pytestmark = pytest.mark.gpu


def _maps(h, w, kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "uniform":
        return rng.random((h, w), dtype=np.float32)
    if kind == "ties":
        return rng.integers(0, 3, (h, w)).astype(np.float32)
    if kind == "flat":
        return np.ones((h, w), np.float32)
    # a cheap valley that wanders across tile borders
    x = np.arange(w)[None, :]
    c = (w / 2 + (w / 3) * np.sin(np.arange(h)[:, None] / 37.0))
    return (np.abs(x - c) / w + 0.01 * rng.random((h, w))).astype(np.float32)


SHAPES = [(1, 1), (1, 5), (7, 1), (31, 64), (33, 65), (100, 129), (257, 300), (64, 1000),
          (1000, 77), (129, 4097)]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: f"{s[0]}x{s[1]}")
@pytest.mark.parametrize("kind", ["uniform", "ties", "flat", "valley"])
def test_seam_matches_oracle(ctx, shape, kind):
    h, w = shape
    E = _maps(h, w, kind, h * 7 + w)
    got = ctx.seam_find(E)
    assert np.array_equal(got, O.seam_find(E))


def test_seam_device_strided_and_large(ctx):
    import torch
    h, w = 4096, 4096
    E = _maps(h, w, "valley", 1)
    buf = torch.full((h, w + 40), np.nan, dtype=torch.float32, device="cuda")
    buf[:, :w] = torch.from_numpy(E).cuda()
    seam = torch.empty(h, dtype=torch.int32, device="cuda")
    ctx.seam_find_tensor(buf[:, :w], seam)
    torch.cuda.synchronize()
    assert np.array_equal(seam.cpu().numpy(), O.seam_find(E))


@pytest.fixture
def bandwise(ctx):
    """DCTE_OPT_DP_BANDWISE: one DP launch per band of rows (the mode a frame
    too wide for every tile to be resident, or a timed-out search, uses)."""
    ctx.set_option(dctenergy.DCTE_OPT_DP_BANDWISE, 1)
    yield ctx
    ctx.set_option(dctenergy.DCTE_OPT_DP_BANDWISE, 0)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: f"{s[0]}x{s[1]}")
@pytest.mark.parametrize("kind", ["ties", "valley"])
def test_seam_bandwise_matches_oracle(bandwise, shape, kind):
    h, w = shape
    E = _maps(h, w, kind, h * 5 + w)
    assert np.array_equal(bandwise.seam_find(E), O.seam_find(E))


def test_seam_wider_than_resident_tiles(ctx):
    """100000 columns is more DP tiles than the chip holds at once: the search
    runs band by band instead of being refused."""
    h, w = 200, 100000
    E = _maps(h, w, "valley", 3)
    E[:, 65000:65010] *= 0.01          # the valley's exit is past the old width limit
    assert np.array_equal(ctx.seam_find(E), O.seam_find(E))


def test_carve_bandwise_equals_resident(ctx):
    img = load_input("natural_rgb_97x41.npy")
    ref, ref_cols = ctx.carve(img, 12, 8, 0.5, 0.5)
    ctx.set_option(dctenergy.DCTE_OPT_DP_BANDWISE, 1)
    try:
        out, cols = ctx.carve(img, 12, 8, 0.5, 0.5)
    finally:
        ctx.set_option(dctenergy.DCTE_OPT_DP_BANDWISE, 0)
    assert np.array_equal(out, ref) and np.array_equal(cols, ref_cols)


def test_seam_timeout_falls_back_to_bandwise(ctx):
    """DCTE_OPT_DP_SPIN_LIMIT = 1: a tile of the single-launch search gives up
    the first time a neighbour's row is not there yet.  The device entry point
    reports that as seam = -1; the host entry points run the search again one
    launch per band and return the oracle's seam."""
    import torch
    h, w = 16384, 4096               # 512 hand-offs per tile: some must wait
    E = _maps(h, w, "valley", 11)
    ref = O.seam_find(E)
    d_map = torch.from_numpy(E).cuda()
    seam = torch.empty(h, dtype=torch.int32, device="cuda")
    ctx.set_option(dctenergy.DCTE_OPT_DP_SPIN_LIMIT, 1)
    try:
        ctx.seam_find_tensor(d_map, seam)
        torch.cuda.synchronize()
        dev = seam.cpu().numpy()
        host = ctx.seam_find(E)              # times out, then runs band-wise
        again = ctx.seam_find(E)             # this stream stays band-wise
    finally:
        ctx.set_option(dctenergy.DCTE_OPT_DP_SPIN_LIMIT, 0)
    assert (dev == -1).all()
    assert np.array_equal(host, ref) and np.array_equal(again, ref)
    assert np.array_equal(ctx.seam_find(E), ref)   # single launch again


def test_carve_timeout_falls_back_to_bandwise(ctx):
    """dcte_carve whose searches time out runs the whole carve again band-wise."""
    img = np.random.default_rng(5).integers(0, 256, (8192, 320, 3), dtype=np.uint8)
    ref, ref_cols = ctx.carve(img, 3, 8, 0.5, 0.5)
    ctx.set_option(dctenergy.DCTE_OPT_DP_SPIN_LIMIT, 1)
    try:
        out, cols = ctx.carve(img, 3, 8, 0.5, 0.5)
    finally:
        ctx.set_option(dctenergy.DCTE_OPT_DP_SPIN_LIMIT, 0)
    assert np.array_equal(out, ref) and np.array_equal(cols, ref_cols)


def test_seam_bad_arguments(ctx):
    L = dctenergy.lib()
    seam = np.empty(4, np.int32)
    E = np.zeros((4, 4), np.float32)
    assert L.dcte_seam_find(ctx._h, E.ctypes.data, 0, 4, seam.ctypes.data) == dctenergy.DCTE_EINVAL
    assert L.dcte_seam_find(ctx._h, None, 4, 4, seam.ctypes.data) == dctenergy.DCTE_EINVAL


def _gpu_loop(ctx, img, n, e, t, steps):
    """map -> (seam -> carve in place) x steps, all on the device."""
    import torch
    cur = torch.from_numpy(img).cuda()
    h, w = img.shape[:2]
    emap = torch.empty((h, w), dtype=torch.float32, device="cuda")
    ctx.energy_map_tensor(cur, emap, n, e, t)
    seam = torch.empty(h, dtype=torch.int32, device="cuda")
    seams, maps = [], []
    for k in range(steps):
        wk = w - k
        maps.append(emap[:, :wk].cpu().numpy())
        ctx.seam_find_tensor(emap[:, :wk], seam)
        ctx.seam_carve_tensor(cur[:, :wk], seam, emap[:, :wk], cur[:, :wk - 1], emap[:, :wk - 1],
                              n, e, t)
        seams.append(seam.cpu().numpy().copy())
    torch.cuda.synchronize()
    return seams, maps, cur[:, :w - steps].cpu().numpy(), emap[:, :w - steps].cpu().numpy()


@pytest.mark.parametrize("n", [4, 8, 16])
def test_carve_loop_refined_equals_cpu_reference_loop(ctx, n):
    """With every pixel refined (the reference's own arithmetic) the device
    loop reproduces the CPU loop exactly: same seams, frame and energies."""
    img = load_input("wilber_rgb_74x59.npy")
    ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, 1.0)
    try:
        seams, _, frame, E = _gpu_loop(ctx, img, n, 0.3, 0.7, 10)
    finally:
        ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, -1)   # the per-N defaults
    host = img
    for k in range(10):
        ref_seam = O.seam_find(O.energy_map(host, n, 0.3, 0.7))
        assert np.array_equal(seams[k], ref_seam), f"seam {k}"
        host = carve(host, ref_seam)
    assert np.array_equal(frame, host)
    assert np.array_equal(E, O.energy_map(host, n, 0.3, 0.7))


def test_carve_loop_default_mode(ctx):
    """Default (fast fp32 map): each device seam is the oracle's seam of the
    device map it was found on."""
    img = load_input("natural_rgb_97x41.npy")
    seams, maps, frame, _ = _gpu_loop(ctx, img, 8, 0.5, 0.5, 12)
    for k, (s, m) in enumerate(zip(seams, maps)):
        assert np.array_equal(s, O.seam_find(m)), f"seam {k}"
    host = img
    for s in seams:
        host = carve(host, s)
    assert np.array_equal(frame, host)


# ---- dcte_carve: the whole loop behind one host call ----------------------
@pytest.mark.parametrize("n", [4, 8])
def test_host_carve_refined_equals_cpu_reference_loop(ctx, n):
    """Refine-all mode: every seam and the final frame equal the CPU loop on
    the reference's arithmetic."""
    img = load_input("wilber_rgb_74x59.npy")
    ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, 1.0)
    try:
        out, cols = ctx.carve(img, 10, n, 0.3, 0.7)
    finally:
        ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, -1)   # the per-N defaults
    host = img
    for k in range(10):
        ref_seam = O.seam_find(O.energy_map(host, n, 0.3, 0.7))
        assert np.array_equal(cols[k], ref_seam), f"seam {k}"
        host = carve(host, ref_seam)
    assert np.array_equal(out, host)


def test_host_carve_equals_device_loop(ctx):
    img = load_input("natural_rgb_97x41.npy")
    out, cols = ctx.carve(img, 12, 8, 0.5, 0.5)
    seams, _, frame, _ = _gpu_loop(ctx, img, 8, 0.5, 0.5, 12)
    assert np.array_equal(out, frame)
    assert np.array_equal(cols, np.stack(seams))


def test_host_carve_transposed(ctx):
    """Horizontal seams == vertical seams of the transposed frame, transposed back."""
    img = load_input("natural_rgb_73x59.npy")
    out, cols = ctx.carve(img, 9, 8, 0.3, 0.7, transposed=True)
    tr = np.ascontiguousarray(np.swapaxes(img, 0, 1))
    out_t, cols_t = ctx.carve(tr, 9, 8, 0.3, 0.7)
    assert out.shape == (59 - 9, 73, 3)
    assert np.array_equal(out, np.swapaxes(out_t, 0, 1))
    assert np.array_equal(cols, cols_t)


def test_host_carve_edges(ctx):
    img = load_input("natural_grey_200x120.npy")
    out, cols = ctx.carve(img, 0, 8)
    assert np.array_equal(out, img) and cols.shape == (0, img.shape[0])
    # strided source rows, carved down to one column
    view = img[:, 3:8]
    assert view.strides[0] != view.shape[1]
    out, cols = ctx.carve(view, 4, 8, 0.3, 0.7)
    assert out.shape == (img.shape[0], 1)
    host = np.ascontiguousarray(view)
    for s in cols:
        host = carve(host, s)
    assert np.array_equal(out, host)
    with pytest.raises(dctenergy.DcteError):
        ctx.carve(view, 5, 8)
    L = dctenergy.lib()
    o = np.empty(16, np.uint8)
    assert L.dcte_carve(ctx._h, view.ctypes.data, 5, 4, 1, 5, 8, 0.5, 0.5, 0, 5, 0,
                        o.ctypes.data, None) == dctenergy.DCTE_EINVAL
    assert L.dcte_carve(ctx._h, view.ctypes.data, 5, 4, 1, 5, 6, 0.5, 0.5, 0, 1, 0,
                        o.ctypes.data, None) == dctenergy.DCTE_EINVAL
