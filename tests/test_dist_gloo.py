"""Multi-rank path on CPU: world_size 2 and 3 with gloo.

The band geometry + halo exchange (dctenergy.dist) must hand every rank
exactly the rows of the global frame its outputs read; the per-band oracle
maps then concatenate to the full-frame map bit-exactly.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, weak, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "dct-carver_amd"), os.path.join(root, "tests")]
    import oracle_py as O
    from dctenergy import dist as D
    from dctenergy import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W = 37
        rows_per_rank = 23 if weak else None
        H = world * 23 if weak else 61
        band = D.make_band(H, rank, world, n, rows_per_rank)
        buf = torch.zeros((band.rows, W, 3), dtype=torch.uint8)
        own = synth.natural_rows(band.Y0, band.own, W, 3, seed=7, device="cpu")
        buf[band.top:band.top + band.own] = own
        for r in D.exchange_halos(buf, band):
            r.wait()
        full = synth.natural_rows(0, H, W, 3, seed=7, device="cpu")
        expect = full[band.row0:band.row0 + band.rows]
        halo_ok = bool(torch.equal(buf, expect))
        # band-local oracle map: rows [Y0, Y1) from band rows only
        img = buf.numpy()
        r = n // 2
        outs = []
        for y in range(band.Y0, band.Y1):
            rows = [min(max(y + j, 0), H - 1) - band.row0 for j in range(-(r - 1), r + 1)]
            win_rows = np.stack([img[i] for i in rows])
            outs.append(O.energy_map(win_rows, n, 0.3, 0.7, y0=r - 1, y1=r)[0])
        part = np.stack(outs)
        # frame-wide min/max by one all-reduce, each band's
        # u8 rows normalised with it; §8e(3): bands gathered to rank 0
        mm = D.global_minmax(torch.tensor([part.min(), part.max()], dtype=torch.float32))
        u8 = O.normalize_lqr(part, minmax=mm.numpy())
        u8p = O.normalize_preview(part, 3, minmax=mm.numpy())
        whole = D.gather_bands(torch.from_numpy(part), band)
        whole_u8 = D.gather_bands(torch.from_numpy(u8), band)
        whole_u8p = D.gather_bands(torch.from_numpy(u8p), band)
        if rank == 0:
            ref = O.energy_map(full.numpy(), n, 0.3, 0.7)
            ok = (np.array_equal(whole.numpy(), ref)
                  and mm.tolist() == [float(ref.min()), float(ref.max())]
                  and np.array_equal(whole_u8.numpy(), O.normalize_lqr(ref))
                  and np.array_equal(whole_u8p.numpy(), O.normalize_preview(ref, 3)))
            q.put((halo_ok, bool(ok)))
        else:
            assert whole is None and whole_u8 is None
            q.put((halo_ok, True))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,weak", [(2, 8, False), (2, 16, True), (3, 4, False), (2, 2, True)])
def test_band_halo_exchange_gloo(world, n, weak):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, weak, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(h for h, _ in res), "halo rows differ from the global frame"
    assert all(m for _, m in res), "band maps do not compose to the full-frame map"


def test_band_geometry():
    from dctenergy import dist as D
    b = D.make_band(16384 * 4, 2, 4, 8, 16384)
    assert (b.Y0, b.Y1, b.top, b.bot, b.rows, b.row0) == (32768, 49152, 3, 4, 16391, 32765)
    assert b.interior() == (32771, 49148)
    assert b.edges() == [(32768, 32771), (49148, 49152)]
    b0 = D.make_band(100, 0, 1, 16)
    assert (b0.top, b0.bot, b0.interior(), b0.edges()) == (0, 0, (0, 100), [])
    with pytest.raises(ValueError):
        D.make_band(12, 1, 4, 16)


def test_band_geometry_strong_bench():
    """bench.py --strong: one 16384^2 frame over 1/2/4/8 ranks (configs[3])."""
    from dctenergy import dist as D
    for world in (1, 2, 4, 8):
        bands = [D.make_band(16384, k, world, 8) for k in range(world)]
        assert [b.own for b in bands] == [16384 // world] * world
        assert bands[0].Y0 == 0 and bands[-1].Y1 == 16384
        assert all(a.Y1 == b.Y0 for a, b in zip(bands, bands[1:]))
        for b in bands:
            assert b.top == (3 if b.Y0 > 0 else 0) and b.bot == (4 if b.Y1 < 16384 else 0)
