"""One rank of tests/test_dist_rccl.py: the row-band path over RCCL (backend
"nccl") with the ranks sharing one device (bench.rank_env(shared_gpu=True)).

Each rank holds its band of ONE frame, receives its halo rows from its
neighbours by RCCL point-to-point (dctenergy.dist.exchange_halos, the rows
src/render.c:146-152 reads across the band edge), maps its own rows on the
device, builds its rows of the 8-bit energy layer with the frame-wide
{min, max} from one RCCL all-reduce, and gathers the bands to
rank 0 (§8e(3)).  Rank 0 compares everything with the single-device map of
the whole frame and prints one JSON line.
    python tests/rccl_worker.py H W N SEMANTICS     (RANK/WORLD_SIZE/... in env)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def main():
    import torch
    import torch.distributed as dist

    import dctenergy
    from dctenergy import dist as D
    from dctenergy import synth

    H, W, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    e, t = 0.3, 0.7
    ctx = dctenergy.Context(ngpus=1)
    try:
        band = D.make_band(H, rank, world, n)
        buf = torch.zeros((band.rows, W, 3), dtype=torch.uint8, device=dev)
        buf[band.top:band.top + band.own] = synth.natural_rows(band.Y0, band.own, W, 3, seed=5,
                                                               device=dev)
        part = torch.empty((band.own, W), dtype=torch.float32, device=dev)

        def rows(y0, y1):
            ctx.energy_map_tensor(buf, part[y0 - band.Y0:], n, e, t, h=H, in_row0=band.row0,
                                  y0=y0, y1=y1)

        reqs = D.exchange_halos(buf, band)
        i0, i1 = band.interior()
        rows(i0, i1)                          # own rows only, beside the exchange
        for r in reqs:
            r.wait()
        for a, b in band.edges():
            rows(a, b)
        full = synth.natural_rows(0, H, W, 3, seed=5, device=dev)
        halo_ok = torch.equal(buf, full[band.row0:band.row0 + band.rows])

        u8 = torch.empty((band.own, W), dtype=torch.uint8, device=dev)
        D.energy_image_u8(ctx, part, u8, dctenergy.DCTE_NORM_LQR)
        whole = D.gather_bands(part, band)
        whole_u8 = D.gather_bands(u8, band)
        torch.cuda.synchronize()
        ok = torch.tensor([int(halo_ok)], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if rank == 0:
            ref = torch.empty((H, W), dtype=torch.float32, device=dev)
            ctx.energy_map_tensor(full, ref, n, e, t)
            ref_u8 = ctx.energy_image_u8(full.cpu().numpy(), n, e, t, dctenergy.DCTE_NORM_LQR)
            torch.cuda.synchronize()
            print(json.dumps({
                "world": world, "frame": [H, W], "n": n,
                "rows_per_rank": [b - a for a, b in (D.band_rows(H, k, world) for k in range(world))],
                "halo_exact": bool(ok.item()),
                "map_bit_exact": bool(torch.equal(whole, ref)),
                "u8_bit_exact": bool((whole_u8.cpu().numpy() == ref_u8).all()),
            }), flush=True)
        else:
            assert whole is None and whole_u8 is None
    finally:
        ctx.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
