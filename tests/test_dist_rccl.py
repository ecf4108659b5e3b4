"""The row-band path over RCCL on the GPU: halo exchange by
RCCL point-to-point, the frame-wide {min, max} all-reduce of the 8-bit layer
and the band gather, checked bit-exactly against the single-device map.

A one-GPU box hosts the ranks on one device: each rank gets its own
NCCL_HOSTID (bench.rank_env(shared_gpu=True)), so RCCL connects them through
its socket transport on loopback instead of xGMI -- the transport differs
from an 8-GPU node, the RCCL calls and stream ordering are the same ones.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _launch(world, H, W, n):
    import bench
    port = bench.free_port()
    procs = []
    for r in range(world):
        env = bench.rank_env(r, world, port, shared_gpu=True)
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "tests", "rccl_worker.py"), str(H), str(W), str(n)],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=150))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, (_, err) in zip(procs, outs):
        assert p.returncode == 0, err[-3000:]
    lines = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1, outs[0][0]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("world,H,W,n", [(2, 1003, 517, 8), (3, 700, 301, 16)])
def test_bands_over_rccl(world, H, W, n):
    res = _launch(world, H, W, n)
    print(res)
    assert res["world"] == world and sum(res["rows_per_rank"]) == H
    assert res["halo_exact"], "halo rows received over RCCL differ from the global frame"
    assert res["map_bit_exact"], "gathered band maps differ from the single-device map"
    assert res["u8_bit_exact"], "band-normalised u8 layer differs from the single-device layer"
