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


@pytest.mark.gpu
def test_config4_bench_eight_ranks_on_one_gpu():
    """BASELINE configs[3] as the driver's scaling run executes it, rehearsed
    on one GPU: bench.py --gpus 8 self-launches 8 RCCL ranks (one 16384^2 RGB
    frame, 2048-row bands, halos over RCCL point-to-point; distinct
    NCCL_HOSTIDs so RCCL accepts 8 ranks on one device), times 3 steps, then
    re-maps every band from regenerated rows without any exchange and
    requires bit-equality (check_bands_bit_exact), and gathers the bands to
    rank 0 (end_to_end).  Basis: the band halo of src/render.c:146-152."""
    import signal
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--shared-gpu",
           "--steps", "3", "--warmup", "1"]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=150)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)      # the rank processes too
        p.communicate()
        raise
    assert p.returncode == 0, err[-3000:]
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    res = json.loads(lines[0])
    print(json.dumps(res))
    assert res["n_gpus"] == 8 and res["scaling"] == "strong"
    assert res["config"]["global_frame"] == [16384, 16384] and res["config"]["rows_per_gpu"] == 2048
    assert res["check_bands_bit_exact"] is True
    assert res["end_to_end"]["gather_ms"] > 0
    assert res["value"] > 0 and res["roofline"]["launches_timed"] > 0
    # self-describing N > 1 lines: which RCCL transport carried the halos (here
    # the socket transport of the one-GPU rehearsal), each rank's kernel time,
    # the exchange time per step
    assert len(res["per_rank_kernel_ms"]) == 8 and min(res["per_rank_kernel_ms"]) > 0
    x = res["halo_exchange"]
    assert x["ms_per_exchange"] > 0 and x["halo_bytes_per_rank"] == (3 + 4) * 16384 * 3
    assert len(x["transport_per_rank"]) == 8 and all(x["transport_per_rank"]), x
    assert any("NET" in t for t in x["transport_per_rank"][0]), x
