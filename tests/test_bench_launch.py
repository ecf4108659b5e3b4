"""bench.py's own rank launcher on CPU (no GPU): `--gpus N` without an
external torch.distributed.run starts N rank processes, they rendezvous on
127.0.0.1 over gloo, split ONE frame into row bands (strong scaling, BASELINE
configs[3]) or stack per-rank bands (--weak), exchange the halo rows and find
them equal to the global frame (src/render.c:146-152 reads N/2-1 rows above
and N/2 below)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-rehearsal", *args],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 prints exactly one line
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus,n", [(2, 8), (3, 16), (4, 8)])
def test_self_launch_strong(gpus, n):
    res = _run("--gpus", str(gpus), "--n", str(n), "--size", "101")
    assert res["n_gpus"] == gpus and res["scaling"] == "strong"
    assert res["global_frame"] == [101, 101]
    assert sum(res["rows_per_rank"]) == 101
    assert res["check_halo_exact"] is True


def test_self_launch_weak():
    res = _run("--gpus", "2", "--n", "8", "--size", "40", "--weak")
    assert res["scaling"] == "weak" and res["global_frame"] == [80, 40]
    assert res["rows_per_rank"] == [40, 40] and res["check_halo_exact"] is True


def test_single_rank():
    res = _run("--size", "33")
    assert res["n_gpus"] == 1 and res["rows_per_rank"] == [33]


def test_failing_rank_fails_the_launch():
    """A rank that dies (here: a band too small for the window, which
    dctenergy.dist rejects) makes the launcher stop the others and exit
    non-zero instead of hanging in the rendezvous or a collective."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-rehearsal",
                        "--gpus", "4", "--n", "16", "--size", "20"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "needs >=" in r.stderr


def test_rank_env_shared_gpu():
    """--shared-gpu: every rank names its own host to RCCL (NCCL_HOSTID), so
    ranks that share a device are not refused as duplicates; plain launches
    leave RCCL's host detection alone."""
    sys.path.insert(0, ROOT)
    import bench
    envs = [bench.rank_env(r, 3, 4242, shared_gpu=True) for r in range(3)]
    assert len({e["NCCL_HOSTID"] for e in envs}) == 3
    assert all(e["NCCL_SOCKET_IFNAME"] == "lo" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert [e["RANK"] for e in envs] == ["0", "1", "2"] and envs[0]["WORLD_SIZE"] == "3"
    plain = bench.rank_env(1, 2, 4242)
    assert "NCCL_HOSTID" not in plain or plain["NCCL_HOSTID"] == os.environ.get("NCCL_HOSTID")
