"""world_size-2 gloo test of the multi-GPU path's exchange step (eppamd.dist): the
all-gather of ragged waypoint sets and the max-over-ranks timing reduction that bench.py
uses over RCCL."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from conftest import PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    import sys
    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    from eppamd.dist import Dist, env
    d = Dist(*env(), backend="gloo")
    wp = np.arange(3 * (4 + 3 * rank), dtype=np.float64).reshape(-1, 3) + 100 * rank
    sets = d.all_gather_waypoints(wp)
    mx = d.max(float(rank + 1))
    sm = d.sum(float(rank + 1))
    empty = d.all_gather_waypoints(np.zeros((0, 3)) if rank == 0 else wp)
    d.barrier()
    d.close()
    q.put((rank, [s.tolist() for s in sets], mx, sm, [len(e) for e in empty]))


def test_all_gather_waypoints_gloo_ws2():
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, sets, mx, sm, empty in res:
        assert mx == 2.0 and sm == 3.0
        assert len(sets) == 2
        for r in range(ws):
            exp = np.arange(3 * (4 + 3 * r), dtype=np.float64).reshape(-1, 3) + 100 * r
            assert np.array_equal(np.array(sets[r]), exp)
        assert empty == [0, 7]


def test_bench_spawns_ranks_gloo_ws2():
    """`bench.py --gpus 2` without a launcher spawns one process per rank (RANK/LOCAL_RANK/
    WORLD_SIZE set before any device call) and reports n_gpus = 2 from rank 0; the
    --launcher-check mode runs that plumbing with gloo instead of the GPU work."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launcher-check"],
                         env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["ranks_seen"] == [0, 1] and r["waypoints_per_track"] == [5, 6]
    assert r["max_over_ranks"] == 2.0 and r["local_rank"] == 0


def test_bench_rejects_mismatched_world_size():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launcher-check"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr
