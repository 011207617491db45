"""world_size-2 gloo tests of the multi-GPU path's plumbing (eppamd.dist): the all-gather
of ragged waypoint sets, the max-over-ranks timing reduction and the error protocol that
bench.py runs over the product's RCCL communicator, plus the file
rendezvous that bootstraps that communicator without torch."""
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
    from eppamd.dist import env, make_group
    ws_, rank_, _ = env()
    d = make_group(ws_, rank_, "gloo")
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
    # the fields the GPU bench line carries for the multi-GPU leg: the communicator's own
    # rank count and every rank's value (full_plan.comm_n_ranks / ms_per_track_per_rank)
    assert r["comm_n_ranks"] == 2 and r["per_rank"] == [1.0, 2.0]
    # the bench line's parity at N > 1 (bench.py rank_parity / reduce_parity): every rank's
    # own counters, reduced -- sums of the mismatches, all-ranks of the equalities
    p = r["parity"]
    assert p["ranks"] == 2 and p["ok"] is True
    assert p["per_rank"]["c2_batch0_mismatches"] == [0, 0] and p["per_rank"]["c2_batch0_compared"] == [4096, 4096]
    assert p["c2_batch0_mismatches"] == 0 and p["c2_batch0_compared"] == 8192
    assert p["gathered_set_equal"] is True and p["per_rank"]["gathered_set_equal"] == [True, True]
    assert p["comm_n_ranks_equal"] is True


def test_bench_parity_mismatch_on_one_rank_is_reported():
    """One rank's mismatch reaches rank 0's line: its per-rank counter, the sum, ok false."""
    import json
    out = _run_bench_ws2(["--parity-flip-rank", "1"])
    assert out.returncode == 0, out.stderr[-2000:]
    p = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])["parity"]
    assert p["per_rank"]["c2_batch0_mismatches"] == [0, 1] and p["c2_batch0_mismatches"] == 1 and p["ok"] is False


def test_bench_rejects_mismatched_world_size():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launcher-check"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr


def _run_bench_ws2(extra, timeout=240):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launcher-check"] + extra,
                          env=env, capture_output=True, text=True, timeout=timeout)


def test_bench_rank_failure_in_plan_fails_every_rank():
    """Rank 1's plan fails: both ranks leave through the collective check (no rank waits in
    the next collective) and the job exits non-zero well inside the timeout."""
    import time
    t = time.monotonic()
    out = _run_bench_ws2(["--fail-rank", "1", "--fail-at", "plan"], timeout=180)
    assert out.returncode != 0
    assert time.monotonic() - t < 150
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    # both ranks report the same failed rank
    assert "rank 0: full plan failed on rank(s) [1]" in out.stderr, out.stderr[-2000:]
    assert "rank 1: full plan failed on rank(s) [1]" in out.stderr
    assert "Path not found" in out.stderr


def test_bench_rank_failure_at_exchange_fails_every_rank():
    """A rank that joins the waypoint all-gather with no set (count -1, the protocol of
    epp_comm_allgather_waypoints) makes the all-gather raise on every rank."""
    out = _run_bench_ws2(["--fail-rank", "0", "--fail-at", "exchange"], timeout=180)
    assert out.returncode != 0
    assert out.stderr.count("reported a failure") >= 2, out.stderr[-2000:]


def test_bench_rank_dying_after_counts_fails_every_rank():
    """A rank that dies after sending its count (its peers are then inside the data
    all-gather) must not leave them waiting: both ranks exit non-zero within the timeout,
    rank 0 through the exchange's own error (LegFailed), not the spawner's termination."""
    import time
    t = time.monotonic()
    out = _run_bench_ws2(["--fail-rank", "1", "--fail-at", "after-count"], timeout=180)
    assert out.returncode != 0
    assert time.monotonic() - t < 120
    assert "rank 1: dying after the counts" in out.stderr, out.stderr[-2000:]
    assert "bench.py rank 0: all-gather: a peer failed during the data exchange" in out.stderr, out.stderr[-2000:]
    assert "exit codes [1, 7]" in out.stderr, out.stderr[-2000:]


def _exchange_worker(rank, ws, d, q):
    import sys
    sys.path.insert(0, PKG)
    os.environ["EPP_RDV_DIR"] = d
    from eppamd.dist import file_exchange
    q.put((rank, file_exchange("init", rank, ws, {"rank": rank, "uid": "ab" * 64 if rank == 0 else ""})))


def test_file_rendezvous_ws2(tmp_path):
    """The torch-free bootstrap of the RCCL communicator: every rank sees every rank's
    payload (rank 0's id included)."""
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_exchange_worker, args=(r, ws, str(tmp_path), q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(ws):
        assert [x["rank"] for x in res[r]] == [0, 1] and res[r][0]["uid"] == "ab" * 64


def test_file_rendezvous_missing_rank_times_out(tmp_path, monkeypatch):
    """A rank that never arrives (died before the rendezvous) ends the wait with an error
    instead of a hang."""
    import pytest
    monkeypatch.setenv("EPP_RDV_DIR", str(tmp_path))
    import sys
    sys.path.insert(0, PKG)
    from eppamd.dist import file_exchange
    with pytest.raises(TimeoutError, match=r"ranks \[1\]"):
        file_exchange("init", 0, 2, {"ok": True}, timeout=0.5)


def test_spawn_ranks_terminates_hung_peers():
    """spawn_ranks: when one rank exits non-zero the others get a grace period and are
    then terminated (a rank stuck in a collective cannot hang the job)."""
    import sys
    import time
    sys.path.insert(0, PKG)
    from eppamd.dist import spawn_ranks
    code = "import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(600)"
    t = time.monotonic()
    rc = spawn_ranks(2, [sys.executable, "-c", code], grace_s=1.0)
    assert rc != 0 and time.monotonic() - t < 60
