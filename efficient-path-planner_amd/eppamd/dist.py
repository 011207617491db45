"""Multi-GPU plumbing of the hot path: one process per GPU, independent
tracks per rank, and one exchange step — the all-gather of the final waypoint sets.

Groups (the collectives a multi-rank caller needs: barrier, max/sum over ranks, the
waypoint all-gather, and a collective error check):

* ``RcclGroup`` — the GPU path.  Torch-free: the product's own RCCL communicator
  (``epp_comm_*`` in libepp.so, over xGMI), bootstrapped by a file rendezvous (rank 0
  writes the 128-byte RCCL id), so libepp runs on the same HIP runtime (ROCm's) at every
  rank count.
* ``Solo`` — one rank: every collective is the identity.
* ``GlooGroup`` — the same interface over torch.distributed "gloo" on CPU tensors (the
  world_size-2 tests in this container).

Error protocol: a leg that fails on some rank must fail on every rank, or the others
wait in the next collective forever.  ``Group.check(err)`` is a collective: every rank
passes its own exception (or None), the flags are summed over the ranks, and every rank
raises ``LegFailed`` naming the failed ranks if any did.  The waypoint all-gather carries
the same protocol inside the product (a failed rank sends count -1, epp.h).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np


class LegFailed(RuntimeError):
    """Raised on every rank when a leg failed on at least one rank."""

    def __init__(self, failed: list[int], msg: str):
        super().__init__(msg)
        self.failed = failed


def env():
    """(world_size, rank, local_rank) from the launcher's environment (torchrun or
    spawn_ranks)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str], extra_env: dict | None = None, grace_s: float = 30.0) -> int:
    """Runs `argv` as n processes, one per GPU of this node (RANK = LOCAL_RANK = i,
    WORLD_SIZE = n, a fresh rendezvous directory in EPP_RDV_DIR), and returns the first
    non-zero exit code (0 if every rank succeeded).  When a rank fails the others get
    `grace_s` seconds to finish (they normally fail too, through the error protocol) and
    are then terminated, so one failed rank cannot leave the job hanging.  The caller must
    not have initialised the GPU: the children each bind their own device."""
    port = str(free_port())
    rdv = tempfile.mkdtemp(prefix="epp_rdv_")
    procs = []
    for r in range(n):
        e = dict(os.environ)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port, "EPP_RDV_DIR": rdv})
        e.update(extra_env or {})
        procs.append(subprocess.Popen(argv, env=e))
    failed_at = None
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            break
        if failed_at is None and any(rc not in (None, 0) for rc in rcs):
            failed_at = time.monotonic()
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.05)
    rcs = [p.wait() for p in procs]
    _rmtree(rdv)
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        print(f"spawn_ranks: exit codes {rcs}", file=sys.stderr)
    return bad[0] if bad else 0


def _rmtree(d: str) -> None:
    import shutil
    shutil.rmtree(d, ignore_errors=True)


def rendezvous_dir() -> str:
    """Directory the ranks of one job share: EPP_RDV_DIR (spawn_ranks) or, under torchrun,
    one keyed by the launcher process (every worker's parent) and the job's port."""
    d = os.environ.get("EPP_RDV_DIR")
    if d:
        return d
    port = os.environ.get("MASTER_PORT", "0")
    restart = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    return os.path.join(tempfile.gettempdir(), f"epp_rdv_{os.getppid()}_{port}_{restart}")


def file_exchange(tag: str, rank: int, ws: int, payload: dict, timeout: float = 120.0) -> list[dict]:
    """Every rank's JSON payload, through files in rendezvous_dir() (one node).  Each rank
    writes `<tag>.<rank>` atomically and waits for all ws files; raises TimeoutError if a
    rank has not written within `timeout` (it died before the rendezvous)."""
    d = rendezvous_dir()
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"{tag}.{rank}")
    tmp = path + f".tmp{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(payload, f)
    os.replace(tmp, path)
    out, t0 = [None] * ws, time.monotonic()
    while True:
        for r in range(ws):
            if out[r] is None:
                try:
                    with open(os.path.join(d, f"{tag}.{r}")) as f:
                        out[r] = json.load(f)
                except (OSError, ValueError):
                    pass
        if all(o is not None for o in out):
            return out
        if time.monotonic() - t0 > timeout:
            missing = [r for r in range(ws) if out[r] is None]
            raise TimeoutError(f"rendezvous {tag!r} in {d}: ranks {missing} did not arrive within {timeout:.0f} s")
        time.sleep(0.01)


class Group:
    ws: int = 1
    rank: int = 0
    kind: str = ""

    def barrier(self) -> None:
        raise NotImplementedError

    def _reduce(self, x: np.ndarray, op: str) -> np.ndarray:
        raise NotImplementedError

    def max(self, x: float) -> float:
        return float(self._reduce(np.array([x], np.float64), "max")[0])

    def sum(self, x: float) -> float:
        return float(self._reduce(np.array([x], np.float64), "sum")[0])

    def gather(self, x: float) -> list[float]:
        """Every rank's value of x, in rank order (a sum over one-hot vectors)."""
        v = np.zeros(self.ws, np.float64)
        v[self.rank] = x
        return [float(y) for y in self._reduce(v, "sum")]

    def all_gather_waypoints(self, wp: np.ndarray | None) -> list[np.ndarray]:
        raise NotImplementedError

    def n_ranks(self) -> int:
        """The ranks the group's own communicator reports (RCCL's count on the GPU path),
        not the launcher's WORLD_SIZE."""
        raise NotImplementedError

    def check(self, err: BaseException | None, what: str = "leg") -> None:
        """Collective: raises LegFailed on every rank if `err` is set on any rank."""
        flags = np.zeros(self.ws, np.float64)
        flags[self.rank] = 1.0 if err is not None else 0.0
        flags = self._reduce(flags, "sum")
        failed = [r for r in range(self.ws) if flags[r] > 0]
        if failed:
            mine = f": {type(err).__name__}: {err}" if err is not None else ""
            raise LegFailed(failed, f"{what} failed on rank(s) {failed} (this is rank {self.rank}{mine})")

    def run(self, fn, what: str = "leg"):
        """fn() on this rank, then check(): either every rank returns or every rank raises."""
        err, res = None, None
        try:
            res = fn()
        except Exception as e:  # noqa: BLE001 — reported to every rank by check()
            err = e
        self.check(err, what)
        return res

    def close(self) -> None:
        pass


class Solo(Group):
    kind = "solo"

    def barrier(self) -> None:
        pass

    def _reduce(self, x, op):
        return np.asarray(x, np.float64)

    def n_ranks(self) -> int:
        return 1

    def all_gather_waypoints(self, wp):
        if wp is None:
            raise LegFailed([0], "all-gather: rank 0 reported a failure")
        return [np.ascontiguousarray(np.asarray(wp, np.float64).reshape(-1, 3))]


class RcclGroup(Group):
    """The product's RCCL communicator (libepp epp_comm_*) as the job's process group.
    Bootstrap (collective, through file_exchange): every rank reports whether RCCL loads;
    rank 0 adds the RCCL unique id; all ranks init only if every rank is ready, else all
    raise — a rank that cannot join never leaves the others inside ncclCommInitRank."""
    kind = "rccl (epp_comm)"
    # deadline of every collective (epp_comm_set_timeout): a peer that died without an RCCL
    # asynchronous error fails the job after this long instead of the library's 120 s default
    COLLECTIVE_TIMEOUT_S = 30.0

    def __init__(self, ws: int, rank: int, timeout: float = 120.0, collective_timeout_s: float = COLLECTIVE_TIMEOUT_S):
        from eppamd import capi
        self.capi, self.ws, self.rank = capi, ws, rank
        ok, msg, uid = True, "", ""
        try:
            capi.check(capi.lib().epp_comm_available())
            if rank == 0:
                uid = capi.Comm.unique_id().hex()
        except Exception as e:  # noqa: BLE001 — shared with every rank below
            ok, msg = False, f"{type(e).__name__}: {e}"
        if ws == 1:
            if not ok:
                raise RuntimeError(f"RcclGroup: {msg}")
            peers = [{"ok": True, "uid": uid}]
        else:
            peers = file_exchange("init", rank, ws, {"ok": ok, "msg": msg, "uid": uid}, timeout)
            bad = {r: p["msg"] for r, p in enumerate(peers) if not p["ok"]}
            if bad:
                raise LegFailed(sorted(bad), f"RcclGroup: ranks not ready: {bad}")
        self.comm = capi.Comm(bytes.fromhex(peers[0]["uid"]), ws, rank)
        self.comm.set_timeout(collective_timeout_s)
        self.collective_timeout_s = collective_timeout_s
        if ws > 1:
            self.comm.barrier()  # every rank has read the rendezvous files
            if rank == 0:
                _rmtree(rendezvous_dir())

    def barrier(self) -> None:
        self.comm.barrier()

    def n_ranks(self) -> int:
        return int(self.comm.n_ranks)  # epp_comm_rank: RCCL's own rank count

    def _reduce(self, x, op):
        c = self.capi
        return self.comm.allreduce(x, {"sum": c.EPP_REDUCE_SUM, "max": c.EPP_REDUCE_MAX, "min": c.EPP_REDUCE_MIN}[op])

    def all_gather_waypoints(self, wp):
        try:
            return self.comm.allgather_waypoints(wp)
        except self.capi.EppError as e:
            if e.code == self.capi.EPP_ERR_PEER:
                raise LegFailed([r for r, c in enumerate(e.counts) if c < 0], str(e)) from e
            raise

    def close(self) -> None:
        self.comm.close()


class GlooGroup(Group):
    """torch.distributed "gloo" (CPU tensors): the world_size > 1 tests without a GPU."""
    kind = "gloo"

    def __init__(self, ws: int, rank: int, timeout_s: float = 60.0):
        import datetime

        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.ws, self.rank = torch, dist, ws, rank
        if ws > 1:  # (a collective a peer never joins fails after timeout_s, as epp_comm's deadline)
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=timeout_s))

    def barrier(self) -> None:
        if self.ws > 1:
            self.dist.barrier()

    def n_ranks(self) -> int:
        return int(self.dist.get_world_size()) if self.ws > 1 else 1

    def _reduce(self, x, op):
        x = np.asarray(x, np.float64)
        if self.ws == 1:
            return x
        t = self.torch.from_numpy(x.copy())
        rop = {"sum": self.dist.ReduceOp.SUM, "max": self.dist.ReduceOp.MAX, "min": self.dist.ReduceOp.MIN}[op]
        self.dist.all_reduce(t, op=rop)
        return t.numpy()

    def all_gather_waypoints(self, wp):
        """Counts first (-1 = this rank failed: every rank raises LegFailed), then the sets
        padded to the longest — the protocol of epp_comm_allgather_waypoints."""
        torch, dist = self.torch, self.dist
        wp = None if wp is None else np.ascontiguousarray(np.asarray(wp, np.float64).reshape(-1, 3))
        if self.ws == 1:
            return Solo().all_gather_waypoints(wp)
        n = torch.tensor([-1 if wp is None else len(wp)], dtype=torch.int64)
        ns = [torch.zeros_like(n) for _ in range(self.ws)]
        dist.all_gather(ns, n)
        counts = [int(x.item()) for x in ns]
        failed = [r for r, c in enumerate(counts) if c < 0]
        if failed:
            raise LegFailed(failed, f"all-gather: rank(s) {failed} reported a failure")
        buf = torch.zeros((max(max(counts), 1), 3), dtype=torch.float64)
        if len(wp):
            buf[:len(wp)] = torch.from_numpy(wp)
        outs = [torch.zeros_like(buf) for _ in range(self.ws)]
        try:  # a peer that dies (or hangs) past the counts: an error here, not a hang
            dist.all_gather(outs, buf)
        except RuntimeError as e:
            raise LegFailed([], f"all-gather: a peer failed during the data exchange ({e})") from e
        return [o[:c].numpy() for o, c in zip(outs, counts)]

    def close(self) -> None:
        if self.ws > 1:
            self.dist.destroy_process_group()


def make_group(ws: int, rank: int, backend: str) -> Group:
    """backend "rccl": the product communicator (GPU ranks; Solo at ws = 1); "gloo": CPU."""
    if backend == "gloo":
        return GlooGroup(ws, rank)
    if backend == "rccl":
        return Solo() if ws == 1 else RcclGroup(ws, rank)
    raise ValueError(f"unknown backend {backend!r}")
