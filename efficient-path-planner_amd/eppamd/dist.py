"""Multi-GPU plumbing of the hot path: one process per GPU, independent
tracks per rank, and one exchange step — the all-gather of the final waypoint sets.

Backend "nccl" is RCCL on ROCm (xGMI between the GPUs of a node); "gloo" runs the same
code on CPU tensors (used by the world_size-2 tests in this container).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import numpy as np


def env():
    """(world_size, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str], extra_env: dict | None = None) -> int:
    """Runs `argv` as n processes, one per GPU of this node (RANK = LOCAL_RANK = i,
    WORLD_SIZE = n, rendezvous on 127.0.0.1), and returns the first non-zero exit code
    (0 if every rank succeeded).  The caller must not have initialised the GPU: the
    children each bind their own device."""
    port = str(free_port())
    procs = []
    for r in range(n):
        e = dict(os.environ)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port})
        e.update(extra_env or {})
        procs.append(subprocess.Popen(argv, env=e))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        print(f"spawn_ranks: exit codes {rcs}", file=sys.stderr)
    return bad[0] if bad else 0


class Dist:
    def __init__(self, ws: int, rank: int, local: int, backend: str = "nccl"):
        self.ws, self.rank, self.local, self.backend = ws, rank, local, backend
        self.device = "cpu"
        if ws > 1:
            import torch
            import torch.distributed as dist
            self.torch, self.dist = torch, dist
            if backend == "nccl":
                torch.cuda.set_device(local)
                self.device = f"cuda:{local}"
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group(backend)

    def barrier(self):
        if self.ws > 1:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.ws == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if self.ws == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def broadcast_bytes(self, b: bytes | None, n: int) -> bytes:
        """Rank 0's n bytes on every rank (bootstraps the product's RCCL communicator)."""
        if self.ws == 1:
            return b
        torch = self.torch
        t = torch.zeros(n, dtype=torch.uint8, device=self.device)
        if self.rank == 0:
            t.copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
        self.dist.broadcast(t, 0)
        return bytes(t.cpu().numpy().tobytes())

    def all_gather_waypoints(self, wp: np.ndarray) -> list[np.ndarray]:
        """All-gather of every rank's (W_r, 3) float64 waypoint set: the counts first, then
        the sets padded to max W (two collectives, a few KB each)."""
        wp = np.ascontiguousarray(np.asarray(wp, np.float64).reshape(-1, 3))
        if self.ws == 1:
            return [wp]
        torch, dist = self.torch, self.dist
        n = torch.tensor([len(wp)], dtype=torch.int64, device=self.device)
        ns = [torch.zeros_like(n) for _ in range(self.ws)]
        dist.all_gather(ns, n)
        counts = [int(x.item()) for x in ns]
        buf = torch.zeros((max(counts), 3), dtype=torch.float64, device=self.device)
        if len(wp):
            buf[:len(wp)] = torch.from_numpy(wp).to(self.device)
        outs = [torch.zeros_like(buf) for _ in range(self.ws)]
        dist.all_gather(outs, buf)
        return [o[:c].cpu().numpy() for o, c in zip(outs, counts)]

    def close(self):
        if self.ws > 1:
            self.dist.destroy_process_group()
