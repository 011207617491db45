"""RCCL probe (diagnostics): the product's exchange step (epp_comm_*) on one rank, with
PyTorch imported before libepp.so ("torch-first": the process then runs on torch's bundled
HIP runtime and RCCL), after it ("epp-first": ROCm's), or not at all ("no-torch").
python scripts/rccl_probe.py {torch-first|epp-first|no-torch}"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
mode = sys.argv[1]
if mode == "torch-first":
    import torch  # noqa: F401
from eppamd import capi  # noqa: E402

L = capi.lib()
if mode == "epp-first":
    import torch  # noqa: F401,E402
import numpy as np  # noqa: E402


def loaded(sub):
    return sorted({ln.split()[-1] for ln in open("/proc/self/maps") if sub in ln and ln.split()[-1].startswith("/")})


try:
    uid = capi.Comm.unique_id()
    c = capi.Comm(uid, 1, 0)
    wp = np.arange(30, dtype=np.float64).reshape(10, 3)
    ok = np.array_equal(c.allgather_waypoints(wp, cap=16)[0], wp)
    c.close()
    res = "ok" if ok else "WRONG"
except capi.EppError as e:
    res = f"error: {e}"
print(mode, res, "| hip:", loaded("libamdhip64"), "| rccl:", loaded("librccl"), flush=True)
