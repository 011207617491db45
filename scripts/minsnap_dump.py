"""Dump the GPU's min-snap coefficients of chosen C5 bench problems (diagnostics, round 6):
the batch kernel with its own Nfabian times and with the oracle's times given
(epp_minsnap_batch_times), so the accuracy analysis can run on the CPU side.
    python scripts/minsnap_dump.py OUT.npz [problem ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "efficient-path-planner_amd")]
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from eppamd import capi, synth  # noqa: E402

ids = [int(a) for a in sys.argv[2:]] or [184, 1540, 1742, 2942]
tracks = [synth.random_track_waypoints(10_000 + k, 12) for k in ids]
Ts, Cs, st = capi.minsnap_batch(tracks, 1.0, 2.0)
Tr = np.array([O.minsnap_track(w, 1.0, 2.0)[0] for w in tracks])
Ct, st2 = capi.minsnap_batch_times(tracks, list(Tr))
np.savez(sys.argv[1], ids=np.array(ids), wp=np.array(tracks), T_gpu=np.array(Ts), C_gpu=np.array(Cs),
         T_oracle=Tr, C_gpu_oracle_times=np.array(Ct))
print("saved", sys.argv[1])
