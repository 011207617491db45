"""OnlineTrajGenerator.pre_compute_traj on the bench's C4 track without kernel
serialisation (diagnostics).  argv[1]: repetitions."""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
from eppamd import capi, config, synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
    cfg["world_properties"]["lower_bound"] = [-6, -6, 0]
    cfg["world_properties"]["upper_bound"] = [6, 6, 2]
    cfg["path_planner_properties"]["samples_fmt"] = 65536
    geom = config.geometry(cfg)
    gates, obstacles = synth.track_world(100)
    cps = synth.gate_checkpoints(gates, geom.gate_height, 0.55)
    import online_traj_planner as otp

    fd, path = tempfile.mkstemp(suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(cfg, f)
    otg = otp.OnlineTrajGenerator(cps[0], cps[-1], gates, obstacles, path)
    for r in range(reps):
        print("pre_compute_traj", r, flush=True)
        otg.pre_compute_traj(0.0)
        print("  stats", otg.planner_stats(), flush=True)
    capi.sync()
    print("done", otg.get_planned_traj().shape, flush=True)


if __name__ == "__main__":
    main()
