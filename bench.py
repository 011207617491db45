"""bench.py — validity checks/sec on MI355X (BASELINE.json metric), one JSON line.

Workload at N=1 = BASELINE configs[1] (C2): one track, 8 gates, 64 OBBs (40 gate + 24
obstacle), 1,048,576 uniformly sampled states per step, StateValidator semantics
(World::checkPointValidity(p, canPassGate=false), src/World.cpp:80-104).  Every step
checks a FRESH batch of 1M states (a sampler streaming new samples): 16 resident batches
(400 MB, larger than the 256 MB Infinity Cache) are rotated, so the timed kernels stream
from HBM.  Inputs are resident in HBM before the timed region.

Multi-GPU: one process per GPU (torchrun, or `--gpus N` spawning its own ranks); every
rank checks its own stream of states against its own copy of the world (independent
samplers, no data-path collective: "scaling": "weak"); ranks synchronise with a barrier
and the slowest rank's time is used.  The ranks' collectives (barrier, max over ranks, the
waypoint all-gather) go through the product's own RCCL communicator (epp_comm_* in
libepp.so, bootstrapped by a file rendezvous: eppamd/dist.py) — no torch in a GPU rank, so
libepp runs on ROCm's HIP runtime at every N.  A leg that fails on one rank fails on every
rank (Group.check / the all-gather's count -1) and the job exits non-zero.

Full plan ms/track (the metric's second half, BASELINE configs[3] = C4): every rank plans
its own randomised track (world seed 100 + rank, 8 gates, 24 obstacles, bounds
[-6,6]^2 x [0,2]) end to end through the C++ API (OnlineTrajGenerator::preComputeTraj:
9 gate-to-gate batch plans with 65,536 samples and k = 16 neighbours each, includeGates2,
min-snap fit, sampling at dt = 0.1), then the final waypoint sets of all tracks are
all-gathered over RCCL (the path's only exchange step).

Side measurements (same JSON line, not the headline value): C3 motion checks (512 OBBs,
analytic and 32-step discretised), the C5 batched min-snap refit (4096 x 12 segments),
and the CPU oracle timed on the host (cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]

N_STATES = 1 << 20
N_BATCHES = 16
BYTES_PER_STATE = 25  # 24 B xyz read + 1 B flag written
BYTES_PER_EDGE = 49
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def timed_kernel_ms(capi, stream, fn, reps):
    """Average device time per launch of `fn`: HIP events on `stream` around `reps`
    back-to-back launches (the steady state the timed region runs in; per-launch event
    pairs would add the host launch latency to every launch)."""
    import ctypes as C
    L = capi.lib()
    e0, e1 = C.c_void_p(), C.c_void_p()
    capi.check(L.epp_event_create(C.byref(e0)))
    capi.check(L.epp_event_create(C.byref(e1)))
    capi.check(L.epp_event_record(e0, stream))
    for r in range(reps):
        fn(r)
    capi.check(L.epp_event_record(e1, stream))
    ms = C.c_float()
    capi.check(L.epp_event_elapsed_ms(e0, e1, C.byref(ms)))
    L.epp_event_destroy(e0)
    L.epp_event_destroy(e1)
    return ms.value / reps


def json_stdout():
    """stdout carries only the one JSON line: everything else written to fd 1 from here on
    (the library's own messages, e.g. PathWriter's "Folder created") goes to stderr."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)  # ~17 ms timed: host hiccups amortised
    ap.add_argument("--warmup", type=int, default=200)  # ~2 ms of GPU work: clocks settle
    ap.add_argument("--no-side", action="store_true", help="skip the side measurements (C3, C5)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--no-plan", action="store_true", help="skip the full-plan (C4) leg")
    ap.add_argument("--plan-reps", type=int, default=20)  # the seed changes per call: ~1 in 6 takes the slower symmetrised search
    ap.add_argument("--host-loop", action="store_true",
                    help="launch the timed steps from a host loop instead of replaying a captured HIP graph")
    ap.add_argument("--launcher-check", action="store_true",
                    help="CPU-only: run the rank launch + gloo exchange plumbing and print one JSON line")
    ap.add_argument("--fail-rank", type=int, default=-1,
                    help="with --launcher-check: this rank's (simulated) plan fails (error-protocol test)")
    ap.add_argument("--fail-at", choices=("plan", "exchange", "after-count"), default="plan",
                    help="with --fail-rank: fail inside the plan leg (collective check), at the all-gather (count -1) "
                         "or die right after sending its count (the peers are then inside the data all-gather)")
    ap.add_argument("--parity-flip-rank", type=int, default=-1,
                    help="with --launcher-check: this rank reports one C2 flag mismatch (parity reduction test)")
    args = ap.parse_args()

    from eppamd.dist import LegFailed, env, make_group, spawn_ranks
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` without a launcher: one child process per GPU (rank = local
        # rank = GPU index), started before this process touches the GPU
        sys.exit(spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    out_stream = json_stdout()
    ws, rank, local = env()
    if ws != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws} (launch one process per GPU)")
    try:
        if args.launcher_check:
            return launcher_check(ws, rank, local, out_stream, args.fail_rank, args.fail_at, args.parity_flip_rank)
        run(args, ws, rank, local, out_stream)
    except LegFailed as e:
        # exit at once: a process group whose peer died can abort the interpreter's teardown
        # (a joinable transport thread -> std::terminate, exit -6 instead of 1)
        print(f"bench.py rank {rank}: {e}", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(1)


def run(args, ws, rank, local, out_stream):
    import ctypes as C

    from eppamd import capi, config, synth
    from eppamd.dist import make_group

    L = capi.lib()
    capi.check(L.epp_set_device(local))
    dist = make_group(ws, rank, "rccl")  # the product's communicator (Solo at N = 1)
    stream = C.c_void_p()
    capi.check(L.epp_stream_create(C.byref(stream)))
    stream = stream.value

    cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
    geom = config.geometry(cfg)
    rg, ro = config.inflate_radii(cfg)
    gates, obstacles = synth.track_world(42)
    obbs = capi.build_obbs(geom, gates, obstacles)
    world = capi.World(obbs, rg, ro)
    lo, hi = synth.C2_BOUNDS

    # ---- the metric's second half and the side legs (before the headline's timed region)
    plan = full_plan(dist, rank, args.plan_reps) if not args.no_plan else None
    side, c5_inputs = {}, None
    if not args.no_side:  # rank 0 only; collective so that a failure there ends every rank
        side, c5_inputs = dist.run(lambda: side_measurements(capi, L, stream, geom, cfg, rg, ro)
                                   if rank == 0 else ({}, None), "side legs")

    # ---- resident inputs: 16 fresh 1M-state batches per rank ------------------------
    d_states = capi.DeviceBuffer(N_BATCHES * N_STATES * 24)
    for b in range(N_BATCHES):
        pts = synth.sample_states(7 + 1000 * rank, lo, hi, N_STATES, start=b * N_STATES)
        capi.check(L.epp_memcpy_h2d(d_states.ptr + b * N_STATES * 24, pts.ctypes.data, pts.nbytes, stream))
    d_valid = capi.DeviceBuffer(N_STATES)

    def step(i):
        world.check_states_dev(d_states.ptr + (i % N_BATCHES) * N_STATES * 24, N_STATES, 0, d_valid.ptr,
                               stream=stream)

    for i in range(args.warmup):
        step(i)
    capi.check(L.epp_stream_sync(stream))
    # The K timed steps (the same K launches the host loop would make) are captured once
    # into a HIP graph and replayed, so the kernels dispatch back to back whatever the
    # host launch path costs (an ~8 us kernel is about one host-side launch; under
    # rocprofv3's kernel trace a host loop runs at ~11 us per launch).
    graph = None
    ev0, ev1 = C.c_void_p(), C.c_void_p()
    for ev in (ev0, ev1):
        capi.check(L.epp_event_create(C.byref(ev)))
    if not args.host_loop:
        g = C.c_void_p()
        try:
            capi.check(L.epp_graph_begin(stream))
            for i in range(args.steps):
                step(i)
            capi.check(L.epp_graph_end(stream, C.byref(g)))
            graph = g.value
            # one untimed replay: the graph's first launch pays its upload to the device;
            # the timed replay below is the steady state (the same K launches, same work)
            capi.check(L.epp_graph_launch(graph, stream))
        except capi.EppError as e:
            print(f"bench: graph capture failed ({e}); timing the host loop", file=sys.stderr)
            if L.epp_graph_end(stream, C.byref(g)) == 0:  # leave capture mode if still in it
                L.epp_graph_destroy(g)
            graph = None
        capi.check(L.epp_stream_sync(stream))

    def run_steps():
        if graph is not None:
            capi.check(L.epp_graph_launch(graph, stream))
        else:
            for i in range(args.steps):
                step(i)

    dist.barrier()
    capi.check(L.epp_stream_sync(stream))
    t0 = time.perf_counter()
    capi.check(L.epp_event_record(ev0, stream))
    run_steps()
    capi.check(L.epp_event_record(ev1, stream))
    capi.check(L.epp_stream_sync(stream))
    dist.barrier()
    t1 = time.perf_counter()
    elapsed = dist.max(t1 - t0)
    value = ws * N_STATES * args.steps / elapsed

    # dominant kernel's average launch time: HIP events on the launch stream bracketing
    # the timed region's K back-to-back launches (the only kernel in it).  The bracket
    # also holds the graph's submission; a replay queued behind a host-released gate
    # kernel (events around the kernels only) measured the same per-launch time (8.40 vs
    # 8.33 us at K = 20, round 6), so the submission is not what the short region adds.
    evms = C.c_float()
    capi.check(L.epp_event_elapsed_ms(ev0, ev1, C.byref(evms)))
    kms = evms.value / args.steps
    for ev in (ev0, ev1):
        L.epp_event_destroy(ev)
    if graph is not None:
        capi.check(L.epp_graph_destroy(graph))
    achieved = BYTES_PER_STATE * N_STATES / (kms * 1e-3) / 1e9
    n_valid = int(d_valid.download(np.uint8, N_STATES).sum())
    # parity: the flags of resident batch 0 (the cpu_baseline leg checks the same batch on
    # the oracle and counts the mismatches)
    step(0)
    capi.check(L.epp_stream_sync(stream))
    c2_flags = d_valid.download(np.uint8, N_STATES)

    traffic, traffic_src = committed_traffic()

    cpu = None
    parity_gpu = dict((c5_inputs or {}).get("parity_gpu", {}))
    first = plan.pop("_first") if plan else None
    gathered_ok = plan.pop("_gathered_own_equal", None) if plan else None
    # every rank, at every N: its own C2 batch 0 and its own track against the oracle,
    # reduced over the ranks (rank 0 prints the sums and every rank's counters)
    rparity = None
    if not args.no_cpu:
        rparity = reduce_parity(dist, dist.run(lambda: rank_parity(
            rank, geom, rg, ro, gates, obstacles, lo, hi, c2_flags, first, gathered_ok,
            plan["comm_n_ranks"] if plan else None, ws), "parity"), ws)
    if not args.no_cpu and ws == 1:
        cpu = cpu_baseline(geom, rg, ro, gates, obstacles, lo, hi, c5_inputs, parity_gpu)
    if c5_inputs:
        os.unlink(c5_inputs["cfg_path"])
    parity = dict(cpu.pop("parity", None) or {}) if cpu else {}
    if rparity:
        parity.update(rparity)
    if parity:
        parity.update(parity_verdict(parity))

    if rank == 0:
        out = {
            "metric": "validity checks/sec + full plan ms/track, 1/2/4/8 MI355X vs CPU ref",
            "value": value,
            "unit": "state validity checks/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (counter-based uniform states, seeded track world)",
            "config": {"workload": "C2: 1 track, 8 gates, 64 OBBs, 1,048,576 sampled states per step",
                       "states_per_step_per_gpu": N_STATES, "obbs": int(len(obbs)),
                       "can_pass_gate": False, "valid_fraction": n_valid / N_STATES,
                       "parallelism": f"replicas x{ws} (independent samplers)", "process_group": dist.kind,
                       "launch": "hip graph of the K steps" if graph is not None else "host loop"},
            "roofline": {"bound": "hbm", "kernel": "k_states_v5", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_unit": "bytes per launch",
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": BYTES_PER_STATE * N_STATES,
                         "bytes_per_state": BYTES_PER_STATE, "kernel_ms": kms},
            "full_plan_ms_per_track": plan["ms_per_track"] if plan else None,
            "full_plan": plan,
            "cpu_baseline": cpu,
            # the GPU results above against the CPU oracle on the same inputs: every rank's
            # own C2 batch and track (reduced over the ranks, any N), the side legs' (N = 1,
            # in the cpu_baseline leg); null with --no-cpu
            "parity": parity or None,
            "side": side,
        }
        print(json.dumps(out), file=out_stream, flush=True)
    capi.check(L.epp_stream_destroy(stream))
    dist.close()


def launcher_check(ws, rank, local, out_stream, fail_rank=-1, fail_at="plan", parity_flip_rank=-1):
    """The multi-rank plumbing of this bench without a GPU (gloo): the same launch, env,
    barrier, max-over-ranks reduction, error protocol and ragged waypoint all-gather as the
    GPU run (eppamd.dist.Group; the GPU run's group is the product's RCCL communicator).
    fail_rank >= 0 makes that rank's simulated plan fail, inside the leg (fail_at="plan":
    Group.run's collective check) or at the exchange (fail_at="exchange": count -1)."""
    from eppamd.dist import make_group
    dist = make_group(ws, rank, "gloo")
    dist.barrier()

    def plan():
        if rank == fail_rank and fail_at == "plan":
            raise RuntimeError("Path not found")
        return np.arange(3 * (5 + rank), dtype=np.float64).reshape(-1, 3) + 1000 * rank

    wp = dist.run(plan, "full plan")
    per_rank = dist.gather(float(rank + 1))
    if rank == fail_rank and fail_at == "after-count":
        # this rank's process dies between the two steps of the exchange: its count is sent,
        # its set never is (the peers must leave the data all-gather with an error)
        import torch
        n = torch.tensor([len(wp)], dtype=torch.int64)
        dist.dist.all_gather([torch.zeros_like(n) for _ in range(ws)], n)
        print(f"bench.py rank {rank}: dying after the counts (test)", file=sys.stderr, flush=True)
        os._exit(7)
    sets = dist.all_gather_waypoints(None if (rank == fail_rank and fail_at == "exchange") else wp)
    t = dist.max(float(rank + 1))
    # the per-rank parity and its reduction, as the GPU run does them: this rank's C2 batch 0
    # (a 4096-state prefix; the oracle's own flags stand in for the GPU's, with one flipped
    # on --parity-flip-rank), the gathered set at this rank's slot, the group's rank count
    from eppamd import config, synth
    cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
    geom = config.geometry(cfg)
    rg, ro = config.inflate_radii(cfg)
    gates, obstacles = synth.track_world(42)
    lo, hi = synth.C2_BOUNDS
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    n = 4096
    flags = O.check_states(O.world_build(geom, gates, obstacles, rg, ro), rg, ro,
                           synth.sample_states(7 + 1000 * rank, lo, hi, n), False, threads=2)
    if rank == parity_flip_rank:
        flags[17] ^= 1
    own = len(sets) == ws and np.array_equal(np.asarray(sets[rank]), wp)
    parity = reduce_parity(dist, dist.run(lambda: rank_parity(rank, geom, rg, ro, gates, obstacles, lo, hi, flags,
                                                              None, own, dist.n_ranks(), ws, c2_n=n, threads=2),
                                          "parity"), ws)
    parity.update(parity_verdict(parity))
    if rank == 0:
        print(json.dumps({"n_gpus": ws, "ranks_seen": [int(s[0, 0] // 1000) for s in sets],
                          "waypoints_per_track": [len(s) for s in sets], "max_over_ranks": t,
                          "local_rank": local, "process_group": dist.kind, "comm_n_ranks": dist.n_ranks(),
                          "per_rank": per_rank, "parity": parity}), file=out_stream, flush=True)
    dist.close()


PLAN_SAMPLES = 65536


def committed_traffic():
    """HBM bytes per k_states launch from the newest committed PMC summary
    (profiles/rNN_traffic.json, written by scripts/profile_summary.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this bench)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")))
    if not files:
        return None, None
    try:
        d = json.load(open(files[-1]))
    except (OSError, ValueError):
        return None, None
    # the headline launch: the plain (no minDistance, no compaction) state kernel with
    # the most launches in the PMC passes
    cands = [(v["launches"], v) for name, v in d.items()
             if "k_states" in name and "<false, false" in name]
    if cands:
        return max(cands, key=lambda c: c[0])[1]["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)
    return None, None


def committed_motions_valu():
    """Per-launch VALU instruction counts of the C3 motion kernels (analytic, discrete32)
    from the newest committed profiles/rNN_motions_valu.json (scripts/gpu_pmc_motions.sh ->
    scripts/motions_valu.py: rocprofv3 --pmc passes over the same C3 launch)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_motions_valu.json")))
    if not files:
        return None, None
    try:
        d = json.load(open(files[-1]))
    except (OSError, ValueError):
        return None, None
    out = {}
    for name, v in d.items():
        if "true>" in name:  # (the planner's k-NN-table form)
            continue
        out.setdefault(v.get("mode"), v)
    return out, os.path.relpath(files[-1], ROOT)


def full_plan(dist, rank, reps):
    """C4: plan this rank's track end to end (OnlineTrajGenerator.preComputeTraj), time it,
    all-gather the waypoint sets through the product's RCCL communicator.  Returns the
    slowest rank's mean ms per track.  Collective: a rank whose plan fails makes every rank
    raise (dist.run / the all-gather's count -1)."""
    import online_traj_planner as otp
    from eppamd import config, synth
    from eppamd.dist import RcclGroup

    cfg, path = _track_config()
    geom = config.geometry(cfg)
    gates, obstacles = synth.track_world(100 + rank)
    state = {}

    def setup():
        cps = synth.gate_checkpoints(gates, geom.gate_height, 0.55)
        otg = otp.OnlineTrajGenerator(cps[0], cps[-1], gates, obstacles, path)
        otg.pre_compute_traj(0.0)  # warm-up: allocations, first launches
        state["otg"] = otg
        # the first call (planner call numbers 0..8): what the cpu_baseline leg's CPU
        # restatement of the rank-0 track plans (parity)
        state["first"] = {"wp": np.array(otg.get_waypoints()), "traj": np.array(otg.get_planned_traj())}

    def timed():
        per, stats = [], []
        for _ in range(reps):
            t = time.perf_counter()
            state["otg"].pre_compute_traj(0.0)
            per.append((time.perf_counter() - t) * 1e3)
            stats.append(state["otg"].planner_stats())
        state["stats"] = stats
        # one gate-to-gate segment alone, with the planner's device / host split: a fresh
        # PathPlanner's first plan (cold: its construction included) and its second (warm)
        all_cps = state["otg"].get_checkpoints()
        t = time.perf_counter()
        pp = otp.PathPlanner(gates, obstacles, path)
        pp.plan_path(all_cps[2], all_cps[3], 2.0)
        cold = dict(pp.last_stats(), wall_ms_with_construction=(time.perf_counter() - t) * 1e3)
        pp.plan_path(all_cps[4], all_cps[5], 2.0)
        return per, {"cold": cold, "warm": pp.last_stats()}

    try:
        dist.run(setup, "full plan (warm-up)")
        dist.barrier()
        per, seg = dist.run(timed, "full plan")
    finally:
        os.unlink(path)
    ms = float(np.mean(per))
    ms_max = dist.max(ms)
    per_rank = dist.gather(ms)  # every rank's own mean (the headline takes the slowest)
    st = state.get("stats", [])
    # the batched planner's phases per call (rank 0's): device stages up to the emitted
    # rows, the searches, the shortcut; the rest of pre_compute_traj (includeGates2, the
    # min-snap refit and sampling, the path dump)
    phases = {k: float(np.median([x[k] for x in st])) for k in ("ms_batch", "ms_solve", "ms_shortcut")} if st else None
    if phases:
        phases["ms_outside_planner"] = float(np.median([t - x["ms"] for t, x in zip(per, st)]))
        phases["fallbacks_per_call"] = float(np.mean([x["fallbacks"] for x in st]))
        phases["restricted_rows_per_call"] = float(np.median([x["restricted_rows"] for x in st]))
    otg = state["otg"]
    wp = np.ascontiguousarray(otg.get_waypoints())
    traj = otg.get_planned_traj()
    # the exchange step through the product's RCCL communicator (epp_comm_allgather_waypoints):
    # the job's group at N > 1; a one-rank communicator at N = 1
    via = "RCCL (epp_comm_allgather_waypoints)"
    gather_ms, sets, comm_ranks = None, [wp], None
    if isinstance(dist, RcclGroup):
        comm = dist
    else:
        try:
            comm = RcclGroup(1, 0)
        except Exception as e:  # noqa: BLE001 — N = 1 only: reported in the leg, not hidden
            print(f"bench: product communicator unavailable at N=1 ({e})", file=sys.stderr)
            comm, via = None, f"FAILED: {e}"
    if comm is not None:
        comm.all_gather_waypoints(wp)  # (first call: connection setup)
        dist.barrier()
        t = time.perf_counter()
        sets = comm.all_gather_waypoints(wp)
        gather_ms = dist.max((time.perf_counter() - t) * 1e3)
        comm_ranks = comm.n_ranks()  # RCCL's own rank count (epp_comm_rank), not WORLD_SIZE
        if comm is not dist:
            comm.close()
    # (parity of the exchange: this rank's slot of the gathered sets is its own set)
    own_ok = len(sets) == dist.ws and np.array_equal(np.asarray(sets[rank if len(sets) > 1 else 0]), wp)
    return {"_first": state["first"], "_gathered_own_equal": bool(own_ok),
            "ms_per_track": ms_max, "ms_per_track_p50": dist.max(float(np.median(per))), "tracks": dist.ws,
            "ms_per_track_per_rank": per_rank, "comm_n_ranks": comm_ranks, "ms_per_call": per,
            "planner_phases_p50": phases,
            "collective_timeout_s": getattr(comm, "collective_timeout_s", None),
            "samples_per_segment": PLAN_SAMPLES, "k": 16,
            "segments_per_track": 9, "reps": reps, "waypoints_per_track": [len(x) for x in sets],
            "traj_rows": int(len(traj)), "traj_duration_s": float(traj[-1, 9] - traj[0, 9]),
            "all_gather_ms": gather_ms, "all_gather": via, "one_segment": seg,
            "reference_configured_budget_ms": 9 * 2000.0,  # RRT* solve(time_limit_offline=2 s) x 9 segments
            "workload": "C4: per rank one track (seed 100+rank), 8 gates + 24 obstacles, 9 gate-to-gate "
                        "batch plans (65,536 samples, k=16) + includeGates2 + min-snap + sampling"}


C1_REPS = 20


def c1_plan(reps=C1_REPS, cpu_threads=None):
    """BASELINE C1 (single gate + 4 OBB obstacles, bounds [-2,2]^2 x [0,2], the shipped
    config: samples_fmt 4096): ms per plan through the pybind module, as a Python caller of
    the reference's online_traj_planner sees it (src/pybind.cpp:10-27): OnlineTrajGenerator
    -> pre_compute_traj (2 gate-to-gate plans + includeGates2 + min-snap + sampling).  The
    first plan of a fresh generator (cold: construction, workspaces, first launches) is
    reported apart from the steady state.  cpu_threads: the same plans on the CPU
    restatement (oracle/track_planner.OnlineTrajGeneratorCPU; equal waypoints,
    tests/test_gpu_planner.py)."""
    from eppamd import config, synth
    path = os.path.join(ROOT, "configs", "config.json")
    cfg = config.load(path)
    geom = config.geometry(cfg)
    g, o, start, goal = synth.c1_world()
    if cpu_threads:
        import track_planner as TP

        def make():
            return TP.OnlineTrajGeneratorCPU(geom, cfg, start, goal, g, o, threads=cpu_threads)
    else:
        import online_traj_planner as otp

        def make():
            return otp.OnlineTrajGenerator(start, goal, g, o, path)
    t = time.perf_counter()
    otg = make()
    otg.pre_compute_traj(0.0)
    cold = (time.perf_counter() - t) * 1e3
    per = []
    for _ in range(reps):
        t = time.perf_counter()
        otg.pre_compute_traj(0.0)
        per.append((time.perf_counter() - t) * 1e3)
    out = {"ms_per_plan": float(np.mean(per)), "ms_per_plan_p50": float(np.median(per)), "reps": reps,
           "cold_first_plan_ms": cold, "segments": 2, "samples_per_segment": int(cfg["path_planner_properties"]
                                                                                ["samples_fmt"]),
           "workload": "C1: single gate + 4 obstacles, OnlineTrajGenerator.pre_compute_traj (2 batch plans + "
                       "includeGates2 + min-snap + sampling)"}
    if cpu_threads:
        out["threads"] = cpu_threads
    return out


def side_measurements(capi, L, stream, geom, cfg, rg, ro):
    from eppamd import synth
    res = {"c1_plan": c1_plan()}
    # C3: 512 OBBs, 1M edges (analytic) and 32-step discretised
    g3, o3 = synth.track_world(42, n_obstacles=472)
    w3 = capi.World(capi.build_obbs(geom, g3, o3), rg, ro)
    lo, hi = synth.C2_BOUNDS
    n = N_STATES
    s1, s2 = synth.edges(43, 8, lo, hi, n)
    d1, d2 = capi.DeviceBuffer.from_array(s1, stream), capi.DeviceBuffer.from_array(s2, stream)
    dv = capi.DeviceBuffer(n)
    parity_gpu = {}
    for mode, key in ((0, "c3_motion_analytic"), (1, "c3_motion_discrete32")):
        f = lambda r: w3.check_motions_dev(d1.ptr, d2.ptr, n, 0, mode, dv.ptr, stream=stream)  # noqa: E731
        f(0)
        ms = timed_kernel_ms(capi, stream, f, 10)
        res[key] = {"edges_per_s": n / (ms * 1e-3), "kernel_ms": ms,
                    "hbm_frac": BYTES_PER_EDGE * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        capi.check(L.epp_stream_sync(stream))
        parity_gpu[key] = dv.download(np.uint8, C3_CPU_EDGES[mode])  # (the prefix the CPU leg checks)
    # (point-equivalents: 32 step points per edge, the work a plain discretised validator
    # does; the kernel itself evaluates only the 1-3 steps per candidate pair that can hit)
    res["c3_motion_discrete32"]["point_equivalents_per_s"] = 32 * res["c3_motion_discrete32"]["edges_per_s"]
    # the VALU roofline of the two motion kernels (VALU-issue bound, not HBM): per-launch
    # instruction counts from the newest committed PMC summary, over this run's duration
    valu, valu_src = committed_motions_valu()
    for key, mode in (("c3_motion_analytic", "analytic"), ("c3_motion_discrete32", "discrete32")):
        v = valu.get(mode) if valu else None
        if v:
            s_ = res[key]["kernel_ms"] * 1e-3
            res[key]["valu_issue_frac"] = v["valu_issue_cycles_per_launch"] / (s_ * 2.4e9 * 1024)
            res[key]["fp64_frac"] = v["fp64_flops_per_launch"] / s_ / 78.6e12
            res[key]["valu_source"] = valu_src
    # C5 batched: 4096 independent 12-segment refits per launch
    nt = 4096
    tracks = [synth.random_track_waypoints(10_000 + k, 12) for k in range(nt)]
    wp = np.ascontiguousarray(np.concatenate(tracks))
    off = np.arange(nt + 1, dtype=np.int32) * 13
    d_wp, d_off = capi.DeviceBuffer.from_array(wp, stream), capi.DeviceBuffer.from_array(off, stream)
    d_T, d_C, d_st = capi.DeviceBuffer(8 * 12 * nt), capi.DeviceBuffer(240 * 12 * nt), capi.DeviceBuffer(4 * nt)

    def ms_fn(r):
        capi.check(L.epp_minsnap_batch(d_wp.ptr, d_off.ptr, nt, 1.0, 2.0, None, None, d_T.ptr, d_C.ptr, d_st.ptr,
                                       stream))
    ms_fn(0)
    ms = timed_kernel_ms(capi, stream, ms_fn, 10)
    res["c5_minsnap_batch"] = {"problems_per_s": nt / (ms * 1e-3), "ms_per_launch": ms, "problems": nt,
                               "segments": 12}
    capi.check(L.epp_stream_sync(stream))
    parity_gpu["c5_batch"] = (d_T.download(np.float64, 12 * nt).reshape(nt, 12),
                              d_C.download(np.float64, 30 * 12 * nt).reshape(nt, 12, 3, 10),
                              d_st.download(np.int32, nt))
    # C5 single refit latency (host buffers in/out, includes sampling at dt=0.1): the
    # C++ entry through ctypes, 200 calls
    wp1 = tracks[0]
    lat = np.zeros(200)
    for r in range(len(lat)):
        t = time.perf_counter()
        rows1 = capi.generate_trajectory(wp1, 1.0, 2.0, 0.1)
        lat[r] = time.perf_counter() - t
    res["c5_refit"] = _pct(lat[20:] * 1e6)
    parity_gpu["c5_refit_rows"] = np.array(rows1)
    # C5 online replanning loop (1000 steps of gate update + A11 + refit + sampling)
    tg = cfg["trajectory_generator_properties"]
    c5cfg, c5path, c5geom, c5g, c5o, wp, window = c5_setup()
    lat = c5_online(c5path, c5geom, c5g, c5o, wp, window, tg["max_velocity"], tg["max_acceleration"],
                    tg["sampling_interval"], cfg["path_planner_properties"]["min_dist_check_traj_collision"])
    res["c5_online"] = dict(_pct(lat), workload="C5: 1000 steps of gate-pose perturbation (+-0.1 m, +-0.1 rad) -> "
                            "World update -> A11 check of 100 lookahead rows -> 12-segment min-snap refit (W = 13) "
                            "-> sampling at dt = 0.1", waypoints=int(len(wp)), window_gates=[g for g, _ in window],
                            via="Python (pybind PathPlanner / polynomial_trajectory)")
    md = cfg["path_planner_properties"]["min_dist_check_traj_collision"]
    # the same two loops natively through the product's C++ API (tools/c5_native), from an
    # input file the CPU leg's native driver (oracle/cpu_bench) reads as well
    c5_file = write_c5_input(c5geom, c5g, c5o, rg, ro, md, tg["max_velocity"], tg["max_acceleration"],
                             tg["sampling_interval"], wp, window, tracks[0])
    res["c5_native"] = run_native([os.path.join(ROOT, "tools", "c5_native"), c5path, c5_file],
                                  "tools/c5_native (C++ API over libepp, no Python)")
    # the reference's own entry point: OnlineTrajGenerator.update_gate_pos events
    res["c5_update_gate_pos"] = c5_events(c5path, c5geom, c5g, c5o)
    # the same loop's inputs for the CPU leg
    c5_inputs = dict(cfg_path=c5path, geom=c5geom, gates=c5g, obstacles=c5o, wp=wp, window=window,
                     vmax=tg["max_velocity"], amax=tg["max_acceleration"], dt=tg["sampling_interval"],
                     md=md, native_input=c5_file, cfg=c5cfg, parity_gpu=parity_gpu)
    return res, c5_inputs


C5_STEPS = 1000
C3_CPU_EDGES = {0: 1 << 18, 1: 1 << 16}  # the CPU leg's bounded C3 samples (a prefix of the GPU's edges)


def _track_config(samples=PLAN_SAMPLES):
    """configs/config.json with the C2/C4 track bounds [-6,6]^2 x [0,2] (a temp file)."""
    import tempfile

    from eppamd import config
    cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
    cfg["world_properties"]["lower_bound"] = [-6, -6, 0]
    cfg["world_properties"]["upper_bound"] = [6, 6, 2]
    cfg["path_planner_properties"]["samples_fmt"] = samples
    fd, path = tempfile.mkstemp(suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(cfg, f)
    return cfg, path


def c5_setup(seed=42):
    """The C5 track: the C2 world (8 gates, 24 obstacles), planned once end to end; the
    refit window is its first 13 waypoints (12 segments), which include the centres of the
    first gates (includeGates2 inserts them)."""
    import online_traj_planner as otp
    from eppamd import config, synth
    cfg, path = _track_config()
    geom = config.geometry(cfg)
    gates, obstacles = synth.track_world(seed)
    cps = synth.gate_checkpoints(gates, geom.gate_height, 0.55)
    otg = otp.OnlineTrajGenerator(cps[0], cps[-1], gates, obstacles, path)
    otg.pre_compute_traj(0.0)
    wp = np.ascontiguousarray(otg.get_waypoints()[:13])
    centres = gates[:, :3] + np.stack([np.zeros(len(gates)), np.zeros(len(gates)),
                                       geom.gate_height[gates[:, 6].astype(int)]], 1)
    window = []  # (gate, waypoint index) of the gates whose centre is a window waypoint
    for g, c in enumerate(centres):
        d = np.linalg.norm(wp - c, axis=1)
        if d.min() < 1e-9:
            window.append((g, int(d.argmin())))
    return cfg, path, geom, gates, obstacles, wp, window


C5_V0, C5_A0 = np.array([0.4, -0.2, 0.1]), np.array([0.0, 0.3, 0.0])


def c5_steps(window, steps=C5_STEPS):
    """The C5 perturbation sequence: (window gate, its waypoint index), (dx, dy, dyaw)."""
    rs = np.random.RandomState(5)
    return [(window[s % len(window)], rs.uniform(-0.1, 0.1, 3)) for s in range(steps)]


def write_c5_input(geom, gates, obstacles, rg, ro, md, vmax, amax, dt, wp, window, refit_wp, steps=C5_STEPS):
    """The C5 loops' inputs as the native drivers read them (oracle/cpu_bench.cpp
    read_input): OBB descriptions, world, limits, the refit window, the first lookahead
    rows (100 rows of the window's trajectory, computed by the oracle), the single-refit
    track, v0 / a0 and the perturbation steps.  Returns the file path (a temp file)."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    rows = O.generate_trajectory(wp, vmax, amax, dt, 0.0, C5_V0, C5_A0)[:100]
    f17 = lambda x: "%.17g" % x  # noqa: E731

    def desc(d):
        return [str(len(d))] + [" ".join(map(f17, list(r["pos"]) + list(r["size"]))) + f" {int(r['filling'])}"
                                for r in d]

    def mat(m, cols):
        m = np.asarray(m, float).reshape(-1, cols)
        return [str(len(m))] + [" ".join(map(f17, r)) for r in m]

    lines = desc(geom.gate_desc) + [str(len(geom.gate_desc_off)), " ".join(map(str, geom.gate_desc_off))]
    lines += desc(geom.obst_desc) + mat(gates, 7) + mat(obstacles, 6)
    lines += [" ".join(map(f17, (rg, ro, md, vmax, amax, dt)))]
    lines += mat(wp, 3) + mat(rows[:, [0, 3, 6]], 3) + mat(refit_wp, 3)
    lines += [" ".join(map(f17, C5_V0)), " ".join(map(f17, C5_A0))]
    st = c5_steps(window, steps)
    lines += [str(len(st))] + [f"{g} {wi} " + " ".join(map(f17, d)) for (g, wi), d in st]
    fd, path = tempfile.mkstemp(suffix="_c5.txt")
    with os.fdopen(fd, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def run_native(argv, via, timeout=120):
    """One native timing driver (its JSON line), or the failure, visibly."""
    import subprocess
    try:
        r = subprocess.run(argv, capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0:
            raise RuntimeError(f"exit {r.returncode}: {r.stderr[-500:]}")
        out = json.loads(r.stdout.strip().splitlines()[-1])
        out["via"] = via
        return out
    except Exception as e:  # noqa: BLE001 — a side leg: reported, not hidden
        print(f"bench: {argv[0]} failed: {e}", file=sys.stderr)
        return {"error": f"{type(e).__name__}: {e}", "via": via}


C5_EVENT_TRACKS = 24  # 192 events: ~100 replans, so the replan class has a p99 worth the name
# How far ahead of a gate it is observed.  The tracks pass their gate centres slowly
# (0.08-0.4 m/s: the centre is a min-snap waypoint), so with the round-5 lead of 1 s the
# advanced start recomputeTraj replans from (t + time_limit_online + 0.01 s,
# src/OnlineTrajGenerator.cpp:290-310) lay within ~3-19 cm of the old centre, where the
# +-0.1 m / 0.1 rad move put it inside the moved gate's inflated frame: 38 % of the events
# took the no-recomputation exit (9 of 24 on 3 tracks, CPU restatement); at 2 s, 2 of 24.
C5_EVENT_LEAD_S = 2.0


def c5_events(cfg_path, geom, gates, obstacles, n_tracks=C5_EVENT_TRACKS, cpu_threads=None, lead_s=C5_EVENT_LEAD_S):
    """C5 through the reference's entry point, OnlineTrajGenerator.update_gate_pos
    (src/OnlineTrajGenerator.cpp:123-226): every gate of a planned track is observed once
    (as the reference allows), lead_s of flight before the trajectory reaches its centre, at
    a pose perturbed by +-0.1 m / +-0.1 rad; the call checks the lookahead (checkGatePassed
    + A11) and, when the trajectory no longer passes or collides, calls recomputeTraj
    (inline: recalculate_online false).  Each event is timed and filed by what it ran:
      check_only             -- returned False (no recomputation);
      skipped_invalid_start  -- returned True, but recomputeTraj took the reference's
                                "Advanced trajectory does not end at valid position" exit
                                (:304-310): no plan, no refit;
      replan                 -- returned True after two segment plans + includeGates2 +
                                refit + merge.
    (The product reports the exit through OnlineTrajGenerator.recompute_counts(); the CPU
    restatement through its planner call counter: +2 per replan.)  n_tracks fresh
    generators (planned untimed), the same tracks and perturbations for cpu_threads: the
    CPU restatement (oracle/track_planner.OnlineTrajGeneratorCPU: planner in C++, driven
    from Python) -- the same events, so the two distributions compare."""
    rs = np.random.RandomState(11)
    from eppamd import synth
    cps = synth.gate_checkpoints(gates, geom.gate_height, 0.55)
    centres = gates[:, :3] + np.stack([np.zeros(len(gates)), np.zeros(len(gates)),
                                       geom.gate_height[gates[:, 6].astype(int)]], 1)
    perturb = [[rs.uniform(-0.1, 0.1, 3) for _ in range(len(gates))] for _ in range(n_tracks)]
    us = {"check_only": [], "skipped_invalid_start": [], "replan": []}
    if cpu_threads:
        import track_planner as TP
        cfg = cfg_json(cfg_path)
    else:
        import online_traj_planner as otp
    for k in range(n_tracks):
        if cpu_threads:
            otg = TP.OnlineTrajGeneratorCPU(geom, cfg, cps[0], cps[-1], gates, obstacles, threads=cpu_threads)
            otg.pre_compute_traj(0.0)
            traj_of = lambda: otg.traj  # noqa: E731
        else:
            otg = otp.OnlineTrajGenerator(cps[0], cps[-1], gates, obstacles, cfg_path)
            otg.pre_compute_traj(0.0)
            traj_of = otg.get_planned_traj
        for g in range(len(gates)):
            cur = traj_of()
            i_c = int(np.argmin(np.linalg.norm(cur[:, [0, 3, 6]] - centres[g], axis=1)))
            t_obs = max(float(cur[i_c, -1]) - lead_s, 0.0)
            i = int(np.argmin(np.abs(cur[:, -1] - t_obs)))
            drone = cur[i, [0, 3, 6]].copy()
            pose = gates[g, :6].copy()
            pose[[0, 1, 5]] += perturb[k][g]
            before = otg.calls if cpu_threads else otg.recompute_counts()["planned"]
            t = time.perf_counter()
            r = otg.update_gate_pos(g, pose, drone, True, t_obs)
            el = (time.perf_counter() - t) * 1e6
            after = otg.calls if cpu_threads else otg.recompute_counts()["planned"]
            planned = (after - before) == (2 if cpu_threads else 1)
            us["replan" if planned else ("skipped_invalid_start" if r else "check_only")].append(el)
    out = {"events": sum(len(v) for v in us.values()), "tracks": n_tracks,
           "counts": {k: len(v) for k, v in us.items()},
           **{k: (_pct(np.array(v)) if v else None) for k, v in us.items()},
           "lead_s": lead_s,
           "workload": f"C5 via OnlineTrajGenerator.update_gate_pos: each gate observed once, {lead_s:g} s ahead, pose +-0.1 m / "
                       "+-0.1 rad; check_only (checkGatePassed + A11, returned False), skipped_invalid_start "
                       "(returned True, the reference's no-recomputation exit) and replan (2 segment plans of "
                       f"{PLAN_SAMPLES:,} samples + includeGates2 + refit) timed separately"}
    if cpu_threads:
        out["threads"] = cpu_threads
    return out


def c5_online(cfg_path, geom, gates, obstacles, wp, window, vmax, amax, dt, md, steps=C5_STEPS, cpu=False):
    """C5 (BASELINE configs[4]): the 50 Hz online replanning step, `steps` times.  Per
    step: one window gate gets a perturbed pose (+-0.1 m in x, y; +-0.1 rad yaw around its
    nominal pose) -> World update (World::updateGatePosition, src/World.cpp:20-27) -> A11
    re-check of the 100 lookahead rows (PathPlanner::checkTrajectoryValidity with
    min_dist_check_traj_collision, src/PathPlanner.cpp:267-280) -> 12-segment min-snap refit
    (W = 13, the gate's centre waypoint moved) from the current state -> sampled at dt
    (poly_traj::generateTrajectory).  The GPU step runs the product (PathPlanner:
    update_gate_pos, then check_trajectory_validity_and_generate -- the check and the refit
    in one launch); cpu=True runs the same step on the CPU oracle (world
    rebuild, minDistance check, min-snap + sampling).  Returns per-step microseconds."""
    gates = np.array(gates, float)
    perturb = c5_steps(window, steps)
    v0, a0 = C5_V0, C5_A0
    lat = np.zeros(steps)
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        rg, ro = float(cfg_json(cfg_path)["world_properties"]["inflate_radius"]["gate"]), \
            float(cfg_json(cfg_path)["world_properties"]["inflate_radius"]["obstacle"])
        rows = O.generate_trajectory(wp, vmax, amax, dt, 0.0, v0, a0)
        for s, ((g, wi), d) in enumerate(perturb):
            t = time.perf_counter()
            gs = gates.copy()
            gs[g, 0] += d[0]
            gs[g, 1] += d[1]
            gs[g, 5] += d[2]
            w = O.world_build(geom, gs, obstacles, rg, ro)
            O.check_states_mindist(w, rows[:100][:, [0, 3, 6]], md)
            wp2 = wp.copy()
            wp2[wi, :2] = gs[g, :2]
            rows = O.generate_trajectory(wp2, vmax, amax, dt, 0.0, v0, a0)
            lat[s] = time.perf_counter() - t
        return lat * 1e6
    import online_traj_planner as otp
    import polynomial_trajectory as pt
    pp = otp.PathPlanner(gates, obstacles, cfg_path)
    rows = pt.generate_trajectory(wp, vmax, amax, dt, 0.0, v0, a0)
    pp.check_trajectory_validity(rows[:100], md)  # first upload of the world
    for s, ((g, wi), d) in enumerate(perturb):
        t = time.perf_counter()
        pose = gates[g, :6].copy()
        pose[0] += d[0]
        pose[1] += d[1]
        pose[5] += d[2]
        pp.update_gate_pos(g, pose)
        wp2 = wp.copy()
        wp2[wi, :2] = pose[:2]
        # the A11 check of the lookahead rows and the refit in one launch (the product's
        # online step; the same flags and rows as the two calls, tests/test_gpu_minsnap.py)
        _, rows = pp.check_trajectory_validity_and_generate(rows[:100], md, wp2, vmax, amax, dt, 0.0, v0, a0)
        lat[s] = time.perf_counter() - t
    return lat * 1e6


def cfg_json(path):
    with open(path) as f:
        return json.load(f)


def _pct(lat):
    return {"p50_us": float(np.percentile(lat, 50)), "p99_us": float(np.percentile(lat, 99)),
            "mean_us": float(lat.mean()), "steps": int(len(lat))}


def host_info():
    """The host the CPU legs ran on: logical CPUs of the machine, the CPUs this process
    may run on, and the CPU model (/proc/cpuinfo, as lscpu reports it)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity_cpus": affinity, "cpu_model": model}


# host threads for the all-cores legs: the box's CPU share of one GPU (16; the machine
# reports more logical CPUs than a one-GPU job may use, and the pool's rules size worker
# pools to that share).  States and C3 are also sampled briefly at 32 threads and at every
# logical CPU (states_wide, c3_*.edges_per_s_<T>_threads).
CPU_SHARE_THREADS = 16


def cpu_baseline(geom, rg, ro, gates, obstacles, lo, hi, c5_inputs=None, parity_gpu=None):
    """The CPU oracle (a port of the reference's World / min-snap semantics, kind "port") on
    bounded samples of the same workloads, ~15 s in total:

    * value: state validity checks/s on 1 thread (OMPL calls the plugins one query at a
      time) over the C2 batch; all_cores_value: the same on CPU_SHARE_THREADS threads;
    * c3_*: C3 motion checks (512 OBBs) analytic / discrete32 on CPU_SHARE_THREADS threads;
    * full_plan_ms_per_track: the C4 track planned by the CPU restatement of the same batch
      planner (paths equal to the GPU's, tests/test_gpu_planner.py), CPU_SHARE_THREADS threads;
    * c5_online: the C5 loop on the oracle (world rebuild, minDistance check, min-snap +
      sampling), per-step latency, 1 thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from eppamd import synth
    nt = min(CPU_SHARE_THREADS, host_info()["affinity_cpus"] or 1)
    w = O.world_build(geom, gates, obstacles, rg, ro)
    pts = synth.sample_states(7, lo, hi, N_STATES)
    reps = 0
    parity_gpu = parity_gpu or {}
    parity = {}
    t = time.perf_counter()
    while True:
        ref_flags = O.check_states(w, rg, ro, pts, False, threads=1)
        reps += 1
        if time.perf_counter() - t > 6.0:
            break
    dt = time.perf_counter() - t
    t2 = time.perf_counter()
    for _ in range(3):
        O.check_states(w, rg, ro, pts, False, threads=nt)
    dt2 = (time.perf_counter() - t2) / 3
    host = host_info()
    # wider sweeps, short samples: 32 threads (256 logical CPUs / 8 GPUs: one GPU's share
    # on an 8-GPU node) and every logical CPU the box reports (measured, not the bound;
    # on a shared box other jobs' threads compete for those cores)
    # (131,072 states per thread and call, so thread start-up is amortised: one 1M-state
    # call on 256 threads measured start-up, 1.3e8/s against 4.2e8/s on 32)
    wide = {}
    for tw in sorted({32, host["affinity_cpus"] or 1}):
        big = np.tile(pts, (max(1, tw // 8), 1))
        t3 = time.perf_counter()
        for _ in range(3):
            O.check_states(w, rg, ro, big, False, threads=tw)
        wide[str(tw)] = {"value": 3 * len(big) / (time.perf_counter() - t3), "threads": tw, "checks": 3 * len(big)}
        del big
    out = {"value": reps * N_STATES / dt, "unit": "state validity checks/s", "cores": 1, "kind": "port",
           "sample": f"{reps} passes over the same {N_STATES:,}-state C2 batch ({reps * N_STATES} checks, {dt:.1f} s)",
           "all_cores_value": N_STATES / dt2, "all_cores_threads": nt, "host": host,
           # NOT a measurement: the single-thread rate times every logical CPU of the host
           # (perfect scaling, no memory-bandwidth or SMT limits) -- the most CPU-favourable
           # bound for "all host cores"; running that wide exceeds one GPU job's CPU share
           "all_cores_ideal_bound": {"value": reps * N_STATES / dt * (host["nproc"] or 1),
                                     "threads": host["nproc"], "kind": "bound: 1-thread rate x nproc"},
           "states_wide": wide}
    # C3 motions: 512 OBBs, the same edge generator as the GPU leg (bounded edge counts)
    g3, o3 = synth.track_world(42, n_obstacles=472)
    w3 = O.world_build(geom, g3, o3, rg, ro)
    e1, e2 = synth.edges(43, 8, lo, hi, N_STATES)  # the GPU leg's edges; the CPU checks a prefix
    for mode, key in ((0, "c3_motion_analytic"), (1, "c3_motion_discrete32")):
        n = C3_CPU_EDGES[mode]
        s1, s2 = np.ascontiguousarray(e1[:n]), np.ascontiguousarray(e2[:n])
        t = time.perf_counter()
        ref3 = O.check_motions(w3, rg, ro, s1, s2, False, mode, threads=nt)
        el = time.perf_counter() - t
        out[key] = {"edges_per_s": n / el, "threads": nt, "edges": n}
        if key in parity_gpu:
            parity[f"{key}_mismatches"] = int(np.count_nonzero(parity_gpu[key] != ref3))
            parity[f"{key}_compared"] = n
        for tw in sorted({32, host["affinity_cpus"] or 1}):  # (edges per thread as at 16 threads)
            b1, b2 = np.tile(s1, (max(1, tw // 16), 1)), np.tile(s2, (max(1, tw // 16), 1))
            t = time.perf_counter()
            O.check_motions(w3, rg, ro, b1, b2, False, mode, threads=tw)
            out[key][f"edges_per_s_{tw}_threads"] = len(b1) / (time.perf_counter() - t)
    # C4 full plan on the CPU: the same batch planner restated (oracle/track_planner.py):
    # 9 gate-to-gate plans (65,536 samples, k = 16; each plan's checks and k-NN on nt
    # threads) + includeGates2 + min-snap + sampling, the rank-0 track (seed 100)
    import track_planner as TP
    from eppamd import config as cfgmod
    c4, c4path = _track_config()
    os.unlink(c4path)
    g4, o4 = synth.track_world(100)
    w4 = O.world_build(geom, g4, o4, rg, ro)
    ends = synth.gate_checkpoints(g4, geom.gate_height, 0.55)
    cps = np.vstack([ends[0], synth.gate_checkpoints(g4, geom.gate_height,
                                                     c4["path_planner_properties"]["checkpoint_gate_offset"]), ends[-1]])
    tg = c4["trajectory_generator_properties"]
    lo4, hi4 = cfgmod.bounds(c4)
    t = time.perf_counter()
    wp4, rows4 = TP.plan_track(w4, rg, ro, lo4, hi4, cps, PLAN_SAMPLES, tg["max_velocity"], tg["max_acceleration"],
                               tg["sampling_interval"], threads=nt)
    out["full_plan_ms_per_track"] = (time.perf_counter() - t) * 1e3
    out["full_plan"] = {"threads": nt, "tracks": 1, "waypoints": int(len(wp4)), "traj_rows": int(len(rows4)),
                        "workload": "C4 rank-0 track: 9 batch plans (65,536 samples, k=16) + includeGates2 + "
                                    "min-snap + sampling, the planner restated on the CPU (oracle/track_planner.py)"}
    out["c1_plan"] = c1_plan(reps=5, cpu_threads=1)
    if c5_inputs:
        c = c5_inputs
        lat = c5_online(c["cfg_path"], c["geom"], c["gates"], c["obstacles"], c["wp"], c["window"], c["vmax"],
                        c["amax"], c["dt"], c["md"], cpu=True)
        out["c5_online"] = dict(_pct(lat), threads=1)
        wp1 = synth.random_track_waypoints(10_000, 12)
        lat = np.zeros(200)
        for r in range(len(lat)):
            t = time.perf_counter()
            O.generate_trajectory(wp1, 1.0, 2.0, 0.1)
            lat[r] = time.perf_counter() - t
        out["c5_refit"] = dict(_pct(lat[20:] * 1e6), threads=1, via="Python (ctypes oracle)")
        # C5 batched: the GPU leg's 4096 x 12-segment problems, one generateTrajectory solve
        # each (the reference's per-problem shape), on the CPU share and on 32 threads
        tracks = [synth.random_track_waypoints(10_000 + k, 12) for k in range(4096)]
        out["c5_minsnap_batch"] = {"problems": len(tracks), "segments": 12,
                                   "workload": "4096 x 12-segment min-snap solves (or_minsnap_track: Nfabian times + "
                                               "QP), the GPU leg's problems, contiguous ranges per thread"}
        for tw in sorted({nt, 32}):
            O.minsnap_batch(tracks[:256], 1.0, 2.0, threads=tw)  # (thread start-up, page faults)
            t = time.perf_counter()
            reps = 0
            while reps < 3 or time.perf_counter() - t < 0.5:
                O.minsnap_batch(tracks, 1.0, 2.0, threads=tw)
                reps += 1
            el = (time.perf_counter() - t) / reps
            out["c5_minsnap_batch"][f"problems_per_s_{tw}_threads"] = len(tracks) / el
        out["c5_minsnap_batch"]["problems_per_s"] = out["c5_minsnap_batch"][f"problems_per_s_{nt}_threads"]
        if "c5_batch" in parity_gpu:  # the GPU leg's 4096 problems against the oracle's solves
            Tg, Cg, sg = parity_gpu["c5_batch"]
            Tr, Cr, sr = O.minsnap_batch(tracks, 1.0, 2.0, threads=nt)
            # (success: status 0 on the GPU, a non-negative return code from the oracle)
            parity["c5_batch_solved_equal"] = bool(np.array_equal(np.asarray(sg) == 0, np.asarray(sr) >= 0))
            parity["c5_batch_coeff_max_abs"] = float(max(np.abs(Cg[k] - Cr[k]).max() for k in range(len(tracks))))
            parity["c5_batch_times_max_rel"] = float(max((np.abs(Tg[k] - Tr[k]) / Tr[k]).max()
                                                         for k in range(len(tracks))))
            # both against the truth (the reference's formulation in long double, refined;
            # pinned to 40-digit mpmath in tests/test_oracle.py): how much of the GPU-vs-oracle
            # difference is the oracle's own rounding
            import minsnap_np as MN
            truth = MN.track_batch_refined(np.asarray(tracks), np.asarray(Tr))
            parity["c5_batch_gpu_vs_truth_max_abs"] = float(np.abs(np.asarray(Cg) - truth).max())
            parity["c5_batch_oracle_vs_truth_max_abs"] = float(np.abs(np.asarray(Cr) - truth).max())
        if "c5_refit_rows" in parity_gpu:  # the single refit (native generateTrajectory) vs the oracle's
            rg1 = parity_gpu["c5_refit_rows"]
            rr1 = O.generate_trajectory(wp1, 1.0, 2.0, 0.1)
            same = rg1.shape == rr1.shape
            parity["c5_refit_time_column_equal"] = bool(same and np.array_equal(rg1[:, 9], rr1[:, 9]))
            parity["c5_refit_max_abs"] = float(np.abs(rg1[:, :9] - rr1[:, :9]).max()) if same else None
        out["c5_minsnap_batch"]["threads"] = nt
        out["c5_online"]["via"] = "Python (ctypes oracle)"
        # native: the same loops from the same input file, C++ calls into the oracle
        nat = run_native([os.path.join(ROOT, "oracle", "cpu_bench"), c["native_input"]],
                         "oracle/cpu_bench (C++ calls into liboracle, no Python)")
        for key in ("c5_refit_native", "c5_online_native"):
            if key in nat:
                out[key] = dict(nat[key], via=nat["via"])
        if "error" in nat:
            out["c5_native_error"] = nat["error"]
        os.unlink(c["native_input"])
        # the update_gate_pos events on the CPU restatement: the GPU leg's tracks and
        # perturbations (planner on nt threads)
        out["c5_update_gate_pos"] = c5_events(c["cfg_path"], c["geom"], c["gates"], c["obstacles"],
                                              cpu_threads=nt)
    if parity:
        out["parity"] = parity
    return out


PARITY_THREADS = 16  # one GPU's CPU share on the pool (and on an 8-GPU node: 256 / 8 = 32)


def rank_parity(rank, geom, rg, ro, gates, obstacles, lo, hi, c2_flags, first, gathered_ok, comm_n_ranks, ws,
                c2_n=None, threads=PARITY_THREADS):
    """This rank's own GPU results against the oracle on the same inputs, at any N:

    * C2: the flags of its resident batch 0 (seed 7 + 1000 * rank) -- `c2_flags`, the
      first c2_n states (all by default; ~4 ms of oracle work on 16 threads per 1M);
    * C4: its first plan of its own track (world seed 100 + rank, planner calls 0..8) --
      `first` = {"wp", "traj"} -- against the CPU restatement of the whole track
      (oracle/track_planner.plan_track, ~0.4 s on 16 threads): waypoints and the time
      column equal, the other columns' max-abs difference;
    * the exchange: the all-gathered set at this rank's index equals its own waypoints
      (`gathered_ok`) and RCCL's own rank count equals the world size.

    Returns flat counters (reduce_parity sums / ands / maxes them over the ranks)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from eppamd import synth
    out = {}
    if c2_flags is not None:
        w = O.world_build(geom, gates, obstacles, rg, ro)
        n = len(c2_flags) if c2_n is None else c2_n
        pts = synth.sample_states(7 + 1000 * rank, lo, hi, n)
        ref = O.check_states(w, rg, ro, pts, False, threads=threads)
        out["c2_batch0_mismatches"] = int(np.count_nonzero(np.asarray(c2_flags[:n]) != ref))
        out["c2_batch0_compared"] = int(n)
    if first is not None:
        wp4, rows4 = _cpu_track(geom, rg, ro, rank, threads)
        gw, gt = np.asarray(first["wp"]), np.asarray(first["traj"])
        out["c4_waypoints_equal"] = bool(gw.shape == wp4.shape and np.array_equal(gw, wp4))
        same = gt.shape == rows4.shape
        out["c4_traj_time_column_equal"] = bool(same and np.array_equal(gt[:, 9], rows4[:, 9]))
        out["c4_traj_max_abs"] = float(np.abs(gt[:, :9] - rows4[:, :9]).max()) if same else float("inf")
    if gathered_ok is not None:
        out["gathered_set_equal"] = bool(gathered_ok)
    if comm_n_ranks is not None:
        out["comm_n_ranks_equal"] = bool(comm_n_ranks == ws)
    return out


def _cpu_track(geom, rg, ro, rank, threads):
    """The CPU restatement of full_plan's first plan of this rank's track (world seed
    100 + rank, planner calls 0..8): waypoints and sampled rows."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import track_planner as TP
    from eppamd import config as cfgmod, synth
    c4, c4path = _track_config()
    os.unlink(c4path)
    g4, o4 = synth.track_world(100 + rank)
    w4 = O.world_build(geom, g4, o4, rg, ro)
    ends = synth.gate_checkpoints(g4, geom.gate_height, 0.55)
    cps = np.vstack([ends[0], synth.gate_checkpoints(g4, geom.gate_height,
                                                     c4["path_planner_properties"]["checkpoint_gate_offset"]), ends[-1]])
    tg = c4["trajectory_generator_properties"]
    lo4, hi4 = cfgmod.bounds(c4)
    return TP.plan_track(w4, rg, ro, lo4, hi4, cps, PLAN_SAMPLES, tg["max_velocity"], tg["max_acceleration"],
                         tg["sampling_interval"], threads=threads)


def reduce_parity(dist, local, ws):
    """Collective: every rank's rank_parity counters -> the job's.  Sums for *_mismatches /
    *_compared, all-ranks for *_equal, the max for *_max_abs; every rank's own value under
    per_rank (rank order).  Every rank must hold the same keys (they come from the same
    legs)."""
    keys = sorted(local)
    per_rank, red = {}, {"ranks": ws}
    for k in keys:
        v = local[k]
        vals = dist.gather(float(v))
        if k.endswith("_equal"):
            per_rank[k] = [bool(x) for x in vals]
            red[k] = all(per_rank[k])
        elif k.endswith("_max_abs"):
            per_rank[k] = vals
            red[k] = float(max(vals))
        else:
            per_rank[k] = [int(x) for x in vals]
            red[k] = int(sum(per_rank[k]))
    red["per_rank"] = per_rank
    return red


def parity_verdict(parity):
    """ok = every mismatch count 0, every *_equal true, every *_max_abs within 1e-6."""
    return {"ok": bool(all(parity.get(k, 0) == 0 for k in parity if k.endswith("_mismatches")) and
                       all(parity.get(k, True) for k in parity if k.endswith("_equal")) and
                       all((parity.get(k) is not None and parity[k] <= 1e-6)
                           for k in parity if k.endswith("_max_abs"))),
            "tolerance_f64": 1e-6}


if __name__ == "__main__":
    main()
