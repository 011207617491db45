"""The in-flight failure cases of the multi-track exchange (csrc/comm.cpp), run in its own
process on the test-hooks build of the library.

A collective whose peer never takes part stays queued on the communicator's stream.  The
test-hooks build (efficient-path-planner_amd/testhooks/, -DEPP_TEST_HOOKS) queues a
bounded stall (EPP_TEST_COMM_STALL_MS, 2.5 s here) ahead of every collective, which keeps
a one-rank collective in flight that long — the one-GPU stand-in for a peer that has not
joined.  Checked:
  * the deadline (epp_comm_set_timeout) ends the call with EPP_ERR_TIMEOUT: the wait's
    checks ran while the collective was in flight.  Had anything ahead of the wait blocked
    in the runtime (a device-to-host copy into pageable caller memory), the
    call would have sat out the stall and then found the collective complete: EPP_OK;
  * an abort requested from another thread (epp_comm_abort) ends a call waiting on a
    30 s deadline with EPP_ERR_PEER, likewise;
  * ncclCommAbort itself returns once the work queued on the stream has left it: RCCL's
    own kernels leave a collective at the abort flag, the stand-in stall does not, so both
    calls return when the stall ends (bounded here, long before the 30 s deadline);
  * every later call on the aborted communicator fails at once, its caller buffers are
    never written after the call returned, destroy works, and a new communicator works.

usage: python tests/comm_stall_case.py
"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "efficient-path-planner_amd")
sys.path[:0] = [PKG]
os.environ["EPP_LIB"] = os.path.join(PKG, "testhooks", "libepp.so")
STALL_S = 2.5
os.environ["EPP_TEST_COMM_STALL_MS"] = str(int(STALL_S * 1000))

import numpy as np  # noqa: E402

from eppamd import capi, synth  # noqa: E402

assert capi.LIB_PATH == os.environ["EPP_LIB"]


def main() -> None:
    wp = synth.sample_states(6, [-6, -6, 0], [6, 6, 2], 5)
    # 1. the deadline, with the collective in flight
    c = capi.Comm(capi.Comm.unique_id(), 1, 0)
    c.set_timeout(0.3)
    t0 = time.perf_counter()
    try:
        c.allgather_waypoints(wp, cap=8)
        raise AssertionError("no timeout")
    except capi.EppError as e:
        dt = time.perf_counter() - t0
        assert e.code == capi.EPP_ERR_TIMEOUT, (e.code, str(e))
        assert "no completion within" in str(e)
    assert dt < STALL_S + 5.0, dt
    try:
        c.barrier()
        raise AssertionError("aborted communicator usable")
    except capi.EppError as e:
        assert e.code == capi.EPP_ERR_PEER
    x = np.array([4.0, 5.0])
    try:
        c.allreduce(x, capi.EPP_REDUCE_SUM)
        raise AssertionError("aborted communicator usable")
    except capi.EppError as e:
        assert e.code == capi.EPP_ERR_PEER
    c.close()
    t_timeout = dt

    # 2. an abort from another thread while the call waits on a 30 s deadline
    c = capi.Comm(capi.Comm.unique_id(), 1, 0)
    c.set_timeout(30.0)
    # the caller's buffers, handed to the C ABI as they are and filled with sentinels: the
    # one-rank gather would write 6 and the points into them
    counts = np.full(1, -7, np.int32)
    out = np.full((1, 8, 3), -7.0)
    th = threading.Thread(target=lambda: (time.sleep(0.3), c.abort()))
    th.start()
    t0 = time.perf_counter()
    rc = capi.lib().epp_comm_allgather_waypoints(c.handle, capi._ptr(wp), len(wp), 8, capi._ptr(out),
                                                  capi._ptr(counts))
    dt = time.perf_counter() - t0
    err = capi.lib().epp_last_error().decode()
    assert rc == capi.EPP_ERR_PEER and "aborted" in err, (rc, err)
    th.join()
    assert dt < STALL_S + 5.0, dt  # the abort, not the 30 s deadline
    time.sleep(0.5)
    # nothing was copied into them, before or after the return
    assert counts[0] == -7 and np.all(out == -7.0), (counts, out[0, :2])
    c.close()

    # 3. a new communicator works (the stall only delays it)
    c = capi.Comm(capi.Comm.unique_id(), 1, 0)
    got = c.allgather_waypoints(wp, cap=8)[0]
    assert np.array_equal(got, wp)
    c.close()
    print(f"comm stall case ok: timeout after {t_timeout:.2f} s, abort after {dt:.2f} s")


if __name__ == "__main__":
    main()
