"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of the "optimal" trajectory type.

Follows external/time_parametrization (Kunz & Stilman's time-optimal path
parametrisation as vendored by the reference):

- src/Path.cpp:48-186    line pieces and circular corner blends,
- src/Path.cpp:191-238   the blended path and its switching points,
- src/Path.cpp:240-283   piece lookup / next switching point,
- src/Trajectory.cpp:53-96    the forward/backward integration driver,
- src/Trajectory.cpp:124-237  acceleration / velocity switching points,
- src/Trajectory.cpp:240-377  forward and backward integration,
- src/Trajectory.cpp:379-445  phase-plane limits,
- src/Trajectory.cpp:459-503  sampling at time t,
- src/OptimalTimeParametrizer.cpp:11-108  rows [x vx ax y vy ay z vz az yaw t+t0].

Floating-point operation order follows the reference (Eigen's 3-vector reductions are
((x0 . y0) + (x1 . y1)) + (x2 . y2)).  Parity is UNPINNED against the reference itself:
its sources need Eigen (absent here and on the GPU box) and no reference test or fixture
covers this component; the C++ product path (csrc/host_timeopt.cpp) is checked against
this restatement (tests/test_timeopt_cpu.py), and both against the physical bounds.
"""
from __future__ import annotations

import bisect
import math

EPS = 0.000001
STEP = 0.001
DBL_MAX = 1.7976931348623157e308


def _div(a, b):
    """IEEE division (C++ semantics) where Python would raise on b == 0."""
    try:
        return a / b
    except ZeroDivisionError:
        if a != a or a == 0.0:
            return math.nan
        return math.copysign(math.inf, a) * math.copysign(1.0, b)


def _sq(v):
    return (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]


def _norm(v):
    return math.sqrt(_sq(v))


def _sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def _normalized(v):
    z = _sq(v)
    if not z > 0.0:
        return tuple(v)
    r = math.sqrt(z)
    return (v[0] / r, v[1] / r, v[2] / r)


class _Line:
    """Path.cpp:48-87."""

    def __init__(self, a, b):
        self.a, self.b = tuple(a), tuple(b)
        self.length = _norm(_sub(b, a))
        self.position = 0.0

    def config(self, s):
        s = s / self.length
        s = max(0.0, min(1.0, s))
        return tuple((1.0 - s) * self.a[i] + s * self.b[i] for i in range(3))

    def tangent(self, s):
        return tuple((self.b[i] - self.a[i]) / self.length for i in range(3))

    def curvature(self, s):
        return (0.0, 0.0, 0.0)

    def switching(self):
        return []


class _Arc:
    """Path.cpp:90-186."""

    def __init__(self, start, corner, end, max_dev):
        self.position = 0.0
        self.length, self.radius, self.center = 0.0, 1.0, tuple(corner)
        self.x = self.y = (0.0, 0.0, 0.0)
        if _norm(_sub(corner, start)) < 0.000001 or _norm(_sub(end, corner)) < 0.000001:
            return
        sd = _normalized(_sub(corner, start))
        ed = _normalized(_sub(end, corner))
        if _norm(_sub(sd, ed)) < 0.000001:
            return
        dist = min(_norm(_sub(start, corner)), _norm(_sub(end, corner)))
        angle = math.acos((sd[0] * ed[0] + sd[1] * ed[1]) + sd[2] * ed[2])
        dist = min(dist, max_dev * math.sin(0.5 * angle) / (1.0 - math.cos(0.5 * angle)))
        self.radius = dist / math.tan(0.5 * angle)
        self.length = angle * self.radius
        n = _normalized(_sub(ed, sd))
        c = math.cos(0.5 * angle)
        self.center = tuple(corner[i] + n[i] * self.radius / c for i in range(3))
        self.x = _normalized(tuple((corner[i] - dist * sd[i]) - self.center[i] for i in range(3)))
        self.y = sd

    def config(self, s):
        a = s / self.radius
        c, sn = math.cos(a), math.sin(a)
        return tuple(self.center[i] + self.radius * (self.x[i] * c + self.y[i] * sn) for i in range(3))

    def tangent(self, s):
        a = s / self.radius
        c, sn = math.cos(a), math.sin(a)
        return tuple(-self.x[i] * sn + self.y[i] * c for i in range(3))

    def curvature(self, s):
        a = s / self.radius
        c, sn = math.cos(a), math.sin(a)
        k = -1.0 / self.radius
        return tuple(k * (self.x[i] * c + self.y[i] * sn) for i in range(3))

    def switching(self):
        out = []
        for i in range(3):
            ang = math.atan2(self.y[i], self.x[i])
            if ang < 0.0:
                ang += math.pi
            p = ang * self.radius
            if p < self.length:
                out.append(p)
        return sorted(out)


class Path:
    """Path.cpp:191-283."""

    def __init__(self, pts, max_dev):
        pts = [tuple(map(float, p)) for p in pts]
        if len(pts) < 2:
            raise ValueError("need at least 2 waypoints")
        self.segs = []
        start = pts[0]
        for k in range(1, len(pts)):
            if max_dev > 0.0 and k + 1 < len(pts):
                c1, c2, c3 = pts[k - 1], pts[k], pts[k + 1]
                blend = _Arc(tuple(0.5 * (c1[i] + c2[i]) for i in range(3)), c2,
                             tuple(0.5 * (c2[i] + c3[i]) for i in range(3)), max_dev)
                end = blend.config(0.0)
                if _norm(_sub(end, start)) > 0.000001:
                    self.segs.append(_Line(start, end))
                self.segs.append(blend)
                start = blend.config(blend.length)
            else:
                self.segs.append(_Line(start, pts[k]))
                start = pts[k]
        self.length = 0.0
        self.switching = []
        for seg in self.segs:
            seg.position = self.length
            for p in seg.switching():
                self.switching.append((self.length + p, False))
            self.length += seg.length
            while self.switching and self.switching[-1][0] >= self.length:
                self.switching.pop()
            self.switching.append((self.length, True))
        self.switching.pop()
        self._pos = [s.position for s in self.segs]

    def _seg(self, s):
        k = max(bisect.bisect_right(self._pos, s, 1) - 1, 0)
        return self.segs[k], s - self.segs[k].position

    def config(self, s):
        seg, t = self._seg(s)
        return seg.config(t)

    def tangent(self, s):
        seg, t = self._seg(s)
        return seg.tangent(t)

    def curvature(self, s):
        seg, t = self._seg(s)
        return seg.curvature(t)

    def next_switching(self, s):
        for p, disc in self.switching:
            if p > s:
                return p, disc
        return self.length, True


class Trajectory:
    """Trajectory.cpp:53-503 for equal per-axis bounds vmax, amax."""

    def __init__(self, path: Path, vmax: float, amax: float):
        self.path, self.vmax, self.amax = path, vmax, amax
        self.valid = True
        self.traj = [[0.0, 0.0, 0.0]]  # [s, sdot, t]
        after = self._acc(0.0, 0.0, True)
        while self.valid and not self._forward(after) and self.valid:
            res = self._next_switch(self.traj[-1][0])
            if res is None:
                break
            sw, before, after = res
            self._backward(sw[0], sw[1], before)
        if self.valid:
            self._backward(path.length, 0.0, self._acc(path.length, 0.0, False))
        if self.valid:
            self.traj[0][2] = 0.0
            for k in range(1, len(self.traj)):
                p, c = self.traj[k - 1], self.traj[k]
                c[2] = p[2] + _div(c[0] - p[0], (c[1] + p[1]) / 2.0)
        self._times = [st[2] for st in self.traj]

    # --- limits (Trajectory.cpp:379-445) ---
    def _acc(self, s, sd, upper):
        t, c = self.path.tangent(s), self.path.curvature(s)
        f = 1.0 if upper else -1.0
        m = DBL_MAX
        for i in range(3):
            if t[i] != 0.0:
                m = min(m, self.amax / abs(t[i]) - f * c[i] * sd * sd / t[i])
        return f * m

    def _slope(self, s, sd, upper):
        return _div(self._acc(s, sd, upper), sd)

    def _acc_limit(self, s):
        m = math.inf
        t, c = self.path.tangent(s), self.path.curvature(s)
        for i in range(3):
            if t[i] != 0.0:
                for j in range(i + 1, 3):
                    if t[j] != 0.0:
                        a = c[i] / t[i] - c[j] / t[j]
                        if a != 0.0:
                            m = min(m, math.sqrt((self.amax / abs(t[i]) + self.amax / abs(t[j])) / abs(a)))
            elif c[i] != 0.0:
                m = min(m, math.sqrt(self.amax / abs(c[i])))
        return m

    def _vel_limit(self, s):
        t = self.path.tangent(s)
        m = DBL_MAX
        for i in range(3):
            m = min(m, self.vmax / abs(t[i]) if t[i] != 0.0 else math.inf)
        return m

    def _acc_limit_d(self, s):
        return (self._acc_limit(s + EPS) - self._acc_limit(s - EPS)) / (2.0 * EPS)

    def _vel_limit_d(self, s):
        t = self.path.tangent(s)
        m, act = DBL_MAX, 0
        for i in range(3):
            v = self.vmax / abs(t[i]) if t[i] != 0.0 else math.inf
            if v < m:
                m, act = v, i
        return -(self.vmax * self.path.curvature(s)[act]) / (t[act] * abs(t[act]))

    # --- switching points (Trajectory.cpp:124-237) ---
    def _next_switch(self, s):
        acc_sw, acc_b, acc_a = (s, 0.0), 0.0, 0.0
        while True:
            r = self._next_acc_switch(acc_sw[0])
            acc_end = r is None
            if not acc_end:
                acc_sw, acc_b, acc_a = r
            if acc_end or not acc_sw[1] > self._vel_limit(acc_sw[0]):
                break
        vel_sw, vel_b, vel_a = (s, 0.0), 0.0, 0.0
        while True:
            r = self._next_vel_switch(vel_sw[0])
            vel_end = r is None
            if not vel_end:
                vel_sw, vel_b, vel_a = r
            if not (not vel_end and vel_sw[0] <= acc_sw[0]
                    and (vel_sw[1] > self._acc_limit(vel_sw[0] - EPS) or vel_sw[1] > self._acc_limit(vel_sw[0] + EPS))):
                break
        if acc_end and vel_end:
            return None
        if not acc_end and (vel_end or acc_sw[0] <= vel_sw[0]):
            return acc_sw, acc_b, acc_a
        return vel_sw, vel_b, vel_a

    def _next_acc_switch(self, s):
        while True:
            s, disc = self.path.next_switching(s)
            if s > self.path.length - EPS:
                return None
            if disc:
                vb, va = self._acc_limit(s - EPS), self._acc_limit(s + EPS)
                sd = min(vb, va)
                before = self._acc(s - EPS, sd, False)
                after = self._acc(s + EPS, sd, True)
                if ((vb > va or self._slope(s - EPS, sd, False) > self._acc_limit_d(s - 2.0 * EPS))
                        and (vb < va or self._slope(s + EPS, sd, True) < self._acc_limit_d(s + 2.0 * EPS))):
                    return (s, sd), before, after
            else:
                sd = self._acc_limit(s)
                if self._acc_limit_d(s - EPS) < 0.0 and self._acc_limit_d(s + EPS) > 0.0:
                    return (s, sd), 0.0, 0.0

    def _next_vel_switch(self, s):
        step, accuracy = 0.001, 0.000001
        started = False
        s -= step
        while True:
            s += step
            if self._slope(s, self._vel_limit(s), False) >= self._vel_limit_d(s):
                started = True
            if not ((not started or self._slope(s, self._vel_limit(s), False) > self._vel_limit_d(s))
                    and s < self.path.length):
                break
        if s >= self.path.length:
            return None
        lo, hi = s - step, s
        while hi - lo > accuracy:
            s = (lo + hi) / 2.0
            if self._slope(s, self._vel_limit(s), False) > self._vel_limit_d(s):
                lo = s
            else:
                hi = s
        before = self._acc(lo, self._vel_limit(lo), False)
        after = self._acc(hi, self._vel_limit(hi), True)
        return (hi, self._vel_limit(hi)), before, after

    # --- integration (Trajectory.cpp:240-377) ---
    def _forward(self, acc):
        s, sd = self.traj[-1][0], self.traj[-1][1]
        sws = self.path.switching
        nd = 0
        while True:
            while nd < len(sws) and (sws[nd][0] <= s or not sws[nd][1]):
                nd += 1
            s0, sd0 = s, sd
            sd += STEP * acc
            s += STEP * 0.5 * (sd0 + sd)
            if nd < len(sws) and s > sws[nd][0]:
                sd = sd0 + (sws[nd][0] - s0) * (sd - sd0) / (s - s0)
                s = sws[nd][0]
            if s > self.path.length:
                self.traj.append([s, sd, 0.0])
                return True
            if sd < 0.0:
                self.valid = False
                return True
            if sd > self._vel_limit(s) and self._slope(s0, self._vel_limit(s0), False) <= self._vel_limit_d(s0):
                sd = self._vel_limit(s)
            self.traj.append([s, sd, 0.0])
            acc = self._acc(s, sd, True)
            if sd > self._acc_limit(s) or sd > self._vel_limit(s):
                over = self.traj.pop()
                lo, vlo = self.traj[-1][0], self.traj[-1][1]
                hi, vhi = over[0], over[1]
                while hi - lo > EPS:
                    mid = 0.5 * (lo + hi)
                    vmid = 0.5 * (vlo + vhi)
                    if vmid > self._vel_limit(mid) and self._slope(lo, self._vel_limit(lo), False) <= self._vel_limit_d(lo):
                        vmid = self._vel_limit(mid)
                    if vmid > self._acc_limit(mid) or vmid > self._vel_limit(mid):
                        hi, vhi = mid, vmid
                    else:
                        lo, vlo = mid, vmid
                self.traj.append([lo, vlo, 0.0])
                if self._acc_limit(hi) < self._vel_limit(hi):
                    if nd < len(sws) and hi > sws[nd][0]:
                        return False
                    if self._slope(lo, vlo, True) > self._acc_limit_d(lo):
                        return False
                elif self._slope(lo, vlo, False) > self._vel_limit_d(lo):
                    return False

    def _backward(self, s, sd, acc):
        T = self.traj
        if len(T) < 2:
            self.valid = False
            return
        i2 = len(T) - 1
        i1 = i2 - 1
        back = []  # newest last (= the reference list's front)
        slope = 0.0
        while i1 != 0 or s >= 0.0:
            if T[i1][0] <= s:
                back.append([s, sd, 0.0])
                sd -= STEP * acc
                s -= STEP * 0.5 * (sd + back[-1][1])
                acc = self._acc(s, sd, False)
                slope = _div(back[-1][1] - sd, back[-1][0] - s)
                if sd < 0.0:
                    self.valid = False
                    return
            else:
                if i1 == 0:
                    break
                i1 -= 1
                i2 -= 1
            if not back:
                continue
            a, b = T[i1], T[i2]
            cs = _div(b[1] - a[1], b[0] - a[0])
            xs = _div(a[1] - sd + slope * s - cs * a[0], slope - cs)
            if max(a[0], s) - EPS <= xs <= EPS + min(b[0], back[-1][0]):
                xsd = a[1] + cs * (xs - a[0])
                del T[i2:]
                T.append([xs, xsd, 0.0])
                T.extend(reversed(back))
                return
        self.valid = False

    # --- sampling (Trajectory.cpp:459-503) ---
    def duration(self):
        return self.traj[-1][2]

    def state(self, t):
        if t >= self.traj[-1][2]:
            k = len(self.traj) - 1
        else:
            k = bisect.bisect_right(self._times, t)
        p, c = self.traj[k - 1], self.traj[k]
        h = c[2] - p[2]
        acc = 2.0 * (c[0] - p[0] - h * p[1]) / (h * h)
        h = t - p[2]
        s = p[0] + h * p[1] + 0.5 * h * h * acc
        return s, p[1] + h * acc


def _yaw(vx, vy):
    if vx == 0 and vy == 0:
        return 0.0
    if vx == 0:
        return math.pi / 2 if vy > 0 else -math.pi / 2
    if vy == 0:
        return 0.0 if vx > 0 else math.pi
    return math.atan2(vy, vx)


def calculate_trajectory(waypoints, pre_waypoints, v_max, a_max, t0, dt, max_dev):
    """OptimalTimeParametrizer.cpp:11-108 -> list of 11-column rows."""
    pts = [tuple(map(float, p)) for p in pre_waypoints] + [tuple(map(float, p)) for p in waypoints]
    path = Path(pts, max_dev)
    traj = Trajectory(path, v_max, a_max)
    if not traj.valid:
        raise RuntimeError("Trajectory is not valid")
    n = int(traj.duration() / dt)
    first = tuple(map(float, waypoints[0]))
    offset, best = 0, 1000.0
    for i in range(n):
        s, _ = traj.state(i * dt)
        d = _norm(_sub(path.config(s), first))
        if d < best:
            offset, best = i, d
    rows = []
    for i in range(n - offset):
        s, sd = traj.state((i + offset) * dt)
        pos, tan, cur = path.config(s), path.tangent(s), path.curvature(s)
        r = []
        for d in range(3):
            r += [pos[d], tan[d] * sd, cur[d] * sd * sd]
        r += [_yaw(r[1], r[4]), (i * dt) + t0]
        rows.append(r)
    return rows
