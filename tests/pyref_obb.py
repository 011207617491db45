"""Pure-Python restatement of the reference's World/OBB semantics (small cases only).

An independent second transcription of src/OBB.cpp:10-123 and src/World.cpp:80-162,
used to cross-check oracle/epp_oracle.cpp.  Python floats are IEEE doubles and
Python never fuses a multiply-add, matching the reference's x86-64 build.
"""
import math


def _local(o, p):
    d = [p[i] - o["center"][i] for i in range(3)]
    R = o["rot"]
    # (R^T)(i,k) = R(k,i); Eigen: localPoint = rotation.transpose() * (point - center)
    return [(R[i] * d[0] + R[3 + i] * d[1]) + R[6 + i] * d[2] for i in range(3)]


def point_hit(o, p, inflate):
    l = _local(o, p)
    h = list(o["half"])
    if not o["filling"]:
        h = [x + inflate for x in h]
    return abs(l[0]) <= h[0] and abs(l[1]) <= h[1] and abs(l[2]) <= h[2]


def ray_hit(o, s, e, inflate):
    if point_hit(o, s, inflate) or point_hit(o, e, inflate):
        return True
    ls, le = _local(o, s), _local(o, e)
    ld = [le[i] - ls[i] for i in range(3)]
    tmin, tmax = 0.0, 1.0
    for i in range(3):
        ih = o["half"][i] + inflate
        bmin, bmax = -ih, ih
        if abs(ld[i]) < 1e-6:
            if ls[i] < bmin or ls[i] > bmax:
                return False
        else:
            inv = 1.0 / ld[i]
            t1 = (bmin - ls[i]) * inv
            t2 = (bmax - ls[i]) * inv
            te = t2 if t2 < t1 else t1
            tx = t2 if t1 < t2 else t1
            tmin = te if tmin < te else tmin
            tmax = tx if tx < tmax else tmax
            if tmin > tmax:
                return False
    return 0 <= tmin <= 1 and 0 <= tmax <= 1


def _r(o, rg, ro):
    return rg if o["is_gate"] else ro


def point_valid(world, rg, ro, p, can_pass):
    for o in world:
        lo, hi = o["aabb_lo"], o["aabb_hi"]
        if not all(lo[i] < p[i] < hi[i] for i in range(3)):
            continue
        if o["filling"] and can_pass:
            continue
        if point_hit(o, p, _r(o, rg, ro)):
            return False
    return True


def point_valid_mindist(world, p, md):
    for o in world:
        lo, hi = o["aabb_lo"], o["aabb_hi"]
        if not all(lo[i] < p[i] < hi[i] for i in range(3)):
            continue
        if o["filling"]:
            continue
        if point_hit(o, p, md):
            return False
    return True


def ray_valid(world, rg, ro, s, e, can_pass):
    lo = [min(s[i], e[i]) for i in range(3)]
    hi = [max(s[i], e[i]) for i in range(3)]
    for o in world:
        if any(o["aabb_hi"][i] < lo[i] or hi[i] < o["aabb_lo"][i] for i in range(3)):
            continue
        if o["filling"] and can_pass:
            continue
        if ray_hit(o, s, e, _r(o, rg, ro)):
            return False
    return True


def ray_valid_d32(world, rg, ro, s, e, can_pass):
    for k in range(1, 33):
        t = k / 32.0
        p = [s[i] + (e[i] - s[i]) * t for i in range(3)]
        if not point_valid(world, rg, ro, p, can_pass):
            return False
    return True


def build(geom_gate_desc, gate_off, obst_desc, gates, obstacles, rg, ro):
    """World build (src/Object.cpp:52-85, src/OBB.cpp:93-123) into dicts."""
    out = []

    def obj(g, rot, descs, is_gate, infl):
        c, s = math.cos(rot[2]), math.sin(rot[2])
        R = [c, -s, 0.0, s, c, 0.0, 0.0, 0.0, 1.0]
        gc = [0.0 + g[0], 0.0 + g[1], 0.0 + g[2]]
        for d in descs:
            half = [float(x) / 2 for x in d["size"]]
            ctr = [float(d["pos"][i]) + g[i] for i in range(3)]
            rel = [ctr[i] - gc[i] for i in range(3)]
            ctr = [((R[3 * i] * rel[0] + R[3 * i + 1] * rel[1]) + R[3 * i + 2] * rel[2]) + gc[i] for i in range(3)]
            o = {"center": ctr, "half": half, "rot": R, "filling": bool(d["filling"]), "is_gate": is_gate}
            sx = [-1, 1, 1, -1, -1, 1, 1, -1]
            sy = [-1, -1, 1, 1, -1, -1, 1, 1]
            sz = [-1, -1, -1, -1, 1, 1, 1, 1]
            lo, hi = [0.0] * 3, [0.0] * 3
            for j in range(8):
                cr = [sx[j] * half[0], sy[j] * half[1], sz[j] * half[2]]
                for i in range(3):
                    v = ((R[3 * i] * cr[0] + R[3 * i + 1] * cr[1]) + R[3 * i + 2] * cr[2]) + ctr[i]
                    lo[i] = v if j == 0 else min(lo[i], v)
                    hi[i] = v if j == 0 else max(hi[i], v)
            if not o["filling"]:
                lo = [x - infl for x in lo]
                hi = [x + infl for x in hi]
            o["aabb_lo"], o["aabb_hi"] = lo, hi
            out.append(o)

    for row in gates:
        t = int(row[6])
        descs = geom_gate_desc[gate_off[t]:gate_off[t + 1]]
        obj([row[0], row[1], 0.0], [row[3], row[4], row[5]], descs, True, rg)
    for row in obstacles:
        obj([row[0], row[1], row[2]], [row[3], row[4], row[5]], obst_desc, False, ro)
    return out
