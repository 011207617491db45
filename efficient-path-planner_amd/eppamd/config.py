"""Planner configuration (the reference's ConfigParser, src/ConfigParserYAML.cpp:10-118).

The reference loads the file with yaml-cpp; JSON is the subset both files in the
repositories use.  Geometry is returned as flat description arrays that both the
C ABI (``epp_obb_desc``) and the test oracle (``or_obb_desc``) accept.
"""
from __future__ import annotations

import json
from dataclasses import dataclass

import numpy as np

# struct epp_obb_desc / or_obb_desc: pos[3], size[3], int32 filling, int32 pad
OBB_DESC_DTYPE = np.dtype([("pos", "<f8", 3), ("size", "<f8", 3), ("filling", "<i4"), ("pad", "<i4")])


@dataclass
class Geometry:
    gate_desc: np.ndarray      # OBB_DESC_DTYPE, all gate types concatenated
    gate_desc_off: np.ndarray  # int32 [n_types + 1]
    obst_desc: np.ndarray      # OBB_DESC_DTYPE
    gate_height: np.ndarray    # float64 [n_types]  (component_properties.<comp>.height)


def _descs(component: dict) -> np.ndarray:
    out = np.zeros(len(component), dtype=OBB_DESC_DTYPE)
    for i, (_name, obb) in enumerate(component.items()):  # document order, as yaml-cpp
        out[i]["pos"] = [float(v) for v in obb["position"]]
        out[i]["size"] = [float(v) for v in obb["size"]]
        t = obb["type"]
        if t not in ("collision", "filling"):
            raise ValueError(f"unknown OBB type {t!r}")
        out[i]["filling"] = 1 if t == "filling" else 0
    return out


def load(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


def geometry(cfg: dict) -> Geometry:
    """ConfigParser::parseGeometries / getGateGeometryByTypeId (src/ConfigParserYAML.cpp:21-73)."""
    mapping = cfg["gate_id_to_name_mapping"]
    n_types = len(mapping)
    descs, off, heights = [], [0], []
    for t in range(n_types):
        name = mapping[str(t)]
        d = _descs(cfg["component_geometry"][name])
        descs.append(d)
        off.append(off[-1] + len(d))
        heights.append(float(cfg["component_properties"][name]["height"]))
    gate_desc = np.concatenate(descs) if descs else np.zeros(0, OBB_DESC_DTYPE)
    obst = _descs(cfg["component_geometry"]["obstacle"])
    return Geometry(gate_desc, np.asarray(off, np.int32), obst, np.asarray(heights))


def inflate_radii(cfg: dict) -> tuple[float, float]:
    r = cfg["world_properties"]["inflate_radius"]
    return float(r["gate"]), float(r["obstacle"])


def bounds(cfg: dict) -> tuple[np.ndarray, np.ndarray]:
    w = cfg["world_properties"]
    return np.asarray(w["lower_bound"], float), np.asarray(w["upper_bound"], float)
