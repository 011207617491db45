"""Per-block timing of the tiled k-NN kernel (diagnostics; EPP_KNN_TILE_DBG prints to stderr)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd"), ROOT]
from eppamd import capi, synth  # noqa: E402

nodes = synth.sample_states(5, [-6, -6, 0], [6, 6, 2], 63000)
capi.knn(nodes, 16, method="grid")
os.environ["EPP_KNN_TILE_DBG"] = "1"
os.environ["EPP_KNN_TILE"] = sys.argv[1] if len(sys.argv) > 1 else "1"
capi.knn(nodes, 16, method="grid")
