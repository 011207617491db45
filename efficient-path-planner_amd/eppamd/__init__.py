"""Host-side Python helpers of the MI355X-native Efficient-Path-Planner hot path.

capi   — ctypes binding of include/epp.h (libepp.so: HIP kernels, no CPU fallback)
config — planner config reader (src/ConfigParserYAML.cpp)
synth  — deterministic synthetic worlds / query batches for tests and bench.py
dist   — one-process-per-GPU plumbing: max-over-ranks timing, RCCL all-gather of waypoints
"""
