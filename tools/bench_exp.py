"""EXPERIMENT: bench.py with the gemm256 block-stagger knob set (A/B timing only).
usage: python tools/bench_exp.py ITERS MODE [bench args...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "transformer-stm_amd"))
from vitmi import _lib  # noqa: E402

it, mode = int(sys.argv[1]), int(sys.argv[2])
sys.argv = [sys.argv[0]] + sys.argv[3:]
lib = _lib.lib()
lib.vitmi_gemm_experiment.argtypes = [ctypes.c_int, ctypes.c_int]
lib.vitmi_gemm_experiment(it, mode)
import bench  # noqa: E402

bench.main()
