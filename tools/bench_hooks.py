#!/usr/bin/env python3
"""Same-build A/B of a test hook on a bench line (GPU): sets the hooks in
BENCH_HOOKS (JSON object, include/mgr_instrument.h) in this process, then
runs bench.py with the remaining arguments; one JSON line per run (the
bench's own).  Example: BENCH_HOOKS='{"msel_lists": 1}' python
tools/bench_hooks.py --no-cpu-baseline --exchange --config 3 --overload 0.05"""
import json
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpi_grid_redistribute_amd import _lib  # noqa: E402

for k, v in json.loads(os.environ.get("BENCH_HOOKS", "{}")).items():
    _lib.test_hook(k, v)
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")
