#!/usr/bin/env python3
"""Halo selection tile size A/B (GPU): the --exchange --config 3 --overload
0.05 bench line with halo.SELECT_TILE_ROWS set per run (HALO_TILE env), one
JSON line per run (the bench's own)."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_grid_redistribute_amd.halo as halo  # noqa: E402

halo.SELECT_TILE_ROWS = int(os.environ.get("HALO_TILE", halo.SELECT_TILE_ROWS))
sys.argv = ["bench.py", "--no-cpu-baseline", "--exchange", "--config", "3", "--overload", "0.05",
            "--steps", "20", "--warmup", "5"]
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "bench.py"), run_name="__main__")
