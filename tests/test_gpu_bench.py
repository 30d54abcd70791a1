"""GPU: bench.py's JSON line keeps the driver's contract (metric, value,
unit, steps, roofline with achieved / peak / frac / traffic, config
workload ...) -- run as a child process on a small config-2 input."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--particles", "4194304",
                        "--steps", "3", "--warmup", "1", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    rec = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True and rec["unit"] == "particles/s"
    assert abs(rec["value"] - 4194304 / (rec["ms_per_step"] / 1e3)) / rec["value"] < 1e-6
    assert rec["config"]["workload"].startswith("cfg2_")
    rl = rec["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(rl)
    assert rl["bound"] == "hbm" and rl["unit"] == "GB/s" and rl["peak"] == 8000.0
    assert abs(rl["frac"] - rl["achieved"] / rl["peak"]) < 1e-9
