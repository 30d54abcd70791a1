"""CPU tests of bench.py's bare multi-GPU launch (`python bench.py --gpus N`
with no WORLD_SIZE): the parent starts N rank processes as children, relays
rank 0's JSON line, and fails loudly -- on a failing rank, on a timeout, or
when rank 0 prints no line -- instead of hanging or exec'ing.  The children
here are a tiny stand-in script (no GPU), driven by its argv."""
import io
import json
import os
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

CHILD = textwrap.dedent("""
    import json, os, sys, time
    mode = sys.argv[1]
    r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["MASTER_PORT"]) > 0
    assert os.environ["LOCAL_RANK"] == str(r)
    if mode == "fail" and r == 1:
        sys.exit(7)
    if mode == "hang" or (mode == "fail" and r != 1):
        time.sleep(600)
    if mode == "silent":
        sys.exit(0)
    if r == 0:
        print(json.dumps({"metric": "x", "value": 1.0, "n_gpus": w,
                          "ranks_seen": [os.environ["RANK"], os.environ["WORLD_SIZE"]]}))
""")


@pytest.fixture
def child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return str(p)


def test_relays_rank0_line(child):
    out = io.StringIO()
    rc = bench.launch_ranks(3, ["ok"], 60, script=child, out=out)
    assert rc == 0
    lines = [ln for ln in out.getvalue().splitlines() if ln.strip()]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 3 and rec["ranks_seen"] == ["0", "3"]


def test_failing_rank_kills_peers(child):
    t0 = time.monotonic()
    rc = bench.launch_ranks(3, ["fail"], 120, script=child, grace_s=1.0, out=io.StringIO())
    assert rc == 7
    assert time.monotonic() - t0 < 30      # peers stuck "in a collective" were killed


def test_timeout_kills_all(child):
    t0 = time.monotonic()
    rc = bench.launch_ranks(2, ["hang"], 2.0, script=child, out=io.StringIO())
    assert rc == 124
    assert time.monotonic() - t0 < 30


def test_no_json_line_is_a_failure(child):
    assert bench.launch_ranks(2, ["silent"], 60, script=child, out=io.StringIO()) == 3


def test_cpu_baseline_c_is_repeatable():
    """bench.py's threaded C baseline reports the median of its iterations
    (no allocation or first touch inside a timed call): two runs agree within
    20 % (best-of-3 picked a 3.7x outlier in round 5)."""
    a, b = bench.cpu_baseline_c(iters=5), bench.cpu_baseline_c(iters=5)
    assert a["stat"] == "median" and a["spread"][0] <= a["value"] <= a["spread"][1]
    assert abs(a["value"] - b["value"]) / max(a["value"], b["value"]) < 0.2, (a, b)
