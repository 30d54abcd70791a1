"""GPU: the C ABI from a host program with no Python or torch in it
(examples/c_abi_partition.cpp: hipMalloc'd buffers -> mgr_bin_count ->
mgr_scan -> mgr_pack), checked inside the program byte for byte against a C++
restatement of redist.py:157-198 (wrapped positions, counts, partitioned
rows).  Run as a child process, bounded by a timeout."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "bin", "c_abi_partition")


@pytest.mark.parametrize("n", [1, 4097, 1 << 22])
def test_c_abi_program_partition_exact(n):
    if not os.path.exists(EXE):
        pytest.fail("examples/bin/c_abi_partition missing: run __graft_entry__.build()")
    r = subprocess.run([EXE, str(n)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"c_abi_partition ok: n={n} " in r.stdout, r.stdout
