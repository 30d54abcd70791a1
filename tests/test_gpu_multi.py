"""Multi-process parity of the product transport (RcclComm over RCCL):
world 2 / 4 / 8 ranks, one process each (tests/rccl_worker.py), every rank's
output bit-exact against the reference's fixtures and the oracle.

* With >= world GPUs: rank r on GPU r, RCCL over xGMI (the BASELINE config
  3-5 deployment).
* With fewer GPUs (the 1-GPU test box): all ranks on GPU 0, each with its own
  NCCL_HOSTID so RCCL connects them with its socket transport -- the same
  mgr_exchange_counts / mgr_exchange_rows / mgr_group_p2p calls, offsets,
  ring order, skewed and empty counts, between distinct ranks.
Replaces ``comm.alltoall`` (redist.py:199) and the halo's isend/irecv pairs
(redist.py:289-303).
"""
import json
import os
import signal
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TIMEOUT_S = int(os.environ.get("MGR_MULTI_TIMEOUT", "300"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_multi_rank(world, tmp_path):
    _run_world(world, tmp_path, {})


def test_rccl_full_size_cfg3_cfg4(tmp_path):
    """BASELINE configs 3 and 4 at their full per-GPU size: 125M rows per rank
    (uniform, then clustered), world 2, the product path over RCCL, checked by
    properties against the C oracle (rccl_worker.case_full_size)."""
    _run_world(2, tmp_path, {"MGR_TEST_SET": "fullsize", "MGR_CASE_TIMEOUT": "300"},
               timeout=900)


def _run_world(world, tmp_path, extra_env, timeout=TIMEOUT_S):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    shared = torch.cuda.device_count() < world
    port = _free_port()
    # worker logs go to files (gpurun_out/ on the GPU box: progress stays visible)
    logdir = os.path.join(ROOT, "gpurun_out") if os.environ.get("GRAFT_REPO_ROOT") else str(tmp_path)
    os.makedirs(logdir, exist_ok=True)
    procs, logs = [], []
    for r in range(world):
        env = dict(os.environ)
        env.update(RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   MGR_TEST_OUT=str(tmp_path / f"rank{r}.json"),
                   MGR_TEST_SHARED_GPU="1" if shared else "0")
        env.update(extra_env)
        tag = extra_env.get("MGR_TEST_SET", "")
        logs.append(open(os.path.join(logdir, f"multi_w{world}{tag}_rank{r}.log"), "w"))
        procs.append(subprocess.Popen([sys.executable, "-u", "-m", "tests.rccl_worker"], cwd=ROOT,
                                      env=env, start_new_session=True, stdout=logs[-1],
                                      stderr=subprocess.STDOUT))
    codes = []
    try:
        for p in procs:
            codes.append(p.wait(timeout=timeout))
    except subprocess.TimeoutExpired:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
        for p in procs:
            p.wait()
        pytest.fail(f"world {world}: ranks did not finish within {timeout} s")
    finally:
        for fh in logs:
            fh.close()
    failures = {}
    for r in range(world):
        path = tmp_path / f"rank{r}.json"
        assert path.exists(), f"rank {r} exited {codes[r]} without results"
        res = json.loads(path.read_text())
        assert res, f"rank {r}: no cases ran"
        failures.update({f"rank{r}:{k}": v for k, v in res.items() if v != "ok"})
    assert not failures, "\n".join(f"{k}: {v}" for k, v in failures.items())
    assert all(c == 0 for c in codes), codes
