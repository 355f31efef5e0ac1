"""The first multi-GPU run's safety net, exercised: bench.py's N > 1 path with
two ranks sharing the box's GPU over gloo (WGSR_BENCH_BACKEND=gloo,
WGSR_BENCH_SHARE_GPU=1; the driver's 8-GPU run takes the same code path
over RCCL), with faults injected into the exchange (wgsr.dp._fault):

* none                       -> exchange_check ok, the views exchange timed;
* the exchange raises        -> fallback "allreduce", a valid bench line, rc 0;
* one rank's result is off   -> both ranks fall back (the decision is a MIN
                                over the gloo control group), rc 0;
* exchange AND the fallback all-reduce raise -> non-zero exit, no bench line.

SURVEY.md 8(e); VERDICT round 3, "Next round" item 2.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(extra_env, timeout=150):
    env = dict(os.environ, WGSR_BENCH_BACKEND="gloo", WGSR_BENCH_SHARE_GPU="1", WGSR_BENCH_PG_TIMEOUT="60",
               OMP_NUM_THREADS="4", **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--P", "20000", "--width", "320", "--height", "240",
           "--no-profile", "--no-knn"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr[-3000:]


@pytest.mark.parametrize("fault", ["none", "raise", "perturb_rank1"])
def test_bench_dp_exchange_check_and_fallback(fault):
    env = {"none": {}, "raise": {"WGSR_DP_FAULT": "raise"},
           "perturb_rank1": {"WGSR_DP_FAULT": "perturb", "WGSR_DP_FAULT_RANKS": "1"}}[fault]
    rc, line, err = _run(env)
    assert rc == 0, err
    assert line is not None, err
    chk = line["config"]["exchange_check"]
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["ms_per_step"] > 0
    if fault == "none":
        assert chk["ok"] and "fallback" not in chk and chk["rel_l1_vs_allreduce"] <= 1e-5
        assert line["config"]["dp_exchange"] == "views"
    else:
        assert not chk["ok"] and chk["fallback"] == "allreduce"
        assert line["config"]["dp_exchange"] == "allreduce"
        if fault == "raise":
            assert "injected exchange failure" in chk.get("error", "")
        else:   # rank 0's own result agreed: the fallback came from rank 1's vote
            assert chk["rel_l1_vs_allreduce"] <= 1e-5 and "error" not in chk


def test_bench_dp_failed_fallback_exits_nonzero():
    rc, line, err = _run({"WGSR_DP_FAULT": "raise", "WGSR_DP_FAULT_ALLREDUCE": "raise"})
    assert rc != 0
    assert line is None
    assert "all-reduce fallback failed" in err
