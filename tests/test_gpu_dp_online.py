"""The online mapper data-parallel over keyframe views (wgsr.dp_online,
SURVEY.md 8(e)) on two ranks sharing the box's GPU over gloo (the 8-GPU
run takes the same code over RCCL): tests/_dp_online_worker.py runs the loop
through initialisation, keyframe insertions, densify_and_prune, the opacity
resets, the exposure and MLP steps, then one step checked against its
definition.

* the replicas are identical after the run (every rank's digest of its
  Gaussians, MLP and exposures);
* one data-parallel step equals the Adam step on the SUM of the two views'
  single-process gradients (8(e)'s parity bar: rel L1 <= 1e-5 of the update;
  the two-operand sum is exact, so it is bit-identical in practice);
* the steady state as graph replays (DPIterationGraphs) keeps the replicas
  identical and stays within the MLP sum order of the eager data-parallel
  loop (the single-GPU bar of test_gpu_online_graph);
* every branch ran and the map is usable (finite, PSNR as in
  test_gpu_online)."""
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


def test_dp_online_mapper_two_ranks(tmp_path):
    out = tmp_path / "dp_online.json"
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "_dp_online_worker.py"), str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    if r.returncode != 0:
        errs = "".join(f"--- rank {k} ---\n" + open(f"{out}.rank{k}.err").read()[-3000:]
                       for k in range(2) if os.path.exists(f"{out}.rank{k}.err"))
        raise AssertionError(errs or r.stderr[-4000:])
    res = json.loads(out.read_text())
    assert res["world"] == 2
    d = res["digest"]
    assert d[0] == d[1], d
    kinds = res["events"]
    assert kinds.count("densify") >= 3 and "reset_opacity" in kinds and "reset_opacity_nonvisible" in kinds
    assert res["finite"] and res["psnr"] > 12.0
    for name, v in res["step_vs_summed_views"].items():
        assert v["moved_l1"] > 0, name
        assert v["rel_l1_of_update"] <= 1e-5, (name, v)
    # the graph-replayed data-parallel steady state: replicas identical, most
    # iterations replayed, the state within the MLP sum order of the eager loop
    g = res["graphs"]
    assert g["disabled"] is None
    assert g["digest_graphs"][0] == g["digest_graphs"][1], g["digest_graphs"]
    assert g["digest_eager"][0] == g["digest_eager"][1], g["digest_eager"]
    assert g["replays"] > 100 and g["captures"] >= 2 and g["overflows"] == 0, g
    bad = {k: r for k, r in g["rel_vs_eager"].items() if r is None or r > 2e-3}
    assert not bad, (g["rel_vs_eager"], g.get("exposure_eager"), g.get("exposure_graphs"), g.get("kopt_steps"),
                     g.get("iterations"))
