"""One rank of tests/test_gpu_dp_online.py (launched by torch.distributed.run,
two ranks sharing the box's GPU over gloo).

1. The whole online loop data-parallel (wgsr.dp_online.DPOnlineMapper):
   initialisation with densify / reset_opacity, keyframe insertions with
   densify_and_prune and reset_opacity_nonvisible -> every rank's replica
   digest, the events, the final PSNR.
2. One data-parallel mapping step against its definition:
   from the same state, rank r's view fwd+bwd, the flat gradient
   all-reduce and Adam, versus one process summing the two views'
   gradients before the same Adam step.
Rank 0 writes the results as JSON to argv[1]."""
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"), ROOT, HERE):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

DEV = torch.device("cuda:0")


def main(out_path):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from test_gpu_online import _keyframes, _psnr
    from wgsr.dp_online import DPOnlineMapper, allreduce_flat
    kfs = _keyframes(4)
    cfg = {"init_itr_num": 24, "init_gaussian_update": 10, "init_gaussian_reset": 15, "mapping_itr_num": 24,
           "gaussian_th": 0.05, "gaussian_update_every": 12, "gaussian_update_offset": 5, "gaussian_reset": 19,
           "window_size": 3}
    m = DPOnlineMapper(sh_degree=0, device=DEV, config=cfg, seed=1)
    m.initialize(kfs[:2])
    for kf in kfs[2:]:
        m.insert_keyframe(kf)
    torch.cuda.synchronize()
    digest = m.replica_digest().cpu()
    kinds = [k for _, k, _ in m.events]
    psnr = _psnr(m, kfs)

    # 2. one step from the current state: DP versus the summed single-view gradients
    ms = m.ms
    st = ms.store
    names = ms.GROUPS
    snap = {n: (st.param(n).clone(), st.exp_avg(n).clone(), st.exp_avg_sq(n).clone()) for n in names}
    steps0, skip0 = dict(ms.steps), set(getattr(ms, "_skip", set()))

    def restore():
        for n in names:
            for dst, src in zip((st.param(n), st.exp_avg(n), st.exp_avg_sq(n)), snap[n]):
                dst.copy_(src)
        ms.steps = dict(steps0)
        ms._skip = set(skip0)

    def view_grad(kf):
        ms.forward_backward(kf.cam, kf.image, kf.depth, kf.exposure_a, kf.exposure_b, m.bg)

    views = kfs[:world]
    view_grad(views[rank])
    allreduce_flat([st.grad(n) for n in names])
    ms.optimizer_step()
    dp = {n: st.param(n).clone() for n in names}
    restore()
    acc = {n: torch.zeros_like(st.grad(n)) for n in names}
    for kf in views:
        view_grad(kf)
        for n in names:
            acc[n] += st.grad(n)
    for n in names:
        st.grad(n).copy_(acc[n])
    ms.optimizer_step()
    rel = {}
    for n in names:
        ref = st.param(n)
        moved = (ref - snap[n][0]).abs().sum().item()
        rel[n] = {"max_abs": float((dp[n] - ref).abs().max()), "moved_l1": moved,
                  "rel_l1_of_update": float((dp[n] - ref).abs().sum()) / max(moved, 1e-30)}
    graphs = graph_phase(kfs, rank)
    with open(f"{out_path}.rank{rank}.graphs.json", "w") as f:
        json.dump(graphs, f)
    if "error" in graphs:
        raise RuntimeError(f"graph phase on rank {rank}: {graphs}")
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"world": world, "digest": digest.tolist(), "events": kinds, "psnr": psnr, "P": int(ms.P),
                       "finite": all(bool(torch.isfinite(st.param(n)).all()) for n in names),
                       "step_vs_summed_views": rel, "psnr_finite": math.isfinite(psnr), "graphs": graphs}, f)
    dist.barrier()
    dist.destroy_process_group()


def graph_phase(kfs, rank):
    """3. The steady state as graph replays (wgsr.dp_online.DPIterationGraphs:
    graph A, the two all-reduces, graph B, the exposure steps) against the
    eager data-parallel loop from the same seeds: the replicas' digests, the
    replay counts and the state's distance to the eager run (the MLP
    gradient's sum order differs, as on one GPU)."""
    from wgsr.dp_online import DPOnlineMapper
    cfg = {"init_itr_num": 30, "init_gaussian_update": 100, "init_gaussian_reset": 10_000, "mapping_itr_num": 60,
           "gaussian_update_every": 100_000, "gaussian_update_offset": 99_999, "gaussian_reset": 100_001,
           "window_size": 4}

    def run(graphs, holder=None):
        # (fresh keyframes per run: a mapper's bank adopts a keyframe's CURRENT
        # fields, and the previous run's bank would hand over its exposures)
        from test_gpu_online import _keyframes
        kfs = _keyframes(4)
        m = DPOnlineMapper(sh_degree=0, device=DEV, config=cfg, seed=3)
        if holder is not None:
            holder["m"] = m
        if not graphs:
            m.graphs = None
        m.initialize(kfs[:2])
        for kf in kfs[2:]:
            m.insert_keyframe(kf, iters=60)
        m.iterations_after_densify_or_reset = 1000
        m.final_refine(40)
        torch.cuda.synchronize()
        return m

    def state(m):
        out = {n: m.ms.store.param(n).clone() for n in m.ms.GROUPS}
        out.update({f"mlp{i}": p.detach().clone() for i, p in enumerate(m.net.parameters())})
        out["exposure"] = m.bank.ex[:, 0].clone()
        return out
    eager = run(False)
    a = state(eager)
    holder = {}
    try:
        mg = run(True, holder)
    except Exception as e:  # (the capacity history and the error, for the test's message)
        g = holder["m"].graphs
        return {"error": f"{type(e).__name__}: {e}", "cap_log": g.stats.get("cap_log"), "stats": {
            k: v for k, v in g.stats.items() if k != "cap_log"}}
    b = state(mg)
    rel = {k: float((a[k] - b[k]).norm() / a[k].norm().clamp_min(1e-12)) if a[k].shape == b[k].shape else None
           for k in a}
    st = mg.graphs.stats
    return {"digest_graphs": mg.replica_digest().cpu().tolist(), "digest_eager": eager.replica_digest().cpu().tolist(),
            "replays": st["replays"], "captures": st["captures"], "overflows": st["overflows"],
            "allreduce_ms_per_replay": 1e3 * st["allreduce_s"] / max(1, st["replays"]),
            "rel_vs_eager": rel, "disabled": mg.graphs.disabled, "cap_log": st.get("cap_log"),
            "exposure_eager": a["exposure"].tolist(), "exposure_graphs": b["exposure"].tolist(),
            "kopt_steps": [eager.kopt_steps, mg.kopt_steps], "iterations": [eager.iteration_count, mg.iteration_count]}


if __name__ == "__main__":
    try:
        main(sys.argv[1])
    except BaseException:
        # every rank's own traceback next to the result file (the launcher
        # keeps only the tail of the interleaved stderr)
        import traceback
        with open(f"{sys.argv[1]}.rank{os.environ.get('RANK', '?')}.err", "w") as f:
            traceback.print_exc(file=f)
        raise
