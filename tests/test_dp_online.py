"""The data-parallel online mapper's exchange logic (wgsr.dp_online) over
gloo, world_size 2, on CPU tensors: the flat gradient all-reduce, the
statistics reduction before a densify, the visibility union of
reset_opacity_nonvisible, the gathered exposure steps and occlusion masks,
and the per-rank keyframe draw.  The GPU run of the whole loop on two ranks
is tests/test_gpu_dp_online.py."""
import os
import socket
import sys
from types import SimpleNamespace

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Store:
    def __init__(self, rank):
        g = torch.Generator().manual_seed(10 + rank)
        # the gradients as views of one flat buffer (GaussianStore.grad_flat)
        widths = (("xyz", 3), ("features", 3), ("opacity", 1), ("scaling", 3), ("rotation", 4))
        self.flat = torch.randn(5 * sum(k for _, k in widths), generator=g)
        self.t, off = {}, 0
        for n, k in widths:
            self.t[n] = self.flat[off:off + 5 * k].view(5, k)
            off += 5 * k
        self.s = {"xyz_gradient_accum": torch.rand(5, 1, generator=g), "denom": torch.randint(0, 3, (5, 1)).float(),
                  "max_radii2D": torch.rand(5, generator=g) * 10}

    def grad(self, n):
        return self.t[n]

    def grad_flat(self):
        return self.flat

    def stat(self, n):
        return self.s[n]


def _worker(rank, port, out_dir):
    for p in (os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python"), ROOT):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from wgsr.dp_online import DPOnlineMapper, allreduce_flat, gather_exposure, gather_rows
    res = {}
    # flat all-reduce of tensors of different shapes, in place
    a = torch.full((2, 3), float(rank + 1))
    b = torch.arange(4, dtype=torch.float32) * (rank + 1)
    allreduce_flat([a, None, b])
    res["a"], res["b"] = a, b
    res["rows"] = gather_rows(torch.tensor([rank * 10.0, rank + 0.5]))
    # exposure gathering: the same keyframe on both ranks, then two different ones
    part = torch.full((3, 2), float(rank + 1))
    res["exp_same"] = gather_exposure(5, part)
    res["exp_diff"] = gather_exposure(3 + 4 * rank, part)
    # the per-rank draw: every rank consumes world draws and keeps its own
    it = iter(range(100))
    fake = SimpleNamespace(world=WORLD, rank=rank)
    res["picks"] = [DPOnlineMapper._pick(fake, lambda: next(it)) for _ in range(3)]
    res["next_draw"] = next(it)
    # the after-backward reduction on a stand-in mapper state
    st = _Store(rank)
    net = torch.nn.Linear(2, 2)
    for p in net.parameters():
        p.grad = torch.full_like(p, float(rank + 1))
    fake = SimpleNamespace(ms=SimpleNamespace(store=st, GROUPS=("xyz", "features", "opacity", "scaling", "rotation")),
                           net=net, group=None)
    res["grads_in"] = {n: t.clone() for n, t in st.t.items()}
    res["stats_in"] = {n: t.clone() for n, t in st.s.items()}
    radii = torch.tensor([0, 1, 0, 2, 0], dtype=torch.int32) if rank == 0 else torch.tensor([0, 0, 3, 0, 0],
                                                                                            dtype=torch.int32)
    vis = DPOnlineMapper._after_backward(fake, {"radii": radii}, True, True)
    res["grads_out"] = st.t
    res["stats_out"] = st.s
    res["vis"] = vis
    res["mlp_grad"] = [p.grad for p in net.parameters()]
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def test_dp_online_exchange(tmp_path):
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    r = [torch.load(tmp_path / f"rank{k}.pt", weights_only=True) for k in range(WORLD)]
    for k in range(WORLD):
        assert torch.equal(r[k]["a"], torch.full((2, 3), 3.0))
        assert torch.equal(r[k]["b"], torch.arange(4, dtype=torch.float32) * 3)
        assert torch.equal(r[k]["rows"], torch.tensor([[0.0, 0.5], [10.0, 1.5]]))
        same = r[k]["exp_same"]
        assert len(same) == 1 and same[0][0] == 5
        assert torch.equal(same[0][1], torch.cat([torch.full((3, 2), 1.0), torch.full((3, 2), 2.0)]))
        diff = r[k]["exp_diff"]
        assert [u for u, _ in diff] == [3, 7]
        assert torch.equal(diff[1][1], torch.full((3, 2), 2.0))
        assert r[k]["picks"] == [k, 2 + k, 4 + k] and r[k]["next_draw"] == 6
        for n in r[k]["grads_out"]:
            assert torch.equal(r[k]["grads_out"][n], r[0]["grads_in"][n] + r[1]["grads_in"][n]), n
        for n in ("xyz_gradient_accum", "denom"):
            assert torch.equal(r[k]["stats_out"][n], r[0]["stats_in"][n] + r[1]["stats_in"][n]), n
        assert torch.equal(r[k]["stats_out"]["max_radii2D"],
                           torch.maximum(r[0]["stats_in"]["max_radii2D"], r[1]["stats_in"]["max_radii2D"]))
        assert r[k]["vis"].tolist() == [False, True, True, True, False]
        for g in r[k]["mlp_grad"]:
            assert torch.equal(g, torch.full_like(g, 3.0))
