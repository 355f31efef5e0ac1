"""Generate tests/golden/dino_cases.npz (build container): inputs, value and
uncertainty gradient of the reference's OWN compute_dino_regularization_loss
(src/utils/dyn_uncertainty/mapping_utils.py:332-389) on CPU -- the DINO
feature-similarity regulariser of the mapper (mapper.py:1140-1164, 986-997).

Features are clustered (so that many pairs pass the 0.75 cosine threshold)
and the three call shapes are covered: a [1, N] sampled-uncertainty with
[1, N, C] features (map_opt_online), lists of one strided [h, w, 1] map and
one [h, w, C] feature map (initialize_map_opt), and fewer samples than the
top-k of 128.  loss_utils.py imports cv2 (absent here, unused): a stub module.

Usage:  python tests/golden/make_dino_fixtures.py
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def main():
    sys.path.insert(0, REF)
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    from src.utils.dyn_uncertainty import mapping_utils as mu
    g = torch.Generator().manual_seed(31)
    out = {}
    for ci, (shape, C, n_clusters) in enumerate([((1, 300), 64, 6), ((9, 7), 32, 3), ((1, 60), 16, 4)]):
        n = shape[0] * shape[1]
        centers = torch.randn(n_clusters, C, generator=g)
        lab = torch.randint(0, n_clusters, (n,), generator=g)
        feat = centers[lab] + 0.35 * torch.randn(n, C, generator=g)
        unc = (0.1 + 2 * torch.rand(n, generator=g)).reshape(shape).requires_grad_(True)
        if ci == 1:  # list inputs as initialize_map_opt passes them
            loss = mu.compute_dino_regularization_loss([unc.unsqueeze(-1)], [feat.reshape(shape + (C,))])
        else:
            loss = mu.compute_dino_regularization_loss(unc, feat.reshape(shape + (C,)))
        loss.backward()
        k = f"c{ci}_"
        out[k + "unc"] = unc.detach().numpy()
        out[k + "feat"] = feat.reshape(shape + (C,)).numpy()
        out[k + "loss"] = np.array(float(loss))
        out[k + "grad"] = unc.grad.numpy()
        out[k + "as_list"] = np.array(ci == 1)
    np.savez_compressed(os.path.join(HERE, "dino_cases.npz"), **out)
    print("dino_cases.npz:", {k: float(v) for k, v in out.items() if k.endswith("loss")})


if __name__ == "__main__":
    main()
