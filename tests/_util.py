"""Shared test helpers: golden-fixture loading and error metrics."""
from __future__ import annotations

import glob
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SETTING_KEYS = ("H", "W", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix",
                "projmatrix", "projmatrix_raw", "sh_degree", "campos")
INPUT_KEYS = ("means3D", "opacities", "shs", "colors_precomp", "scales", "rotations",
              "cov3D_precomp")
GRAD_KEYS = ("dL_dmeans3D", "dL_dmeans2D", "dL_dopacity", "dL_dsh", "dL_dcolors", "dL_dscales",
             "dL_drotations", "dL_dcov3D")


def scene_names():
    return sorted(os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(GOLDEN, "scene_*.npz")))


def load_scene(name):
    z = np.load(os.path.join(GOLDEN, f"scene_{name}.npz"))
    inputs = {k: torch.from_numpy(z["in_" + k]) for k in INPUT_KEYS if "in_" + k in z}
    settings = {}
    for k in SETTING_KEYS:
        v = z["set_" + k]
        if v.ndim == 0:
            v = v.item()
            if k in ("H", "W", "sh_degree"):
                v = int(v)
            else:
                v = float(v)
        else:
            v = torch.from_numpy(v)
        settings[k] = v
    expect = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    expect["num_rendered"] = int(expect["num_rendered"])
    for k in GRAD_KEYS + ("dL_dtau",):
        if k in z:
            expect[k] = z[k]
    grads = (torch.from_numpy(z["grad_color"]), torch.from_numpy(z["grad_depth"]))
    return inputs, settings, expect, grads


def rel_l1(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.abs(b).sum()
    num = np.abs(a - b).sum()
    if den == 0:
        return float(num)
    return float(num / den)
