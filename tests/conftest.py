"""pytest configuration: registers the ``gpu`` marker and puts the package's
python directory (``wildgs-slam-blackwell_amd/python``) and the repo root on
sys.path so tests import ``diff_gaussian_rasterization``, ``simple_knn``,
``wgsr`` and ``oracle`` the way a WildGS caller would."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG_PY = os.path.join(ROOT, "wildgs-slam-blackwell_amd", "python")
for p in (PKG_PY, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
