"""Drop-in ``simple_knn`` for MI355X: ``from simple_knn._C import distCUDA2``
(thirdparty/gaussian_splatting/scene/gaussian_model.py:18,201-207)."""
