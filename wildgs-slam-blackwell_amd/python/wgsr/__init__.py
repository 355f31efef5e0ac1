"""wgsr: MI355X-native WildGS-SLAM Gaussian-splatting hot path (host side).

* ``wgsr._lib``     ctypes binding of libwgsr.so (include/wgsr.h)
* ``wgsr.camera``   the reference's camera / pose matrices (restated)
* ``wgsr.scene``    BASELINE.md synthetic scenes
* ``wgsr.dp``       keyframe-view data parallelism over RCCL
* ``wgsr.render``   the reference ``render()`` contract for a plain scene
"""
__version__ = "0.1.0"
