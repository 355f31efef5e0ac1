#!/usr/bin/env python
"""Host-side (Python / ctypes / launch) cost of a small-scale mapping
iteration: cProfile over tools/bench_mapping_step.py's fused path, top
functions by own time.  usage: python tools/host_profile.py [bench args...]"""
import cProfile
import io
import os
import pstats
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
args = sys.argv[1:] or ["--loss", "uncertainty", "--only", "fused", "--P", "100000", "--width", "512",
                        "--height", "384", "--iters", "200"]
sys.argv = ["bench_mapping_step.py"] + args
import bench_mapping_step as b  # noqa: E402

pr = cProfile.Profile()
pr.enable()
b.main()
pr.disable()
s = io.StringIO()
st = pstats.Stats(pr, stream=s)
st.sort_stats("tottime").print_stats(40)
st.print_callers(r"method 'to' of|_foreach_sqrt|torch.rsub|method 'clamp'")
print(s.getvalue())
