#!/usr/bin/env python
"""Host-side cost of the configs[4]-shaped online mapper loop: cProfile over
tools/bench_online.py (short schedule), top functions by own time.
usage: python tools/host_profile_online.py [bench_online args...]"""
import cProfile
import io
import os
import pstats
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
args = sys.argv[1:] or ["--keyframes", "5", "--init-iters", "100", "--iters", "100"]
sys.argv = ["bench_online.py"] + args
import bench_online as b  # noqa: E402

pr = cProfile.Profile()
pr.enable()
b.main()
pr.disable()
s = io.StringIO()
st = pstats.Stats(pr, stream=s)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumulative").print_stats(45)
print(s.getvalue())
