#!/usr/bin/env python
"""Stage times of the A/B bench runs written by tools/gpu_check.sh (step ab)."""
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
rows = []
for f in sorted(glob.glob(os.path.join(root, "ab_*.json"))):
    try:
        d = json.load(open(f))
    except Exception:
        continue
    st = d.get("stages_ms_per_step", {})
    rows.append((os.path.basename(f)[3:-5], d["ms_per_step"], st))
keys = list(rows[0][2]) if rows else []
print(f"{'variant':18s} {'ms/step':>8s} " + " ".join(f"{k[:10]:>10s}" for k in keys))
for name, ms, st in rows:
    print(f"{name:18s} {ms:8.3f} " + " ".join(f"{st.get(k, float('nan')):10.3f}" for k in keys))
