#!/usr/bin/env python
"""Per-kernel vector-memory-path summary of a gpu_check.sh `pmc_ta` pass.

Counters are summed over instances (one TA / TD / TCP per CU); GRBM_GUI_ACTIVE
is the busy clock count summed over the 8 XCDs (~8.3x the kernel's duration
in clocks on the bench's kernels), so a block's busy fraction is
X_sum / (256 CUs x GRBM_GUI_ACTIVE / 8).  TCP_TCC_READ_REQ_LATENCY_sum over
the tag accesses is a rough mean L2 latency per access (cycles).

usage: python tools/pmc_ta.py gpurun_out/pmc_ta[_sfx]/run_counter_collection.csv
"""
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import load  # noqa: E402

N_CU, N_XCD = 256, 8


def main():
    path = sys.argv[1]
    d = load(path)
    rows = []
    for (k, grid), c in d.items():
        if not c.get("GRBM_GUI_ACTIVE"):
            continue
        n = len(c["GRBM_GUI_ACTIVE"])
        avg = {name: sum(v) / max(len(v), 1) for name, v in c.items() if name != "_ns"}
        gui = avg["GRBM_GUI_ACTIVE"] or 1.0
        frac = lambda name: avg.get(name, 0.0) / (N_CU * gui / N_XCD)  # noqa: E731
        rows.append((avg.get("GRBM_GUI_ACTIVE", 0), k, grid, n, frac("TA_TA_BUSY_sum"),
                     frac("TA_ADDR_STALLED_BY_TC_CYCLES_sum"), frac("TD_TD_BUSY_sum"), frac("TD_TC_STALL_sum"),
                     frac("TCP_TCP_TA_DATA_STALL_CYCLES_sum"), frac("TCP_PENDING_STALL_CYCLES_sum"),
                     avg.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0) / 1e3))
    rows.sort(reverse=True)
    print(f"{'kernel':24s} {'grid':>8s} {'n':>3s} {'gui_kcyc':>8s} {'TA_busy':>7s} {'TA_stTC':>7s} {'TD_busy':>7s} "
          f"{'TD_stTC':>7s} {'TCP_stTA':>8s} {'TCP_pend':>8s} {'tags_k':>9s}")
    for gui, k, grid, n, ta, tast, td, tdst, tcpst, pend, tags in rows:
        print(f"{k[:24]:24s} {grid:8d} {n:3d} {gui / 1e3:8.1f} {ta:7.3f} {tast:7.3f} {td:7.3f} {tdst:7.3f} "
              f"{tcpst:8.3f} {pend:8.3f} {tags:9.1f}")


if __name__ == "__main__":
    main()
