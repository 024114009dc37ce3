"""Summaries of a rocprofv3 kernel-trace CSV.

    python tools/ktrace.py <run_kernel_trace.csv> [--epoch K] [--start KERNEL]

Prints per-kernel totals per epoch (an epoch starts at each k_probe, or at
each KERNEL, e.g. k_tpcc_resolve for TPC-C epochs) and the
dispatch timeline of epoch K (duration and gap to the previous dispatch).
"""
import csv
import sys
from collections import defaultdict


def short(name):
    name = name.split("(")[0]
    for p in ("void ", "dvcc::"):
        if name.startswith(p):
            name = name[len(p):]
    return name


def main():
    path = sys.argv[1]
    show = int(sys.argv[sys.argv.index("--epoch") + 1]) if "--epoch" in sys.argv else 3
    start = sys.argv[sys.argv.index("--start") + 1] if "--start" in sys.argv else "k_probe"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    epochs, cur = [], None
    for r in rows:
        name = short(r["Kernel_Name"])
        if name.startswith(start):
            cur = []
            epochs.append(cur)
        if cur is not None:
            cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Grid_Size_X"]))
    print(f"{len(epochs)} epochs")
    for k, ep in enumerate(epochs):
        tot = defaultdict(float)
        cnt = defaultdict(int)
        for n, s, e, _ in ep:
            tot[n] += (e - s) / 1e3
            cnt[n] += 1
        wall = (ep[-1][2] - ep[0][1]) / 1e3
        busy = sum(tot.values())
        print(f"epoch {k}: wall {wall:.1f} us, busy {busy:.1f} us, "
              + ", ".join(f"{n}x{cnt[n]}={t:.1f}" for n, t in sorted(tot.items(), key=lambda x: -x[1])))
    if show < len(epochs):
        ep = epochs[show]
        prev = ep[0][1]
        print(f"--- epoch {show} timeline (us): name dur gap grid")
        for n, s, e, g in ep:
            print(f"{n:32s} {(e - s) / 1e3:8.1f} {(s - prev) / 1e3:7.1f} {g}")
            prev = e


if __name__ == "__main__":
    main()
