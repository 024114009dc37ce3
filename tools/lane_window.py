"""Timeline of a short pipelined run from a rocprofv3 kernel trace: the last
window of kernels (gaps over --gap us split windows) -- per hardware queue
(decision lane) its first start and last end relative to the window's start,
its busy time, and the window's span.  Shows whether a 20-epoch run loses
its time at the start (lanes starting late), at the end (lanes idle while
the last epochs finish) or in between.
    python tools/lane_window.py run_kernel_trace.csv [--gap 200]"""
import csv
import sys


def main():
    path = sys.argv[1]
    gap = float(sys.argv[sys.argv.index("--gap") + 1]) * 1e3 if "--gap" in sys.argv else 200e3
    rows = [r for r in csv.DictReader(open(path)) if "rocclr" not in r["Kernel_Name"]]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                 r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]) for r in rows)
    wins, cur, end = [], [ks[0]], ks[0][1]
    for k in ks[1:]:
        if k[0] - end > gap:
            wins.append(cur)
            cur = []
        cur.append(k)
        end = max(end, k[1])
    wins.append(cur)
    for w in wins[-2:]:
        t0 = w[0][0]
        t1 = max(e for _, e, _, _ in w)
        print(f"window: {len(w)} kernels, span {(t1 - t0) / 1e3:.1f} us")
        for q in sorted({q for _, _, q, _ in w}):
            mine = [k for k in w if k[2] == q]
            busy = 0
            last = 0
            for s, e, _, _ in mine:  # union of intervals
                s = max(s, last)
                if e > s:
                    busy += e - s
                last = max(last, e)
            n_clear = sum(1 for k in mine if k[3] == "k_epoch_clear")
            print(f"  queue {q}: {len(mine)} kernels, {n_clear} epochs, first {(mine[0][0] - t0) / 1e3:.1f} us, "
                  f"last end {(max(e for _, e, _, _ in mine) - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
