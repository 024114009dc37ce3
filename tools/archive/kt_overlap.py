"""Overlap of kernels across queues in a rocprofv3 kernel trace (decision
lanes): per queue its kernel time, the union of all kernels' intervals, and
the sum of durations over that union (> 1: kernels of two lanes ran at once).
Windows are the stretches between host gaps longer than --gap us.
    python tools/kt_overlap.py run_kernel_trace.csv [--gap 200]"""
import csv
import sys


def main():
    path = sys.argv[1]
    gap = float(sys.argv[sys.argv.index("--gap") + 1]) * 1e3 if "--gap" in sys.argv else 200e3
    rows = [r for r in csv.DictReader(open(path)) if "rocclr" not in r["Kernel_Name"]]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows)
    wins, cur = [], [ks[0]]
    end = ks[0][1]
    for k in ks[1:]:
        if k[0] - end > gap:
            wins.append(cur)
            cur = []
        cur.append(k)
        end = max(end, k[1])
    wins.append(cur)
    print(f"{len(ks)} kernels, {len(wins)} windows (host gaps > {gap / 1e3:.0f} us)")
    for i, w in enumerate(wins):
        if len(w) < 40:
            continue
        busy = sum(e - s for s, e, _, _ in w)
        union, ce = 0, None
        cs = None
        for s, e, _, _ in w:
            if ce is None or s > ce:
                if ce is not None:
                    union += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        union += ce - cs
        span = w[-1][1] - w[0][0]
        per_q = {}
        for s, e, q, _ in w:
            per_q[q] = per_q.get(q, 0) + e - s
        clears = sum(1 for k in w if "k_epoch_clear" in k[3])
        print(f"window {i}: {len(w)} kernels, {clears} epochs, span {span / 1e3:.1f} us, union {union / 1e3:.1f} us, "
              f"kernel time {busy / 1e3:.1f} us, concurrency {busy / union:.2f}, "
              f"per queue {', '.join(f'q{q} {t / 1e3:.1f}' for q, t in sorted(per_q.items()))}"
              + (f", {span / 1e3 / clears:.1f} us per epoch" if clears else ""))


if __name__ == "__main__":
    main()
