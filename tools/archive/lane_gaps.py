"""Where decision lanes sit idle: in the busiest multi-queue window of a
rocprofv3 kernel trace, per queue its busy fraction and the idle time before
each kernel, summed by that kernel's name (a gap before k_lane_gate / the
execution is a wait for the previous epoch's execution on another lane; a gap
before k_epoch_clear is the lane waiting for the host to queue its next epoch).
Also each kernel's mean duration in that window (on its lane's CU share).
    python tools/lane_gaps.py run_kernel_trace.csv [--gap 200]"""
import csv
import sys


def short(name):
    return name.split("(")[0].split("<")[0].split("::")[-1]


def main():
    path = sys.argv[1]
    gap = float(sys.argv[sys.argv.index("--gap") + 1]) * 1e3 if "--gap" in sys.argv else 200e3
    rows = [r for r in csv.DictReader(open(path)) if "rocclr" not in r["Kernel_Name"]]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], short(r["Kernel_Name"]))
                for r in rows)
    wins, cur, end = [], [ks[0]], ks[0][1]
    for k in ks[1:]:
        if k[0] - end > gap:
            wins.append(cur)
            cur = []
        cur.append(k)
        end = max(end, k[1])
    wins.append(cur)
    multi = [w for w in wins if len({q for _, _, q, _ in w}) >= 2]
    if not multi:
        print("no multi-queue window")
        return
    w = max(multi, key=len)
    span = w[-1][1] - w[0][0]
    epochs = sum(1 for k in w if k[3] == "k_epoch_clear")
    print(f"window: {len(w)} kernels, {epochs} epochs, span {span / 1e3:.1f} us, "
          f"{span / 1e3 / max(1, epochs):.1f} us per epoch")
    by_q = {}
    for k in w:
        by_q.setdefault(k[2], []).append(k)
    tot_gap = {}
    for q, lst in sorted(by_q.items()):
        lst.sort()
        busy = sum(e - s for s, e, _, _ in lst)
        gaps = {}
        for a, b in zip(lst, lst[1:]):
            g = b[0] - a[1]
            if g > 0:
                gaps[b[3]] = gaps.get(b[3], 0) + g
                tot_gap[b[3]] = tot_gap.get(b[3], 0) + g
        top = sorted(gaps.items(), key=lambda kv: -kv[1])[:5]
        print(f"queue {q}: {len(lst)} kernels, busy {busy / 1e3:.1f} us ({busy / span:.2f} of the span); idle before: "
              + ", ".join(f"{n} {t / 1e3:.1f}" for n, t in top))
    print("idle before, all queues: " + ", ".join(f"{n} {t / 1e3:.1f}" for n, t in
                                                 sorted(tot_gap.items(), key=lambda kv: -kv[1])[:8]))
    # each kernel's duration beside the other lanes (its CU share), per epoch
    dur = {}
    for s_, e_, _, n in w:
        d = dur.setdefault(n, [0, 0])
        d[0] += 1
        d[1] += e_ - s_
    print("kernel durations in the window (launches per epoch, mean us, us per epoch):")
    for n, (c, t) in sorted(dur.items(), key=lambda kv: -kv[1][1]):
        print(f"  {n:24s} x {c / max(1, epochs):5.2f} {t / c / 1e3:8.1f} {t / 1e3 / max(1, epochs):8.1f}")


if __name__ == "__main__":
    main()
