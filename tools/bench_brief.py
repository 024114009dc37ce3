"""One-screen summary of a bench.py JSON line: headline, roofline, kernel table."""
import json
import os
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
if os.path.exists(str(d.get("detail"))):  # (the compact line: the full record is in the detail file)
    line = d
    d = json.load(open(d["detail"]))
    print(f"stdout line {len(json.dumps(line))} B; detail {line['detail']}")
if "value" not in d:  # (--tpcc-only: the TPC-C leg alone)
    for size, leg in [("", d.get("tpcc", {}))] + [(k, v) for k, v in d.get("tpcc", {}).items() if k.startswith("window")]:
        for cc, v in leg.items():
            if isinstance(v, dict) and "ms_per_epoch" in v:
                print(f"tpcc {size or 'main'} {cc}: {v['ms_per_epoch']:.4f} ms/epoch, {v['committed_per_s']:.4g} committed/s")
    sys.exit(0)
print(f"value {d['value']:.4g} {d['unit']}  ms/step {d['ms_per_step']:.4f}  abort {d.get('abort_rate', 0):.4f}")
r = d["roofline"]
print(f"roofline {r['kernel']}: {r['achieved']:.1f} GB/s frac {r['frac']:.4f} share {r.get('share_of_epoch', 0):.3f}")
if "k_probe" in r:
    p = r["k_probe"]
    print(f"  k_probe: {p['achieved']:.1f} GB/s frac {p['frac']:.4f} avg {p['avg_launch_ms'] * 1e3:.1f} us")
print(f"kernel us/epoch {d.get('kernel_us_per_epoch', 0):.1f}; stages {d.get('stage_ms_mean')}")
for k in d.get("kernels", []):
    print(f"  {k['kernel']:<22} x{k['launches_per_epoch']:5.2f} {k['avg_us']:8.1f} us  {k['us_per_epoch']:8.1f} us/ep"
          f"  {k['share']:.3f}  frac {k.get('frac', float('nan')):.4f}")
for key in ("cpu_baseline", "closed_loop_retry", "sort"):
    if key in d:
        v = d[key]
        print(key, {a: b for a, b in v.items() if not isinstance(b, (dict, list)) and a != "sample"})
