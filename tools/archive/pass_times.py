"""Mean k_round_pass duration per round position (3 rounds per epoch) from a
rocprofv3 kernel trace of tools/exp_pass.py, skipping the first epoch.

    python tools/pass_times.py <run_kernel_trace.csv> <label>
"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_round_pass" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in rows]
per = [d[i::3][1:] for i in range(3)]
print(sys.argv[2], " ".join(f"r{i}={sum(p) / max(1, len(p)):.1f}us" for i, p in enumerate(per)))
