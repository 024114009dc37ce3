"""Calibrated HBM traffic of k_probe (MI355X_MICROARCH.md "HBM": FETCH_SIZE
is exact only after calibration on the kernel's own access mix).

    python tools/pmc_probe_cal.py <pmc summary json> <fetch.csv of the no-gather build> <n_acc>

The no-gather build (DVCC_CAL_NO_GATHER) reads exactly the probe's streams --
key 8 + type 1 + txn id 4 B per access -- so its FETCH_SIZE per launch gives
the counter's factor for these streaming loads; what the real build fetches
beyond that is the key-tag gather, taken at the counter's face value (one
64-B request per line).  Writes: WRITE_SIZE as is.  Adds
"hbm_bytes_per_launch_calibrated" to k_probe in the summary.
"""
import csv
import json
import sys


def main():
    path, cal_fetch, n_acc = sys.argv[1], sys.argv[2], int(sys.argv[3])
    res = json.load(open(path))
    vals = [float(r["Counter_Value"]) * 1024.0 for r in csv.DictReader(open(cal_fetch))
            if r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1] == "k_probe"
            and r["Counter_Name"] == "FETCH_SIZE"]
    raw_stream = sum(vals) / len(vals)
    stream = 13.0 * n_acc
    k = res["kernels"]["k_probe"]
    gather = max(0.0, k["fetch_raw_bytes_per_launch"] - raw_stream)
    k["calibration"] = {"stream_bytes": stream, "stream_fetch_raw": raw_stream, "factor": stream / raw_stream,
                        "gather_fetch_raw": gather}
    k["hbm_bytes_per_launch_calibrated"] = stream + gather + k["write_bytes_per_launch"]
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(k))


if __name__ == "__main__":
    main()
