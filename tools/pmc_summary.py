"""Per-launch HBM traffic of kernels from rocprofv3 --pmc CSVs.

    python tools/pmc_summary.py <fetch.csv> <write.csv> <out.json> <kernel,kernel,...> [key=value ...]

FETCH_SIZE and WRITE_SIZE come from separate passes (they cannot share one on
gfx950) and are reported in KiB.  Per MI355X_MICROARCH.md "HBM": on gfx950
FETCH_SIZE counts half the bytes of a wide coalesced streaming read, so the
corrected figure doubles it; reads of other widths (byte gathers) are
uncalibrated, so the raw figure is kept beside it.  WRITE_SIZE is taken as
is.  The launches of each kernel are averaged.
"""
import csv
import json
import sys


def per_launch(path, kernel, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1] == kernel and r["Counter_Name"] == counter]
    return (sum(vals) / len(vals) * 1024.0 if vals else 0.0), len(vals)


def main():
    fetch, write, out, kernels = sys.argv[1:5]
    res = {"correction": "hbm = 2 x FETCH_SIZE (gfx950 half-count of wide streaming reads) + WRITE_SIZE; "
                         "byte gathers uncalibrated (fetch_raw kept)", "kernels": {}}
    for kernel in kernels.split(","):
        f, nf = per_launch(fetch, kernel, "FETCH_SIZE")
        w, nw = per_launch(write, kernel, "WRITE_SIZE")
        res["kernels"][kernel] = {"fetch_raw_bytes_per_launch": f, "write_bytes_per_launch": w,
                                  "hbm_bytes_per_launch": 2.0 * f + w, "launches": [nf, nw]}
    for kv in sys.argv[5:]:
        k, v = kv.split("=", 1)
        res[k] = int(v) if v.isdigit() else v
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
