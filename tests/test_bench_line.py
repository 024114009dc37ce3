"""bench.py's stdout record: one compact JSON line that
the driver parses -- the headline keys, the dominant kernel's roofline and the
CPU baseline -- with kernel tables and leg detail in the side file.  Built
from round 4's full 29.7-KB record (which the driver could not parse) and from
a synthetic N>1 record; no GPU."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

FULL = os.path.join(ROOT, "profiles", "r04_final3", "bench.json")
REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _check(line, out):
    assert "\n" not in line and len(line) < bench.LINE_LIMIT, len(line)
    rec = json.loads(line)
    for k in REQUIRED:
        assert k in rec, k
    assert rec["value"] == pytest.approx(out["value"], rel=1e-3)
    assert rec["ms_per_step"] == pytest.approx(out["ms_per_step"], rel=1e-3)
    rf = rec["roofline"]
    for k in ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic", "bytes_per_launch",
              "avg_launch_ms", "launches_per_epoch"):
        assert k in rf, k
    assert rf["kernel"] == out["roofline"]["kernel"]
    assert rf["frac"] == pytest.approx(out["roofline"]["frac"], rel=1e-3)
    for k in ("value", "unit", "cores", "kind"):
        assert k in rec["cpu_baseline"], k
    return rec


@pytest.mark.skipif(not os.path.exists(FULL), reason="round-4 record not in the tree")
def test_round4_record_compacts_under_the_limit(tmp_path):
    out = json.load(open(FULL))
    assert len(json.dumps(out)) > 20_000  # (the line the driver could not parse)
    path = bench.write_detail(out, str(tmp_path / "detail.json"))
    rec = _check(bench.headline_record(out, path), out)
    assert json.load(open(tmp_path / "detail.json")) == out
    legs = rec["legs"]
    assert legs["config_b"]["ms_per_epoch"] == pytest.approx(out["config_b"]["ms_per_epoch"], rel=1e-3)
    assert legs["config_c"]["roofline"]["kernel"] == out["config_c"]["roofline"]["kernel"]
    assert legs["tpcc"]["WAIT_DIE"]["ms_per_epoch"] == pytest.approx(out["tpcc"]["WAIT_DIE"]["ms_per_epoch"],
                                                                     rel=1e-3)
    assert "window_10000_CALVIN" in legs["tpcc"]
    assert legs["cpu_config_a"]["cores"] == 4


def test_synthetic_multi_gpu_record():
    kern = [{"kernel": f"k_{i}", "avg_us": 1.0 * i, "share": 0.01, "bytes": "x" * 300} for i in range(60)]
    out = {"metric": bench.METRIC, "value": 1.5e9, "unit": "committed txns/s", "n_gpus": 8, "steps": 20,
           "warmup": 5, "ms_per_step": 0.7, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "u64", "data": "synthetic", "config": {"workload": "w", "parallelism": "partitioned x8",
                                                            "sequence_order": "p" * 500},
           "roofline": {"kernel": "k_round_async", "bound": "hbm", "achieved": 30.0, "peak": 8000.0,
                        "unit": "GB/s", "frac": 0.004, "traffic": None, "bytes_per_launch": 1.5e6,
                        "avg_launch_ms": 0.05, "launches_per_epoch": 2.0, "share_of_epoch": 0.3,
                        "timed_by": "z" * 400, "algorithmic_bytes": "y" * 400},
           "cpu_baseline": {"value": 2e6, "unit": "committed txns/s", "cores": 16, "kind": "port",
                            "sample": "s" * 2000, "threads_scaling": {"1": 1e6, "4": 3e6, "16": 2e6}},
           "kernels": kern, "mpr_sweep": [{"mpr": m / 10, "committed_per_s": 1e9, "ms_per_step": 0.7,
                                           "abort_rate": 0.9, "steps": 10, "rounds_mean": 30.0}
                                          for m in range(6)],
           "strong_scaling": {"txns_per_epoch": 1 << 20, "ms_per_epoch": 0.5, "committed_per_s": 1e8},
           "tpcc_partitioned": {"warehouses": 256, "WAIT_DIE": {"txns_per_epoch": 65536, "ms_per_epoch": 0.3,
                                                                "committed_per_s": 1e6}}}
    rec = _check(bench.headline_record(out, "gpurun_out/bench_detail.json"), out)
    assert len(rec["legs"]["mpr_sweep"]) == 6 and "kernels" not in rec
    assert rec["legs"]["tpcc_partitioned"]["WAIT_DIE"]["ms_per_epoch"] == 0.3
