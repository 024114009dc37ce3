"""Deneva-compatible [summary] line (stats.cpp:425-500, 1541-1560), parsed the
way scripts/helper.py does (get_summary strips the 10-character prefix,
process_results splits on ',' and '=' and keeps float values,
helper.py:755-815, 934-944)."""
import re
import types

from dvcc.stats import summary_line


def _process_results(summary, results):  # helper.py:934-944, restated
    for r in results:
        try:
            (name, val) = re.split("=", r)
            val = float(val)
        except ValueError:
            continue
        summary.setdefault(name, []).append(val)


def test_summary_line_parses_like_helper_py():
    st = [types.SimpleNamespace(committed=100, aborted=28, n_txn=128, write_cnt=500),
          types.SimpleNamespace(committed=50, aborted=78, n_txn=128, write_cnt=250)]
    line = summary_line(2.0, st)
    assert line.startswith("[summary] ")
    s = {}
    _process_results(s, re.split(",", line.rstrip("\n")[10:]))
    assert s["txn_cnt"] == [150.0] and s["total_txn_abort_cnt"] == [106.0]
    assert s["tput"] == [75.0] and s["total_runtime"] == [2.0]
    assert s["local_txn_start_cnt"] == [256.0] and s["record_write_cnt"] == [750.0]
    assert summary_line(1.0, st, prog=True).startswith("[prog] ")
    # single / multi-partition counts and parts touched are commit-time
    # counters (txn.cpp:581-587, 600-602), not per started txn
    assert s["single_part_txn_cnt"] == [150.0] and s["multi_part_txn_cnt"] == [0.0]
    assert s["parts_touched"] == [150.0] and s["avg_parts_touched"] == [1.0]
    s2 = {}
    _process_results(s2, re.split(",", summary_line(2.0, st, multi_part_txn_cnt=30, parts_touched=180)[10:]))
    assert s2["single_part_txn_cnt"] == [120.0] and s2["avg_parts_touched"] == [1.2]
    # txn_run_time: each committed txn's latency is its epoch's time (txn.cpp:580)
    assert s["txn_run_time"] == [150.0] and s["txn_run_avg_time"] == [1.0]
    s3 = {}
    _process_results(s3, re.split(",", summary_line(2.0, st, epoch_seconds=[0.5, 2.0])[10:]))
    assert s3["txn_run_time"] == [150.0] and s3["txn_run_avg_time"] == [1.0]


def test_summary_line_without_partition_counts():
    """A partitioned run that did not count its multi-partition commits leaves
    the four partition counters out instead of printing the one-partition
    default (multi_part_txn_cnt=0, avg_parts_touched=1)."""
    st = [types.SimpleNamespace(committed=100, aborted=28, n_txn=128, write_cnt=500)]
    s = {}
    _process_results(s, re.split(",", summary_line(1.0, st, part_counts=False)[10:]))
    assert s["txn_cnt"] == [100.0]
    for k in ("multi_part_txn_cnt", "single_part_txn_cnt", "parts_touched", "avg_parts_touched"):
        assert k not in s
