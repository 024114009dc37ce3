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
