"""Deneva-compatible statistics lines.

`summary_line` prints the counters this path owns in the format of
Stats_thd::print (statistics/stats.cpp:425-500) behind the "[summary] " /
"[prog] " prefix of Stats::print (stats.cpp:1541-1560), so Deneva's
scripts/helper.py (get_summary / process_results, helper.py:755-815, 934-944)
parses engine runs like rundb output.  Times are seconds, as the reference
prints them (x / BILLION).  Counters of subsystems outside this path
(network, queues, latency breakdowns) are not printed.
"""


def summary_fields(total_runtime_s, stats, multi_part_txn_cnt=0, parts_touched=None, epoch_seconds=None,
                   part_counts=True):
    """stats: dv_stats of the epochs run in total_runtime_s (one partition's
    view; committed/aborted are global per epoch, as every rank decides every
    txn).  multi_part_txn_cnt / parts_touched: over the COMMITTED txns, as
    TxnManager::commit_stats counts them (txn.cpp:581-587, 600-602); by default
    every committed txn touched one partition.  txn_run_time sums the
    committed txns' latencies (txn.cpp:580): an epoch's txns start together
    and commit when it is decided, so each one's latency is its epoch's time --
    epoch_seconds[e] when given, else the epoch's share of the run (a lower
    bound when epochs overlap on decision lanes).  part_counts=False leaves
    the four partition counters out (a partitioned run that did not count
    them: the one-partition default would understate them)."""
    txn_cnt = sum(int(s.committed) for s in stats)       # INC_STATS(txn_cnt) on commit (txn.cpp:578)
    aborts = sum(int(s.aborted) for s in stats)           # total_txn_abort_cnt (stats.cpp:447)
    started = sum(int(s.n_txn) for s in stats)
    writes = sum(int(s.write_cnt) for s in stats)
    run = float(total_runtime_s)
    if epoch_seconds is None:
        epoch_seconds = [run / len(stats)] * len(stats) if stats else []
    run_time = sum(int(s.committed) * float(e) for s, e in zip(stats, epoch_seconds))
    tput = txn_cnt / run if run > 0 else 0.0             # stats.cpp:436-437
    parts = txn_cnt if parts_touched is None else int(parts_touched)
    single = txn_cnt - int(multi_part_txn_cnt)
    out = [
        ("total_runtime", run),
        ("tput", tput),
        ("txn_cnt", txn_cnt),
        ("remote_txn_cnt", 0),
        ("local_txn_cnt", txn_cnt),
        ("local_txn_start_cnt", started),
        ("total_txn_commit_cnt", txn_cnt),
        ("local_txn_commit_cnt", txn_cnt),
        ("remote_txn_commit_cnt", 0),
        ("total_txn_abort_cnt", aborts),
        ("unique_txn_abort_cnt", aborts),
        ("local_txn_abort_cnt", aborts),
        ("remote_txn_abort_cnt", 0),
        ("txn_run_time", run_time),
        ("txn_run_avg_time", run_time / txn_cnt if txn_cnt else 0.0),
        ("multi_part_txn_cnt", int(multi_part_txn_cnt)),
        ("single_part_txn_cnt", single),
        ("txn_write_cnt", writes),
        ("record_write_cnt", writes),
        ("parts_touched", parts),
        ("avg_parts_touched", parts / txn_cnt if txn_cnt else 0.0),
    ]
    if not part_counts:
        drop = {"multi_part_txn_cnt", "single_part_txn_cnt", "parts_touched", "avg_parts_touched"}
        out = [kv for kv in out if kv[0] not in drop]
    return out


def summary_line(total_runtime_s, stats, prog=False, **kw):
    body = ",".join(f"{k}={v:f}" if isinstance(v, float) else f"{k}={v:d}"
                    for k, v in summary_fields(total_runtime_s, stats, **kw))
    return ("[prog] " if prog else "[summary] ") + body
