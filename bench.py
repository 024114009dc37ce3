"""Benchmark: committed txns/sec of the batched CC engine on YCSB (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cc NO_WAIT|WAIT_DIE|OCC|CALVIN]
                    [--config D|C|B] [--mpr 0.1] [--mpr-sweep 0,0.1,0.2,0.3,0.4,0.5]

A step is one epoch through the hot path (probe -> sort -> decide -> execute)
with its accesses already resident in HBM.  Default workload: config D of
SURVEY.md 8(d), the headline "YCSB zipf 0.9 at 1/2/4/8 GPUs" -- 16,777,216
rows per partition, an epoch of 1,048,576 txns IN TOTAL (1,048,576 / N per
GPU), 10 requests/txn, zipf 0.9, 50 % of the accesses writes (TXN_WRITE_PERC
1.0, TUP_WRITE_PERC 0.5), NO_WAIT.

--gpus N > 1 starts its own N rank processes (torch.distributed.run) when no
launcher did; one process per GPU, rank r owns partition r (16,777,216 rows),
all collectives from the engine over RCCL (dv_comm_init).  The headline runs
config D's epochs -- 1,048,576 txns each IN TOTAL, every rank's client batch
1,048,576 / N of them, multi-partition txns per the MPR gate (2 partitions) --
as epoch groups (dv_epoch_group_run): a step is one group of N consecutive
epochs, rank e receives every batch of epoch e (all-to-allv), decides it with
the single-GPU path and forwards the committed accesses to their owners, who
execute the N epochs in order.  Per-GPU work is one epoch decided per step,
so the line says "scaling": "weak".  Beside it: one epoch per step over
dv_epoch_run_part (strong scaling; replicated sequencing), the
1,048,576-txn-per-GPU epochs of the list protocol, and the MPR sweep.
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))
# HIP graphs in packet-capture mode (the epoch graphs' replay: ~4 us of host
# time instead of 15-50), before anything initialises the HIP runtime
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import dvcc  # noqa: E402

METRIC = "committed txns/sec (node) YCSB zipf0.9 at 1/2/4/8 GPUs; abort-set bit-exact"
HBM_PEAK_GBPS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_ACCESS = 67        # algorithmic bytes per access
SCAN_BYTES = 9               # SURVEY.md 8d per access: scan read 8 B + conflict flag write 1 B
TIMING = {"full": True, "kernel": "kernel", "off": False}
PROBE_ACC, PROBE_TXN = 17, 9  # k_probe algorithmic bytes per access / per txn (roofline)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_config_d.json")  # tools/pmc_summary.py

CONFIGS = {
    # name: rows per partition, txns per epoch (in total, over all GPUs), zipf theta, description
    "D": (16_777_216, 1_048_576, 0.9, "YCSB config D: 16,777,216 rows/partition, 1,048,576-txn epoch in total"),
    "C": (100_000_000, 1_048_576, 0.9, "YCSB config C: 100,000,000 rows, 1,048,576-txn epoch"),
    "B": (16_777_216, 65_536, 0.6, "YCSB config B: 16,777,216 rows, 65,536-txn epoch"),
}
TPCC_EPOCHS = 3  # distinct TPC-C epochs (coprime to the four lanes)
CPU_SHARE = 16  # host threads the GPU box gives one GPU's job (nproc shows the whole machine)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cc", default="NO_WAIT")
    ap.add_argument("--config", default="D")
    ap.add_argument("--mpr", type=float, default=0.1, help="N>1: multi-partition txn ratio of the headline")
    ap.add_argument("--mpr-sweep", default="0,0.1,0.2,0.3,0.4,0.5",
                    help="N>1: config D's MPR values, each a short extra run ('' = none)")
    ap.add_argument("--no-weak", action="store_true", help="N>1: skip the 1,048,576-txn-per-GPU run")
    ap.add_argument("--protocol", choices=["group", "part"], default="group",
                    help="N>1 headline: epoch groups (dv_epoch_group_run) or one epoch per step "
                         "(dv_epoch_run_part, --part-mode)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one dv_epoch_run_device (N=1) / dv_epoch_group_run (epoch groups) call per step "
                         "instead of the batch call")
    ap.add_argument("--part1", action="store_true",
                    help="N=1 through the partitioned drivers on a one-rank RCCL communicator (their overhead)")
    ap.add_argument("--part-mode", type=int, default=0,
                    help="N>1: dv_comm_set_mode -- 0 replicated when the epoch fits, else the list protocol; "
                         "1 list protocol; 2 replicated; + 4: 8-byte epoch-group batches (DV_COMM_WIDE_BATCHES)")
    ap.add_argument("--order", choices=["position", "origin"], default="position",
                    help="N>1 epoch groups, NO_WAIT / WAIT_DIE / OCC: the origins' batches of an epoch sequenced txn "
                         "by txn (DV_COMM_POSITION_ORDER, origin q's txn j at j * N + q -- clients of all nodes "
                         "arriving together) or batch by batch (Calvin's lock order, which CALVIN always keeps)")
    ap.add_argument("--prefix", type=int, default=0,
                    help="prefix-kill decisions (dv_set_prefix): 0 automatic, -1 off, K txns")
    ap.add_argument("--epochs", type=int, default=5,
                    help="distinct pre-generated epochs (coprime to --lanes, so every epoch is decided on every "
                         "lane in turn)")
    ap.add_argument("--ipc-rehearsal", action="store_true",
                    help="N>1 ranks sharing fewer GPUs (a rehearsal of the N>1 path on a one-GPU box): torch "
                         "collectives over gloo, the engine's over dv_comm_init_ipc (a test transport); the "
                         "numbers are no scaling result")
    ap.add_argument("--lanes", type=int, default=4,
                    help="one GPU: decision lanes (dv_epoch_run_device_lanes) -- epochs decided on this many "
                         "contexts in turn, executions in epoch order; 1 = dv_epoch_run_device_batch")
    ap.add_argument("--group-lanes", type=int, default=4,
                    help="N>1 epoch groups: ordered decision lanes per rank (dv_lanes_order, one RCCL "
                         "communicator per lane, each lane stream on a hardware queue of its own -- checked by "
                         "dv_lanes_order, DESIGN.md 6; 1 = one context per rank)")
    ap.add_argument("--part-lanes", type=int, default=1,
                    help="N>1 TPC-C leg: ordered decision lanes per rank for dv_tpcc_epoch_run_part "
                         "(dv_lanes_order; opt-in)")
    ap.add_argument("--no-txn-begin", action="store_true",
                    help="A/B: device epochs without their txn boundaries (dv_epoch_dev::txn_begin), so prefix-kill "
                         "epochs derive ranges from acc_txn and probe every access up front")
    ap.add_argument("--no-recs32", action="store_true",
                    help="A/B: device epochs without their 4-byte records (dv_epoch_dev::recs32): keys and types "
                         "read instead")
    ap.add_argument("--lsd-sort", action="store_true",
                    help="A/B: sort with the plain LSD passes (DV_FLAG_LSD_SORT), no bucket sort")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="the full record (kernel tables, every leg) as JSON; stdout carries one compact line "
                         "('' = not written)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-tpcc", action="store_true", help="skip the TPC-C (config E) leg")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the config B (CALVIN) / C (OCC, 100M rows) legs and the CPU config A line")
    ap.add_argument("--tpcc-only", action="store_true", help="run and print only the TPC-C leg (profiling)")
    ap.add_argument("--tpcc-no-async", action="store_true",
                    help="A/B: TPC-C decisions without the asynchronous round launch (DV_FLAG_NO_ASYNC: pipelined "
                         "rounds, then the one-workgroup LDS tail)")
    ap.add_argument("--tpcc-wh", type=int, default=32, help="warehouses per GPU (config E: 256 / 8)")
    ap.add_argument("--tpcc-part-wh", type=int, default=256,
                    help="N>1 (or --part1): warehouses of the partitioned TPC-C leg, split over the ranks")
    ap.add_argument("--no-tpcc-part", action="store_true", help="N>1: skip the partitioned TPC-C leg")
    ap.add_argument("--tpcc-txns", default="65536,10000",
                    help="txns per TPC-C epoch, comma-separated (the first is the leg's line; 10000 is the "
                         "reference's concurrency window, 8 nodes x 1250 in-flight txns)")
    ap.add_argument("--timing", choices=["full", "kernel", "off"], default="off",
                    help="engine timing inside the timed region: per-stage events, only the "
                         "scatter/pass dispatch timestamps, or none (default: the timed region "
                         "runs as the product does; the roofline and stage legs follow it)")
    return ap.parse_args()


def gen_epochs(gen, n_txn, rank, count):
    with ThreadPoolExecutor(max_workers=min(count, 8)) as ex:  # dv_ycsb_gen releases the GIL
        futs = [ex.submit(gen.gen, n_txn, dvcc.epoch_seed(rank, e), rank) for e in range(count)]
        return [f.result() for f in futs]


def cpu_baseline(epochs, rows, cc_name, seconds):
    """The oracle (single-thread E-schedule restatement of the reference CC,
    not the reference binary) on the same epochs, cycled for ~`seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    cc = {"NO_WAIT": O.NO_WAIT, "WAIT_DIE": O.WAIT_DIE, "OCC": O.OCC, "CALVIN": O.CALVIN}[cc_name]
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    committed = txns = 0
    t0 = time.perf_counter()
    i = 0
    while True:
        e = epochs[i % len(epochs)]
        _, _, st = O.epoch_run(cc, tab.ix, f0, e.n_txn, e.txn_begin, e.keys, e.types)
        committed += st.committed
        txns += e.n_txn
        i += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": committed / el, "unit": "committed txns/s", "cores": 1, "kind": "port",
            "sample": f"oracle E-schedule ({cc_name}) over {i} epoch(s) of {epochs[0].n_txn} txns "
                      f"of the bench workload, {txns} txns in {el:.1f} s on 1 host core; "
                      f"restatement of the reference CC, not the reference binary"}


def cpu_baseline_mt(epochs, rows, seconds):
    """a Deneva-style multi-threaded NO_WAIT engine
    (oracle/mt_engine.c: per-row lock words, index probe, run_ycsb_1, no
    retry) on the same epochs.  The headline figure uses the box's CPU share
    for one GPU, CPU_SHARE threads: the GPU box gives one GPU's job 16 host
    cores and asks that worker pools stay within them, while nproc reports
    the whole machine (256).  Beside it the same engine at 1 and 4 threads
    (its scaling), and the CPU_SHARE rate scaled to every core nproc counts,
    labelled as an extrapolation (linear in threads: an upper bound, not a
    measurement).  Its aborts depend on the interleaving (THREAD_CNT txns in
    flight), not the E-schedule's 1M; a throughput reference only."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    tab = O.YcsbTable(rows)

    def run(threads, secs):
        f0 = tab.f0.copy()
        lock = O.mt_lock(rows)
        committed = txns = 0
        t0 = time.perf_counter()
        i = 0
        while True:
            e = epochs[i % len(epochs)]
            c, _ = O.mt_epoch_run(tab.ix, f0, lock, e.n_txn, e.txn_begin, e.keys, e.types, threads)
            committed += c
            txns += e.n_txn
            i += 1
            el = time.perf_counter() - t0
            if el >= secs:
                return committed / el, txns, i, el, committed

    threads = max(1, min(CPU_SHARE, avail))
    v, txns, i, el, committed = run(threads, seconds)
    scaling = {}
    for t in (1, 4):
        if t < threads:
            scaling[str(t)] = run(t, min(3.0, seconds))[0]
    scaling[str(threads)] = v
    nproc = os.cpu_count() or threads
    return {"value": v, "unit": "committed txns/s", "cores": threads, "kind": "port",
            "nproc": nproc, "affinity": avail, "threads_scaling": scaling,
            "all_cores_extrapolated": {"value": v * nproc / threads, "cores": nproc,
                                       "note": f"{threads}-thread rate x {nproc}/{threads}, linear: an upper bound, "
                                               "not measured (the box asks one GPU's job to keep its worker "
                                               f"pools within its {CPU_SHARE}-core share)"},
            "sample": f"Deneva-style multi-threaded NO_WAIT engine (per-row lock words, {threads} "
                      f"threads = the box's CPU share for one GPU; nproc {nproc}, affinity {avail}) "
                      f"over {i} epoch(s) of {epochs[0].n_txn} txns of the bench workload, "
                      f"{txns} txns in {el:.1f} s, abort rate {1 - committed / max(1, txns):.3f}; "
                      "restatement of the reference CC, not the reference binary"}


def tpcc_bytes_per_txn(e):
    """SURVEY.md 8(d) algorithmic bytes of one TPC-C epoch: 67 B per access,
    plus execution and inserts -- Payment 160 B (3 row updates + HISTORY),
    NewOrder 148 B per order line (stock update + ORDER_LINE; ORDER/NEW_ORDER
    and the district counted in the 592 + 888 B of a 10-line order)."""
    n = np.diff(e.txn_begin.astype(np.int64))
    pay = e.txn_type == 1
    per = np.where(pay, 67 * n + 160, 67 * n + 148 * ((n - 3) // 2))
    return int(per.sum())


def tpcc_leg(a, cc_names=("WAIT_DIE", "CALVIN")):
    """Config E on one GPU: TPC-C Payment + NewOrder (PERC_PAYMENT 0.5, MPR 1.0,
    remote customer 15 %, remote item 1 %), this GPU's share of 256
    warehouses (32), full item / customer counts; a step = one epoch of
    --tpcc-txns txns through last-name lookup -> probe -> sort -> decide ->
    execute, epochs resident in HBM.  The first size is the leg's line; each
    further size (the reference's 10,000-txn window) is reported under
    "window_<n>".  Beside the first size the oracle (single thread) on one of
    the same epochs."""
    from dvcc import tpcc as T
    p = T.tpcc_params(a.tpcc_wh)
    sizes = [int(x) for x in str(a.tpcc_txns).split(",") if x]
    out = {}
    for si, n_txn in enumerate(sizes):
        eps = [T.gen(p, n_txn, dvcc.epoch_seed(0, e)) for e in range(TPCC_EPOCHS)]
        res = {"workload": f"TPC-C config E share: {a.tpcc_wh} warehouses/GPU, {n_txn}-txn epochs, "
                           "Payment 50 % / NewOrder 50 %, full schema counts (100,000 items, 3,000 customers/district)",
               "bytes_per_txn_mean": tpcc_bytes_per_txn(eps[0]) / n_txn}
        for cc_name in cc_names:
            eng = T.TpccEngine(cc_name, p, n_txn, seed=1, lsd_sort=a.lsd_sort, asynchronous=not a.tpcc_no_async)
            lanes = [eng.open_lane() for _ in range(max(1, a.lanes) - 1)]  # decision lanes, as config D
            dev = [T.device_epoch(e) for e in eps]
            d_commit = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
            d_oid = torch.zeros(n_txn, dtype=torch.int64, device="cuda")
            # (the window's epochs are short: 200 of them amortise the lanes'
            # fill and drain, ~2 ms in all)
            k = max(a.steps, 50) if si == 0 else max(4 * a.steps, 200)

            def batch(m):  # the pipelined entry point (epoch k+1 queued before k is read back)
                ne = len(dev)
                return eng.run_tpcc_epochs_device([dev[i % ne][0] for i in range(m)],
                                                  [dev[i % ne][1] for i in range(m)], d_commit, d_oid, lanes=lanes)
            if a.warmup:
                batch(max(a.warmup, 2 * (1 + len(lanes))))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sts = batch(k)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            committed = sum(s.committed for s in sts)
            byts = sum(tpcc_bytes_per_txn(eps[i % len(eps)]) for i in range(k))
            res[cc_name] = {"committed_per_s": committed / el, "decided_txns_per_s": k * n_txn / el,
                            "ms_per_epoch": el / k * 1e3, "abort_rate": 1 - committed / (k * n_txn),
                            "epochs": k, "decision_lanes": 1 + len(lanes),
                            "epoch_roofline": {"achieved_GBps": byts / el / 1e9,
                                                            "frac": byts / el / 1e9 / HBM_PEAK_GBPS}}
            eng.close()
        if si == 0 and not a.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import _oracle as O
            po = O.tpcc_params(a.tpcc_wh)
            e = eps[0]
            for cc_name in cc_names:
                db = O.TpccDB(po, 1)
                cc = {"WAIT_DIE": O.WAIT_DIE, "CALVIN": O.CALVIN, "NO_WAIT": O.NO_WAIT, "OCC": O.OCC}[cc_name]
                t0 = time.perf_counter()
                commit, _, st = db.epoch(cc, e.keys, e.types, e.tables, e.args, e.txn_begin)
                el = time.perf_counter() - t0
                res[cc_name]["cpu_baseline"] = {
                    "value": st.committed / el, "unit": "committed txns/s", "cores": 1, "kind": "port",
                    "sample": f"oracle (tpcc.c, E-schedule {cc_name}) on 1 epoch of {n_txn} txns of this "
                              f"workload in {el:.2f} s on 1 host core; restatement, not the reference binary"}
        if si == 0:
            out.update(res)
        else:
            out[f"window_{n_txn}"] = res
    return out


def closed_loop_leg(eng, gen, n_txn, k, d_commit, open_ms=None):
    """Closed loop with retries on the device
    (dv_epoch_run_closed_loop): every epoch holds n_txn txns, the previous
    epoch's aborted ones first, new ones from a pre-generated pool (2 x n_txn
    txns, drawn in order, wrapping) filling the rest -- built on the device
    behind the previous epoch's execution, nothing read back between epochs,
    epoch k+1 queued before epoch k's outcome is read.  Committed txns/s over
    k epochs in one call, the carry-over and epoch assembly included."""
    pool_n = 2 * n_txn
    pool = gen.gen(pool_n, dvcc.epoch_seed(0, 999))
    dpool = dvcc.DeviceEpoch(pool)
    pb = torch.from_numpy(pool.txn_begin.astype(np.int32)).cuda()
    commits = [torch.zeros(n_txn, dtype=torch.uint8, device="cuda") for _ in range(k)]
    sts, bufs, cursor = eng.closed_loop(dpool, pb, n_txn, 2, d_commits=commits[:2])  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sts, bufs, cursor = eng.closed_loop(dpool, pb, n_txn, k, cursor=cursor, bufs=bufs, d_commits=commits,
                                        resume=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    committed = sum(s.committed for s in sts)
    carried = sum(s.n_txn - s.committed for s in sts[:-1])
    out = {"committed_per_s": committed / el, "ms_per_epoch": el / k * 1e3, "epochs": k,
           "carried_per_epoch": carried / max(1, k - 1),
           "entry_point": "dv_epoch_run_closed_loop",
           "note": "aborted txns retried in the next epoch ahead of new ones (one-epoch penalty); "
                   "the next epoch built on the device (no host readback)"}
    if open_ms:
        out["vs_open_loop_ms"] = out["ms_per_epoch"] / open_ms
    return out


def closed_loop_lanes_leg(eng, lanes, gen, n_txn, k, open_ms=None):
    """The same closed loop over the decision lanes
    (dv_epoch_run_closed_loop_lanes): epoch k decided on lane k % L, each
    lane's aborted txns retried in its next epoch (L epochs later), the pool
    drawn in epoch order; k a multiple of 2 L."""
    nl = 1 + len(lanes)
    k = max(2 * nl, (k + 2 * nl - 1) // (2 * nl) * 2 * nl)
    pool = gen.gen(2 * n_txn, dvcc.epoch_seed(0, 999))
    dpool = dvcc.DeviceEpoch(pool)
    pb = torch.from_numpy(pool.txn_begin.astype(np.int32)).cuda()
    commits = [torch.zeros(n_txn, dtype=torch.uint8, device="cuda") for _ in range(k)]
    sts, bufs, cursor = eng.closed_loop_lanes(lanes, dpool, pb, n_txn, 2 * nl, d_commits=commits[:2 * nl])  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sts, bufs, cursor = eng.closed_loop_lanes(lanes, dpool, pb, n_txn, k, cursor=cursor, bufs=bufs,
                                              d_commits=commits, resume=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    committed = sum(s.committed for s in sts)
    out = {"committed_per_s": committed / el, "ms_per_epoch": el / k * 1e3, "epochs": k, "decision_lanes": nl,
           "carried_per_epoch": sum(s.n_txn - s.committed for s in sts[:-nl]) / max(1, k - nl),
           "entry_point": "dv_epoch_run_closed_loop_lanes",
           "note": f"aborted txns retried {nl} epochs later (each lane's next epoch) ahead of new ones; "
                   "epochs built on the device, executed in epoch order"}
    if open_ms:
        out["vs_open_loop_ms"] = out["ms_per_epoch"] / open_ms
    return out


def config_leg(a, cfg, cc_name):
    """BASELINE configs B (CALVIN, 65,536-txn epochs, zipf 0.6, 16,777,216
    rows) and C (OCC, 1,048,576-txn epochs, zipf 0.9, 100,000,000 rows) on one
    GPU, through the headline's entry point (decision lanes, pipelined, epochs
    resident in HBM, 3 distinct epochs cycled), with their own kernel table
    and roofline from one context right after the timed region, as the
    headline's.  Not `value`."""
    rows, n_txn, theta, desc = CONFIGS[cfg]
    R = 10
    gen = dvcc.YCSBQueryGenerator(rows, part_cnt=1, req_per_query=R, zipf_theta=theta, txn_write_perc=1.0,
                                  tup_write_perc=0.5, part_per_txn=1, strict_ppt=1, mpr=-1.0)
    t0 = time.perf_counter()
    epochs = gen_epochs(gen, n_txn, 0, 3)
    deps = [dvcc.DeviceEpoch(e, txn_begin=not a.no_txn_begin, recs32=not a.no_recs32) for e in epochs]
    t_gen = time.perf_counter() - t0
    eng = dvcc.CCEngine(cc_name, n_txn, max(e.n_acc for e in epochs), device=0, lsd_sort=a.lsd_sort)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.load_ycsb_partition(rows)
    lanes = [eng.open_lane() for _ in range(max(1, a.lanes) - 1)]
    d_commit = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
    ne = len(deps)

    def batch(first, count):
        run = [deps[(first + i) % ne] for i in range(count)]
        return eng.run_epochs_lanes(lanes, run, d_commit) if lanes else eng.run_epochs_device(run, d_commit)
    k = max(12, min(a.steps, 24))
    k = (k + max(1, len(lanes) + 1) - 1) // (len(lanes) + 1) * (len(lanes) + 1)
    stats, el = timed(None, 0, a.warmup, k, 1, batch)
    # the kernel table: one context, each launch with its own dispatch timestamps
    eng.set_timing(False, profile=True)
    eng.kernel_times(reset=True)
    pstats = eng.run_epochs_device([deps[i % ne] for i in range(6)], d_commit)
    ktimes = eng.kernel_times(reset=True)
    eng.set_timing(False)
    table, kus = kernel_table(ktimes, pstats, rows, R, a, cc_name, 1, tb=not a.no_txn_begin,
                              recs=not a.no_txn_begin and not a.no_recs32)
    committed = sum(s.committed for s in stats)
    out = {"workload": desc, "cc_alg": cc_name, "zipf_theta": theta, "txn_write_perc": 1.0, "tup_write_perc": 0.5,
           "committed_per_s": committed / el, "decided_txns_per_s": k * n_txn / el, "ms_per_epoch": el / k * 1e3,
           "abort_rate": 1 - committed / (k * n_txn), "epochs": k, "distinct_epochs": ne,
           "decision_lanes": 1 + len(lanes), "gen_seconds": t_gen,
           "epoch_roofline": {"bytes_per_txn": BYTES_PER_ACCESS * R + 1,
                              "achieved_GBps": k * n_txn / el * (BYTES_PER_ACCESS * R + 1) / 1e9,
                              "frac": k * n_txn / el * (BYTES_PER_ACCESS * R + 1) / 1e9 / HBM_PEAK_GBPS},
           "roofline": roofline(table, len(pstats), a), "kernels": table, "kernel_us_per_epoch": kus,
           "stage_sizes_mean": {kk: float(np.mean([getattr(st, kk) for st in pstats]))
                                for kk in ("n_txn", "n_acc", "prefix_txn", "prefix_acc", "surv_txn", "surv_acc")}}
    for ln in lanes:
        ln.close()
    eng.close()
    return out


def cpu_config_a(seconds):
    """BASELINE config A's CPU reference setting: NO_WAIT, THREAD_CNT = 4, zipf
    0.6, 16,777,216 rows, the Deneva YCSB mix (TXN_WRITE_PERC 0.5,
    TUP_WRITE_PERC 0.5, experiments.py:65-72), 10 requests -- on the
    Deneva-style multi-threaded engine (oracle/mt_engine.c: per-row NO_WAIT
    lock words, index probe, run_ycsb_1, no retry), 4 worker threads, epochs
    of 65,536 txns, ~`seconds` of work.  A restatement of the reference CC on
    the box's cores, not the reference binary."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    rows, threads, n = 16_777_216, 4, 65_536
    gen = dvcc.YCSBQueryGenerator(rows, part_cnt=1, req_per_query=10, zipf_theta=0.6, txn_write_perc=0.5,
                                  tup_write_perc=0.5, part_per_txn=1, strict_ppt=1, mpr=-1.0)
    epochs = gen_epochs(gen, n, 0, 4)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    lock = O.mt_lock(rows)
    committed = txns = i = 0
    t0 = time.perf_counter()
    while True:
        e = epochs[i % len(epochs)]
        c, _ = O.mt_epoch_run(tab.ix, f0, lock, e.n_txn, e.txn_begin, e.keys, e.types, threads)
        committed += c
        txns += e.n_txn
        i += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": committed / el, "unit": "committed txns/s", "cores": threads, "kind": "port",
            "abort_rate": 1 - committed / max(1, txns),
            "sample": f"config A: NO_WAIT, THREAD_CNT=4, zipf 0.6, 16,777,216 rows, TXN_WRITE_PERC 0.5 / "
                      f"TUP_WRITE_PERC 0.5, 10 requests; Deneva-style multi-threaded engine (oracle/mt_engine.c) "
                      f"over {i} epoch(s) of {n} txns, {txns} txns in {el:.1f} s on 4 threads; restatement of the "
                      "reference CC, not the reference binary"}


def wire_ingress_leg(eng, epoch, rows, d_commit, reps=3):
    """Deneva's wire format in front of the engine (never the `value`): the
    epoch as runcl's client batches (CL_QRY mbufs of at most 4 KB,
    tests/wire_fmt.py builds them as synthetic traffic), decoded by
    dv_wire_decode_batches into a host epoch on one core, run on the GPU --
    its commit bytes must equal the generated epoch's -- and the replies
    (CL_RSP per committed txn) packed by dv_wire_respond."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import wire_fmt as W
    from dvcc.wire import WireIngress
    buf, off = W.ycsb_epoch_buffer_np(epoch, 0, 1)
    w = WireIngress(dvcc._lib.YCSB, epoch.n_txn, epoch.n_acc, node_id=0, node_cnt=1, synth_table_size=rows)
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        closed = w.feed_buffer(buf, off)
        ep = w.take()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    if closed or not ((ep.keys == epoch.keys).all() and (ep.types == epoch.types).all()
                      and (ep.txn_begin == epoch.txn_begin).all()):
        return {"error": "decoded epoch differs from the generated one"}
    d_ref = torch.zeros_like(d_commit)
    eng.run_epoch_device(dvcc.DeviceEpoch(epoch), d_ref)
    st = eng.run_epoch_device(dvcc.DeviceEpoch(ep), d_commit)
    commit = d_commit.cpu().numpy()[:ep.n_txn]
    if not (commit == d_ref.cpu().numpy()[:ep.n_txn]).all():
        return {"error": "commit bytes of the decoded epoch differ"}
    t0 = time.perf_counter()
    replies = w.respond(ep, commit)
    t_rsp = time.perf_counter() - t0
    return {"decoded_txns_per_s": ep.n_txn / best, "wire_MBps": len(buf) / best / 1e6, "batches": len(off) - 1,
            "wire_bytes": int(len(buf)), "decode_ms": best * 1e3, "committed": int(st.committed),
            "reply_batches": len(replies), "respond_txns_per_s": ep.n_txn / t_rsp, "cores": 1,
            "entry_points": "dv_wire_decode_batches, dv_wire_respond (include/dvcc.h)",
            "note": "host-side ingress of one config-D epoch (1,048,576 CL_QRY messages); decode time is the "
                    "best of %d passes on one core; the GPU run checks the decoded epoch's commit bytes "
                    "against the generated epoch's" % reps}


def e2e_host_leg(eng, epochs, k):
    """SURVEY.md 8(d)'s second reading: epochs from host buffers, so the H2D
    copy of the 16-B access records is inside the time (pinned host memory,
    as a caller that batches epochs would hold them).  Serial: dv_epoch_run
    (copy, then decide).  Double-buffered: dv_epoch_stage_host of epoch k+1
    on the copy stream before dv_epoch_run_staged of epoch k, so the copy
    overlaps the decisions -- per epoch max(H2D, compute).  Never `value`."""
    bufs = []
    for e in epochs:
        acc = torch.from_numpy(e.to_access_array().view(np.uint8)).pin_memory()
        tb = torch.from_numpy(np.ascontiguousarray(e.txn_begin, dtype=np.uint32)).pin_memory()
        bufs.append((acc, tb, e.n_acc, e.n_txn))
    commit = torch.zeros(max(b[3] for b in bufs), dtype=torch.uint8).pin_memory()
    eng.run_epoch_host(*bufs[0], commit)  # staging buffers allocated outside the timing
    t0 = time.perf_counter()
    committed = 0
    for i in range(k):
        committed += eng.run_epoch_host(*bufs[i % len(bufs)], commit).committed
    el = time.perf_counter() - t0
    out = {"committed_per_s": committed / el, "ms_per_epoch": el / k * 1e3, "epochs": k,
           "bytes_h2d_per_epoch": int(bufs[0][0].numel()),
           "note": "dv_epoch_run: H2D of the access records, then the same device path"}
    # double-buffered
    eng.stage_host(0, *bufs[0])  # both slots allocated outside the timing
    eng.stage_host(1, *bufs[1 % len(bufs)])
    eng.run_staged(0, commit)
    eng.run_staged(1, commit)
    t0 = time.perf_counter()
    committed = 0
    eng.stage_host(0, *bufs[0])
    for i in range(k):
        if i + 1 < k:
            eng.stage_host((i + 1) % 2, *bufs[(i + 1) % len(bufs)])
        committed += eng.run_staged(i % 2, commit).committed
    el = time.perf_counter() - t0
    dst = torch.empty(bufs[0][0].numel(), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(k):  # the record copies alone (pinned -> HBM)
        dst.copy_(bufs[i % len(bufs)][0], non_blocking=True)
    torch.cuda.synchronize()
    h2d = (time.perf_counter() - t1) / k
    out["double_buffered"] = {"committed_per_s": committed / el, "ms_per_epoch": el / k * 1e3, "epochs": k,
                              "h2d_ms_per_epoch": h2d * 1e3,
                              "note": "dv_epoch_stage_host(k+1) on the copy stream, then dv_epoch_run_staged(k)"}
    # double-buffered from 4-byte records (key | write << 31) + txn_begin
    rbufs = [(torch.from_numpy(e.to_row_records()).pin_memory(), b[1], b[2], b[3]) for e, b in zip(epochs, bufs)]
    eng.stage_host_rows(0, *rbufs[0])
    eng.run_staged(0, commit)
    t0 = time.perf_counter()
    committed = 0
    eng.stage_host_rows(0, *rbufs[0])
    for i in range(k):
        if i + 1 < k:
            eng.stage_host_rows((i + 1) % 2, *rbufs[(i + 1) % len(rbufs)])
        committed += eng.run_staged(i % 2, commit).committed
    el = time.perf_counter() - t0
    out["double_buffered_rows"] = {
        "committed_per_s": committed / el, "ms_per_epoch": el / k * 1e3, "epochs": k,
        "bytes_h2d_per_epoch": int(rbufs[0][0].numel() * 4 + rbufs[0][1].numel() * 4),
        "note": "dv_epoch_stage_host_rows(k+1): 4-byte records + txn_begin, then dv_epoch_run_staged(k)"}
    return out


class stdout_to_stderr:
    """RCCL prints its version banner on stdout when a communicator is made;
    the bench's stdout carries exactly one JSON line, so the C-level stdout
    points at stderr meanwhile."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def launch_ranks(a):
    """--gpus N > 1 without a launcher: run this script as N rank processes
    under torch.distributed.run (one per GPU) as a child, and return its exit
    status.  Nothing in this process has touched the GPU."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def timed(step, first, warmup, steps, world, batch=None):
    """W untimed steps, then exactly K steps between barrier + synchronize
    on both sides; the slowest rank's time.  batch(first, count): the steps
    as one pipelined call (dv_epoch_run_device_batch), one epoch per step."""
    if batch is not None and warmup:
        batch(first, warmup)
    for i in range(warmup if batch is None else 0):
        step(first + i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if batch is not None:
        stats = batch(first + warmup, steps)
    else:
        stats = [step(first + warmup + i) for i in range(steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cpu" if dist.get_backend() == "gloo" else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return stats, el


def pmc_traffic(a, cc_name, world, kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (tools/pmc_summary.py), only if it was measured on these sources, this
    config and GPU count."""
    if not os.path.exists(PMC_SUMMARY):
        return None, "no PMC summary"
    pmc = json.load(open(PMC_SUMMARY))
    want = {"config": a.config, "cc": cc_name, "n_gpus": world, "src_hash": dvcc._lib.source_hash()}
    stale = {k: (pmc.get(k), v) for k, v in want.items() if pmc.get(k) != v}
    if stale:
        return None, f"PMC summary does not match this run: {stale}"
    k = pmc.get("kernels", {}).get(kernel)
    if not k:
        return None, f"no {kernel} in the PMC summary"
    if "hbm_bytes_per_launch_calibrated" in k:  # tools/pmc_probe_cal.py
        return k["hbm_bytes_per_launch_calibrated"], os.path.relpath(PMC_SUMMARY, ROOT) + " (calibrated)"
    return k["hbm_bytes_per_launch"], os.path.relpath(PMC_SUMMARY, ROOT)


def epoch_bytes(st, rows, R, bucket=False, tb=False, recs=False):
    """SURVEY.md 8(d) algorithmic bytes of each kernel for ONE epoch with the
    stats `st` (mean over the profiled epochs), counted on what the launches of
    that kernel actually processed: {kernel: (bytes per epoch, what is counted)}.
    A stage's bytes are counted once per launch that reads them (a sort pass
    reads and writes its keys; the decision launches read each live access
    once, rounds being overhead).  Kernels not listed move only counters."""
    n_acc, n_txn = st["n_acc"], st["n_txn"]
    ka, kb = st["prefix_acc"], st["surv_acc"]          # keys the prefix's / survivors' sorts order
    ta, tb_ = st["prefix_txn"], st["surv_txn"]
    keys = (ka + kb) if (ka or kb) else n_acc           # (no prefix: the whole epoch is sorted)
    stage_txn = (ta + tb_) if (ka or kb) else n_txn
    # bucket sorts (k_bucket_sort, small sorts): one histogram / scan /
    # scatter pass, then the bucket launch; else sort_passes LSD passes
    passes = 1 if bucket else max(1, st["sort_passes"])
    tiles = sum((k + 4095) // 4096 for k in ((ka, kb) if (ka or kb) else (n_acc,)))
    later = max(0, n_acc - ka)
    per_txn = n_acc / max(1, n_txn)
    surv_all = st["surv_txn"] * per_txn if tb else 0  # tb: every access of a survivor probed by k_kill_emit
    out = {
        "k_epoch_clear": (10 * n_txn + (rows // 4 + (1 << 17) if ka else 0),
                          "per txn: status 1 + access range 8 + length 1 written; prefix epochs: the 2-bit "
                          "row-state bitmap + Bloom filter zeroed"),
        "k_probe": (PROBE_ACC * n_acc + PROBE_TXN * n_txn + 8 * ka,
                    f"{PROBE_ACC} B per access (key 8, type 1, txn id 4 read; row word 4 written; a dense YCSB "
                    f"table's key check is arithmetic) + {PROBE_TXN} B per txn (access range, length) + 8 B per "
                    "prefix sort key written"),
        "k_radix_hist": (8 * passes * keys, "8 B per key read, per pass"),
        "k_radix_scan": (8 * 256 * passes * tiles, "per pass: 256 digit counts per 4096-key tile, read + written"),
        "k_radix_scatter": (16 * passes * keys, "per pass: 8 B per key read + 8 B written"),
        "k_bucket_sort": (16 * keys, "8 B per key read + 8 B written (the bucket's sort by the rest of the row "
                                     "hash, in LDS)"),
        "k_round_pass": (SCAN_BYTES * (keys + st["pass_live"]),
                         f"{SCAN_BYTES} B per live access read (scan 8 + verdict 1): round 0 of each stage scans "
                         "every sorted key once, a later pass its live accesses"),
        "k_round_settle": (17 * stage_txn, "per txn of the stage: length 1, status 1 + 1, verdict bytes 10, "
                                           "fact word 4"),
        "k_round_async": (SCAN_BYTES * st["async_live"],
                          f"{SCAN_BYTES} B per live access entering the launch (scan 8 + verdict 1), once: "
                          "its iterations are rounds, overhead (SURVEY.md 8d)"),
        "k_round_finalize": (5 * stage_txn, "per txn of the stage: fact word 4 read, status 1 written"),
        "k_prefix_mark": (9 * ta + 4 * ka * 0, "per prefix txn: status 1 + access range 8 (lower bound: the "
                                              "committed txns' rows are not counted)"),
        "k_probe_tb": (4 * n_txn + (16 if recs else 21) * ka + ta,
                       "per txn: its boundary 4 read; per prefix access: " + ("4-byte record" if recs else
                                                                            "key 8 + type 1") +
                       " read, row word 4 + sort key 8 written; 1 B of length per prefix txn (the later accesses are "
                       "probed by k_kill)"),
        "k_kill": ((4 if (recs or not tb) else 9) * later + later // 8,
                   ("per access after the prefix: " + ("its 4-byte record" if recs else "key 8 + type 1") +
                    " read (the probe is here), kill bit written") if tb else
                   "per access after the prefix: row word 4 read + kill bit written"),
        "k_kill_count": (13 * max(0, n_txn - ta) + later // 4,
                         "per later txn: access range 8 + status 1 + info word 4 written; kill and skip bits read"),
        "k_kill_emit": (8 * max(0, n_txn - ta) + (12 if (recs or not tb) else 17) * kb + 6 * tb_ +
                        int((8 if recs else 13) * surv_all),
                        "per later txn: first access 4 + info word 4; per survivor access kept: "
                        + ("its record 4 read, " if (tb and recs) else ("key 8 + type 1 read, " if tb else
                                                                        "row word 4 read + ")) +
                        "sort key 8 written; per survivor: map 4 + length 1 + status 1"
                        + (("; every access of a survivor: " + ("record 4" if recs else "key 8 + type 1") +
                            " read, row word 4 written") if tb else "")),
        "k_sub_scatter_back": (6 * tb_, "per survivor: map 4 + status 1 read, status 1 written"),
        "k_exec_txn": (10 * n_txn + int(12 * st["committed"] * per_txn),
                       "per txn: status 1 + access range 8 + commit byte 1; per committed access: row word 4 + "
                       "the 8-byte F0 field"),
        # CALVIN (config B): row queues of the whole epoch, grant groups, execution in queue order
        "k_seg_prepare": (16 * n_acc, "per access: sorted pair 8 read, queue element 8 written"),
        "k_calvin_pass": (13 * n_acc, "per access: queue element 8 read, grant group 4 + read-after-write flag 1 "
                                      "written"),
        "k_exec": (13 * n_acc, "per launch (reads, then writes) and access: queue element 8 + flag 1 read, the "
                               "8-byte F0 field of the half this launch executes"),
        "k_commit_out": (2 * n_txn, "per txn: status 1 read, commit byte 1 written"),
    }
    return out


def kernel_table(ktimes, sts, rows, R, a, cc_name, world, txn_div=1, tb=False, recs=False):
    """Per-kernel table of the profiled epochs: launches per epoch, average
    launch time (its own dispatch timestamps), share of the epoch's kernel
    time, algorithmic bytes per launch (epoch_bytes), achieved GB/s and
    fraction of the HBM peak, and PMC traffic per launch where profiles/ holds
    it for these sources."""
    ep = max(1, len(sts))
    mean = {k: float(np.mean([getattr(s, k) for s in sts])) for k in
            ("n_acc", "n_txn", "prefix_acc", "surv_acc", "prefix_txn", "surv_txn", "pass_live", "async_live",
             "committed", "sort_passes")}
    mean["n_txn"] /= txn_div  # (epoch groups: the stats count the group's txns, n_acc the decided epoch's)
    mean["committed"] /= txn_div
    eb = epoch_bytes(mean, rows, R, bucket="k_bucket_sort" in ktimes, tb=tb, recs=recs)
    total_ms = sum(ms for _, ms in ktimes.values())
    rows_out = []
    for name, (launches, ms) in sorted(ktimes.items(), key=lambda kv: -kv[1][1]):
        lpe = launches / ep
        avg = ms / max(1, launches)
        r = {"kernel": name, "launches_per_epoch": lpe, "avg_us": avg * 1e3,
             "us_per_epoch": ms / ep * 1e3, "share": ms / total_ms if total_ms else 0.0}
        if name in eb and lpe > 0:
            b = eb[name][0] / lpe
            ach = b / (avg * 1e-3) / 1e9 if avg > 0 else 0.0
            r.update({"bytes_per_launch": b, "achieved_GBps": ach, "frac": ach / HBM_PEAK_GBPS,
                      "bytes": eb[name][1]})
            tr, src = pmc_traffic(a, cc_name, world, name)
            r["traffic"] = tr
            if tr is None:
                r["traffic_note"] = src
        rows_out.append(r)
    return rows_out, total_ms / ep * 1e3


def roofline(table, epochs, a):
    """`roofline` of the line: the kernel with the largest share of the
    epoch's kernel time (its algorithmic bytes per launch over its average
    launch time), with the index probe beside it."""
    def entry(r):
        return {"kernel": r["kernel"], "bound": "hbm", "achieved": r.get("achieved_GBps", 0.0),
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": r.get("frac", 0.0), "traffic": r.get("traffic"),
                "bytes_per_launch": r.get("bytes_per_launch"), "avg_launch_ms": r["avg_us"] * 1e-3,
                "launches_per_epoch": r["launches_per_epoch"], "share_of_epoch": r["share"],
                "algorithmic_bytes": r.get("bytes")}
    timed = [r for r in table if "bytes_per_launch" in r]
    if not timed:
        return {"kernel": None, "bound": "hbm", "achieved": 0.0, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": 0.0, "traffic": None}
    top = max(timed, key=lambda r: r["share"])
    out = entry(top)
    out["timed_by"] = (f"each launch's own dispatch timestamps (hipExtLaunchKernelGGL events, "
                       f"dv_kernel_times) over {epochs} epochs run right after the timed region, same epochs "
                       "and stream, as the timed region runs them")
    probe = next((r for r in table if r["kernel"] in ("k_probe", "k_probe_hist", "k_probe_tb")), None)
    if probe is not None and probe is not top:
        out["k_probe"] = entry(probe)
    return out


def measure_legs(a, eng, step, nxt, stats, batch=None):
    """Legs after the timed region, on the same epochs and stream: per-launch
    kernel timing (every launch dispatched with its own timestamps; it adds
    launch latency, so the timed region runs without it), then per-stage
    events.  Returns (profiled stats, stage-timed stats, kernel times)."""
    eng.set_timing(False, profile=True)
    eng.kernel_times(reset=True)
    if batch is not None:
        pstats = batch(nxt, a.steps)
    else:
        pstats = [step(nxt + i) for i in range(a.steps)]
    ktimes = eng.kernel_times(reset=True)
    eng.set_timing(False)
    nxt += a.steps
    if a.timing != "full":
        eng.set_timing(True)
        sstats = [step(nxt + i) for i in range(min(a.steps, 5))]
    else:
        sstats = stats
    eng.set_timing(False)
    return pstats, sstats, ktimes


def stage_summary(stats, sstats, table, el, R):
    committed = sum(s.committed for s in stats)
    txns = sum(s.n_txn for s in stats)
    acc_local = sum(s.n_acc for s in stats)
    n_acc_step = acc_local / max(1, len(stats))
    epoch_gbps = (txns / el) * (BYTES_PER_ACCESS * R + 1) / 1e9
    stage = {k: float(np.mean([getattr(s, k) for s in sstats]))
             for k in ("ms_probe", "ms_sort", "ms_decide", "ms_exec", "ms_total")}
    # SURVEY.md 8(d) counts every stage once: the scan stage's 9 B per access
    # over the whole decide stage (rounds are overhead, not algorithmic)
    dec = stage["ms_decide"]
    scan_stage_gbps = n_acc_step * SCAN_BYTES / (dec * 1e-3) / 1e9 if dec > 0 else 0.0
    out = {
        "epoch_roofline": {"bytes_per_txn": BYTES_PER_ACCESS * R + 1, "achieved_GBps": epoch_gbps,
                           "frac": epoch_gbps / HBM_PEAK_GBPS},
        "decide_stage_roofline": {"bytes": f"{SCAN_BYTES} B per access of this partition, counted once "
                                           "(SURVEY.md 8d: rounds are overhead)",
                                  "achieved_GBps": scan_stage_gbps, "frac": scan_stage_gbps / HBM_PEAK_GBPS},
        "abort_rate": 1.0 - committed / max(1, txns),
        "decided_txns_per_s": txns / el,
        "rounds_mean": float(np.mean([s.rounds for s in stats])),
        "async_tries": {"launches": int(sum(s.async_launches for s in stats)),
                        "declined": int(sum(s.async_declined for s in stats)),
                        "yields": int(sum(s.async_yields for s in stats)), "epochs": len(stats)},
        "stage_ms_mean": stage,
    }
    sc = next((r for r in table if r["kernel"] == "k_radix_scatter" and "bytes_per_launch" in r), None)
    if sc is not None:  # keys each scatter launch actually ordered (the prefix's and the survivors' sorts)
        keys = sc["bytes_per_launch"] / 16
        # the whole sort stage: every launch of it (histogram, digit scan, scatter, bucket sort) per epoch
        stage_kernels = ("k_radix_hist", "k_radix_scan", "k_radix_scatter", "k_bucket_sort")
        stage_us = sum(r["us_per_epoch"] for r in table if r["kernel"] in stage_kernels)
        keys_epoch = keys * sc["launches_per_epoch"]
        sorts = sc["launches_per_epoch"] if "k_bucket_sort" in {r["kernel"] for r in table} else 1.0
        out["sort"] = {"keys_per_epoch": keys_epoch, "sorts_per_epoch": sorts,
                       "stage_us_per_epoch": stage_us, "stage_us_per_sort": stage_us / max(1e-9, sorts),
                       "keys_per_s": keys_epoch / (stage_us * 1e-6) if stage_us > 0 else 0.0,
                       "keys_per_s_counts": "every launch of the sort stage: " + " + ".join(
                           k for k in stage_kernels if any(r["kernel"] == k for r in table)),
                       "scatter": {"kernel": "k_radix_scatter", "avg_launch_ms": sc["avg_us"] * 1e-3,
                                   "keys_per_launch": keys, "keys_per_s": keys / (sc["avg_us"] * 1e-6),
                                   "achieved_GBps": sc["achieved_GBps"], "frac": sc["frac"],
                                   "bytes": "16 B per key per pass (read 8 + write 8)"}}
    return out


def engine_comm_init(a, eng, world, rank, tag):
    """The engine's communicator: RCCL (dv_comm_init), or for --ipc-rehearsal
    the process-boundary test transport (dv_comm_init_ipc), ranks meeting at a
    shared-memory name rank 0 picks."""
    if a.ipc_rehearsal:
        name = [f"/dvcc_bench_{os.getpid()}_{tag}" if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(name, src=0)
        eng.comm_init_ipc(name[0], world, rank)
        return
    uid = [dvcc.comm_unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(uid, src=0)
    with stdout_to_stderr():
        eng.comm_init(uid[0], world, rank)


class PartitionedBench:
    """One rank of a partitioned run: the engine bound to partition `rank`,
    its RCCL communicator (dv_comm_init) and device-resident home batches."""

    def __init__(self, a, cc_name, rows, world, rank, local_rank, max_txn_rank, R):
        self.a, self.world, self.rank, self.R = a, world, rank, R
        # received accesses: this rank's share of every origin's batch (keys
        # spread evenly by key % PART_CNT; multi-partition txns add ~MPR / 2)
        # ... or the whole epoch, which the replicated protocol decides on every
        # rank (dv_comm_set_mode 0 picks it when the epoch fits)
        cap = max(int(max_txn_rank * R * 1.4), CONFIGS[a.config][1] * R) + 65536
        self.eng = dvcc.CCEngine(cc_name, max_txn_rank * world, cap, device=local_rank, part_cnt=world,
                                 part_id=rank, timing=TIMING[a.timing], lsd_sort=a.lsd_sort)
        self.eng.set_stream(torch.cuda.current_stream().cuda_stream)
        self.eng.load_ycsb_partition(rows)
        # epoch groups over ordered decision lanes (dv_lanes_order): L contexts
        # over this partition's tables, each with its own communicator, group
        # g decided on lane g % L, executions in group order
        # (one rank: --lanes; N ranks: --group-lanes; dv_lanes_order refuses
        # lanes whose streams share a hardware queue -- two lanes' RCCL
        # kernels could then queue in opposite orders on two GPUs -- and the
        # bench then runs one context per rank, saying so in the line)
        nl = (max(1, a.lanes) if world == 1 else max(1, a.group_lanes)) \
            if a.protocol == "group" and not a.no_pipeline else 1
        self.lanes = [self.eng.open_lane() for _ in range(nl - 1)]
        engine_comm_init(a, self.eng, world, rank, "ycsb")
        # (the order flag matters to epoch groups only)
        mode = a.part_mode | (dvcc._lib.DV_COMM_POSITION_ORDER if a.order == "position" else 0)
        self.eng.comm_set_mode(mode)
        for ln, lane in enumerate(self.lanes):
            engine_comm_init(a, lane, world, rank, f"ycsb_lane{ln + 1}")
            lane.comm_set_mode(mode)
        self.lanes_refused = None
        if self.lanes:
            ok = 1
            try:
                self.eng.lanes_order(self.lanes)
            except dvcc.DvccError as ex:  # (a shared hardware queue: no ordered lanes on this box)
                self.lanes_refused = repr(ex)
                ok = 0
            if world > 1:  # every rank takes the same path
                t = torch.tensor([ok], dtype=torch.int32, device="cpu" if dist.get_backend() == "gloo" else "cuda")
                dist.all_reduce(t, op=dist.ReduceOp.MIN)
                ok = int(t.item())
            if not ok:
                if self.lanes_refused is None:
                    self.eng.lanes_order([])
                    self.lanes_refused = "refused on another rank"
                self.lanes = []
        self.rows = rows
        self.d_commit = torch.zeros(max_txn_rank * world, dtype=torch.uint8, device="cuda")
        self.d_commits = [self.d_commit] + [torch.zeros_like(self.d_commit) for _ in self.lanes]

    def unorder(self):
        """After the timed region: the engine alone on the bench's stream
        again (the measurement legs and extras run one context)."""
        if self.lanes:
            self.eng.lanes_order([])
            self.eng.set_stream(torch.cuda.current_stream().cuda_stream)

    def order(self):
        """The ordered lanes again (the MPR sweep runs the headline's path)."""
        if self.lanes:
            self.eng.lanes_order(self.lanes)

    def epochs(self, n_txn_rank, mpr, theta, count):
        gen = dvcc.YCSBQueryGenerator(self.rows * self.world, part_cnt=self.world, req_per_query=self.R,
                                      zipf_theta=theta, txn_write_perc=1.0, tup_write_perc=0.5,
                                      part_per_txn=2, strict_ppt=1, mpr=mpr)
        host = gen_epochs(gen, n_txn_rank, self.rank, count)
        return [dvcc.DeviceEpoch(e) for e in host]

    def stepper(self, deps, n_txn_rank):
        def step(i):
            return self.eng.run_epoch_part(deps[i % len(deps)], n_txn_rank, self.d_commit)
        return step

    def groups(self, n_txn_rank, mpr, theta, count):
        """count epoch groups: group g holds this rank's batches of epochs
        g * N .. g * N + N - 1 (seeded SEED + 97 * part + epoch)."""
        gen = dvcc.YCSBQueryGenerator(self.rows * self.world, part_cnt=self.world, req_per_query=self.R,
                                      zipf_theta=theta, txn_write_perc=1.0, tup_write_perc=0.5,
                                      part_per_txn=2, strict_ppt=1, mpr=mpr)
        with ThreadPoolExecutor(max_workers=8) as ex:
            futs = [[ex.submit(gen.gen, n_txn_rank, dvcc.epoch_seed(self.rank, g * self.world + e), self.rank)
                     for e in range(self.world)] for g in range(count)]
            return [[dvcc.DeviceEpoch(f.result()) for f in grp] for grp in futs]

    def group_stepper(self, groups, n_txn_rank):
        def step(i):
            return self.eng.run_epoch_group(groups[i % len(groups)], n_txn_rank, self.d_commit)
        return step

    def group_batcher(self, groups, n_txn_rank, lanes=True):
        """count consecutive groups in one dv_epoch_group_run_batch call (one
        host wait between two groups), or over the ordered lanes."""
        def batch(first, count):
            run = [groups[(first + i) % len(groups)] for i in range(count)]
            if lanes and self.lanes:
                nl = len(self.d_commits)
                base = self.eng._order_next
                return self.eng.run_epoch_groups_ordered(run, n_txn_rank,
                                                         [self.d_commits[(base + i) % nl] for i in range(count)])
            return self.eng.run_epoch_groups(run, n_txn_rank, self.d_commit)
        return batch


def tpcc_part_leg(a, world, rank, local_rank, first_step):
    """Config E across the ranks (dv_tpcc_epoch_run_part over RCCL):
    --tpcc-part-wh warehouses (256) split over the N ranks, each rank's client
    batch 1/N of a global epoch of each --tpcc-txns size (65,536, and the
    reference's 10,000-txn window), records sent to the partition owning their
    warehouse, decided, executed there, o_ids all-reduced; WAIT_DIE and
    CALVIN.  Max over ranks of the time of K epochs, like the headline."""
    from dvcc import tpcc as T
    pp = T.tpcc_params(a.tpcc_part_wh, part_cnt=world)
    sizes = [int(x) for x in str(a.tpcc_txns).split(",") if x]
    out = {"warehouses": a.tpcc_part_wh, "warehouses_per_gpu": a.tpcc_part_wh / world,
           "protocol": "dv_tpcc_epoch_run_part (owner split, per-round verdict all-reduce, o_id all-reduce)"}
    nxt = first_step
    for cc_name in ("WAIT_DIE", "CALVIN"):
        n_max = max(sizes) // world
        eng = T.TpccEngine(cc_name, pp, n_max * world, device=local_rank, part_id=rank, seed=1)
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        lanes = [eng.open_lane() for _ in range(max(1, a.part_lanes) - 1)]
        engine_comm_init(a, eng, world, rank, "tpcc_" + cc_name)
        for ln, lane in enumerate(lanes):
            engine_comm_init(a, lane, world, rank, f"tpcc_{cc_name}_lane{ln + 1}")
        if lanes:
            eng.lanes_order(lanes)
        out["decision_lanes"] = 1 + len(lanes)
        for total in sizes:
            n_rank = total // world
            batches = [T.gen(pp, n_rank, dvcc.epoch_seed(rank, 500 + e), home_part=rank) for e in range(2)]
            dev = [(T.device_epoch(b), torch.from_numpy(b.owner).cuda()) for b in batches]
            d_commit = torch.zeros(n_rank * world, dtype=torch.uint8, device="cuda")
            d_oid = torch.zeros(n_rank * world, dtype=torch.int64, device="cuda")
            # (lanes: one commit / o_id buffer per lane)
            bufs = [(d_commit, d_oid)] + [(torch.zeros_like(d_commit), torch.zeros_like(d_oid)) for _ in lanes]

            def step(i, dev=dev, n_rank=n_rank, d_commit=d_commit, d_oid=d_oid):
                (dep, d_args), own = dev[i % 2]
                return eng.run_tpcc_epoch_part(dep, d_args, own, n_rank, d_commit, d_oid)

            def batch(first, count, dev=dev, n_rank=n_rank, bufs=bufs):
                ctx_ix = {id(c): j for j, c in enumerate([eng] + lanes)}

                def one(ctx, i):
                    (dep, d_args), own = dev[(first + i) % 2]
                    dc, do = bufs[ctx_ix[id(ctx)]]
                    return ctx.run_tpcc_epoch_part(dep, d_args, own, n_rank, dc, do)
                return eng.run_ordered(count, one)
            k = max(a.steps, 5) if total == sizes[0] else max(a.steps, 20)
            if lanes:  # (whole rounds of the lanes per call)
                k = (k + len(bufs) - 1) // len(bufs) * len(bufs)
            sts, el = timed(step, nxt, a.warmup, k, world, batch if lanes else None)
            nxt += 100
            committed = sum(st.committed for st in sts)
            key = cc_name if total == sizes[0] else f"window_{total}_{cc_name}"
            out[key] = {"txns_per_epoch": n_rank * world, "txns_per_rank": n_rank,
                        "committed_per_s": committed / el, "decided_txns_per_s": k * n_rank * world / el,
                        "ms_per_epoch": el / k * 1e3, "abort_rate": 1 - committed / (k * n_rank * world),
                        "epochs": k}
        eng.close()
    return out


def extra_legs(a, out, pb, mpr, theta, n_txn_rank, n_txn_total, world, group):
    """N>1 extras beside the headline, each with the headline's warmup:
    strong scaling (one 1,048,576-txn epoch per step, dv_epoch_run_part --
    replicated when the epoch fits, mode 0), weak scaling (1,048,576 txns per
    GPU, the list protocol) and the MPR sweep (the headline's path: epoch
    groups through dv_epoch_group_run_batch over the ordered lanes)."""
    nxt = 10_000
    k = max(1, min(a.steps, 10))
    if group:
        sdeps = pb.epochs(n_txn_rank, mpr, theta, 2)
        sst, sel = timed(pb.stepper(sdeps, n_txn_rank), nxt, a.warmup, k, world)
        scm = sum(s.committed for s in sst)
        out["strong_scaling"] = {"txns_per_epoch": n_txn_total, "committed_per_s": scm / sel,
                                 "ms_per_epoch": sel / len(sst) * 1e3, "epochs": len(sst),
                                 "protocol": "dv_epoch_run_part, mode %d" % a.part_mode,
                                 "sequence_order": a.order if a.cc.upper() != "CALVIN" else "origin"}
        del sdeps
        nxt += 100
    if not a.no_weak:
        wdeps = pb.epochs(n_txn_total, mpr, theta, 2)
        wst, wel = timed(pb.stepper(wdeps, n_txn_total), nxt, a.warmup, k, world)
        wc = sum(s.committed for s in wst)
        out["weak_scaling"] = {"txns_per_epoch_per_gpu": n_txn_total, "txns_per_epoch": n_txn_total * world,
                               "committed_per_s": wc / wel, "decided_txns_per_s": len(wst) * n_txn_total * world / wel,
                               "ms_per_epoch": wel / len(wst) * 1e3,
                               "abort_rate": 1 - wc / (len(wst) * n_txn_total * world), "epochs": len(wst),
                               "mpr": mpr,
                               "protocol": ("dv_epoch_run_part, list protocol (the epoch exceeds a context)" if world > 1
                                            else "dv_epoch_run_part on one rank: the strong leg's epoch size, replicated")}
        del wdeps
        nxt += 100
    sweep = []
    if group:
        pb.order()
    for m in [float(x) for x in a.mpr_sweep.split(",") if x.strip()]:
        if group:
            mg = pb.groups(n_txn_rank, m, theta, 3)
            km = (k + len(pb.d_commits) - 1) // len(pb.d_commits) * len(pb.d_commits)
            mst, mel = timed(None, 0, a.warmup, km, world, pb.group_batcher(mg, n_txn_rank))
            mtx = len(mst) * n_txn_total * world
        else:
            mdeps = pb.epochs(n_txn_rank, m, theta, 2)
            mst, mel = timed(pb.stepper(mdeps, n_txn_rank), nxt, a.warmup, k, world)
            mtx = len(mst) * n_txn_total
        mc = sum(s.committed for s in mst)
        sweep.append({"mpr": m, "committed_per_s": mc / mel, "ms_per_step": mel / len(mst) * 1e3,
                      "abort_rate": 1 - mc / mtx, "steps": len(mst),
                      "rounds_mean": float(np.mean([s.rounds for s in mst]))})
        nxt += 100
    if group:
        pb.unorder()
    if sweep:
        out["mpr_sweep"] = sweep
    if not a.no_tpcc_part and not a.no_tpcc:
        out["tpcc_partitioned"] = tpcc_part_leg(a, world, pb.rank, int(os.environ.get("LOCAL_RANK", 0)), nxt)


LINE_LIMIT = 8192  # bytes of the stdout record (the driver parses the tail of stdout)


def _r(v, sig=4):
    """A float at `sig` significant digits (the record's numbers)."""
    if isinstance(v, float):
        return float(f"{v:.{sig}g}")
    return v


def _pick(d, keys):
    return {k: _r(d[k]) for k in keys if isinstance(d, dict) and k in d and not isinstance(d[k], (dict, list))}


def headline_record(out, detail_path=None):
    """The ONE stdout line: the headline (metric, value, unit, n_gpus, steps,
    warmup, ms_per_step, ...), the dominant kernel's roofline, the CPU
    baseline and a few numbers per side leg; everything else -- kernel
    tables, leg detail, samples -- stays in the detail file (`detail_path`).
    Stays under LINE_LIMIT bytes whatever the legs hold."""
    rec = {k: _r(out[k]) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                   "higher_is_better", "scaling", "vs_baseline", "dtype", "data") if k in out}
    cfg = out.get("config", {})
    rec["config"] = {k: cfg[k] for k in ("workload", "cc_alg", "rows_per_partition", "txns_per_epoch",
                                         "txns_per_epoch_per_gpu", "req_per_query", "zipf_theta", "mpr",
                                         "parallelism", "decision_lanes", "epochs_per_step", "sequence_order",
                                         "ordered_lanes_refused") if k in cfg}
    for k in ("sequence_order", "ordered_lanes_refused"):
        if isinstance(rec["config"].get(k), str):
            rec["config"][k] = rec["config"][k][:80]
    rf = out.get("roofline") or {}
    rec["roofline"] = {k: _r(rf.get(k)) for k in ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic",
                                                  "bytes_per_launch", "avg_launch_ms", "launches_per_epoch",
                                                  "share_of_epoch")}
    if isinstance(rf.get("k_probe"), dict):
        rec["roofline"]["k_probe"] = _pick(rf["k_probe"], ("kernel", "frac", "achieved", "avg_launch_ms"))
    cb = out.get("cpu_baseline")
    if isinstance(cb, dict):
        rec["cpu_baseline"] = _pick(cb, ("value", "unit", "cores", "kind"))
        rec["cpu_baseline"]["sample"] = str(cb.get("sample", ""))[:160]
        if isinstance(cb.get("threads_scaling"), dict):
            rec["cpu_baseline"]["threads_scaling"] = {k: _r(v) for k, v in cb["threads_scaling"].items()}
    if isinstance(out.get("cpu_baseline_single_thread"), dict):
        rec["cpu_baseline_single_thread"] = _pick(out["cpu_baseline_single_thread"], ("value", "cores", "kind"))
    for k in ("abort_rate", "decided_txns_per_s"):
        if k in out:
            rec[k] = _r(out[k])
    for k in ("epoch_roofline", "decide_stage_roofline"):
        if isinstance(out.get(k), dict):
            rec[k] = _r(out[k].get("frac"))
    if "kernel_us_per_epoch" in out:
        rec["kernel_us_per_epoch"] = _r(out["kernel_us_per_epoch"])
    legs = {}
    for leg in ("config_b", "config_c"):
        d = out.get(leg)
        if isinstance(d, dict):
            legs[leg] = _pick(d, ("cc_alg", "ms_per_epoch", "committed_per_s", "abort_rate", "error"))
            if isinstance(d.get("roofline"), dict):
                legs[leg]["roofline"] = _pick(d["roofline"], ("kernel", "frac", "avg_launch_ms"))
            if isinstance(d.get("epoch_roofline"), dict):
                legs[leg]["epoch_roofline"] = _r(d["epoch_roofline"].get("frac"))
    tp = out.get("tpcc")
    if isinstance(tp, dict):
        t = {}
        for name, d in [(k, v) for k, v in tp.items() if isinstance(v, dict)]:
            for cc, v in ([(name, d)] if "ms_per_epoch" in d else [(f"{name}_{c}", x) for c, x in d.items()
                                                                  if isinstance(x, dict)]):
                if "ms_per_epoch" in v:
                    t[cc] = _pick(v, ("ms_per_epoch", "committed_per_s", "abort_rate"))
                    if isinstance(v.get("epoch_roofline"), dict):
                        t[cc]["epoch_roofline"] = _r(v["epoch_roofline"].get("frac"))
                    if isinstance(v.get("cpu_baseline"), dict):
                        t[cc]["cpu_baseline"] = _r(v["cpu_baseline"].get("value"))
        legs["tpcc"] = t
    if isinstance(out.get("sort"), dict):
        legs["sort"] = _pick(out["sort"], ("keys_per_s", "stage_us_per_sort", "keys_per_epoch"))
    if isinstance(out.get("wire_ingress"), dict):
        legs["wire_ingress"] = _pick(out["wire_ingress"], ("decoded_txns_per_s", "wire_MBps", "batches",
                                                            "respond_txns_per_s", "cores", "error"))
    if isinstance(out.get("cpu_config_a"), dict):
        legs["cpu_config_a"] = _pick(out["cpu_config_a"], ("value", "unit", "cores", "kind", "abort_rate"))
    cl = out.get("closed_loop_retry")
    if isinstance(cl, dict):
        legs["closed_loop_retry"] = _pick(cl, ("ms_per_epoch", "committed_per_s"))
        if isinstance(cl.get("lanes"), dict):
            legs["closed_loop_retry"]["lanes"] = _pick(cl["lanes"], ("ms_per_epoch", "committed_per_s",
                                                                     "decision_lanes"))
    for leg in ("strong_scaling", "weak_scaling"):
        if isinstance(out.get(leg), dict):
            legs[leg] = _pick(out[leg], ("txns_per_epoch", "ms_per_epoch", "committed_per_s", "abort_rate"))
    if isinstance(out.get("mpr_sweep"), list):
        legs["mpr_sweep"] = [_pick(m, ("mpr", "ms_per_step", "committed_per_s", "abort_rate"))
                             for m in out["mpr_sweep"][:8]]
    tpp = out.get("tpcc_partitioned")
    if isinstance(tpp, dict):
        legs["tpcc_partitioned"] = {k: _pick(v, ("txns_per_epoch", "ms_per_epoch", "committed_per_s"))
                                    for k, v in tpp.items() if isinstance(v, dict)}
    for k in ("extra_legs_error",):
        if k in out:
            legs[k] = str(out[k])[:200]
    rec["legs"] = legs
    for k in ("src_hash", "timing_in_timed_region"):
        if k in out:
            rec[k] = out[k]
    if detail_path:
        rec["detail"] = detail_path
    line = json.dumps(rec)
    if len(line) > LINE_LIMIT:  # (never expected: the legs are the first to go)
        rec["legs"] = {"dropped": f"{len(line)} B > {LINE_LIMIT}: see the detail file"}
        line = json.dumps(rec)
    return line


def write_detail(out, path):
    """The full record (kernel tables, every leg) beside the stdout line."""
    try:
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f)
        return os.path.relpath(os.path.abspath(path), ROOT)
    except OSError as ex:
        print(f"bench: detail file not written: {ex!r}", file=sys.stderr)
        return None


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.ipc_rehearsal:  # (ranks share the box's GPUs)
        local_rank %= max(1, torch.cuda.device_count())
        os.environ["LOCAL_RANK"] = str(local_rank)
    a.gpus = world
    torch.cuda.set_device(local_rank)
    # one stream for torch and the engine: the engine then needs no event
    # wait on torch's stream before each epoch (CCEngine._after_torch)
    if not os.environ.get("DVCC_BENCH_OWN_STREAM"):
        torch.cuda.set_stream(torch.cuda.Stream())
    if world > 1:
        with stdout_to_stderr():
            if a.ipc_rehearsal:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
            dist.barrier()
    if a.tpcc_only:
        print(json.dumps({"tpcc": tpcc_leg(a)}), flush=True)
        return
    cc_name = a.cc.upper()
    rows, n_txn_total, theta, desc = CONFIGS[a.config]
    R = 10
    n_txn_rank = n_txn_total // world
    part = world > 1 or a.part1
    mpr = a.mpr if part else -1.0  # N=1: the reference zipf generator, unmodified
    n_epochs = max(1, min(a.epochs, a.steps + a.warmup))
    t_gen = time.perf_counter()
    extra = {}
    if not part:
        gen = dvcc.YCSBQueryGenerator(rows, part_cnt=1, req_per_query=R, zipf_theta=theta,
                                      txn_write_perc=1.0, tup_write_perc=0.5, part_per_txn=1, strict_ppt=1,
                                      mpr=mpr)
        epochs = gen_epochs(gen, n_txn_total, 0, n_epochs)
        t_gen = time.perf_counter() - t_gen
        eng = dvcc.CCEngine(cc_name, n_txn_total, n_txn_total * R, device=local_rank, timing=TIMING[a.timing],
                            lsd_sort=a.lsd_sort)
        eng.set_prefix(None if a.prefix < 0 else a.prefix)
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        eng.load_ycsb_partition(rows)
        deps = [dvcc.DeviceEpoch(e, txn_begin=not a.no_txn_begin, recs32=not a.no_recs32) for e in epochs]
        d_commit = torch.zeros(n_txn_total, dtype=torch.uint8, device="cuda")

        def step(i):
            return eng.run_epoch_device(deps[i % n_epochs], d_commit)

        # decision lanes: more contexts over the engine's tables, each on its
        # own stream, so one epoch's (latency-bound) rounds overlap the next's
        lanes = [eng.open_lane() for _ in range(max(1, a.lanes) - 1)]

        def batch(first, count):  # the product's pipelined entry point: epoch k+1 queued before k is read
            run = [deps[(first + i) % n_epochs] for i in range(count)]
            if lanes:
                return eng.run_epochs_lanes(lanes, run, d_commit)
            return eng.run_epochs_device(run, d_commit)

        def batch1(first, count):
            return eng.run_epochs_device([deps[(first + i) % n_epochs] for i in range(count)], d_commit)
    else:
        weak = not a.no_weak
        pb = PartitionedBench(a, cc_name, rows, world, rank, local_rank,
                              n_txn_total if weak else n_txn_rank, R)
        eng = pb.eng
        if a.protocol == "group":
            groups = pb.groups(n_txn_rank, mpr, theta, n_epochs)
            step = pb.group_stepper(groups, n_txn_rank)
            batch = pb.group_batcher(groups, n_txn_rank)
            batch1 = pb.group_batcher(groups, n_txn_rank, lanes=False)
        else:
            deps = pb.epochs(n_txn_rank, mpr, theta, n_epochs)
            step = pb.stepper(deps, n_txn_rank)
        t_gen = time.perf_counter() - t_gen

    # the pipelined entry points: dv_epoch_run_device_batch (one GPU),
    # dv_epoch_group_run_batch (epoch groups); the other protocols step
    pipelined = not a.no_pipeline and (not part or a.protocol == "group")
    stats, el = timed(step, 0, a.warmup, a.steps, world, batch if pipelined else None)
    # (the profiling legs time one context's launches: one lane)
    if part:
        pb.unorder()
    pstats, sstats, ktimes = measure_legs(a, eng, step, a.warmup + a.steps, stats,
                                          batch1 if pipelined else None)
    table, kus = kernel_table(ktimes, pstats, rows, R, a, cc_name, world, world if (part and a.protocol == "group") else 1,
                              tb=not part and not a.no_txn_begin, recs=not part and not a.no_txn_begin and not a.no_recs32)
    committed = sum(s.committed for s in stats)  # global: every rank holds the same decisions
    group = part and a.protocol == "group"
    out = {
        "metric": METRIC,
        "value": committed / el,
        "unit": "committed txns/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": el / a.steps * 1e3,
        "higher_is_better": True,
        # per GPU and step: one 1,048,576-txn epoch decided (N = 1 too), N epochs per step at N > 1
        "scaling": "weak" if (group or (world == 1 and a.protocol == "group")) else "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic: Deneva YCSB zipf generator (myrand LCG, seeded SEED+97*part+epoch)",
        "config": {
            "workload": desc, "cc_alg": cc_name, "rows_per_partition": rows,
            "txns_per_epoch": n_txn_total, "txns_per_epoch_per_gpu": n_txn_rank, "req_per_query": R,
            "zipf_theta": theta, "txn_write_perc": 1.0, "tup_write_perc": 0.5,
            "mpr": mpr if part else 0.0, "part_per_txn": min(2, world),
            "parallelism": (f"partitioned x{world} (PART_CNT={world}, "
                            + ("IPC rehearsal: ranks sharing a GPU, not a scaling result)" if a.ipc_rehearsal
                               else "RCCL)")) if world > 1 else "1 GPU",
            "epochs_per_step": world if group else 1,
            "protocol": ("epoch groups (rank e decides epoch e of each group of N; batches all-to-allv'd to "
                         "the decider, committed accesses forwarded to their owners, epochs executed in order)"
                         if group else
                         {0: "replicated (the epoch's accesses all-gathered, decided on every rank, own rows "
                             "executed) when the epoch fits a context, else the list protocol",
                          1: "list protocol (owner split, per-round verdict all-reduce)",
                          2: "replicated"}[a.part_mode] if part else "single GPU"),
            "distinct_epochs": n_epochs,
            "decision_lanes": 1 + (len(pb.lanes) if part else len(lanes)),
            "sequence_order": ("position-major (origin q's txn j at j * N + q, DV_COMM_POSITION_ORDER)"
                               if group and a.order == "position" and cc_name != "CALVIN" else
                               "origin-major (Calvin's lock order)") if part else "one origin",
        },
        "roofline": roofline(table, len(pstats), a),
        "timing_in_timed_region": a.timing,
        "gen_seconds": t_gen,
        "src_hash": dvcc._lib.source_hash(),
    }
    if part and pb.lanes_refused:
        out["config"]["ordered_lanes_refused"] = pb.lanes_refused
    out.update(stage_summary(stats, sstats, table, el, R))
    out["kernels"] = table
    out["kernel_us_per_epoch"] = kus
    out["stage_sizes_mean"] = {k: float(np.mean([getattr(st, k) for st in pstats]))
                               for k in ("n_txn", "n_acc", "prefix_txn", "prefix_acc", "surv_txn", "surv_acc")}
    if not part:
        live, und = eng.round_log()
        out["round_log_last_epoch"] = {"live": live, "undecided": und}
        out["e2e_host_input"] = e2e_host_leg(eng, epochs, min(a.steps, 5))
        try:
            out["wire_ingress"] = wire_ingress_leg(eng, epochs[0], rows, d_commit)
        except Exception as ex:  # noqa: BLE001 -- the headline above is already measured
            out["wire_ingress"] = {"error": repr(ex)[:200]}
        out["closed_loop_retry"] = closed_loop_leg(eng, gen, n_txn_total, max(4, min(a.steps, 10)), d_commit,
                                                   out["ms_per_step"])
        if lanes:
            out["closed_loop_retry"]["lanes"] = closed_loop_lanes_leg(eng, lanes, gen, n_txn_total,
                                                                      max(8, min(a.steps, 16)), out["ms_per_step"])
    else:
        try:
            extra_legs(a, out, pb, mpr, theta, n_txn_rank, n_txn_total, world, group)
        except Exception as ex:  # noqa: BLE001 -- the headline above is already measured
            out["extra_legs_error"] = repr(ex)
    if not part and rank == 0 and not a.no_cpu_baseline:
        # the single-thread E-schedule port (decision-identical) and, for
        # NO_WAIT, the multi-threaded engine, which is then the baseline
        single = cpu_baseline(epochs, rows, cc_name, a.cpu_seconds)
        if cc_name == "NO_WAIT":
            out["cpu_baseline"] = cpu_baseline_mt(epochs, rows, a.cpu_seconds)
            out["cpu_baseline_single_thread"] = single
        else:
            out["cpu_baseline"] = single
    if rank == 0:  # Deneva's [summary] line (stats.cpp:425-500) for scripts/helper.py, on stderr
        from dvcc.stats import summary_line
        # (partitioned runs do not count their multi-partition commits: those
        # four counters are left out rather than printed as one-partition)
        out["deneva_summary"] = summary_line(el, stats, part_counts=not part)
        print(out["deneva_summary"], file=sys.stderr, flush=True)
    if not part and not a.no_tpcc:
        out["tpcc"] = tpcc_leg(a)
    if not part and not a.no_configs and a.config == "D":
        eng.close()  # (the other configs' tables in its place)
        eng = None
        legs = {}
        for cfg, cc in (("B", "CALVIN"), ("C", "OCC")):
            try:
                legs[f"config_{cfg.lower()}"] = config_leg(a, cfg, cc)
            except Exception as ex:  # noqa: BLE001 -- the headline above is already measured
                legs[f"config_{cfg.lower()}"] = {"error": repr(ex)}
        out.update(legs)
        if rank == 0 and not a.no_cpu_baseline:
            out["cpu_config_a"] = cpu_config_a(min(a.cpu_seconds, 10.0))
    if rank == 0:
        path = write_detail(out, a.detail_out) if a.detail_out else None
        sys.stderr.flush()
        print(headline_record(out, path), flush=True)
    if eng is not None:
        eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
