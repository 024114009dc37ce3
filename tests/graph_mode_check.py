"""Epoch graphs under HIP's default graph-capture mode: run by
test_gpu_parity.py::test_epoch_graphs_default_capture_mode in a fresh process
whose environment has DEBUG_CLR_GRAPH_PACKET_CAPTURE unset -- the mode a C++
host linking libdvcc.so gets.  Small YCSB epochs from the same device buffers
again and again (captured at a key's third call, replayed from its fourth),
through the batch and through four decision lanes, every epoch checked
against the oracle (test infrastructure).  Prints "graph mode ok"."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "deneva-plus_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

assert "DEBUG_CLR_GRAPH_PACKET_CAPTURE" not in os.environ

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _oracle as O  # noqa: E402
import dvcc  # noqa: E402

assert "DEBUG_CLR_GRAPH_PACKET_CAPTURE" not in os.environ, "importing dvcc set the HIP switch"
ORACLE_CC = {dvcc.NO_WAIT: O.NO_WAIT, dvcc.OCC: O.OCC, dvcc.CALVIN: O.CALVIN}


def check(cc, lanes):
    rows, n = 1 << 16, 5000
    g = dvcc.YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = dvcc.CCEngine(cc, n, 60_000)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(None)
    extra = [eng.open_lane() for _ in range(lanes - 1)]
    src = [g.gen(n, 1800 + k) for k in range(3)]
    bufs = [dvcc.DeviceEpoch(e) for e in src]
    seq = [k % 3 for k in range(6 * max(lanes, 3))]
    commits = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in seq]
    deps = [bufs[k] for k in seq]
    sts = eng.run_epochs_lanes(extra, deps, commits) if extra else eng.run_epochs_device(deps, commits)
    for i, (k, st) in enumerate(zip(seq, sts)):
        c_ref, _, st_ref = O.epoch_run(ORACLE_CC[cc], tab.ix, f0, n, src[k].txn_begin, src[k].keys, src[k].types,
                                       want_grant=cc == dvcc.CALVIN)
        assert (commits[i].cpu().numpy() == c_ref).all(), (cc, lanes, i)
        assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                               st_ref.write_cnt), (cc, lanes, i)
    assert (eng.read_table(0, rows) == f0).all(), (cc, lanes)
    for ln in extra:
        ln.close()
    eng.close()
    print(f"cc={cc} lanes={lanes}: {len(seq)} epochs ok")


if __name__ == "__main__":
    assert torch.cuda.is_available()
    for cc, lanes in [(dvcc.NO_WAIT, 1), (dvcc.NO_WAIT, 4), (dvcc.CALVIN, 4), (dvcc.OCC, 1)]:
        check(cc, lanes)
    print("graph mode ok")
