"""The partitioned protocol (dv_epoch_run_part over a one-rank RCCL
communicator) on config D at 1/P of the data per rank: per-epoch time and
rounds, i.e. the kernel side of an N-GPU epoch without the network.

    python tools/exp_part1.py [P ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))

import torch  # noqa: E402

import dvcc  # noqa: E402


MODE = int(os.environ.get("DVCC_PART_MODE", "1"))  # 1 list protocol, 2 replicated


def main():
    rows = 16_777_216
    for P in [int(x) for x in sys.argv[1:]] or [1, 2, 8]:
        n_txn = 1_048_576 // P
        gen = dvcc.YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
        eps = [gen.gen(n_txn, dvcc.epoch_seed(0, e)) for e in range(2)]
        eng = dvcc.CCEngine(dvcc.NO_WAIT, n_txn, n_txn * 10)
        eng.load_ycsb_partition(rows)
        eng.comm_init(dvcc.comm_unique_id(), 1, 0)
        eng.comm_set_mode(MODE)
        deps = [dvcc.DeviceEpoch(e) for e in eps]
        d = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
        for i in range(3):
            eng.run_epoch_part(deps[i % 2], n_txn, d)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        k = 10
        sts = [eng.run_epoch_part(deps[i % 2], n_txn, d) for i in range(k)]
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / k
        print(f"1/{P} of config D ({n_txn} txns): {'list' if MODE == 1 else 'replicated'} protocol {el * 1e3:.3f} ms/epoch, "
              f"rounds {sts[-1].rounds}, committed {sts[-1].committed}", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
