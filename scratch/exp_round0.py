# experiment: time round 0 / round 1 with and without the OK-push atomics
import os, sys, time
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "deneva-plus_amd"))
import torch, numpy as np, dvcc
rows, n_txn = 1 << 24, 1 << 20
g = dvcc.YCSBQueryGenerator(rows, zipf_theta=0.9)
e = g.gen(n_txn, 1)
eng = dvcc.CCEngine(dvcc.NO_WAIT, n_txn, e.n_acc)
eng.load_ycsb_partition(rows)
S = torch.cuda.Stream(); torch.cuda.set_stream(S); eng.set_stream(S.cuda_stream)
dep = dvcc.DeviceEpoch(e)
v = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
res = []
for it in range(6):
    eng.begin(dep)
    torch.cuda.synchronize()
    ts = []
    for r in range(3):
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record(); eng.round_local(v); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
        try:
            eng.round_apply(v)
        except Exception as ex:
            break
    try:
        eng.finish()
    except Exception:
        pass
    res.append(ts)
print(os.environ.get("DVCC_LIB", "normal"), np.median(np.array(res[1:]), axis=0))
