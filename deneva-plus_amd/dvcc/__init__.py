"""dvcc -- MI355X batched concurrency-control engine for Deneva's
transaction-scheduling hot path (probe -> lock/validate -> grant/abort ->
execute), exposed through libdvcc.so (include/dvcc.h)."""
import os

# The HIP runtime's packet-capture mode for graphs (DEBUG_CLR_GRAPH_PACKET_CAPTURE=1):
# an epoch graph (dvcc_runtime.hip graph_decide) then replays in ~4 us of host
# time instead of 15-50 (measured, profiles/r05_k).  It is a process-wide HIP
# switch that also changes torch's own graph capture, so importing dvcc does
# not set it: opt in with DVCC_PACKET_CAPTURE=1 (or set the HIP variable
# yourself) before anything touches the GPU -- bench.py and the tests do.
# The epoch graphs are correct either way (tests/test_gpu_parity.py
# test_epoch_graphs_default_capture_mode runs them with it unset).
if os.environ.get("DVCC_PACKET_CAPTURE") == "1":
    os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "1")
try:  # share torch's HIP runtime when torch is present (one libamdhip64 per process)
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    pass

from ._lib import (CALVIN, CC_NAMES, HASH_MOD, HASH_YCSB, NO_WAIT, OCC, RD, SCAN, WAIT_DIE, WR,  # noqa
                   DvccError, lib)
from .engine import CCEngine, ClosedLoopBufs, DeviceEpoch, Epoch, comm_unique_id  # noqa: F401
from .ycsb import YCSBQueryGenerator, epoch_seed, sequence, sequence_position  # noqa: F401
