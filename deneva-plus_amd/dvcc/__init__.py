"""dvcc -- MI355X batched concurrency-control engine for Deneva's
transaction-scheduling hot path (probe -> lock/validate -> grant/abort ->
execute), exposed through libdvcc.so (include/dvcc.h)."""
try:  # share torch's HIP runtime when torch is present (one libamdhip64 per process)
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    pass

from ._lib import (CALVIN, CC_NAMES, HASH_MOD, HASH_YCSB, NO_WAIT, OCC, RD, SCAN, WAIT_DIE, WR,  # noqa
                   DvccError, lib)
from .engine import CCEngine, ClosedLoopBufs, DeviceEpoch, Epoch, comm_unique_id  # noqa: F401
from .ycsb import YCSBQueryGenerator, epoch_seed, sequence, sequence_position  # noqa: F401
