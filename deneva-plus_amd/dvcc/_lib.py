"""ctypes binding of libdvcc.so (the C ABI of include/dvcc.h).

The library is loaded from the in-tree build (deneva-plus_amd/build/libdvcc.so).
If it is missing the import fails loudly: there is no CPU fallback for the
engine -- the HIP path is the product.
"""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("DVCC_LIB") or os.path.join(PKG_DIR, "build", "libdvcc.so")

DV_OK = 0
DV_ERR_ARG = -1
DV_COMM_WIDE_BATCHES = 4  # dv_comm_set_mode: 8-byte epoch-group batches
DV_COMM_POSITION_ORDER = 8  # dv_comm_set_mode: epoch groups sequenced txn by txn across origins
DV_ERR_HIP = -2
DV_ERR_NOMEM = -3
DV_ERR_KEY_NOT_FOUND = -4
DV_ERR_DUP_ROW = -5
DV_ERR_NO_TABLE = -6
DV_ERR_STATE = -7
DV_ERR_NO_DEVICE = -8
DV_ERR_TXN_RANGE = -9

# CC_ALG (config.h)
NO_WAIT, WAIT_DIE, OCC, CALVIN = 1, 2, 8, 10
CC_NAMES = {"NO_WAIT": NO_WAIT, "WAIT_DIE": WAIT_DIE, "OCC": OCC, "CALVIN": CALVIN}
YCSB, TPCC = 1, 2
RD, WR, SCAN = 0, 1, 3
HASH_YCSB, HASH_MOD = 0, 1
FLAG_TIMING = 1
FLAG_NO_TAIL = 2
FLAG_EL64 = 4
FLAG_NO_ASYNC = 8
FLAG_KERNEL_TIMING = 16
FLAG_KERNEL_PROFILE = 32
FLAG_LSD_SORT = 64


class DvccError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = lib().dv_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: dvcc error {code} ({msg})" if what else f"dvcc error {code} ({msg})")


class Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("cc_alg", ctypes.c_int32), ("workload", ctypes.c_int32),
                ("part_cnt", ctypes.c_uint32), ("part_id", ctypes.c_uint32),
                ("max_txn", ctypes.c_uint32), ("max_acc", ctypes.c_uint64),
                ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class Access(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint64), ("txn_seq", ctypes.c_uint32), ("type", ctypes.c_uint8),
                ("table", ctypes.c_uint8), ("flags", ctypes.c_uint16)]


class EpochDev(ctypes.Structure):
    _fields_ = [("keys", ctypes.c_void_p), ("types", ctypes.c_void_p), ("acc_txn", ctypes.c_void_p),
                ("tables", ctypes.c_void_p), ("n_acc", ctypes.c_uint64), ("n_txn", ctypes.c_uint32),
                ("max_txn_acc", ctypes.c_uint32), ("ts", ctypes.c_void_p), ("n_acc_dev", ctypes.c_void_p),
                ("txn_begin", ctypes.c_void_p), ("recs32", ctypes.c_void_p)]


class Stats(ctypes.Structure):
    _fields_ = [("n_txn", ctypes.c_uint64), ("n_acc", ctypes.c_uint64),
                ("committed", ctypes.c_uint64), ("aborted", ctypes.c_uint64),
                ("write_cnt", ctypes.c_uint64), ("read_digest", ctypes.c_uint64),
                ("rounds", ctypes.c_uint32), ("sort_passes", ctypes.c_uint32),
                ("ms_total", ctypes.c_float), ("ms_probe", ctypes.c_float),
                ("ms_sort", ctypes.c_float), ("ms_decide", ctypes.c_float),
                ("ms_exec", ctypes.c_float), ("ms_scatter", ctypes.c_float),
                ("scatter_launches", ctypes.c_uint32), ("pass_launches", ctypes.c_uint32),
                ("ms_pass", ctypes.c_float), ("async_launches", ctypes.c_uint16),
                ("async_declined", ctypes.c_uint16),
                ("pass_live", ctypes.c_uint64), ("async_yields", ctypes.c_uint32),
                ("ms_probe_kernel", ctypes.c_float),
                ("prefix_txn", ctypes.c_uint32), ("surv_txn", ctypes.c_uint32),
                ("prefix_acc", ctypes.c_uint64), ("surv_acc", ctypes.c_uint64),
                ("async_live", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class KernelTime(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 48), ("launches", ctypes.c_uint64), ("ms_total", ctypes.c_double)]


class YcsbParams(ctypes.Structure):
    _fields_ = [("synth_table_size", ctypes.c_uint64), ("part_cnt", ctypes.c_uint32),
                ("req_per_query", ctypes.c_uint32), ("zipf_theta", ctypes.c_double),
                ("txn_write_perc", ctypes.c_double), ("tup_write_perc", ctypes.c_double),
                ("part_per_txn", ctypes.c_uint32), ("strict_ppt", ctypes.c_uint32),
                ("mpr", ctypes.c_double)]


class TpccParams(ctypes.Structure):
    _fields_ = [("num_wh", ctypes.c_uint32), ("dist_per_wh", ctypes.c_uint32),
                ("cust_per_dist", ctypes.c_uint32), ("max_items", ctypes.c_uint32),
                ("max_items_per_txn", ctypes.c_uint32), ("part_cnt", ctypes.c_uint32),
                ("part_per_txn", ctypes.c_uint32), ("wh_update", ctypes.c_uint32),
                ("perc_payment", ctypes.c_double), ("mpr", ctypes.c_double)]


TPCC_MAX_OL, TPCC_MAX_PARTS = 62, 64


class TpccItem(ctypes.Structure):  # dv_tpcc_item (Item_no)
    _fields_ = [("ol_i_id", ctypes.c_uint64), ("ol_supply_w_id", ctypes.c_uint64), ("ol_quantity", ctypes.c_uint64)]


class TpccQuery(ctypes.Structure):  # dv_tpcc_query (TPCCQuery / TPCCClientQueryMessage)
    _fields_ = [("txn_type", ctypes.c_uint64), ("w_id", ctypes.c_uint64), ("d_id", ctypes.c_uint64),
                ("c_id", ctypes.c_uint64), ("d_w_id", ctypes.c_uint64), ("c_w_id", ctypes.c_uint64),
                ("c_d_id", ctypes.c_uint64), ("c_last", ctypes.c_char * 16), ("h_amount", ctypes.c_uint64),
                ("by_last_name", ctypes.c_uint8), ("rbk", ctypes.c_uint8), ("remote", ctypes.c_uint8),
                ("pad_", ctypes.c_uint8 * 5), ("ol_cnt", ctypes.c_uint64), ("o_entry_d", ctypes.c_uint64),
                ("n_parts", ctypes.c_uint32), ("pad2_", ctypes.c_uint32),
                ("parts", ctypes.c_uint64 * TPCC_MAX_PARTS), ("items", TpccItem * TPCC_MAX_OL)]


# Deneva wire format (include/dvcc.h)
WIRE_MSG_MAX, WIRE_HDR = 4096, 12
WIRE_CL_QRY, WIRE_RDONE, WIRE_CL_RSP, WIRE_CALVIN_ACK = 3, 19, 20, 24
WIRE_MORE = 1


class WireCfg(ctypes.Structure):
    _fields_ = [("workload", ctypes.c_int32), ("calvin", ctypes.c_uint32), ("node_id", ctypes.c_uint32),
                ("node_cnt", ctypes.c_uint32), ("part_cnt", ctypes.c_uint32), ("max_req", ctypes.c_uint32),
                ("synth_table_size", ctypes.c_uint64), ("tpcc", ctypes.POINTER(TpccParams))]


class WireEpoch(ctypes.Structure):
    _fields_ = [("max_txn", ctypes.c_uint32), ("pad_", ctypes.c_uint32), ("max_acc", ctypes.c_uint64),
                ("keys", ctypes.c_void_p), ("types", ctypes.c_void_p), ("txn_begin", ctypes.c_void_p),
                ("tables", ctypes.c_void_p), ("args", ctypes.c_void_p), ("txn_type", ctypes.c_void_p),
                ("owner", ctypes.c_void_p), ("txn_id", ctypes.c_void_p), ("client_startts", ctypes.c_void_p),
                ("return_node", ctypes.c_void_p), ("n_txn", ctypes.c_uint32), ("rdone", ctypes.c_uint32),
                ("n_acc", ctypes.c_uint64), ("batch_id", ctypes.c_uint64), ("next_txn", ctypes.c_uint64)]


class WireCursor(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_void_p), ("len", ctypes.c_uint64), ("off", ctypes.c_uint64),
                ("left", ctypes.c_uint32), ("src", ctypes.c_uint32)]


# TPC-C table ids and operation words (include/dvcc.h)
T_WAREHOUSE, T_DISTRICT, T_CUSTOMER, T_ITEM, T_STOCK, T_CUST_LAST = 0, 1, 2, 3, 4, 5
TOP_NONE, TOP_PAY_WH, TOP_PAY_DIST, TOP_PAY_CUST, TOP_NO_DIST, TOP_NO_STOCK = 0, 1, 2, 3, 4, 5

# every symbol include/dvcc.h declares: (name, restype, argtypes)
_P = ctypes.POINTER
_vp = ctypes.c_void_p
SIGNATURES = [
    ("dv_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("dv_device_count", ctypes.c_int, [_P(ctypes.c_int)]),
    ("dv_open", ctypes.c_int, [_P(_vp), _P(Config)]),
    ("dv_close", None, [_vp]),
    ("dv_stream", _vp, [_vp]),
    ("dv_own_stream", _vp, [_vp]),
    ("dv_set_stream", ctypes.c_int, [_vp, _vp]),
    ("dv_set_timing", ctypes.c_int, [_vp, ctypes.c_uint32]),
    ("dv_kernel_times", ctypes.c_int, [_vp, _P(KernelTime), ctypes.c_uint32, ctypes.c_int]),
    ("dv_create_table", ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_uint32]),
    ("dv_load_table", ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp, ctypes.c_uint64]),
    ("dv_load_ycsb_partition", ctypes.c_int, [_vp, ctypes.c_uint64]),
    ("dv_read_rows", ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint64, _vp]),
    ("dv_read_table", ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, _vp]),
    ("dv_epoch_run", ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, _vp, _vp,
                                    _P(Stats)]),
    ("dv_epoch_run_device", ctypes.c_int, [_vp, _P(EpochDev), _vp, _vp, _P(Stats)]),
    ("dv_epoch_begin", ctypes.c_int, [_vp, _P(EpochDev), _vp]),
    ("dv_epoch_carry", ctypes.c_int, [_vp, _P(EpochDev), ctypes.c_uint32, _P(EpochDev)]),
    ("dv_epoch_group_carry", ctypes.c_int, [_vp, _P(EpochDev), ctypes.c_uint32, ctypes.c_uint32, _vp,
                                            ctypes.c_uint32, _P(EpochDev)]),
    ("dv_comm_unique_id", ctypes.c_int, [_vp]),
    ("dv_comm_init", ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int]),
    ("dv_comm_init_local", ctypes.c_int, [_P(_vp), ctypes.c_int]),
    ("dv_comm_init_ipc", ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]),
    ("dv_epoch_run_part", ctypes.c_int, [_vp, _P(EpochDev), ctypes.c_uint32, _vp, _P(Stats)]),
    ("dv_epoch_round_local", ctypes.c_int, [_vp, _vp]),
    ("dv_epoch_round_apply", ctypes.c_int, [_vp, _vp, _P(ctypes.c_uint32)]),
    ("dv_epoch_round_wait", ctypes.c_int, [_vp, ctypes.c_uint32, _P(ctypes.c_uint32)]),
    ("dv_epoch_finish", ctypes.c_int, [_vp, _vp, _P(Stats)]),
    ("dv_round_log", ctypes.c_int, [_vp, _P(ctypes.c_uint32), _P(ctypes.c_uint32), ctypes.c_uint32]),
    ("dv_epoch_errors_local", ctypes.c_int, [_vp, _vp]),
    ("dv_epoch_errors_combined", ctypes.c_int, [_vp, _vp]),
    ("dv_set_async_limits", ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32]),
    ("dv_set_prefix", ctypes.c_int, [_vp, ctypes.c_uint32]),
    ("dv_ycsb_gen", ctypes.c_int, [_P(YcsbParams), ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_uint32, _vp, _vp, _vp]),
    ("dv_tpcc_table_rows", ctypes.c_int, [_P(TpccParams), ctypes.c_uint32, ctypes.c_uint32,
                                          _P(ctypes.c_uint64)]),
    ("dv_tpcc_load", ctypes.c_int, [_vp, _P(TpccParams), ctypes.c_uint64]),
    ("dv_tpcc_table", ctypes.c_int, [_P(TpccParams), ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                     _vp, _vp, _vp, _vp]),
    ("dv_tpcc_gen", ctypes.c_int, [_P(TpccParams), ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("dv_tpcc_epoch_begin", ctypes.c_int, [_vp, _P(EpochDev), _vp, _vp]),
    ("dv_tpcc_epoch_run", ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, _vp, _vp,
                                         _P(Stats)]),
    ("dv_load_table_cols", ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, ctypes.c_uint64]),
    ("dv_read_table_col", ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                         ctypes.c_uint64, _vp]),
    ("dv_tpcc_epoch_run_device", ctypes.c_int, [_vp, _P(EpochDev), _vp, _vp, _vp, _P(Stats)]),
    ("dv_tpcc_epoch_run_device_batch", ctypes.c_int, [_vp, _P(EpochDev), _vp, ctypes.c_uint32, _vp, _vp,
                                                      _P(Stats)]),
    ("dv_comm_set_mode", ctypes.c_int, [_vp, ctypes.c_int]),
    ("dv_epoch_run_device_batch", ctypes.c_int, [_vp, _P(EpochDev), ctypes.c_uint32, _P(_vp), _P(Stats)]),
    ("dv_open_lane", ctypes.c_int, [_vp, _P(_vp)]),
    ("dv_lanes_order", ctypes.c_int, [_P(_vp), ctypes.c_uint32]),
    ("dv_epoch_run_closed_loop_lanes", ctypes.c_int,
     [_P(_vp), ctypes.c_uint32, _P(EpochDev), _vp, _vp, ctypes.c_uint32, _P(EpochDev), ctypes.c_uint64,
      ctypes.c_uint32, ctypes.c_int, _P(_vp), _P(Stats)]),
    ("dv_tpcc_epoch_run_device_lanes", ctypes.c_int,
     [_P(_vp), ctypes.c_uint32, _P(EpochDev), _vp, ctypes.c_uint32, _vp, _vp, _P(Stats)]),
    ("dv_epoch_run_device_lanes", ctypes.c_int,
     [_P(_vp), ctypes.c_uint32, _P(EpochDev), ctypes.c_uint32, _P(_vp), _P(Stats)]),
    ("dv_epoch_run_closed_loop", ctypes.c_int, [_vp, _P(EpochDev), _vp, _vp, ctypes.c_uint32, _P(EpochDev),
                                                 ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, _P(_vp),
                                                 _P(Stats)]),
    ("dv_epoch_group_run", ctypes.c_int, [_vp, _P(EpochDev), ctypes.c_uint32, ctypes.c_uint32, _vp, _P(Stats)]),
    ("dv_epoch_group_run_batch", ctypes.c_int, [_vp, _P(EpochDev), ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint32, _P(_vp), _P(Stats)]),
    ("dv_epoch_stage_host", ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32]),
    ("dv_epoch_stage_host_rows", ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32]),
    ("dv_epoch_run_staged", ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, _P(Stats)]),
    ("dv_tpcc_epoch_run_part", ctypes.c_int, [_vp, _P(EpochDev), _vp, _vp, ctypes.c_uint32, _vp, _vp,
                                              _P(Stats)]),
    ("dv_tpcc_gen_queries", ctypes.c_int, [_P(TpccParams), ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                           _P(TpccQuery)]),
    ("dv_tpcc_expand", ctypes.c_int, [_P(TpccParams), _P(TpccQuery), ctypes.c_uint32, ctypes.c_uint64,
                                      _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("dv_wire_epoch_reset", ctypes.c_int, [_P(WireEpoch)]),
    ("dv_wire_open", ctypes.c_int, [_P(WireCfg), _vp, ctypes.c_uint64, _P(WireCursor)]),
    ("dv_wire_decode", ctypes.c_int, [_P(WireCfg), _P(WireCursor), _P(WireEpoch)]),
    ("dv_wire_decode_batches", ctypes.c_int, [_P(WireCfg), _vp, _vp, ctypes.c_uint32, _P(WireCursor),
                                              _P(ctypes.c_uint32), _P(WireEpoch)]),
    ("dv_wire_respond", ctypes.c_int, [_P(WireCfg), _P(WireEpoch), _vp, _vp, ctypes.c_uint64, _vp,
                                       ctypes.c_uint32, _P(ctypes.c_uint32)]),
]

_lib = None


def lib():
    """Loads libdvcc.so; raises if the HIP extension has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libdvcc.so not found at {LIB_PATH}: build it with "
                f"`python deneva-plus_amd/build.py` (there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def source_hash():
    """12 hex digits over the engine's sources (csrc/, include/dvcc.h): ties a
    committed profile (e.g. the PMC traffic of a kernel) to the code it
    measured."""
    import glob
    import hashlib
    h = hashlib.sha256()
    root = os.path.dirname(PKG_DIR)
    files = sorted(glob.glob(os.path.join(PKG_DIR, "csrc", "*"))) + [os.path.join(root, "include", "dvcc.h")]
    for f in files:
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode())
            h.update(fh.read())
    return h.hexdigest()[:12]


def check(rc, what=""):
    if rc != DV_OK:
        raise DvccError(rc, what)
    return rc
