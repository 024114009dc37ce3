"""CPU checks of the C ABI: the library loads, exports every symbol that
include/dvcc.h declares, and its host-side epoch builder reproduces the
oracle's generator bit for bit.  No GPU compute is called here."""
import ctypes
import os
import re

import numpy as np
import pytest

import _oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "dvcc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dv_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_expected_surface():
    syms = _declared_symbols()
    for s in ["dv_open", "dv_close", "dv_epoch_run", "dv_epoch_run_device", "dv_load_table",
              "dv_read_rows", "dv_epoch_begin", "dv_epoch_round_local", "dv_epoch_round_apply",
              "dv_epoch_finish", "dv_ycsb_gen"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from dvcc import _lib
    L = _lib.lib()
    for s in _declared_symbols():
        assert hasattr(L, s), s
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(_declared_symbols()) == bound


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors against the header itself, compiled by gcc."""
    import subprocess
    from dvcc import _lib
    structs = {"dv_access": _lib.Access, "dv_config": _lib.Config, "dv_epoch_dev": _lib.EpochDev,
               "dv_ycsb_params": _lib.YcsbParams, "dv_stats": _lib.Stats, "dv_tpcc_params": _lib.TpccParams,
               "dv_kernel_time": _lib.KernelTime, "dv_tpcc_item": _lib.TpccItem, "dv_tpcc_query": _lib.TpccQuery,
               "dv_wire_cfg": _lib.WireCfg, "dv_wire_epoch": _lib.WireEpoch, "dv_wire_cursor": _lib.WireCursor}
    src = tmp_path / "sz.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "dvcc.h"', "int main(void) {"]
    for name, cls in structs.items():
        lines.append(f'printf("{name} %zu\\n", sizeof({name}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{name}.{f} %zu\\n", offsetof({name}, {f}));')
    lines.append("return 0; }")
    src.write_text("\n".join(lines))
    exe = tmp_path / "sz"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.check_call(["gcc", "-I", inc, str(src), "-o", str(exe)])
    got = dict(line.split() for line in subprocess.check_output([str(exe)]).decode().splitlines())
    for name, cls in structs.items():
        assert int(got[name]) == ctypes.sizeof(cls), name
        for f, _ in cls._fields_:
            assert int(got[f"{name}.{f}"]) == getattr(cls, f).offset, f"{name}.{f}"


def test_strerror():
    from dvcc import _lib
    assert _lib.lib().dv_strerror(-4) == b"key does not exist in the index"


@pytest.mark.parametrize("cfg", [
    dict(table=1 << 16, P=1, theta=0.9, mpr=-1.0, strict=0, ppt=1),
    dict(table=1 << 16, P=1, theta=0.6, mpr=-1.0, strict=0, ppt=1),
    dict(table=(1 << 14) * 8, P=8, theta=0.9, mpr=0.2, strict=1, ppt=2),
    dict(table=(1 << 14) * 4, P=4, theta=0.9, mpr=-1.0, strict=1, ppt=2),
])
def test_product_generator_equals_oracle(cfg):
    from dvcc import YCSBQueryGenerator
    g = YCSBQueryGenerator(cfg["table"], part_cnt=cfg["P"], zipf_theta=cfg["theta"],
                           part_per_txn=cfg["ppt"], strict_ppt=cfg["strict"], mpr=cfg["mpr"])
    p = O.ycsb_params(cfg["table"], part_cnt=cfg["P"], zipf_theta=cfg["theta"],
                      part_per_txn=cfg["ppt"], strict_ppt=cfg["strict"], mpr=cfg["mpr"])
    for home in range(min(cfg["P"], 3)):
        e = g.gen(3000, 11 + home, home)
        k, t, tb = O.ycsb_gen(p, 11 + home, home, 3000)
        assert (e.keys == k).all() and (e.types == t).all() and (e.txn_begin == tb).all()


def test_open_without_device_fails_cleanly():
    from dvcc import _lib
    n = ctypes.c_int(-1)
    rc = _lib.lib().dv_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a GPU is visible")
    ctx = ctypes.c_void_p()
    cfg = _lib.Config(0, 1, 1, 1, 0, 16, 160, 0, 0)
    assert _lib.lib().dv_open(ctypes.byref(ctx), ctypes.byref(cfg)) == _lib.DV_ERR_NO_DEVICE


def test_sequence_orders_batches_by_origin():
    from dvcc import Epoch, sequence
    a = Epoch(np.array([1, 2], np.uint64), np.array([0, 1], np.uint8), np.array([0, 1, 2], np.uint32))
    b = Epoch(np.array([3, 4, 5], np.uint64), np.array([1, 1, 0], np.uint8), np.array([0, 3], np.uint32))
    e = sequence([a, b])
    assert e.keys.tolist() == [1, 2, 3, 4, 5]
    assert e.txn_begin.tolist() == [0, 1, 2, 5]
    assert e.acc_txn().tolist() == [0, 1, 2, 2, 2]
