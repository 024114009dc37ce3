"""The C++ host mirror of the plugin surface (include/dvcc_host.hpp): a Deneva
workload driver's view -- RC, ycsb_request, TPCCQuery, get_lock /
acquire_locks per txn, one epoch per run -- compiled with g++ against the C
ABI.  CPU: the header compiles on its own and the driver binary was built.
GPU: the driver binary (tests/cpp/host_driver_test.cpp) runs YCSB and TPC-C
epochs for every CC algorithm and checks them against the oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "host_driver_test")


def test_header_compiles_standalone():
    src = '#include "dvcc_host.hpp"\nint main() { dvcc_host::EpochRunner r; return r.txn_cnt(); }\n'
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", "-x", "c++", "-I",
                    os.path.join(ROOT, "include"), "-"], input=src.encode(), check=True)


def test_driver_binary_built():
    if not os.path.exists(BIN):
        import __graft_entry__ as g
        g.build_host_test()
    assert os.access(BIN, os.X_OK)


@pytest.mark.gpu
def test_host_driver_parity():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=240)
    print(r.stdout[-3000:], r.stderr[-2000:])
    assert r.returncode == 0 and "ALL PASS" in r.stdout
