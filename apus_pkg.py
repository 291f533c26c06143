"""Import helpers for the repo's two native libraries.

`rdma-paxos_amd/` (the product package) has a hyphen in its name, so it is
loaded by path as module `rdma_paxos_amd`.  The oracle (test infrastructure
only) is loaded by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg through oracle/oracle.py.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "rdma-paxos_amd")


def load_package():
    if "rdma_paxos_amd" in sys.modules:
        return sys.modules["rdma_paxos_amd"]
    spec = importlib.util.spec_from_file_location(
        "rdma_paxos_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["rdma_paxos_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from oracle import oracle as o  # noqa: E402
    return o
