"""rdma-paxos_amd: MI355X-native engine for the APUS (DARE) quorum/commit hot path.

The product is the C-ABI library csrc/ -> libapus_gpu.so (hand-written HIP for
gfx950).  This package is the Python host-side plumbing around it: a ctypes
mirror of include/apus_gpu.h (abi), group-major batch containers (batch) and
reference-named wrappers (engine).  The directory name contains a hyphen, so
import it through load_package() / importlib as `rdma_paxos_amd`.
"""
from . import abi, batch, shard  # noqa: F401
from .abi import load_library  # noqa: F401


def Engine(*a, **k):  # lazy: importing torch is only needed for device work
    from .engine import Engine as _E
    return _E(*a, **k)
