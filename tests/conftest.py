import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Four full GPU runs of this round stopped on an illegal-address fault raised
# by the first host-to-device copies of the first GPU test after
# tests/test_gpu_streams.py, with the device synchronised clean before that
# test and every host registration confirmed released ("The
# illegal-address fault").  What those runs share on the host side: HIP was
# called from 6 Python threads that then exited, and host buffers that had
# been registered were unregistered and freed.  So the threads that call the
# scalar drop-ins live for the whole session (host_pool), the registered
# buffers are kept (keep_host), and glibc is told not to give freed heap
# memory back to the kernel (no munmap / trim below 32 MiB).
HOST_KEEP = []
_POOL = []


def host_pool(n):
    """a thread pool that lives until the process exits (see above)"""
    if not _POOL:
        from concurrent.futures import ThreadPoolExecutor
        _POOL.append(ThreadPoolExecutor(max_workers=n))
    return _POOL[0]


def keep_host(*objs):
    """keep host memory that was registered with the GPU mapped until the end
    of the session (see above); returns the first object"""
    HOST_KEEP.extend(objs)
    return objs[0] if objs else None


def _no_munmap():
    import ctypes
    try:
        libc = ctypes.CDLL("libc.so.6")
        libc.mallopt(-1, 1 << 30)        # M_TRIM_THRESHOLD
        libc.mallopt(-3, 32 << 20)       # M_MMAP_THRESHOLD (glibc's maximum)
    except OSError:
        pass


_no_munmap()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libapus_gpu.so)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def pkg():
    import apus_pkg
    return apus_pkg.load_package()


@pytest.fixture(scope="session")
def orc():
    import apus_pkg
    o = apus_pkg.load_oracle()
    o.lib()
    return o


@pytest.fixture(scope="session")
def ref(orc):
    r = orc.ref()
    if r is None:
        pytest.skip("oracle/_ref not built (reference tree absent on this machine)")
    return r


@pytest.fixture(autouse=True)
def _gpu_sync(request):
    """synchronize the device before and after every GPU test (APUS_TEST_SYNC=0
    turns it off), so an asynchronously reported device fault is charged to
    the test whose work raised it (the teardown of that test fails)"""
    if os.environ.get("APUS_TEST_SYNC", "1") != "0" and request.node.get_closest_marker("gpu"):
        import torch
        torch.cuda.synchronize()
        yield
        torch.cuda.synchronize()
        # every test releases the host logs it mapped, and the runtime confirmed it
        import ctypes as C
        import apus_pkg
        lib = apus_pkg.load_package().abi.load_library()
        live, failed = C.c_uint32(0), C.c_uint32(0)
        lib.apus_host_registrations(C.byref(live), C.byref(failed))
        assert (live.value, failed.value) == (0, 0), f"host registrations live={live.value} failed={failed.value}"
    else:
        yield
