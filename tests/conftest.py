import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)



class ScalarLog:
    """A dare_log_t (header + ring) for the scalar drop-ins.

    mode "heap":  a numpy buffer the caller owns; the library stages the
                  bytes each call reads (include/apus_gpu.h).
    mode "owned": apus_log_new (pinned, mapped, library-owned); the kernels
                  read it in place.  free() returns it (apus_log_free).
    `buf` is the byte image, `log` the LogHeader view, `ptr` the address."""

    def __init__(self, pkg, ring_len, mode="heap"):
        import ctypes as C

        import numpy as np
        abi = pkg.abi
        self.lib = abi.load_library()
        self.mode = mode
        hdr = C.sizeof(abi.LogHeader)
        self.hdr = hdr
        if mode == "owned":
            p = C.c_void_p()
            assert self.lib.apus_log_new(ring_len, C.byref(p)) == 0
            self.ptr = p
            self.buf = np.ctypeslib.as_array((C.c_uint8 * (hdr + ring_len)).from_address(p.value))
            self.log = abi.LogHeader.from_address(p.value)
            # log_new's initial offsets
            assert (self.log.len, self.log.end, self.log.tail, self.log.old_end) == (ring_len,) * 4
        else:
            self.buf = np.zeros(hdr + ring_len + 64, np.uint8)
            self.ptr = C.c_void_p(self.buf.ctypes.data)
            self.log = abi.LogHeader.from_buffer(self.buf)
            self.log.len = ring_len

    def load(self, hb, g):
        """group g of a host batch into this log: offsets and ring bytes"""
        st = hb.state[g]
        ln = int(st["len"])
        assert ln == self.log.len
        for k in ("head", "apply", "commit", "end", "tail"):
            setattr(self.log, k, int(st[k]))
        self.buf[self.hdr:self.hdr + ln] = hb.group_ring(g)[:ln]
        return self

    def free(self):
        if self.mode == "owned" and self.ptr is not None:
            assert self.lib.apus_log_free(self.ptr) == 0
        self.ptr = None
        self.buf = self.log = None


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
        # every test returns the logs it allocated with apus_log_new
        import ctypes as C
        import apus_pkg
        lib = apus_pkg.load_package().abi.load_library()
        owned = C.c_uint32(0)
        assert lib.apus_scalar_path_stats(None, None, None, C.byref(owned)) == 0
        assert owned.value == 0, f"{owned.value} apus_log_new logs not freed"
    else:
        yield
