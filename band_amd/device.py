"""Device buffers and streams over the thin C ABI (no torch needed).

Used by the Python mirror of the backend, by bench.py and by the GPU tests.
"""
import ctypes

import numpy as np

from . import _abi


class Stream:
    def __init__(self):
        self.lib = _abi.load()
        h = ctypes.c_void_p()
        _abi.check(self.lib.bh_stream_create(ctypes.byref(h)), "bh_stream_create")
        self.handle = h

    def sync(self):
        _abi.check(self.lib.bh_stream_sync(self.handle), "bh_stream_sync")

    def close(self):
        if self.handle:
            self.lib.bh_stream_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBuffer:
    """A hipMalloc'ed byte buffer."""

    def __init__(self, nbytes):
        self.lib = _abi.load()
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        _abi.check(self.lib.bh_malloc(ctypes.byref(p), max(self.nbytes, 16)), "bh_malloc")
        self.ptr = p

    @classmethod
    def from_array(cls, a):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a)
        return b

    def upload(self, a):
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        _abi.check(self.lib.bh_memcpy_h2d(self.ptr, a.ctypes.data_as(ctypes.c_void_p), a.nbytes), "h2d")

    def download(self, dtype, shape):
        out = np.empty(shape, dtype)
        assert out.nbytes <= self.nbytes
        _abi.check(self.lib.bh_memcpy_d2h(out.ctypes.data_as(ctypes.c_void_p), self.ptr, out.nbytes), "d2h")
        return out

    @property
    def value(self):
        return self.ptr.value

    def free(self):
        if self.ptr:
            self.lib.bh_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def device_count():
    lib = _abi.load()
    n = ctypes.c_int(0)
    lib.bh_device_count(ctypes.byref(n))
    return n.value


def device_arch(ordinal=0):
    lib = _abi.load()
    buf = ctypes.create_string_buffer(128)
    _abi.check(lib.bh_device_arch(ordinal, buf, 128), "bh_device_arch")
    return buf.value.decode()
