"""A mock JNIEnv built with ctypes: a 233-slot JNINativeInterface table whose
GetArrayLength (171), GetByteArrayRegion (200), GetIntArrayRegion (203),
GetFloatArrayRegion (205), SetIntArrayRegion (211), SetFloatArrayRegion (213)
and ExceptionCheck (228) slots are Python callbacks over numpy arrays.  Java
arrays are represented by integer handles (0 = null)."""
import ctypes

import numpy as np

SLOTS = 233

_GETLEN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p)
_GETREG = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p)
_EXC = ctypes.CFUNCTYPE(ctypes.c_uint8, ctypes.c_void_p)


class MockJNIEnv:
    def __init__(self):
        self.arrays: dict[int, np.ndarray] = {}
        self._next = 1
        self.calls: list[str] = []
        self._cbs = [
            _GETLEN(self._get_len),
            _GETREG(self._get_region),
            _GETREG(self._get_region),
            _GETREG(self._get_region),
            _GETREG(self._set_region),
            _GETREG(self._set_region),
            _EXC(lambda env: 0),
        ]
        table = (ctypes.c_void_p * SLOTS)()
        for slot, cb in zip((171, 200, 203, 205, 211, 213, 228), self._cbs):
            table[slot] = ctypes.cast(cb, ctypes.c_void_p)
        self.table = table
        self.table_ptr = ctypes.c_void_p(ctypes.addressof(table))
        self.env = ctypes.pointer(self.table_ptr)  # JNIEnv* -> pointer to the function table

    def new_array(self, a: np.ndarray) -> int:
        h = self._next
        self._next += 1
        self.arrays[h] = a
        return h

    def _get_len(self, env, arr):
        self.calls.append("GetArrayLength")
        return int(self.arrays[arr].size)

    def _get_region(self, env, arr, start, length, buf):
        self.calls.append("GetRegion")
        a = self.arrays[arr]
        ctypes.memmove(buf, a[start:start + length].ctypes.data, length * a.itemsize)

    def _set_region(self, env, arr, start, length, buf):
        self.calls.append("SetFloatArrayRegion" if self.arrays[arr].dtype == np.float32 else "SetIntArrayRegion")
        a = self.arrays[arr]
        ctypes.memmove(a[start:start + length].ctypes.data, buf, length * a.itemsize)
