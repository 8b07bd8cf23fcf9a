"""Run rp_selftest_prims (sort + scan self-check, timed pair sorts) for one size, for a
rocprofv3 kernel trace:  rocprofv3 --kernel-trace --stats -d gpurun_out/pp -- python3 tools/prims_prof.py N BITS MODE REPS"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_pkg  # noqa: E402

rpa = load_pkg()
n, bits, mode, reps = (int(x) for x in sys.argv[1:5])
f = rpa.lib().rp_selftest_prims
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
              ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_float)]
bad, ms = ctypes.c_uint64(), ctypes.c_float()
rpa.check(f(n, 5, bits, 0, mode, reps, ctypes.byref(bad), ctypes.byref(ms)))
print("n %d bits %d mode %d bad %d sort_ms %.4f" % (n, bits, mode, bad.value, ms.value))
