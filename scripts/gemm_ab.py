#!/usr/bin/env python3
"""A/B the GEMM screen library against a variant build (same C ABI): best TFLOP/s of N screens each."""
import ctypes
import json
import sys

libs = {name: ctypes.CDLL(path) for name, path in (a.split("=", 1) for a in sys.argv[1:])}
out = {}
for size in (4096, 8192):
    for name, lib in libs.items():
        lib.tkg_screen.argtypes = [ctypes.c_int] * 5 + [ctypes.c_longlong, ctypes.POINTER(ctypes.c_double)]
        best = 0.0
        for _ in range(3):
            o = (ctypes.c_double * 7)()
            assert lib.tkg_screen(0, size, size, size, 5, -1, o) == 0
            assert o[2] == 0 and o[3] == 0, list(o)
            best = max(best, o[0])
        out[f"{name}@{size}"] = round(best, 1)
print(json.dumps(out))
