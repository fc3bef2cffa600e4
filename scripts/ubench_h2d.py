"""Host<->device copy paths for the map-chain boundary (the f2py-shaped calls hand host numpy buffers: ~42 MB of
maps in and ~41 MB of results out at the C4 shape, N^2 = 16). Times, on the GPU box, per direction and size:
  pageable   hipMemcpy from / to an ordinary numpy buffer (the runtime stages it)
  register   hipHostRegister(buffer) + hipMemcpy + hipHostUnregister (the pinning cost included)
  pinned     hipMemcpy from / to a hipHostMalloc buffer (what a context-owned staging buffer reaches), plus a
             host memcpy into / out of it (numpy copyto) timed separately
usage: python scripts/ubench_h2d.py [--mb 42,212]
"""
import argparse
import ctypes as C
import json
import time

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", default="4,42,212")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    hip = C.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
    hip.hipHostUnregister.argtypes = [C.c_void_p]
    hip.hipFree.argtypes = [C.c_void_p]
    hip.hipHostFree.argtypes = [C.c_void_p]
    hip.hipDeviceSynchronize.argtypes = []

    def ok(rc):
        assert rc == 0, rc

    for mb in [int(x) for x in args.mb.split(",")]:
        n = mb * 1000 * 1000
        host = np.ones(n // 8, dtype=np.float64)
        dev = C.c_void_p()
        ok(hip.hipMalloc(C.byref(dev), n))
        pin = C.c_void_p()
        ok(hip.hipHostMalloc(C.byref(pin), n, 0))
        pin_np = np.ctypeslib.as_array(C.cast(pin, C.POINTER(C.c_double)), shape=(n // 8,))
        hp = host.ctypes.data_as(C.c_void_p)
        row = {"MB": mb}
        for name, kind in (("h2d", 1), ("d2h", 2)):
            def cp(src_host):
                if kind == 1:
                    ok(hip.hipMemcpy(dev, src_host, n, 1))
                else:
                    ok(hip.hipMemcpy(src_host, dev, n, 2))
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter(); cp(hp); ts.append(time.perf_counter() - t0)
            row[f"{name}_pageable_ms"] = 1e3 * min(ts)
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                ok(hip.hipHostRegister(hp, n, 0))
                cp(hp)
                ok(hip.hipHostUnregister(hp))
                ts.append(time.perf_counter() - t0)
            row[f"{name}_register_ms"] = 1e3 * min(ts)
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter(); ok(hip.hipHostRegister(hp, n, 0)); ts.append(time.perf_counter() - t0)
                ok(hip.hipHostUnregister(hp))
            row[f"register_only_ms"] = 1e3 * min(ts)
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter(); cp(pin); ts.append(time.perf_counter() - t0)
            row[f"{name}_pinned_ms"] = 1e3 * min(ts)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter(); np.copyto(pin_np, host); ts.append(time.perf_counter() - t0)
        row["host_memcpy_into_pinned_ms"] = 1e3 * min(ts)
        # what an f2py-style call pays: the result array is new (np.zeros: untouched pages, faulted in by the copy)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fresh = np.zeros(n // 8, dtype=np.float64)
            ok(hip.hipMemcpy(fresh.ctypes.data_as(C.c_void_p), dev, n, 2))
            ts.append(time.perf_counter() - t0)
            del fresh
        row["d2h_fresh_zeros_ms"] = 1e3 * min(ts)
        for k in list(row):
            if k.endswith("_ms") and k != "register_only_ms":
                row[k.replace("_ms", "_GBs")] = n / (row[k] * 1e-3) / 1e9
        print(json.dumps(row), flush=True)
        hip.hipFree(dev)
        hip.hipHostFree(pin)


if __name__ == "__main__":
    main()
