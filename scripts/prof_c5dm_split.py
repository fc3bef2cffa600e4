"""Where the c5dm scan's wall time goes (scripts/bench_configs.py run_c5dm, one warm scan): per-function wall time
summed over the three G2_reuse threads (spec assembly, the driver up to the launch, the launch + table download
inside propagate_table, the tau/t1 integrals). usage: python scripts/prof_c5dm_split.py"""
import collections
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "scripts"))

acc = collections.defaultdict(float)
cnt = collections.Counter()
lock = threading.Lock()
on = {"v": False}


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            if on["v"]:
                with lock:
                    acc[name] += time.perf_counter() - t0
                    cnt[name] += 1
    return w


def main():
    import bench_configs
    import pyaceqd_amd.pol_entanglement.G2 as g2
    import pyaceqd_amd.general_system.general_system as gs
    from pyaceqd_amd import engine
    P = g2.PolarizatzionEntanglement
    P._g2_specs = timed("g2_specs", P._g2_specs)
    P._reuse_integrals = timed("reuse_integrals", P._reuse_integrals)
    P._densitymatrix_from = timed("densitymatrix_from", P._densitymatrix_from)
    gs.propagate_table = timed("propagate_table (launch + download)", gs.propagate_table)
    import pyaceqd_amd.six_level_system.linear as lin
    lin.system_ace_stream = timed("system_ace_stream (driver total)", lin.system_ace_stream)
    engine.split_table = timed("split_table", engine.split_table)
    real_scan = g2.densitymatrix_reuse_scan
    calls = {"n": 0}

    def scan(*a, **k):
        calls["n"] += 1
        if calls["n"] == 2:
            on["v"] = True
            t0 = time.perf_counter()
            r = real_scan(*a, **k)
            print("measured scan wall: %.3f s" % (time.perf_counter() - t0), flush=True)
            on["v"] = False
            return r
        return real_scan(*a, **k)
    g2.densitymatrix_reuse_scan = scan
    bench_configs.run_c5dm(1)
    for k, v in sorted(acc.items(), key=lambda x: -x[1]):
        print(f"{k:40s} {v:8.3f} s summed over threads  ({cnt[k]} calls)")


main()
