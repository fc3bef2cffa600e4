"""Host/GPU time split of the c5dm scan (scripts/bench_configs.py run_c5dm): cProfile of one warm scan, top
functions by cumulative and internal time. usage: python scripts/prof_c5dm.py"""
import cProfile
import os
import pstats
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "scripts"))
import bench_configs  # noqa: E402

pr = cProfile.Profile()
orig = bench_configs.run_c5dm


def main():
    import time
    import pyaceqd_amd.pol_entanglement.G2 as g2
    real = g2.densitymatrix_reuse_scan
    calls = {"n": 0}

    def wrapped(*a, **k):
        calls["n"] += 1
        if calls["n"] == 2:
            t0 = time.perf_counter()
            pr.enable()
            r = real(*a, **k)
            pr.disable()
            print("profiled scan: %.2f s" % (time.perf_counter() - t0), flush=True)
            return r
        return real(*a, **k)
    g2.densitymatrix_reuse_scan = wrapped
    print(orig(1))
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(30)
    st.sort_stats("tottime").print_stats(20)


main()
