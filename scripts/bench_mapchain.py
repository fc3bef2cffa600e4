"""Throughput of the map-chain kernels (the reference's Fortran sweeps on the GPU) vs the reference's own Fortran.

BASELINE.md: the reference's calc_onetime_parallel (two_time/propagate_tau.f90:110-187) on 256 trajectories x 10,000
tau-steps of synthetic near-identity maps ran at ~1.5e7 traj-steps/s (N=4, 8 threads), ~3.3e6 (N=6), ~2.2e7 (N=2)
in the survey container. Here the same workload runs through pqd_calc_onetime_parallel (GPU: upload, mc_trunk +
mc_tau kernels, download) and through the reference Fortran compiled in oracle/_ref (TEST INFRASTRUCTURE: timed as
the CPU reference on this host), on identical inputs; the two results must agree.
  onetime   calc_onetime_parallel, dims 2 / 4 / 6
  block     calc_onetime_parallel_block (periodic maps + stationary map), dim 4
  ft8       four_time_8op on n_t = 128 t1 points (all (i, j) pairs), dim 4
  tlmap     calc_tl_dynmap_pseudo on 4,000 maps of size 16
usage: python scripts/bench_mapchain.py [--cases onetime,block,ft8,tlmap] [--cpu-threads 16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def _maps(n, dim, seed, eps=2e-3):
    N2 = dim * dim
    rng = np.random.default_rng(seed)
    m = np.eye(N2)[None] + eps * (rng.normal(size=(n, N2, N2)) + 1j * rng.normal(size=(n, N2, N2))) / np.sqrt(N2)
    return np.asfortranarray(m.transpose(1, 2, 0))


def _ops(dim, seed):
    rng = np.random.default_rng(seed)
    return [np.asfortranarray(rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim))) for _ in range(3)]


def _time(fn, reps):
    """median wall time of `reps` calls after one warm-up call (the same statistic for the GPU and the CPU side)"""
    fn()
    ts = []
    for _ in range(reps):
        out = None  # the previous result is released before the clock starts (its unmapping is not the call's)
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), out


def case_onetime(dim, n_t=256, n_tau=10000, reps=5, cpu=True):
    from pyaceqd_amd.two_time import propagate_tau_module as gpu
    dt = 0.1
    n_tfull = n_t + n_tau + 2
    dm = _maps(n_tfull, dim, seed=dim)
    time_full = dt * np.arange(n_tfull)
    time_sparse = time_full[:n_t] + 1e-9  # t1 points on the map grid (staggered by one map each)
    rho0 = np.zeros(dim * dim, complex)
    rho0[0] = 1
    A, B, C = _ops(dim, 7)
    args = (dm, rho0, n_tau, dim, A, B, C, time_full, time_sparse)
    el, got = _time(lambda: gpu.calc_onetime_parallel(*args), reps)
    row = {"case": f"onetime_d{dim}", "n_t": n_t, "n_tau": n_tau, "N2": dim * dim, "gpu_wall_s": el,
           "gpu_traj_steps_per_s": n_t * n_tau / el}

    def cpu_part():
        from oracle import fref
        if fref.available():
            elc, ref = _time(lambda: fref.calc_onetime_parallel(*args), 3)
            row.update(cpu_ref_wall_s=elc, cpu_ref_traj_steps_per_s=n_t * n_tau / elc,
                       max_rel_diff=float(np.max(np.abs(got - ref)) / np.max(np.abs(ref))),
                       speedup=elc / el)
    return row, (cpu_part if cpu else None)


def case_block(dim=4, n_t=256, n_tb=100, nx_tau=100, reps=5, cpu=True):
    from pyaceqd_amd.two_time import propagate_tau_module as gpu
    dt = 0.1
    dm_block = _maps(n_tb, dim, seed=11)
    dm_s = np.asfortranarray(_maps(1, dim, seed=12)[:, :, 0])
    n_tfull = n_t + n_tb + 2
    time_full = dt * np.arange(n_tfull)
    time_sparse = time_full[:n_t] + 1e-9
    rho0 = np.zeros(dim * dim, complex)
    rho0[0] = 1
    A, B, C = _ops(dim, 8)
    args = (dm_block, dm_s, rho0, n_tb, nx_tau, dim, A, B, C, time_full, time_sparse)
    el, got = _time(lambda: gpu.calc_onetime_parallel_block(*args), reps)
    steps = n_t * n_tb * nx_tau
    row = {"case": f"block_d{dim}", "n_t": n_t, "tau_steps": n_tb * nx_tau, "gpu_wall_s": el,
           "gpu_traj_steps_per_s": steps / el}

    def cpu_part():
        from oracle import fref
        if fref.available():
            elc, ref = _time(lambda: fref.calc_onetime_parallel_block(*args), 3)
            row.update(cpu_ref_wall_s=elc, cpu_ref_traj_steps_per_s=steps / elc,
                       max_rel_diff=float(np.max(np.abs(got - ref)) / np.max(np.abs(ref))), speedup=elc / el)
    return row, (cpu_part if cpu else None)


def case_ft8(dim=4, n_t=128, reps=3, cpu=True):
    from pyaceqd_amd.timebin import timebin_tl as gpu
    dt = 0.1
    n_map = 2 * n_t + 10
    dm1, dm2 = _maps(n_map, dim, seed=21), _maps(n_map, dim, seed=22)
    precalc = np.asfortranarray(np.stack([np.linalg.matrix_power(dm1[:, :, -1], 2 ** b) for b in range(12)], axis=2))
    t1 = dt * np.arange(n_t)
    tb = dt * (n_map - 2)
    rho0 = np.zeros(dim * dim, complex)
    rho0[0] = 1
    rng = np.random.default_rng(3)
    ops8 = [np.asfortranarray(rng.normal(size=(dim, dim)) + 1j * rng.normal(size=(dim, dim))) for _ in range(8)]
    fn = lambda: gpu.four_time_8op(dm1, dm2, rho0, t1, precalc, dt, dim, *ops8, False, False, tb)  # noqa: E731
    el, got = _time(fn, reps)
    row = {"case": f"four_time_8op_d{dim}", "n_t": n_t, "pairs": n_t * (n_t + 1) // 2, "gpu_wall_s": el}

    def cpu_part():
        from oracle import fref
        if fref.available():
            elc, ref = _time(lambda: fref.four_time_8op(dm1, dm2, rho0, t1, precalc, dt, dim, ops8, False, False,
                                                        tb), 3)
            row.update(cpu_ref_wall_s=elc, max_rel_diff=float(np.max(np.abs(got - ref)) / np.max(np.abs(ref))),
                       speedup=elc / el)
    return row, (cpu_part if cpu else None)


def case_tlmap(n_maps=4000, N2=16, reps=3, cpu=True):
    from pyaceqd_amd import tools
    dm = np.ascontiguousarray(_maps(n_maps, int(round(np.sqrt(N2))), seed=31, eps=0.05).transpose(2, 0, 1))
    times = 0.1 * np.arange(n_maps + 1)
    el, got = _time(lambda: tools.calc_tl_dynmap_pseudo(dm, times), reps)
    row = {"case": f"tl_dynmap_N2_{N2}", "maps": n_maps, "gpu_wall_s": el, "maps_per_s": n_maps / el}

    def cpu_part():
        t0 = time.perf_counter()
        ref = [dm[0]] + [dm[i] @ np.linalg.pinv(dm[i - 1], rcond=1e-12) for i in range(1, n_maps)]
        elc = time.perf_counter() - t0
        row.update(cpu_numpy_wall_s=elc, speedup=elc / el,
                   max_rel_diff=float(max(np.max(np.abs(a - b)) for a, b in zip(got, ref))))
    return row, (cpu_part if cpu else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="onetime,block,ft8,tlmap")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    os.environ.setdefault("OMP_NUM_THREADS", str(args.cpu_threads))
    cpu = not args.no_cpu
    # every GPU timing first, then the CPU references: the reference's OpenMP threads keep spinning for a while
    # after each call (libomp blocktime) and would take cores from the GPU calls' host side
    done = []
    for c in args.cases.split(","):
        if c == "onetime":
            for d in (2, 4, 6):
                done.append(case_onetime(d, cpu=cpu))
        elif c == "block":
            done.append(case_block(cpu=cpu))
        elif c == "ft8":
            done.append(case_ft8(cpu=cpu))
        elif c == "tlmap":
            done.append(case_tlmap(cpu=cpu))
    for row, cpu_part in done:
        if cpu_part is not None:
            cpu_part()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
