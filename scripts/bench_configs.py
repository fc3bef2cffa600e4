"""Throughput of the PT sweep on the other SURVEY.md §8d configurations (bench.py measures the C3/C4 metric line).

One JSON line per config: executed traj-steps/s, pt_sweep ms per launch (HIP events) and TFLOP/s in SURVEY §8d's
algorithmic flops (fused half steps: F = 8 (D chi^2 + chi N^4 + n_out N^2), D = N^2, no dictionary).
  c1      TLS, N=2, no PT (chi=1), 1,000 steps: a pulse-area scan of 4096 trajectories
  c2      TLS, N=2, synthetic chi=32 PT, 10,000 steps, 2048 trajectories (area scan)
  c3one   biexciton, N=4, chi=64, 10,000 steps, ONE trajectory (the reference's single-run case: latency)
  c2one   TLS, N=2, chi=32, 10,000 steps, one trajectory;  c5one: six-level, N=6, chi=64, one trajectory
  c3eight eight biexciton runs (a small area scan), chi=64, 10,000 steps; c3twenty: twenty; c5eight: eight six-level runs
  c5      six-level linear model, N=6, chi=64, 32 scan points x 64 t1 points = 2048 trajectories, 2,000 tau steps
  c5d     c5 with a dictionary PT (9 slices for the 36 rows, as a generated physical PT has)
  c3d     the bench workload at n_tau = 2,000 with a dictionary PT (9 slices for the 16 rows)
  c4reuse G2_reuse-shaped biexciton sweep (reference pol_entanglement/G2.py:486-497): 8 scan points x 1024 t1 points
          spread over [0, tend), every trajectory from step 0 to tend = 4,096 steps with its MTOs at t1, chi = 64;
          run without (PQD_BRANCH=0) and with shared trunks: executed vs useful traj-steps and wall per launch
  c3one128 the single biexciton run on a chi = 128 dictionary PT (a generated PT's bond cap): split groups of one
          PT row per workgroup (pt_msplit.hip) where the single-trajectory split kernel stops at chi = 64
  c4d128  the bench workload (8 scan points x 256 t1 x 10,000 tau, biexciton) on a synthetic chi = 128 dictionary PT
          (9 slices for the 16 rows: the shape of a generated biexciton PT at the reference parameters)
  c4g     the same workload on a GPU-generated biexciton PT at dt = 0.1 and the reference's biexciton parameters
          (four_level_system/linear.py: t_mem 20.48 -> K = 205, a_e 3 nm, 4 K, threshold 1e-10, bond cap 128): the
          workload the drop-in produces with phonons; c4g2k: n_tau = 2,000
  c4full  SURVEY §8d C4 literally: 256 t1 x 10,000 tau biexciton G2 sweep, chi = 64, one GPU (north star's 10x
          target workload), auto path vs PQD_MSPLIT=0, plus the CPU port on the same trajectories
  c4shard one rank's 32-t1 block of the same sweep split over 8 GPUs (t1 steps 96..127)
  c5dm    C5 as specified: sixls_linear + polarisation-entanglement tomography (calc_densitymatrix_reuse) over an
          e0 x bx grid (2 x {0, 1, 2, 4} points, tests/six_level_linear.py pulse pair, tend 400 ps, dt 0.1 ps, the
          class's t1 grid, chi = 64 dictionary PT), three launches for the whole grid (densitymatrix_reuse_scan)
usage: python scripts/bench_configs.py [--configs c1,c2,c3one,c5] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

PEAK = 78.6


def _xy(p, t):
    if hasattr(p, "get_total_xy"):
        return p.get_total_xy(t)
    f = p.get_total(t)
    return p.polar_x * f, p.polar_y * f


GEN = {}  # generated PTs of this process (c4g, c4g2k share one)


def generated_pt(bo_mat, dt, K=None):
    """the biexciton PT at the reference's parameters (four_level_system/linear.py:8: t_mem 20.48, a_e 3, 4 K,
    threshold 10), generated on the GPU; K overrides the memory (shorter runs)"""
    from pyaceqd_amd import ptgen_gpu
    key = (dt, K)
    if key not in GEN:
        t0 = time.perf_counter()
        pt = ptgen_gpu.qd_phonon_pt_gpu(bo_mat, dt, t_mem=20.48, ae=3.0, temperature=4, threshold=1e-10, K=K)
        GEN[key] = (pt, time.perf_counter() - t0)
    return GEN[key]


def workload(model, n_scan, n_t1, n_tau, chi, dt=0.1, dictionary=False, generated=False, gen_K=None):
    from pyaceqd_amd import engine, opgrammar, pt as ptmod
    from pyaceqd_amd.constants import hbar
    from pyaceqd_amd.pulses import ChirpedPulse, PulseTrain
    if model == "tls":
        N = 2  # tls.py:24-29 strings
        so, bo, lo, io = [], "1.000*|1><1|_2", [["|0><1|_2", 1 / 100]], [["|1><0|_2", "x"]]
        A, B, C = "|1><0|_2", "|1><1|_2", "|0><1|_2"
        mk = lambda e0: ChirpedPulse(tau_0=3, e_start=0, e0=e0, t0=20)  # noqa: E731
    elif model == "biexciton":
        from pyaceqd_amd.four_level_system.linear import biexciton_ops
        N = 4
        so, bo, lo, io, _ = biexciton_ops(delta_b=4, lindblad=True)
        A, B, C = "|3><1|_4", "|1><1|_4", "|1><3|_4"
        mk = lambda e0: PulseTrain(100, 10, ChirpedPulse(tau_0=3, e_start=-2.0, e0=e0, t0=12, polar_x=1.0))  # noqa
    else:
        from pyaceqd_amd.six_level_system.linear import energies_linear, sixls_ops
        N = 6
        so, bo, lo, io, _ = sixls_ops(delta_b=4, lindblad=True, bx=1.0)
        E_X, _, _, _, E_B = energies_linear(delta_B=4)
        A, B, C = "|5><1|_6", "|1><1|_6", "|1><5|_6"

        class _Two:  # tests/six_level_linear.py:6-8 pulse pair, e0 of the first pulse scanned
            def __init__(self, e0):
                self.p = [ChirpedPulse(tau_0=2.7, e_start=E_X, alpha=40, e0=e0),
                          ChirpedPulse(tau_0=2.7, e_start=E_B - E_X, alpha=40, e0=4.06, t0=120)]

            def get_total_xy(self, t):
                xs = [_xy(p, t) for p in self.p]
                return sum(x for x, _ in xs), sum(y for _, y in xs)
        mk = _Two
    mat = lambda s: opgrammar.to_matrix(s, N)  # noqa: E731
    n_steps = (n_t1 - 1) + n_tau
    ds = dt / 4
    ts = ds * np.arange(4 * n_steps + 1)
    H0 = sum((mat(s) for s in so), np.zeros((N, N), complex))
    lind = [(r, mat(o)) for o, r in lo if r != 0]
    systems = []
    for k in range(n_scan):
        fx, fy = _xy(mk(1.0 + 5.0 * k / max(1, n_scan)), ts)
        chans = [(-0.5 * np.pi * hbar * mat(op), fx if pol == "x" else fy) for op, pol in io]
        systems.append(engine.System(dim=N, H0=H0, lindblad=lind, channels=chans, sample_t0=0.0, sample_dt=ds))
    grid = engine.Grid(0.0, dt, n_steps, 1)
    pt = None
    if generated:
        pt, _ = generated_pt(mat(bo), dt, gen_K)
    elif chi > 1:
        pt = ptmod.synthetic_pt(mat(bo), chi=chi, n_init=min(410, n_steps), n_rep=1, seed=1234, eps=0.05, dt=dt,
                               dictionary=dictionary)
    mtos, beg, end, sysidx = [], [], [], []
    for k in range(n_scan):
        for t1 in range(n_t1):
            t = len(beg)
            if n_t1 > 1:
                mtos.append(engine.MTO(t, t1, False, 2, mat(A)))
                mtos.append(engine.MTO(t, t1, False, 1, mat(C)))
            beg.append(t1 if n_t1 > 1 else 0)
            end.append(t1 + n_tau)
            sysidx.append(k)
    tr = engine.Trajectories(np.array(beg), np.array(end), mtos, system=np.array(sysidx))
    ops = [mat(B), mat(A) @ mat(B) @ mat(C)]
    rho0 = mat("|0><0|_%d" % N)
    return N, (systems if n_scan > 1 else systems[0]), grid, pt, rho0, ops, tr


CONFIGS = {
    "c1": dict(model="tls", n_scan=4096, n_t1=1, n_tau=1000, chi=1),
    "c2": dict(model="tls", n_scan=2048, n_t1=1, n_tau=10000, chi=32),
    "c3one": dict(model="biexciton", n_scan=1, n_t1=1, n_tau=10000, chi=64),
    "c2one": dict(model="tls", n_scan=1, n_t1=1, n_tau=10000, chi=32),
    "c2x64": dict(model="tls", n_scan=2048, n_t1=1, n_tau=10000, chi=64),
    "c5one": dict(model="sixls", n_scan=1, n_t1=1, n_tau=10000, chi=64),
    "c3eight": dict(model="biexciton", n_scan=8, n_t1=1, n_tau=10000, chi=64),
    "c3twenty": dict(model="biexciton", n_scan=20, n_t1=1, n_tau=10000, chi=64),
    "c5eight": dict(model="sixls", n_scan=8, n_t1=1, n_tau=10000, chi=64),
    "c5": dict(model="sixls", n_scan=32, n_t1=64, n_tau=2000, chi=64),
    "c5d": dict(model="sixls", n_scan=32, n_t1=64, n_tau=2000, chi=64, dictionary=True),
    "c3d": dict(model="biexciton", n_scan=8, n_t1=256, n_tau=2000, chi=64, dictionary=True),
    "c4d128": dict(model="biexciton", n_scan=8, n_t1=256, n_tau=10000, chi=128, dictionary=True),
    "c3one128": dict(model="biexciton", n_scan=1, n_t1=1, n_tau=10000, chi=128, dictionary=True),
    "c4d128s": dict(model="biexciton", n_scan=8, n_t1=256, n_tau=2000, chi=128, dictionary=True),
    "c4g": dict(model="biexciton", n_scan=8, n_t1=256, n_tau=10000, chi=128, generated=True),
    "c4g2k": dict(model="biexciton", n_scan=8, n_t1=256, n_tau=2000, chi=128, generated=True),
}


def run(name, steps):
    from pyaceqd_amd import engine
    cfg = CONFIGS[name]
    N, sysd, grid, pt, rho0, ops, tr = workload(**cfg)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    plan.execute()
    plan.synchronize()
    plan.timing(reset=True)
    t0 = time.perf_counter()
    for _ in range(steps):
        plan.execute()
    plan.synchronize()
    el = (time.perf_counter() - t0) / steps
    ms_free, ms_sweep, _ = plan.timing(reset=True)
    res = plan.download()
    assert all(np.all(np.isfinite(r)) for r in res), "non-finite output"
    executed = int(np.sum(tr.out_end + 1))
    chi = pt.chi if pt is not None else cfg["chi"]
    extra = {}
    if cfg.get("generated"):
        _, gen_s = generated_pt(None, cfg.get("dt", 0.1), cfg.get("gen_K"))
        extra = {"pt_chi": pt.chi, "pt_D": pt.D, "pt_slices": pt.n_slices, "pt_gen_s": gen_s,
                 "pt_K": (pt.meta or {}).get("K")}
    F = 8 * (N * N * chi * chi + chi * N ** 4 + len(ops) * N * N) if chi > 1 else 8 * (N ** 4 + len(ops) * N * N)
    tf = executed * F / (ms_sweep * 1e-3) / 1e12
    return {"config": name, **cfg, "N": N, "n_traj": tr.n_traj, "executed_traj_steps": executed,
            "path": plan.info()[0], "traj_per_group_or_block": plan.info()[1],
            "wall_ms_per_launch": el * 1e3, "pt_sweep_ms": ms_sweep, "free_prop_ms": ms_free,
            "traj_steps_per_s": executed / el, "flop_per_traj_step": F, "sweep_TFLOPs": tf, "frac_fp64": tf / PEAK,
            **extra}


def run_c4reuse(steps, n_scan=8, n_t1=1024, n_steps=4096, chi=64):
    import bench
    from pyaceqd_amd import engine
    systems, grid, pt, rho0, ops, tr = bench.build_workload(1, n_steps, chi, scan=n_scan)
    # the same systems and PT on a G2_reuse grid: t1 = k * n_steps / n_t1, windows [t1, tend], MTOs at t1
    A, Cm = [m.op for m in tr.mtos[:2]]
    t1s = (np.arange(n_t1) * n_steps) // n_t1
    mtos, beg, end, sysidx = [], [], [], []
    for k in range(n_scan):
        for t1 in t1s:
            t = len(beg)
            mtos += [engine.MTO(t, int(t1), False, 2, A), engine.MTO(t, int(t1), False, 1, Cm)]
            beg.append(int(t1))
            end.append(n_steps)
            sysidx.append(k)
    tr = engine.Trajectories(np.array(beg), np.array(end), mtos, system=np.array(sysidx))
    grid = engine.Grid(0.0, grid.dt, n_steps, 1)
    useful = int(np.sum(tr.out_end - tr.out_begin + 1))
    row = {"config": "c4reuse", "n_traj": tr.n_traj, "n_steps": n_steps, "chi": chi,
           "useful_traj_steps": useful, "unshared_traj_steps": int(tr.n_traj * (n_steps + 1))}
    ref = None
    for mode in ("0", "1"):
        os.environ["PQD_BRANCH"] = mode
        plan = engine.Plan(systems, grid, rho0, ops, tr, pt=pt)
        os.environ.pop("PQD_BRANCH")
        plan.execute()
        plan.synchronize()
        plan.timing(reset=True)
        t0 = time.perf_counter()
        for _ in range(steps):
            plan.execute()
        plan.synchronize()
        el = (time.perf_counter() - t0) / steps
        ms_free, ms_sweep, _ = plan.timing(reset=True)
        out = np.concatenate([r.ravel() for r in plan.download()])
        if ref is None:
            ref = out
        row["shared" if mode == "1" else "unshared"] = {
            "executed_traj_steps": plan.traj_steps(), "wall_ms_per_launch": el * 1e3, "sweep_ms": ms_sweep,
            "free_prop_ms": ms_free, "useful_traj_steps_per_s": useful / el,
            "max_rel_diff_vs_unshared": float(np.max(np.abs(out - ref)) / np.max(np.abs(ref)))}
    return row


def run_c4_literal(steps, n_t1=256, t1_offset=0, name="c4full", cpu=True):
    """SURVEY §8d C4 as the north star defines it: one biexciton G2(t1, tau) sweep, n_t1 t1 points (t1 = 0.1 ps
    steps from t1_offset) x 10,000 tau steps, chi = 64, the bench PT (bench.build_workload, one scan point).
    c4full = the whole 256-point grid on one GPU; c4shard = one rank's 32-point block of the 8-GPU split
    (t1_offset = 96: rank 3). Timed on the automatic path and, for comparison, with the multi-trajectory split
    groups off (PQD_MSPLIT=0, the previous chooser); the CPU port (oracle/pqd_oracle_blk.c, OpenMP over lockstep
    blocks of 8) on the same trajectories"""
    import bench
    from pyaceqd_amd import engine
    sysd, grid, pt, rho0, ops, tr = bench.build_workload(n_t1, 10000, 64, t1_offset=t1_offset)
    executed = int(np.sum(tr.out_end + 1))
    useful = int(tr.n_traj * 10000)
    row = {"config": name, "n_t1": n_t1, "t1_offset": t1_offset, "n_tau": 10000, "chi": 64, "N": 4,
           "grid_steps": grid.n_steps, "executed_traj_steps": executed, "useful_traj_steps": useful}
    ref = None
    for label, env in (("auto", {}), ("no_msplit", {"PQD_MSPLIT": "0"})):
        for k, v in env.items():
            os.environ[k] = v
        plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
        for k in env:
            os.environ.pop(k)
        plan.execute()
        plan.synchronize()
        plan.timing(reset=True)
        t0 = time.perf_counter()
        for _ in range(steps):
            plan.execute()
        plan.synchronize()
        el = (time.perf_counter() - t0) / steps
        ms_free, ms_sweep, _ = plan.timing(reset=True)
        out = np.concatenate([r.ravel() for r in plan.download()])
        path, bt, fb = plan.info()
        if ref is None:
            ref = out
        row[label] = {"path": path, "traj_per_group_or_block": bt, "split_fallbacks": fb,
                      "wall_ms_per_launch": el * 1e3, "sweep_ms": ms_sweep, "free_prop_ms": ms_free,
                      "traj_steps_per_s": executed / el, "useful_traj_steps_per_s": useful / el,
                      "us_per_grid_step": ms_sweep * 1e3 / (grid.n_steps + 1),
                      "max_rel_diff_vs_auto": float(np.max(np.abs(out - ref)) / np.max(np.abs(ref)))}
    if cpu:
        info = bench.host_cpu()
        threads = bench.cpu_threads(info)
        from oracle import oracle
        t0 = time.perf_counter()
        cres = oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=threads, blocked=bench.CPU_BLOCK)
        cel = time.perf_counter() - t0
        cout = np.concatenate([r.ravel() for r in cres])
        row["cpu_port"] = {"wall_s": cel, "threads": threads, "blocks_of": bench.CPU_BLOCK,
                           "busy_threads": min(threads, (tr.n_traj + bench.CPU_BLOCK - 1) // bench.CPU_BLOCK),
                           "traj_steps_per_s": executed / cel,
                           "max_rel_diff_vs_gpu": float(np.max(np.abs(cout - ref)) / np.max(np.abs(ref)))}
        row["gpu_vs_cpu_wall"] = cel / (row["auto"]["wall_ms_per_launch"] * 1e-3)
    return row


def run_c4_ntraj(steps, n_tau=2000, sizes=(16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512)):
    """where the multi-trajectory split groups stop paying: the C4 sweep shape (bench.build_workload, one scan point,
    chi = 64, n_tau = 2,000) at growing t1 counts, on split groups forced (PQD_MSPLIT=2, past the auto cutoff) and on
    the batched kernel (PQD_MSPLIT=0); sweep ms per launch and the path each took"""
    import bench
    from pyaceqd_amd import engine
    rows = []
    for n in sizes:
        sysd, grid, pt, rho0, ops, tr = bench.build_workload(n, n_tau, 64)
        row = {"n_traj": n, "grid_steps": grid.n_steps}
        for label, env in (("msplit", {"PQD_MSPLIT": "2"}), ("auto", {}), ("batched", {"PQD_MSPLIT": "0"})):
            for k, v in env.items():
                os.environ[k] = v
            try:
                plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
            finally:
                for k in env:
                    os.environ.pop(k)
            plan.execute()
            plan.synchronize()
            plan.timing(reset=True)
            for _ in range(steps):
                plan.execute()
            plan.synchronize()
            _, ms, _ = plan.timing(reset=True)
            path, bt, _ = plan.info()
            row[label] = {"path": path, "bt": bt, "sweep_ms": ms, "us_per_step": ms * 1e3 / (grid.n_steps + 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    return {"config": "c4ntraj", "n_tau": n_tau, "rows": len(rows)}


def run_msx(steps, n_tau=1000, sizes=(16, 32, 64, 128, 256)):
    """the split-groups / batched crossover for the six-level model (N2 = 36, 18 workgroups of two rows per group):
    `workload("sixls", ...)` with the t1 points of one scan point, chi = 64, on split groups forced (PQD_MSPLIT=2), in
    auto mode and on the batched kernel (PQD_MSPLIT=0); us per grid step and the path taken"""
    from pyaceqd_amd import engine
    for n in sizes:
        _, sysd, grid, pt, rho0, ops, tr = workload("sixls", 1, n, n_tau, 64)
        row = {"model": "sixls", "n_traj": n, "grid_steps": grid.n_steps}
        for label, env in (("msplit", {"PQD_MSPLIT": "2"}), ("auto", {}), ("batched", {"PQD_MSPLIT": "0"})):
            for k, v in env.items():
                os.environ[k] = v
            try:
                plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
            finally:
                for k in env:
                    os.environ.pop(k)
            plan.execute()
            plan.synchronize()
            plan.timing(reset=True)
            for _ in range(steps):
                plan.execute()
            plan.synchronize()
            _, ms, _ = plan.timing(reset=True)
            path, bt, _ = plan.info()
            row[label] = {"path": path, "bt": bt, "us_per_step": ms * 1e3 / (grid.n_steps + 1)}
        print(json.dumps(row), flush=True)
    return {"config": "msx", "n_tau": n_tau}


def run_c5dm(steps, n_e0=2, bxs=(0.0, 1.0, 2.0, 4.0), tend=400.0):
    import tempfile
    from pyaceqd_amd import opgrammar, pt as ptmod
    from pyaceqd_amd.pol_entanglement.G2 import PolarizatzionEntanglement, densitymatrix_reuse_scan
    from pyaceqd_amd.pulses import ChirpedPulse
    from pyaceqd_amd.six_level_system.linear import energies_linear, sixls_linear, sixls_ops
    E_X, _, _, _, E_B = energies_linear(delta_B=4)
    pt = ptmod.synthetic_pt(opgrammar.to_matrix(sixls_ops()[1], 6), chi=64, n_init=410, n_rep=1, seed=1234,
                            eps=0.05, dt=0.1, dictionary=True)
    tmp = tempfile.mkdtemp() + "/"
    insts, kws = [], []
    for e0 in np.linspace(1, 10, 64)[:: 64 // n_e0][:n_e0]:
        for bx in bxs:
            p1 = ChirpedPulse(tau_0=2.7, e_start=E_X, alpha=40, e0=e0)
            p2 = ChirpedPulse(tau_0=2.7, e_start=E_B - E_X, alpha=40, e0=4.06, t0=120)
            opts = {"lindblad": True, "gamma_e": 1 / 100, "phonons": True, "pt_file": pt, "temp_dir": tmp}
            insts.append(PolarizatzionEntanglement(sixls_linear, "|0><1|_6 + |1><5|_6", "|0><2|_6 + |2><5|_6",
                                                   "|1><0|_6 + |5><1|_6", "|2><0|_6 + |5><2|_6", p1, p2, dt=0.1,
                                                   tend=tend, options=opts))
            kws.append({"bx": bx})
    densitymatrix_reuse_scan(insts, kws)  # warm-up (PT upload, kernels)
    t0 = time.perf_counter()
    for _ in range(steps):
        conc = densitymatrix_reuse_scan(insts, kws)
    el = (time.perf_counter() - t0) / steps
    n_traj = 3 * sum(len(x.t1) for x in insts)
    n_tau = int(round(tend / 0.1))
    executed = 3 * sum(int(np.sum(n_tau + 1 - np.minimum(n_tau, (np.asarray(x.t1) / 0.1).astype(int))))
                       for x in insts)
    return {"config": "c5dm" if len(insts) == 8 else f"c5dm{len(insts)}", "model": "sixls", "points": len(insts), "e0": n_e0, "bx": list(bxs), "tend": tend,
            "chi": 64, "N": 6, "n_out": "6/8/6", "launches": 3, "n_traj": n_traj,
            "output_traj_steps": executed, "wall_s_per_scan": el, "points_per_s": len(insts) / el,
            "output_traj_steps_per_s": executed / el, "concurrence": [float(c) for c in conc]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2,c3one,c5")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    for name in args.configs.split(","):
        # c5dm32: one rank's share of SURVEY §8d C5 (256 points = 64 e0 x 4 bx over 8 GPUs): 8 e0 x 4 bx
        special = {"c5dm": run_c5dm, "c4reuse": run_c4reuse, "c5dm32": lambda st: run_c5dm(st, n_e0=8),
                   "c4full": run_c4_literal, "c4ntraj": run_c4_ntraj, "msx": run_msx,
                   "c4shard": lambda st: run_c4_literal(st, n_t1=32, t1_offset=96, name="c4shard")}
        print(json.dumps(special[name](args.steps) if name in special else run(name, args.steps)), flush=True)


if __name__ == "__main__":
    main()
