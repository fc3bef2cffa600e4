"""bench.py — propagation steps/s of the 4-level biexciton PT propagator at bond dimension 64.

Workload (BASELINE.json metric; SURVEY.md §8d C3 system, C4 sweep shape, C5 scan structure): each GPU
runs a pulse-area scan of two-time G2(t1, tau) sweeps of the biexciton cascade (N=4, delta_b=4,
lindblad, dt=0.1 ps, pulse train PulseTrain(100, 10, ChirpedPulse(tau_0=3, e_start=-2, e0, t0=12))):
`--scan` pulse areas e0 per GPU (rank r takes scan points [r*scan, (r+1)*scan), e0 = 1 + 0.05 k), each
with the C4 t1 grid of `--t1` points (t1 = 0, 0.1, ... ps). Every (e0, t1) pair is one trajectory
with the MTOs A=|3><1| (right) and C=|1><3| (left) at t1, outputs <B>=<|1><1|> and <ABC> for
tau = 0..1000 ps (n_tau = 10,000). The bath is a chi=64 synthetic PT (I + 0.05 G/sqrt(chi)
per slice, spectral radius <= 1; 410 initial slices + 1 repeated slice; D = N^2 = 16, no dictionary).
Per-GPU work is fixed (weak scaling); there is no data-path collective.

One bench step = one execution of the device-resident plan: free-propagator build for all systems and
half steps + the lock-step PT sweep of every trajectory. Inputs (PT, operators, pulse samples) are
resident in HBM before the timed region. value = whole-job useful trajectory-steps per second
(n_traj * n_tau per GPU; the trunk re-propagation 0 -> t1 (<= 25.5 ps) is executed but not counted).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 (vector == matrix on gfx950), spec
PEAK_HBM_GBS = 8000.0


def build_workload(n_t1, n_tau, chi, scan=1, scan_offset=0, dt=0.1, seed=1234, dictionary=False, t1_offset=0,
                   make_pt=True):
    """(systems, grid, pt, rho0, ops, traj): `scan` pulse-area points x `n_t1` t1 points (t1 steps t1_offset ...);
    make_pt=False leaves the synthetic PT out (pt = None: the caller brings its own)"""
    from pyaceqd_amd import engine, opgrammar, pt as ptmod
    from pyaceqd_amd.constants import hbar
    from pyaceqd_amd.four_level_system.linear import biexciton_ops
    from pyaceqd_amd.pulses import ChirpedPulse, PulseTrain
    N = 4
    so, bo, lo, io, _ = biexciton_ops(delta_b=4, lindblad=True)
    t1_steps = t1_offset + np.arange(n_t1)
    n_steps = int(t1_steps[-1] + n_tau)
    ds = dt / 4
    ts = ds * np.arange(4 * n_steps + 1)
    mat = lambda s: opgrammar.to_matrix(s, N)  # noqa: E731
    H0 = sum(mat(s) for s in so)
    lind = [(r, mat(o)) for o, r in lo]
    systems = []
    for k in range(scan):
        e0 = 1.0 + 0.05 * (scan_offset + k)
        train = PulseTrain(100, 10, ChirpedPulse(tau_0=3, e_start=-2.0, e0=e0, t0=12, polar_x=1.0))
        fx, fy = train.get_total_xy(ts)
        chans = [(-0.5 * np.pi * hbar * mat(op), fx if pol == "x" else fy) for op, pol in io]
        systems.append(engine.System(dim=N, H0=H0, lindblad=lind, channels=chans, sample_t0=0.0, sample_dt=ds))
    grid = engine.Grid(0.0, dt, n_steps, 1)
    pt = ptmod.synthetic_pt(mat(bo), chi=chi, n_init=min(410, n_steps), n_rep=1, seed=seed, eps=0.05, dt=dt,
                            dictionary=dictionary) if make_pt else None
    A, B, Cm = mat("|3><1|_4"), mat("|1><1|_4"), mat("|1><3|_4")
    mtos, beg, end, sysidx = [], [], [], []
    for k in range(scan):
        for t1 in t1_steps:
            t = len(beg)
            mtos.append(engine.MTO(t, int(t1), False, 2, A))
            mtos.append(engine.MTO(t, int(t1), False, 1, Cm))
            beg.append(int(t1))
            end.append(int(t1) + n_tau)
            sysidx.append(k)
    tr = engine.Trajectories(np.array(beg), np.array(end), mtos, system=np.array(sysidx))
    ops = [B, A @ B @ Cm]
    rho0 = mat("|0><0|_4")
    return (systems if scan > 1 else systems[0]), grid, pt, rho0, ops, tr


def flops_per_traj_step(N=4, chi=64, n_out=2, fused=True):
    """F = 8 (D chi^2 + 2 chi N^4 + n_out N^2), D = N^2 PT rows contracted per step. The sweep
    fuses M_b(n-1) and M_a(n) into one N^2 x N^2 operator on steps without MTOs, so the
    executed algorithm does one column product per step: F_fused = 8 (D chi^2 + chi N^4 + n_out N^2)."""
    D = N * N
    if chi <= 1:
        return 8 * ((1 if fused else 2) * N ** 4 + n_out * N * N)
    return 8 * (D * chi * chi + (1 if fused else 2) * chi * N ** 4 + n_out * N * N)


def bytes_per_launch(n_steps, n_init, chi, N=4, n_out=2, n_sys=1, D=16, executed_steps=0):
    """unique HBM bytes one sweep launch must move: every distinct PT slice once; per system and step the fused
    operator F(n) (N^2 x N^2) and the output rows W(n) (n_out x N^2) the sweep reads; the outputs written. The
    augmented states never leave LDS. At the bench config: 411 x 1 MiB + 8 x 10,255 x (4 KiB + 0.5 KiB) + 2 x 16 B
    x 20.48 M = 0.43 + 0.38 + 0.66 = 1.47 GB"""
    slices = min(n_steps, n_init) + 1
    N2 = N * N
    return (slices * D * chi * chi * 16 + n_sys * n_steps * (N2 * N2 + n_out * N2) * 16
            + n_out * 16 * executed_steps)


def pmc_traffic(cfg):
    """HBM bytes per sweep launch from the committed PMC passes (profiles/pmc_traffic.json: FETCH_SIZE x2 +
    WRITE_SIZE, gfx950-corrected) when they were measured on this exact workload; None otherwise"""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None, None
    if any(rec.get("config", {}).get(k) != v for k, v in cfg.items()):
        return None, None
    return float(rec["hbm_bytes_per_launch"]), "profiles/pmc_traffic.json (" + rec.get("passes", "") + ")"


def pmc_mfma(cfg):
    """executed FP64 MFMA flop per sweep launch and the MFMA-busy fraction from the committed SQ counter pass
    (profiles/pmc_mfma.json: SQ_INSTS_VALU_MFMA_MOPS_F64 x 512, SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs) when it
    was measured on this exact workload; None otherwise"""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_mfma.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    if any(rec.get("config", {}).get(k) != v for k, v in cfg.items()):
        return None
    return rec


def host_cpu():
    """what the CPU baseline runs on: model, logical CPUs of the machine, CPUs this process may use (affinity and
    cgroup quota), and whether the reference's ACE binary exists here"""
    import shutil
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0))
    return {"model": model, "nproc": os.cpu_count(), "affinity": aff, "cgroup_cpus": quota,
            "ace_binary": shutil.which("ACE")}


def cpu_threads(info):
    """threads for the CPU baseline: every CPU this process may use. The affinity mask and the cgroup quota bound
    it; when neither does (a GPU box shows the whole multi-GPU machine), the box's documented CPU share per GPU
    (16, the OMP_NUM_THREADS the box exports) is used instead of oversubscribing other tenants' cores."""
    n = info["affinity"]
    if info["cgroup_cpus"]:
        n = min(n, max(1, int(info["cgroup_cpus"])))
    elif n > 64:
        n = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, n)


CPU_BLOCK = 8   # trajectories per lockstep block of the CPU port (oracle/pqd_oracle_blk.c)


def cpu_baseline(chi, target_s=15.0):
    """the CPU port on a bounded sample of the same workload: oracle/pqd_oracle_blk.c (the oracle's algorithm with
    trajectories advanced in lockstep blocks of CPU_BLOCK, so every slice row read serves the whole block; OpenMP
    over blocks), checked against the plain oracle in tests/test_oracle_blocked.py"""
    from oracle import oracle
    info = host_cpu()
    threads = cpu_threads(info)
    unit = threads * CPU_BLOCK        # trajectories per round of blocks over all threads
    # calibrate on the same shape with all threads (setup + free propagators included, as in the sample)
    n_traj = unit
    sysd, grid, pt, rho0, ops, tr = build_workload(n_traj, 300, chi)
    t0 = time.perf_counter()
    oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=threads, blocked=CPU_BLOCK)
    per = (time.perf_counter() - t0) / float(np.sum(tr.out_end + 1))  # seconds per traj-step
    total = target_s / per                                   # traj-steps that fill ~target_s
    steps = int(max(50, min(10000, total / n_traj)))
    n_traj = int(min(4096, max(unit, unit * round(total / steps / unit))))
    sysd, grid, pt, rho0, ops, tr = build_workload(n_traj, steps, chi)
    t0 = time.perf_counter()
    oracle.propagate(sysd, grid, rho0, ops, tr, pt=pt, nthreads=threads, blocked=CPU_BLOCK)
    el = time.perf_counter() - t0
    executed = int(np.sum(tr.out_end + 1))
    return {"value": executed / el, "unit": "traj-steps/s", "cores": threads, "kind": "port", "host": info,
            "sample": f"{n_traj} trajectories x {steps} tau-steps (executed {executed} traj-steps incl. trunk and "
                      f"free-propagator build), chi={chi}, N=4, {el:.1f} s, oracle/pqd_oracle_blk.c OpenMP over "
                      f"lockstep blocks of {CPU_BLOCK} trajectories"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--t1", type=int, default=256, help="t1 points per scan point (C4 grid)")
    ap.add_argument("--scan", type=int, default=8, help="pulse-area scan points per GPU")
    ap.add_argument("--n-tau", type=int, default=10000)
    ap.add_argument("--chi", type=int, default=64)
    ap.add_argument("--pt-dict", type=int, default=0,
                    help="1: dictionary PT (9 slices for the 16 rows, as generated physical PTs have); 0: 16 slices")
    ap.add_argument("--shard", choices=["scan", "t1"], default="scan",
                    help="multi-GPU partition (SURVEY.md §8e): scan = rank r runs scan points [r*scan, (r+1)*scan) with "
                         "the whole t1 grid; t1 = every rank runs the same scan points and its block of a t1 grid of "
                         "t1*world points")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        # nccl (= RCCL over xGMI) on the GPU node; PQD_DIST_BACKEND=gloo rehearses the multi-rank path on one GPU
        backend = os.environ.get("PQD_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    import torch

    from pyaceqd_amd import _lib, engine
    ctx = _lib.context(local)
    from pyaceqd_amd import scan as scanmod
    if args.shard == "t1":
        t1_lo, t1_hi = scanmod.shard_range(args.t1 * world, rank, world)
        sysd, grid, pt, rho0, ops, tr = build_workload(t1_hi - t1_lo, args.n_tau, args.chi, scan=args.scan,
                                                       dictionary=bool(args.pt_dict), t1_offset=t1_lo)
    else:
        sysd, grid, pt, rho0, ops, tr = build_workload(args.t1, args.n_tau, args.chi, scan=args.scan,
                                                       scan_offset=rank * args.scan, dictionary=bool(args.pt_dict))
    n_traj = tr.n_traj
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt, ctx=ctx)

    def barrier():
        if dist is not None:
            if torch.cuda.is_available() and dist.get_backend() == "nccl":
                dist.barrier(device_ids=[local])
            else:
                dist.barrier()

    for _ in range(args.warmup):
        plan.execute()
    plan.synchronize()
    plan.timing(reset=True)
    barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.execute()
    plan.synchronize()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    ms_free, ms_sweep, nexec = plan.timing(reset=True)
    if dist is not None:
        t = torch.tensor([el, ms_sweep, ms_free], dtype=torch.float64,
                         device=f"cuda:{local}" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, ms_sweep, ms_free = [float(x) for x in t.tolist()]

    # the one collective (outside the timed region): every rank's output block gathered to rank 0 in rank order,
    # device buffer to device buffer (RCCL over xGMI point-to-point; scan.gather_tensor); then a finite check of the
    # whole result on rank 0
    t0g = time.perf_counter()
    on_host = dist is not None and dist.get_backend() == "gloo"  # gloo gathers host tensors
    local_out = plan.output_tensor(device="cpu" if on_host else None)
    allout = scanmod.gather_tensor(local_out, dist, dst=0)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    gather_ms = (time.perf_counter() - t0g) * 1e3
    gather = None
    if rank == 0:
        assert bool(torch.isfinite(torch.view_as_real(allout)).all()), "non-finite output"
        gather = {"collective": "gather to rank 0 (send/irecv)" if dist is not None else "none (one rank)",
                  "backend": (dist.get_backend() if dist is not None else None), "values": int(allout.numel()),
                  "bytes": int(allout.numel()) * 16, "ms": gather_ms,
                  "checksum": float(torch.view_as_real(allout).abs().sum())}

    useful = n_traj * args.n_tau
    executed = plan.traj_steps()   # shared trunks (PQD_BRANCH) counted once per workgroup
    value = useful * args.steps * world / el
    fused = os.environ.get("PQD_FUSE", "1") != "0"
    F = flops_per_traj_step(4, args.chi, len(ops), fused=fused)
    achieved_tf = executed * F / (ms_sweep * 1e-3) / 1e12
    wl = {"n_tau": args.n_tau, "traj_per_gpu": n_traj, "chi": args.chi, "scan_points_per_gpu": args.scan,
          "t1_points": args.t1}
    traffic, traffic_src = pmc_traffic(wl)
    algo_bytes = bytes_per_launch(grid.n_steps, 410, args.chi, n_out=len(ops), n_sys=args.scan, executed_steps=executed)
    mf = pmc_mfma(wl)
    line = {
        "metric": "propagation steps/sec (whole node), 4-level biexciton PT bond-dim 64",
        "value": value,
        "unit": "traj-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "c128 (fp64)",
        "data": "synthetic (SURVEY.md §8d: pulse train + synthetic chi=64 PT)",
        "config": {"workload": "biexciton two-time G2 sweep (C3 metric config, C4 shape, C5 scan over ranks)",
                   "N": 4, "chi": args.chi, "D": 16, "dt_ps": 0.1, "n_tau": args.n_tau,
                   "traj_per_gpu": n_traj, "scan_points_per_gpu": args.scan, "t1_points": args.t1,
                   "grid_steps": grid.n_steps,
                   "useful_traj_steps_per_gpu": useful, "executed_traj_steps_per_gpu": executed,
                   "parallelism": f"{args.shard}{world}", "kernel_ms": {"pt_sweep": ms_sweep, "free_prop": ms_free},
                   "gather": gather},
        "roofline": {"bound": "mfma", "achieved": achieved_tf, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved_tf / PEAK_FP64_TFLOPS, "traffic": traffic,
                     "traffic_unit": "HBM bytes per launch", "traffic_source": traffic_src,
                     "kernel": "pt_sweep_kernel<16,64>",
                     "algorithmic": f"{F} flop/traj-step ({'fused' if fused else 'unfused'} half steps) x {executed} "
                                    f"executed traj-steps per launch",
                     "flop_convention": "8 real flops per complex multiply-add (SURVEY.md §8d); with the default 3M "
                                        "products (PQD_PT_MODE=4, PQD_CMUL3=1) the matrix cores execute 6",
                     "hbm_algorithmic_bytes_per_launch": algo_bytes,
                     "hbm_algorithmic_GBs": algo_bytes / (ms_sweep * 1e-3) / 1e9},
    }
    if mf is not None:
        # what the matrix cores actually execute (3M products: 6 real flops per complex MAC), from the counters,
        # priced against this run's kernel time
        line["roofline"]["executed_mfma"] = {
            "flop_per_launch": mf["executed_mfma_flop"],
            "TFLOPs": mf["executed_mfma_flop"] / (ms_sweep * 1e-3) / 1e12,
            "frac": mf["executed_mfma_flop"] / (ms_sweep * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
            "mfma_busy_frac": mf["mfma_busy_frac"], "effective_clock_GHz": mf["effective_clock_GHz"],
            "source": mf["source"]}
    if rank == 0 and world == 1:
        # the reference's single-run case (one trajectory of the same model, chi and length; outside the timed
        # region): a latency figure, carried by N2 split workgroups
        s_sys, s_grid, s_pt, s_rho0, s_ops, s_tr = build_workload(1, args.n_tau, args.chi, scan=1,
                                                                  dictionary=bool(args.pt_dict))
        sp = engine.Plan(s_sys, s_grid, s_rho0, s_ops, s_tr, pt=s_pt, ctx=ctx)
        sp.execute()
        sp.synchronize()
        sp.timing(reset=True)
        for _ in range(3):
            sp.execute()
        sp.synchronize()
        _, s_ms, _ = sp.timing(reset=True)
        sp.download()  # raises on a split timeout that could not be recovered, or on non-finite outputs
        path, bt, fallbacks = sp.info()
        line["single_run"] = {"workload": f"one biexciton G2 trajectory, chi={args.chi}, {args.n_tau} steps",
                              "sweep_ms": s_ms, "us_per_step": s_ms * 1e3 / (args.n_tau + 1),
                              "traj_steps_per_s": (args.n_tau + 1) / (s_ms * 1e-3),
                              "path": path, "split_fallbacks": fallbacks}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.chi, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
