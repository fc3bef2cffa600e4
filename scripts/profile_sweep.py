"""Ablation timing of the PT sweep kernel in one process (interleaved rounds, HIP-event kernel times).

PQD_ABLATE bits (diagnostic builds of the same kernel, outputs wrong by construction):
  1 skip PT contraction, 2 skip the free-propagator column phases, 4 skip outputs.
usage: python scripts/profile_sweep.py [--traj 1024] [--n-tau 2000] [--chi 64] [--rounds 3]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--traj", type=int, default=1024)
    ap.add_argument("--n-tau", type=int, default=2000)
    ap.add_argument("--chi", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0,1,2,4,3,5,6,7")
    ap.add_argument("--pt-modes", default="1", help="PQD_PT_MODE values to cross with the ablations")
    ap.add_argument("--fuse-modes", default="1", help="PQD_FUSE values to cross with the ablations")
    ap.add_argument("--config", default=None, help="a scripts/bench_configs.py config instead of the bench workload")
    ap.add_argument("--scan", type=int, default=None, help="with --config: override its scan points")
    ap.add_argument("--env", default="", help="';'-separated environment variants ('A=1 B=0;A=0') crossed with the rest")
    args = ap.parse_args()
    import bench
    from pyaceqd_amd import engine
    N = 4
    if args.config:
        sys.path.insert(0, os.path.join(HERE, "scripts"))
        import bench_configs
        cfg = dict(bench_configs.CONFIGS[args.config], n_tau=args.n_tau)
        if args.scan:
            cfg["n_scan"] = args.scan
        args.chi = cfg["chi"]
        N, sysd, grid, pt, rho0, ops, tr = bench_configs.workload(**cfg)
        args.traj = tr.n_traj
    else:
        sysd, grid, pt, rho0, ops, tr = bench.build_workload(args.traj, args.n_tau, args.chi)
    plans = {}
    envs = [e.strip() for e in args.env.split(";")] if args.env else [""]
    for ev in envs:
        kv = dict(x.split("=", 1) for x in ev.split()) if ev else {}
        for fm in [int(x) for x in args.fuse_modes.split(",")]:
            for pm in [int(x) for x in args.pt_modes.split(",")]:
                for ab in [int(x) for x in args.variants.split(",")]:
                    os.environ["PQD_ABLATE"] = str(ab)
                    os.environ["PQD_PT_MODE"] = str(pm)
                    os.environ["PQD_FUSE"] = str(fm)
                    os.environ.update(kv)
                    tag = (ev.replace(" ", ",") + "/") if ev else ""
                    plans[f"{tag}fuse{fm}/pt{pm}/ab{ab}"] = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
                    for k in kv:
                        os.environ.pop(k, None)
    for k in ("PQD_ABLATE", "PQD_PT_MODE", "PQD_FUSE"):
        os.environ.pop(k, None)
    res = {v: [] for v in plans}
    for v, p in plans.items():
        p.execute()
        p.synchronize()
        p.timing(reset=True)
    for _ in range(args.rounds):
        for v, p in plans.items():
            p.execute(rebuild_free=False)
            p.synchronize()
            f, w, n = p.timing(reset=True)
            res[v].append(w)
    executed = int(sum(tr.out_end + 1))
    F = bench.flops_per_traj_step(N, args.chi, len(ops), fused=False)  # full-work equivalent (unfused)
    out = {}
    for v, ws in res.items():
        ms = min(ws)
        out[v] = {"ms": ms, "us_per_step": 1e3 * ms / grid.n_steps,
                  "tflops_equiv": executed * F / (ms * 1e-3) / 1e12}
        print(f"{v}: sweep {ms:9.3f} ms  {1e3 * ms / grid.n_steps:7.3f} us/step  "
              f"{out[v]['tflops_equiv']:6.2f} TF/s(full-work equiv)", flush=True)
    print(json.dumps({"traj": args.traj, "n_tau": args.n_tau, "chi": args.chi, "steps": grid.n_steps, "res": out}))


if __name__ == "__main__":
    main()
