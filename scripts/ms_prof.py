"""One multi-trajectory split-group sweep of the C4 shape (bench.build_workload) for counter passes:
python scripts/ms_prof.py [--n-t1 256] [--n-tau 2000]; PQD_* switches from the environment."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-t1", type=int, default=256)
    ap.add_argument("--n-tau", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import bench
    from pyaceqd_amd import engine
    sysd, grid, pt, rho0, ops, tr = bench.build_workload(args.n_t1, args.n_tau, 64, t1_offset=0)
    plan = engine.Plan(sysd, grid, rho0, ops, tr, pt=pt)
    for _ in range(args.reps):
        plan.execute()
        plan.synchronize()
    _, ms, _ = plan.timing(reset=True)
    print("path", plan.info(), f"last sweep {ms:.2f} ms")


if __name__ == "__main__":
    main()
