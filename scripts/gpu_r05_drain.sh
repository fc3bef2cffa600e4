cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05/drain
for r in 1 2; do for a in 0 64; do
PQD_ABLATE=$a timeout -k 10 200 python3 -u scripts/bench_configs.py --configs c3one --steps 3 > gpurun_out/r05/drain/c3_a$a.$r.log 2>&1 || exit 1
echo "ablate=$a $(grep -o '"pt_sweep_ms": [0-9.]*' gpurun_out/r05/drain/c3_a$a.$r.log)"
done; done
