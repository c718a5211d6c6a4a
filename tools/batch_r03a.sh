#!/bin/bash
# round-3 measurement batch: renderer phase profile (grid / sphere), the
# backward-structure difference printout, a C2 bench line, k_bin PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/infer_case.py --profile > gpurun_out/ip_grid.txt 2>&1 || { echo "infer failed"; tail gpurun_out/ip_grid.txt; exit 1; }
timeout -k 10 200 python tools/infer_case.py --profile --sphere > gpurun_out/ip_sphere.txt 2>&1 || { echo "infer sphere failed"; exit 1; }
tail -2 gpurun_out/ip_grid.txt gpurun_out/ip_sphere.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_step_structures.py -k differ -s -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/structures.txt 2>&1 || { echo "structures failed"; tail -20 gpurun_out/structures.txt; exit 2; }
grep -A4 "emb_scale" gpurun_out/structures.txt
timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-traffic --no-infer --no-c5 --no-module-path --no-shading --no-alt-backward > gpurun_out/bench_b.log 2>&1 || { echo "bench failed"; exit 3; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_b.log') if l.startswith('{')][-1]); print(d['ms_per_step'], d['host_issue_ms_per_step'], d['host_cost_ms_per_step'])"
timeout -k 10 900 bash tools/pmc_bin.sh > gpurun_out/pmcbin.txt 2>&1 || { echo "pmc failed"; tail gpurun_out/pmcbin.txt; exit 4; }
tail -40 gpurun_out/pmcbin.txt
