#!/bin/bash
# HBM traffic per kernel of a short bench run: one rocprofv3 pass per counter
# (FETCH_SIZE, WRITE_SIZE), kernel-trace only, then tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmcb
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $out/$c -o run \
        -- python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline --no-kernel-timing \
        > $out/$c.log 2>&1 || { echo "pmc pass $c failed"; tail -5 $out/$c.log; exit 1; }
done
python3 tools/pmc_summary.py $out gpurun_out/pmc_summary.json
