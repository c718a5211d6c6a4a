#!/bin/bash
# rocprofv3 kernel stats of the binned backward per level range.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in ${RANGES:-0-0 9-9 15-15 0-15}; do
    out=gpurun_out/gbl/r$r
    mkdir -p $out
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
        -- python3 tools/grid_bin_case.py --reps 5 --ranges $r > $out/log 2>&1 || { echo "range $r failed"; tail -5 $out/log; exit 1; }
    echo "== $r: $(grep median $out/log)"
    python3 tools/prof_top.py $(find $out -name "*kernel_stats.csv" | head -1) 4
done
