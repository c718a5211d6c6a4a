#!/bin/bash
# rocprofv3 kernel-trace stats of graph-replayed textureless steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_shade
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run \
    -- python tools/shade_steps.py textureless 30 > $OUT/log.txt 2>&1 || { echo "prof failed"; tail -5 $OUT/log.txt; exit 4; }
python tools/prof_top.py $OUT/run_kernel_stats.csv 16 > $OUT/top.txt
cat $OUT/top.txt
