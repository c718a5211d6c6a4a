#!/bin/bash
# rocprofv3 kernel-trace stats of the C2 headline only (graph-replayed train
# steps, no C4 / C5 / shading legs): TAG=name bash tools/prof_c2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-c2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run \
    -- python bench.py --steps ${STEPS:-40} --warmup 10 --no-cpu-baseline --no-kernel-timing \
       --no-traffic --no-infer --no-c5 --no-module-path --no-shading --no-alt-backward ${BENCH_ARGS:-} \
    > $OUT/bench.log 2>&1 || { echo "prof $TAG failed"; tail -5 $OUT/bench.log; exit 4; }
python tools/prof_top.py $OUT/run_kernel_stats.csv ${TOPN:-22} > $OUT/top.txt
cat $OUT/top.txt
