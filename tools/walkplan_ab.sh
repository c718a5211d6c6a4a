#!/bin/bash
# Walk-plan A/B: the default library against variants lib/libdfhip_{s0,t4k}.so
# (s0: no per-segment cost in the part plan, the round-4 plan; t4k:
# 4,096-sample binning tiles for single samples).  Per library: the
# albedo bin-case walk timeline and rocprofv3 kernel stats of the C2 headline
# steps; for s0 and the default also the textureless step (eager-twin walk
# timeline, kernel stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-walkplan}
mkdir -p $OUT
L=$PWD/single-stable-dreamfusion_amd/lib
DFHIP_LIB=$L/libdfhip_t4k.so timeout -k 10 300 python -u -m pytest tests/test_gpu_encoders.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > $OUT/pytest_t4k.log 2>&1 || { echo "pytest t4k failed"; tail -30 $OUT/pytest_t4k.log; exit 1; }
tail -1 $OUT/pytest_t4k.log
for v in ${VARS:-s0 base t4k}; do
  if [ $v = base ]; then unset DFHIP_LIB; else export DFHIP_LIB=$L/libdfhip_$v.so; fi
  timeout -k 10 200 python -u tools/walk_trace.py --mode 0 --reps 3 > $OUT/trace_$v.log 2>&1 \
      || { echo "trace $v failed"; tail -20 $OUT/trace_$v.log; exit 2; }
  echo "=== $v albedo case"; sed -n 2,3p $OUT/trace_$v.log; grep end-time $OUT/trace_$v.log
  TAG=${v}_c2 TOPN=8 bash tools/prof_c2.sh || exit 3
  if [ $v = s0 ] || [ $v = base ]; then
    timeout -k 10 300 python -u tools/walk_trace_bench.py --shade textureless --steps 2 > $OUT/trace7_$v.log 2>&1 \
        || { echo "trace7 $v failed"; tail -20 $OUT/trace7_$v.log; exit 4; }
    echo "=== $v textureless walk"; grep -E "span|duration|end-time" $OUT/trace7_$v.log | tail -3
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shade_$v -o run \
        -- python tools/shade_steps.py textureless 30 > $OUT/shade_$v.log 2>&1 \
        || { echo "shade $v failed"; tail -20 $OUT/shade_$v.log; exit 5; }
    python tools/prof_top.py $OUT/shade_$v/run_kernel_stats.csv 5
  fi
done
