#!/bin/bash
# Resolved-stream iteration: the encoder tests, then the binned backward per
# walk mode on a real march's samples (events), then its kernels by rocprofv3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rs}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_encoders.py} -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u tools/grid_bin_case.py --modes ${MODES:-0,3} --ranges 0-15 --reps 9 > $OUT/case.log 2>&1 \
    || { echo "case failed"; tail -20 $OUT/case.log; exit 2; }
cat $OUT/case.log
for m in ${PMODES:-0 3}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$m -o run \
      -- python tools/grid_bin_case.py --modes $m --ranges 0-15 --reps 9 > $OUT/prof$m.log 2>&1 \
      || { echo "prof failed"; tail -20 $OUT/prof$m.log; exit 3; }
  python tools/prof_top.py $OUT/prof$m/run_kernel_stats.csv 8 > $OUT/top$m.txt
  echo "--- mode $m"; cat $OUT/top$m.txt
done
