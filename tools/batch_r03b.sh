#!/bin/bash
# renderer (lookahead march) + fast binning: parity tests, C4 timing, C2 kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_encoders.py tests/test_gpu_native_step.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_b.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_b.log; exit 1; }
tail -2 gpurun_out/pt_b.log
timeout -k 10 200 python tools/infer_case.py --profile || exit 2
VAR=DFHIP_X A=0 B=1 bash tools/infer_ab.sh || exit 3
TAG=fastbin TOPN=12 bash tools/prof_c2.sh || exit 4
