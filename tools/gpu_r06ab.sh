# C4 final tree: per-wave records of one frame (R0, R1)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 180 python -u $R/tools/infer_case.py --profile --dump gpurun_out/waves_final_r0.npy
timeout -k 10 180 python -u $R/tools/infer_case.py --profile --sphere --dump gpurun_out/waves_final_r1.npy
