# walk timeline (per-workgroup start / end, XCC and CU) of the bench's eager
# twin in the two launch-sequence states (DFHIP_KEPT_CLEAN 1 / 0)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06k}
mkdir -p $O
for v in 1 0 1 0; do
  export DFHIP_KEPT_CLEAN=$v
  echo "=== kept_clean=$v"
  timeout -k 10 300 python -u tools/walk_trace_bench.py --warmup 20 --steps 2 || exit 1
done
