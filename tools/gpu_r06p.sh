# C4 queue layout A/B (tools/infer_case.py): 64-ray row strips vs 8 x 8 pixel
# tiles, both taken in mirrored halves, R0 / R1, interleaved, then one profiled
# frame of each with per-wave records.  The other layouts of
# profiles/r06/c4_queue_layout_ab.txt (dealt queues, mid-round refill,
# iteration caps, mirror blocks, quarters, Morton lanes) were A/B builds
# removed from the tree.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
run() {  # tag, args
  local tag=$1; shift
  echo "== $tag $*"; timeout -k 10 180 python -u $R/tools/infer_case.py "$@"
}
for sc in "" "--sphere"; do
  s=${sc:+r1}; s=${s:-r0}
  for i in 1 2; do
    run ${s}_strips $sc --strips
    run ${s}_tiles $sc
  done
done
timeout -k 10 180 python -u $R/tools/infer_case.py --profile --strips --dump gpurun_out/waves_r0_strips.npy
timeout -k 10 180 python -u $R/tools/infer_case.py --profile --dump gpurun_out/waves_r0_tiles.npy
