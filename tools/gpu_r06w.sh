# C2 native step: the table's corner quads on a side stream beside the march
# (a parallel branch of the captured graph; trainer.overlap_quads, removed
# after this A/B) vs in line: native-step tests, bench C2 alternating, traces
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_step.py tests/test_gpu_graph.py tests/test_gpu_step_structures.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
tail -1 $O/pytest.log
F="--steps 60 --warmup 10 --no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
for i in 1 2 3; do
  for v in 1 0; do
    DFHIP_OVERLAP_QUADS=$v timeout -k 10 300 python -u $R/bench.py $F > $O/b$v$i.log 2>&1 || exit 1
    echo "== overlap $v $(grep -o '"ms_per_step": [0-9.]*' $O/b$v$i.log | head -1)"
  done
done
cd /tmp
for v in 1 0; do
  DFHIP_OVERLAP_QUADS=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$v -o run -- python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path > $O/tr$v.log 2>&1 || exit 1
done
