# C4 with the cooperative drain, every ray stashable: the bench's C4 leg
# (DFHIP_INFER_COOP 0 / 16 / 32 / 64, interleaved twice), then one rocprofv3
# kernel split for 0 and 64
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06n}
mkdir -p $O
F="--no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-traffic --no-c5 --no-module-path --steps 5 --warmup 3"
for rep in 1 2; do
  for v in 0 16 32 64; do
    export DFHIP_INFER_COOP=$v
    timeout -k 10 300 python bench.py $F > $O/c4_$v.$rep.log 2>&1 || exit 1
    python - $O/c4_$v.$rep.log $v <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
inf = json.loads(line)["inference"]
print("coop", sys.argv[2], "R0 ms/frame", inf["ms_per_frame"], "kernel us", inf.get("kernel_avg_us"), "G/s", round(inf["samples_per_sec"] / 1e9, 3))
PY
  done
done
cd /tmp
for v in 0 64; do
  export DFHIP_INFER_COOP=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o run -- python $R/bench.py $F > $O/p$v.log 2>&1 || exit 1
  echo "== rocprof coop $v"; python $R/tools/prof_top.py $O/p$v/run_kernel_stats.csv 40 | grep -E "render|total"
done
