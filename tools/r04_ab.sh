#!/bin/bash
# A/B of environment settings by rocprofv3 kernel stats of the C2 headline
# and the textureless step:  CONFIGS="A=1,B=2 A=0" bash tools/r04_ab.sh
# (each config: comma-separated VAR=value pairs; "-" = no override).
# PMC=1 adds a FETCH_SIZE / WRITE_SIZE pass of the headline per config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for cfg in ${CONFIGS:?}; do
  i=$((i + 1))
  envs=""
  [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' ' ')
  echo "== config $i: $cfg"
  OUT=gpurun_out/ab$i
  mkdir -p $OUT
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2 -o run \
      -- python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-kernel-timing --no-traffic \
         --no-infer --no-c5 --no-module-path --no-shading --no-alt-backward > $OUT/c2.log 2>&1 \
      || { echo "c2 prof failed"; tail -5 $OUT/c2.log; exit 4; }
  python tools/prof_top.py $OUT/c2/run_kernel_stats.csv ${TOPN:-8}
  grep '^{' $OUT/c2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step'], 'M', d['config']['mean_samples_per_step'])"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sh -o run \
      -- python tools/shade_steps.py textureless 30 > $OUT/sh.log 2>&1 \
      || { echo "shade prof failed"; tail -5 $OUT/sh.log; exit 4; }
  python tools/prof_top.py $OUT/sh/run_kernel_stats.csv ${TOPN:-6}
  if [ "${PMC:-0}" = 1 ]; then
    for c in FETCH_SIZE WRITE_SIZE; do
      env $envs timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/pmc_$c -o run \
          -- python bench.py --steps 3 --warmup 47 --no-cpu-baseline --no-kernel-timing --no-traffic \
             --no-infer --no-c5 --no-module-path --no-shading --no-alt-backward > $OUT/pmc_$c.log 2>&1 \
          || { echo "pmc $c failed"; exit 5; }
      for k in k_walk k_bin k_sum; do python tools/pmc_table.py $OUT/pmc_$c $k; done
    done
  fi
done
