# Parity tests, bench lines and kernel stats for the native step (diagnostic).
mkdir -p gpurun_out/ent
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_encoders.py tests/test_gpu_native_step.py tests/test_gpu_field_oracle.py tests/test_gpu_bf16.py -x -q -p no:cacheprovider -m gpu --timeout 180 --timeout-method thread > gpurun_out/ent/pt.log 2>&1 || { tail -40 gpurun_out/ent/pt.log; exit 1; }
tail -1 gpurun_out/ent/pt.log
B="python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path --no-kernel-timing"
for i in 1 2 3; do timeout -k 10 200 $B > gpurun_out/ent/b$i.log 2>&1 || exit 2; done
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ent/b*.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ent/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path > gpurun_out/ent/prof.log 2>&1 || exit 3
python tools/prof_top.py gpurun_out/ent/prof/run_kernel_stats.csv 40 | grep -E "fill|copyBuffer|k_bin"
