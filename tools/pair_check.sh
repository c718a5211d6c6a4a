# Parity of the field-forward gather variants and a bench line (diagnostic).
mkdir -p gpurun_out/pair
timeout -k 10 500 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_field_oracle.py tests/test_gpu_native_step.py tests/test_gpu_shading.py tests/test_gpu_bf16.py tests/test_gpu_graph.py -x -q -p no:cacheprovider -m gpu --timeout 180 --timeout-method thread > gpurun_out/pair/pt.log 2>&1 || { tail -40 gpurun_out/pair/pt.log; exit 1; }
tail -1 gpurun_out/pair/pt.log
timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-alt-backward --no-traffic --no-infer > gpurun_out/pair/bench.log 2>&1 || exit 2
grep '^{' gpurun_out/pair/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('c5',{}).get('ms_per_step'), {k:v for k,v in d.get('shading',{}).items() if 'ms' in k})"
