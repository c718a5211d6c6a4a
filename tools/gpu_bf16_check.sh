set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/bf16
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_field_oracle.py tests/test_gpu_native_step.py tests/test_gpu_field.py tests/test_gpu_network.py -x -v -p no:cacheprovider -m gpu --timeout 180 --timeout-method thread -s > gpurun_out/bf16/pt.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|M=|feature grads|rel" gpurun_out/bf16/pt.log | tail -40
exit $rc
