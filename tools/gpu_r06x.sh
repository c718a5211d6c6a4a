# C4 queue order: k_chunk_order as a ballot-ranked counting sort over 16 waves
# (was 256 threads with a serial scan): render tests, then a kernel trace of
# the C4 frame for the order kernels' times
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06x
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py > $O/test.txt 2>&1
tail -1 $O/test.txt
for i in 1 2; do timeout -k 10 180 python -u $R/tools/infer_case.py | grep res=; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python $R/tools/infer_case.py --reps 5 > $O/tr.log 2>&1
python $R/tools/prof_top.py $O/tr/run_kernel_stats.csv 12
