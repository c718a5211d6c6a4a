# A/B of the native step with and without the corner-quad table (diagnostic; the
# DFHIP_NO_QUADS switch it used was removed after the measurement in DESIGN.md).
mkdir -p gpurun_out/abq
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path"
DFHIP_NO_QUADS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abq/p0 -o run -- $B > gpurun_out/abq/b0.log 2>&1 || exit 1
DFHIP_NO_QUADS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abq/p1 -o run -- $B > gpurun_out/abq/b1.log 2>&1 || exit 1
B2="python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path --no-kernel-timing"
for i in 1 2; do
DFHIP_NO_QUADS=1 timeout -k 10 200 $B2 > gpurun_out/abq/n$i.log 2>&1 || exit 1
DFHIP_NO_QUADS=0 timeout -k 10 200 $B2 > gpurun_out/abq/q$i.log 2>&1 || exit 1
done
grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/abq/[nq]*.log
