# A/B of two builds of the kernel library on one box (diagnostic):
# lib/libdfhip_base.so (before) vs lib/libdfhip.so (after), alternating.
mkdir -p gpurun_out/ablib
B="python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-alt-backward --no-shading --no-infer --no-traffic --no-c5 --no-module-path --no-kernel-timing"
BASE=single-stable-dreamfusion_amd/lib/libdfhip_base.so
for i in 1 2 3; do
  DFHIP_LIB=$BASE timeout -k 10 200 $B > gpurun_out/ablib/base$i.log 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/ablib/new$i.log 2>&1 || exit 1
done
grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/ablib/*.log
