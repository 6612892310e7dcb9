# A/B of a library variant on the config-4 leg of the default line (10 M x 200, 16 pushes).
#   V=j8 bash scripts/gpu_ab_leg4.sh
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
cp distml_amd/libdistml_ps.so /tmp/ab_new.so
for r in 1 2; do
  for v in new $V; do
    if [ $v = new ]; then cp /tmp/ab_new.so distml_amd/libdistml_ps.so; else cp scripts/ab/libdistml_ps_$v.so distml_amd/libdistml_ps.so; fi
    timeout -k 10 300 python bench.py --legs 4 --no-cpu --sparse-steps 0 --steps 50 --warmup 20 > gpurun_out/abl_${v}_$r.json 2> gpurun_out/abl_${v}_$r.err
    python -c "import json;d=json.load(open('gpurun_out/abl_${v}_$r.json'))['config4'];print('$v $r', d['ms_per_step'], d['roofline'].get('avg_kernel_us'))"
  done
done
cp /tmp/ab_new.so distml_amd/libdistml_ps.so
