# A/B of library variants (scripts/build_ab.sh) on the config-2 line: in-order,
# shuffled and in-order-again, with buckets in push-order addresses and in a
# random allocation order (--alloc-seed).  VARIANTS="remap1 remap2" bash scripts/gpu_ab_order.sh
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
cp distml_amd/libdistml_ps.so /tmp/ab_new.so
for r in 1 2; do
  for v in new $VARIANTS; do
    if [ $v = new ]; then cp /tmp/ab_new.so distml_amd/libdistml_ps.so; else cp scripts/ab/libdistml_ps_$v.so distml_amd/libdistml_ps.so; fi
    for a in 0 7; do
      timeout -k 10 120 python bench.py --legs "" --sparse-steps 0 --no-cpu --alloc-seed $a > gpurun_out/ab_${v}_${a}_$r.json 2> gpurun_out/ab_${v}_${a}_$r.err
      python -c "import json;d=json.load(open('gpurun_out/ab_${v}_${a}_$r.json'));s=d['shuffled'];print('$v alloc$a $r', d['roofline']['avg_kernel_us'], s['avg_kernel_us'], s['in_order_again']['avg_kernel_us'], d['ms_per_step'])"
    done
  done
done
cp /tmp/ab_new.so distml_amd/libdistml_ps.so
