# Diagnostic: config-2 steps over buckets in separate allocations or slices of one
# slab, generated into their buffers in order or in a seeded order.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for v in sep0 sep7 slab0 slab7; do
    case $v in sep0) X="";; sep7) X="--alloc-seed 7";; slab0) X="--one-slab";; slab7) X="--one-slab --alloc-seed 7";; esac
    timeout -k 10 150 python bench.py --legs x --sparse-steps 0 --no-cpu $X > gpurun_out/slab_${v}_$r.json 2> gpurun_out/slab_${v}_$r.err
    python -c "import json;d=json.load(open('gpurun_out/slab_${v}_$r.json'));s=d['shuffled'];print('$v $r', d['ms_per_step'], d['roofline']['avg_kernel_us'], s['avg_kernel_us'], s['in_order_again']['avg_kernel_us'], s['buffers_shuffled'].get('avg_kernel_us'), s['buffers_shuffled']['ms_per_step'])"
  done
done
