# Diagnostic of the shuffled-order sub-line: push order vs bucket address order.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for v in def a7 a9 o1; do
    case $v in def) X="";; a7) X="--alloc-seed 7";; a9) X="--alloc-seed 9";; o1) X="--shuffle-orders 1";; esac
    timeout -k 10 120 python bench.py --legs "" --sparse-steps 0 --no-cpu $X > gpurun_out/shuf_${v}_$r.json 2> gpurun_out/shuf_${v}_$r.err
    python -c "import json;d=json.load(open('gpurun_out/shuf_${v}_$r.json'));s=d['shuffled'];print('$v $r', d['roofline']['avg_kernel_us'], s['avg_kernel_us'], s['in_order_again']['avg_kernel_us'])"
  done
done
