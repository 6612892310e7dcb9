set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
A='--legs "" --sparse-steps 0 --no-cpu'
for r in 1 2; do
  for v in def o1 asc perm; do
    case $v in def) X="";; o1) X="--shuffle-orders 1";; asc) X="--shuffle-only asc";; perm) X="--shuffle-only perm";; esac
    timeout -k 10 120 python bench.py --legs "" --sparse-steps 0 --no-cpu $X > gpurun_out/shuf_${v}_$r.json 2> gpurun_out/shuf_${v}_$r.err
    python -c "import json;d=json.load(open('gpurun_out/shuf_${v}_$r.json'));s=d['shuffled'];print('$v $r', d['roofline']['avg_kernel_us'], s['avg_kernel_us'], s['in_order_again']['avg_kernel_us'], s['pushes_per_step'])"
  done
done
