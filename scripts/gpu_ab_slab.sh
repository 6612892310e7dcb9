# Receive slab against one allocation per push for the config-4, 4a and 5 legs,
# alternating, 2 rounds on one box (bench.py --separate-buffers).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
A="--legs 4,4a,5 --sparse-steps 0 --no-cpu --steps 5 --warmup 2 --c4-steps 3 --c4-warmup 1"
for r in 1 2; do
  for v in slab sep; do
    X=""; [ $v = sep ] && X="--separate-buffers"
    timeout -k 10 400 python bench.py $A $X > gpurun_out/abs_${v}_$r.json 2> gpurun_out/abs_${v}_$r.err
    python3 -c "
import json, sys
d = json.load(open(sys.argv[1]))
for leg in ('config4', 'config4_ada', 'config5'):
    x = d[leg]; r = x['roofline']
    print(sys.argv[2], leg, x['ms_per_step'], r['frac'], r['avg_kernel_us'], r['kernel'])
" gpurun_out/abs_${v}_$r.json "$v $r"
  done
done
