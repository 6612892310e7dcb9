# A/B of bench arguments on one box: ROUNDS alternating runs of `python bench.py $ARGS $A`
# and `... $B`; prints each leg in LEGS (frac, kernel µs, floor fraction where the leg has one).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in A B; do
    eval "X=\$$v"
    timeout -k 10 300 python bench.py $ARGS $X > gpurun_out/aba_${v}_$r.json 2> gpurun_out/aba_${v}_$r.err
    python3 -c "
import json, sys
d = json.load(open(sys.argv[1]))
for leg in sys.argv[3].split(','):
    x = d[leg] if leg != 'line' else d
    r = x['roofline']
    print(sys.argv[2], leg, x['ms_per_step'], r['frac'], r['avg_kernel_us'], r.get('frac_of_measured_floor'))
" gpurun_out/aba_${v}_$r.json "$v $r" ${LEGS:-line}
  done
done
