# A/B of several library builds on one box, alternating, the same bench arguments:
# "new" is the in-tree build, the others scripts/ab/libdistml_ps_<V>.so (scripts/build_ab.sh).
#   VARIANTS="new base x" ARGS="--legs 4a ..." LEG=config4_ada ROUNDS=2 bash scripts/ab_multi.sh
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
cp distml_amd/libdistml_ps.so /tmp/ab_new.so
for r in $(seq 1 $ROUNDS); do
  for v in $VARIANTS; do
    if [ $v = new ]; then cp /tmp/ab_new.so distml_amd/libdistml_ps.so; else cp scripts/ab/libdistml_ps_$v.so distml_amd/libdistml_ps.so; fi
    timeout -k 10 300 python bench.py $ARGS > gpurun_out/abm_${v}_$r.json 2> gpurun_out/abm_${v}_$r.err
    python3 -c "
import json, sys
d = json.load(open(sys.argv[1]))
for leg in sys.argv[3].split(','):
    x = d[leg] if leg != 'line' else d
    r = x['roofline']
    print(sys.argv[2], leg, x['ms_per_step'], r['frac'], r['avg_kernel_us'], r['kernel'])
" gpurun_out/abm_${v}_$r.json "$v $r" ${LEG:-line}
  done
done
cp /tmp/ab_new.so distml_amd/libdistml_ps.so
