# A/B of library variants (scripts/build_ab.sh) on per-GPU shard configs:
#   VARIANTS="flatwt" CONFIGS="4 4-perm" bash scripts/gpu_ab_cfg.sh
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
cp distml_amd/libdistml_ps.so /tmp/ab_new.so
for r in 1 2; do
  for v in new $VARIANTS; do
    if [ $v = new ]; then cp /tmp/ab_new.so distml_amd/libdistml_ps.so; else cp scripts/ab/libdistml_ps_$v.so distml_amd/libdistml_ps.so; fi
    for c in $CONFIGS; do
      timeout -k 10 200 python bench.py --config $c --no-cpu > gpurun_out/abc_${v}_${c}_$r.json 2> gpurun_out/abc_${v}_${c}_$r.err
      python -c "import json;d=json.load(open('gpurun_out/abc_${v}_${c}_$r.json'));print('$v $c $r', json.dumps({k: d[k] for k in d if k in ('ms_per_reduce','avg_kernel_us','frac','value')}), json.dumps(d.get('roofline',{}).get('avg_kernel_us')))"
    done
  done
done
cp /tmp/ab_new.so distml_amd/libdistml_ps.so
