# A/B of two library builds on one box: the in-tree build (new) against
# scripts/ab/libdistml_ps_<B>.so (built from the same sources with a -D variant
# switch, e.g. `make -C distml_amd/csrc OUT=... EXTRA=-DDML_AB_X=1`), alternating,
# the same bench arguments.
#   B=base ARGS="--legs 4a --sparse-steps 0 --no-cpu" ROUNDS=2 bash scripts/ab_bench.sh
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
B=${B:-base}; ROUNDS=${ROUNDS:-2}
cp distml_amd/libdistml_ps.so /tmp/ab_new.so
for r in $(seq 1 $ROUNDS); do
  for v in new $B; do
    if [ $v = new ]; then cp /tmp/ab_new.so distml_amd/libdistml_ps.so; else cp scripts/ab/libdistml_ps_$B.so distml_amd/libdistml_ps.so; fi
    timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_${v}_$r.json 2> gpurun_out/ab_${v}_$r.err
    echo "$v $r done"
  done
done
cp /tmp/ab_new.so distml_amd/libdistml_ps.so
