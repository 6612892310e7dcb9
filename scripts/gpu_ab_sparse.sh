# A/B of a library variant on the sparse leg (config 3): the variant's sparse /
# array parity tests first, then the leg for both builds, alternating.
#   V=agg bash scripts/gpu_ab_sparse.sh
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
cp distml_amd/libdistml_ps.so /tmp/ab_new.so
cp scripts/ab/libdistml_ps_$V.so distml_amd/libdistml_ps.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "sparse or array or config3" > gpurun_out/ab_sparse_tests.log 2>&1 || { cp /tmp/ab_new.so distml_amd/libdistml_ps.so; tail -20 gpurun_out/ab_sparse_tests.log; exit 1; }
tail -1 gpurun_out/ab_sparse_tests.log
for r in 1 2 3; do
  for v in new $V; do
    if [ $v = new ]; then cp /tmp/ab_new.so distml_amd/libdistml_ps.so; else cp scripts/ab/libdistml_ps_$v.so distml_amd/libdistml_ps.so; fi
    timeout -k 10 200 python bench.py --legs x --steps 10 --warmup 5 --no-cpu --sparse-steps 40 > gpurun_out/abs_${v}_$r.json 2> gpurun_out/abs_${v}_$r.err
    python -c "import json;d=json.load(open('gpurun_out/abs_${v}_$r.json'))['sparse'];print('$v $r', d['ms_per_step'], d['roofline']['avg_kernel_us'])"
  done
done
cp /tmp/ab_new.so distml_amd/libdistml_ps.so
