# Config 3 leaf A/B: variants in scripts/ab (VARIANTS, the first is the base), their
# sparse / array parity tests, then alternating bench rounds.
export TMPDIR=/tmp; mkdir -p gpurun_out
cp distml_amd/libdistml_ps.so /tmp/keep.so
for v in ${TESTV:-}; do
  cp scripts/ab/libdistml_ps_$v.so distml_amd/libdistml_ps.so
  timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "sparse or array or config3" > gpurun_out/leaf_tests_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc"; tail -1 gpurun_out/leaf_tests_$v.log
  case $rc in 0) ;; *) cp /tmp/keep.so distml_amd/libdistml_ps.so; exit $rc;; esac
done
cp /tmp/keep.so distml_amd/libdistml_ps.so
timeout -k 10 900 bash -c "VARIANTS=\"$VARIANTS\" ARGS=\"--legs x --sparse-steps 40 --no-cpu --steps 20 --warmup 5\" LEG=sparse ROUNDS=${ROUNDS:-3} bash scripts/ab_multi.sh" > gpurun_out/ab_leaf.txt 2>&1; rc=$?
cp /tmp/keep.so distml_amd/libdistml_ps.so
echo "ab rc=$rc"; grep -v "^$" gpurun_out/ab_leaf.txt
for v in $VARIANTS; do for r in $(seq 1 ${ROUNDS:-3}); do python3 -c "import json,sys;d=json.load(open(sys.argv[1]));x=d['sparse'];r=x['roofline'];print(sys.argv[1].split('/')[-1], x['ms_per_step'], r['avg_kernel_us'], r.get('measured_rmw_floor_us'), r.get('frac_of_measured_floor'))" gpurun_out/abm_${v}_$r.json; done; done
