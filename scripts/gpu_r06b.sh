# Round 6, second GPU call: the new GPU tests, k_ada_vec against k_ada_ident (A/B +
# its parity tests on the variant build), the geometry pair alternated in one process.
export TMPDIR=/tmp; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fault/timeout rc=$1, stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "floor or int32_negative or config5_model or flat_kernel or adagrad_ident" > gpurun_out/r06b_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; fatal $rc
DML_PARITY_LOG=gpurun_out/parity_rs.jsonl timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_native_group.py tests/test_jni_shim.py tests/test_gpu_group.py >> gpurun_out/r06b_tests.log 2>&1; rc=$?; echo "group tests rc=$rc"; fatal $rc
grep -E "passed|failed" gpurun_out/r06b_tests.log | tail -3; grep -E "^FAILED|^ERROR" gpurun_out/r06b_tests.log | head
cp distml_amd/libdistml_ps.so /tmp/keep.so
cp scripts/ab/libdistml_ps_adavec2.so distml_amd/libdistml_ps.so
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "adagrad" > gpurun_out/r06b_adavec2_tests.log 2>&1; rc=$?; echo "adavec2 tests rc=$rc"
cp /tmp/keep.so distml_amd/libdistml_ps.so; fatal $rc
tail -3 gpurun_out/r06b_adavec2_tests.log
timeout -k 10 900 bash -c 'VARIANTS="base adavec1 adavec2 adavec4" ARGS="--legs 4a --sparse-steps 0 --no-cpu --steps 20 --warmup 5 --c4a-steps 4" LEG=config4_ada ROUNDS=2 bash scripts/ab_multi.sh' > gpurun_out/ab_ada_vec.txt 2>&1; rc=$?; echo "ab rc=$rc"; cp /tmp/keep.so distml_amd/libdistml_ps.so; fatal $rc
cat gpurun_out/ab_ada_vec.txt | grep -v "^$"
for f in gpurun_out/abm_*_[12].json; do python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['config4_ada']['roofline'];print(sys.argv[1], r['kernel'], r['avg_kernel_us'], r.get('measured_stream_floor_us'), r.get('frac_of_measured_floor'))" $f; done
timeout -k 10 200 scripts/ubench_geom alt 4 > gpurun_out/ubench_geom_alt.jsonl; rc=$?; echo "alt rc=$rc"; fatal $rc
python3 -c "
import json
for l in open('gpurun_out/ubench_geom_alt.jsonl'):
    d=json.loads(l); print(d['case'], d['round'], 'U', d['U_KiB_per_wave'], d['mode'], d['best_us'], d['frac_best'])
"
