# Sparse leaf size A/B: DML_SP_SL_BIAS = 0 (leaves of ~kSpLeafCap/4..kSpLeafCap/2 records), 1 (twice as large), -1.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
DML_SP_SL_BIAS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "array or sparse or config3" -x -q --timeout 200 --timeout-method thread > gpurun_out/leaf_tests_sl.log 2>&1 || { tail -20 gpurun_out/leaf_tests_sl.log; exit 1; }
tail -1 gpurun_out/leaf_tests_sl.log
for rep in 1 2 3; do
for b in 0 1 -1; do
DML_SP_SL_BIAS=$b timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --sparse-steps 20 > gpurun_out/sp.log 2>&1
tail -1 gpurun_out/sp.log | python3 -c "import sys,json; l=json.loads(sys.stdin.read())['sparse']; print('bias $b', l['ms_per_step'], l['apply_kernel_us_avg'])"
done
done
