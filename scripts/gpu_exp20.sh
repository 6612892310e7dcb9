set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
DML_REDUCE_VARIANT=38 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k config2_dense --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t38.log 2>&1 || { tail -30 gpurun_out/t38.log; exit 1; }
echo "v38 config2 parity: $(tail -1 gpurun_out/t38.log)"
timeout -k 10 200 python scripts/exp_variants.py 0,38 4 > gpurun_out/var.log 2>&1; grep variant gpurun_out/var.log
for pairs in 1 0; do
DML_PAIRS=$pairs timeout -k 10 600 python scripts/bench_configs.py 5 4 > gpurun_out/cfg_$pairs.log 2>&1
echo "pairs=$pairs"; grep config gpurun_out/cfg_$pairs.log | python3 -c "import sys,json; [print(' ', json.loads(l)['config'][:8], json.loads(l)['ms_per_step'], json.loads(l)['reduce_kernel_us_avg'], json.loads(l)['kernel_TBps']) for l in sys.stdin]"
done
