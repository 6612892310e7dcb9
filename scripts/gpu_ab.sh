# GPU tests, then k_reduce shape A/B on the config-2 row orders (scripts/exp_order.py).
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for v in ${VARIANTS:-0 10 21 24 27}; do
  DML_REDUCE_VARIANT=$v timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/ab_v$v.log 2>&1
  echo "v=$v"; grep row_order gpurun_out/ab_v$v.log
done
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
