set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/c_0.log 2>&1
echo "overlap $(python3 scripts/summ_order.py gpurun_out/c_0.log)"
DML_SERIAL_INDEX=1 timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/c_ser.log 2>&1
echo "serial $(python3 scripts/summ_order.py gpurun_out/c_ser.log)"
done
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 --group > gpurun_out/bench_group.json 2> gpurun_out/bench_group.err
cat gpurun_out/bench_group.json
