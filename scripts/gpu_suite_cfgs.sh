# GPU parity suite, then configs 5 and 4 (one GPU's shard) through bench.py --config.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --config 5 > gpurun_out/cfg5.log 2>&1
for c in 4 4-32 4-ada; do
timeout -k 10 300 python bench.py --config $c > gpurun_out/cfg$c.log 2>&1
done
for c in 5 4 4-32 4-ada; do tail -1 gpurun_out/cfg$c.log; done
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 > gpurun_out/cfg2.log 2>&1
tail -1 gpurun_out/cfg2.log | python3 -c "import sys,json; l=json.loads(sys.stdin.read()); print('config2', l['value'], l['ms_per_step'], l['roofline']['avg_kernel_us'], l['roofline']['frac'])"
