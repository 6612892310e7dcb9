# GPU parity suite, then the configs the identity-push path touches.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for c in 4-asc 4 5; do
timeout -k 10 200 python bench.py --config $c --no-cpu > gpurun_out/c.log 2>&1
tail -1 gpurun_out/c.log | python3 -c "import sys,json; l=json.loads(sys.stdin.read()); print(sys.argv[1], l['ms_per_step'], l['roofline']['kernel_us_avg'], l['roofline']['achieved'])" $c
done
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 > gpurun_out/cfg2.log 2>&1
tail -1 gpurun_out/cfg2.log | python3 -c "import sys,json; l=json.loads(sys.stdin.read()); print('config2', l['value'], l['ms_per_step'], l['roofline']['avg_kernel_us'], l['roofline']['frac'])"
