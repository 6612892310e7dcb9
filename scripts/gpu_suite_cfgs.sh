# GPU parity suite, then configs 5 and 4 per-GPU shard measurements.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python scripts/bench_configs.py 5 4 > gpurun_out/cfg45.log 2>&1
grep config gpurun_out/cfg45.log
