# AdaGrad store path: GPU parity suite, then config 4 per-GPU measurement.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --config 4-ada --cpu-seconds 0.5 > gpurun_out/cfg4.log 2>&1
grep config gpurun_out/cfg4.log
