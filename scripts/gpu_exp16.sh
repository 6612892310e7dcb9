set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "native_group or rccl_world1 or prereduce" > gpurun_out/ng.log 2>&1 || { tail -40 gpurun_out/ng.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/ng.log | tail -8
