set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "flat_kernel_widths" > gpurun_out/flatw.log 2>&1 || { tail -30 gpurun_out/flatw.log; exit 1; }
tail -1 gpurun_out/flatw.log
V=prent bash scripts/gpu_ab_group4.sh
