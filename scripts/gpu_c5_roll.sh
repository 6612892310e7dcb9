# DEPTH-3 loop as select / issue / consume of load groups (new), with two groups in
# flight (roll), against the previous build (head): parity, then the config-5 leg,
# alternating, 2 rounds.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "int32_negative or batch_error or config5 or matrix_random or pipelined or empty_and_single or identity_speculation or flat_kernel_widths" > gpurun_out/c5roll_tests.log 2>&1 || { tail -30 gpurun_out/c5roll_tests.log; exit 1; }
tail -1 gpurun_out/c5roll_tests.log
VARIANTS="new roll head" ARGS="--legs 5 --sparse-steps 0 --no-cpu --steps 5 --warmup 2" LEG=line,config5 ROUNDS=2 bash scripts/ab_multi.sh
