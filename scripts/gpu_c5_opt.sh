# k_reduce_rows instruction trim (aligned rows, OR-accumulated negativity check): the GPU
# parity suite, then the config-5 leg against the previous build (head) and a 3-waves
# per SIMD register cap (d3w3), alternating, 2 rounds.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/c5opt_tests.log 2>&1 || { tail -30 gpurun_out/c5opt_tests.log; exit 1; }
tail -1 gpurun_out/c5opt_tests.log
VARIANTS="new head d3w3" ARGS="--legs 5 --sparse-steps 0 --no-cpu --steps 20 --warmup 5" LEG=line,config5 ROUNDS=2 bash scripts/ab_multi.sh
