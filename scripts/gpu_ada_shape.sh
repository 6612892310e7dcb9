# k_ada_ident at 8 vectors per lane, 2-wave blocks, 64-B aligned waves (new) against the
# previous build (head: 4 vectors, 4-wave blocks) and J 2 / 4-wave blocks (aij2): parity,
# then the config-4 AdaGrad leg, alternating, 2 rounds.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "adagrad" > gpurun_out/adashape_tests.log 2>&1 || { tail -30 gpurun_out/adashape_tests.log; exit 1; }
tail -1 gpurun_out/adashape_tests.log
VARIANTS="new head aij2" ARGS="--legs 4a --sparse-steps 0 --no-cpu --steps 5 --warmup 2" LEG=config4_ada ROUNDS=2 bash scripts/ab_multi.sh
