# Whole-vector DEPTH-3 instantiation (ALN, 3 waves per SIMD) for config 5: parity, then
# the config-5 leg against ALN at 2 waves per SIMD (alnw1) and the generic instantiation
# (noaln), alternating, 2 rounds.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "int32_negative or batch_error or config5 or matrix_random or pipelined or empty_and_single" > gpurun_out/c5aln_tests.log 2>&1 || { tail -30 gpurun_out/c5aln_tests.log; exit 1; }
tail -1 gpurun_out/c5aln_tests.log
VARIANTS="new alnw1 noaln" ARGS="--legs 5 --sparse-steps 0 --no-cpu --steps 5 --warmup 2" LEG=config5 ROUNDS=2 bash scripts/ab_multi.sh
