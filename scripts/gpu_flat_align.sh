# k_reduce_flat / k_ada_flat rows per wave lowered to whole 64-B sectors (new) against the
# unaligned count (noalign): parity, then the config-4 leg with permuted pushes (the
# k_reduce_flat path), alternating, 2 rounds.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "adagrad_flat or flat_kernel_widths or identity_speculation or config4 or matrix_random or prereduce or slot_reuse" > gpurun_out/flatalign_tests.log 2>&1 || { tail -30 gpurun_out/flatalign_tests.log; exit 1; }
tail -1 gpurun_out/flatalign_tests.log
VARIANTS="new noalign" ARGS="--legs 4 --c4-order perm --sparse-steps 0 --no-cpu --steps 5 --warmup 2 --c4-steps 3 --c4-warmup 1" LEG=config4 ROUNDS=2 bash scripts/ab_multi.sh
