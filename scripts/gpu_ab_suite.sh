# A kernel change on the GPU: the -m gpu suite on the in-tree build, then alternating
# bench rounds against scripts/ab variants (VARIANTS, "new" = in-tree; ARGS, LEG, ROUNDS).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
fi
timeout -k 10 900 bash scripts/ab_multi.sh > gpurun_out/ab.txt 2>&1 || { tail -20 gpurun_out/ab.txt; exit 1; }
cat gpurun_out/ab.txt
