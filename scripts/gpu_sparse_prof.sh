# Compact GPU call: the -m gpu suite, then the sparse leg's profile (stats + FETCH_SIZE
# + WRITE_SIZE passes) for the partition / leaf kernels.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
TAG=sparse ARGS="--legs x --no-cpu --steps 10 --warmup 5 --sparse-steps 20" bash scripts/gpu_prof.sh
grep -h '"sparse"' gpurun_out/prof_sparse_stats.log | head -1 | cut -c1-100 || true
