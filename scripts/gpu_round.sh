# One GPU call: the whole -m gpu suite, smoke, the default bench line and the line
# profile (kernel stats + separate FETCH_SIZE / WRITE_SIZE passes, scripts/gpu_prof.sh).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
timeout -k 10 200 python bench.py --group --no-cpu --sparse-steps 0 --legs "" > gpurun_out/bench_group.json 2> gpurun_out/bench_group.err
cat gpurun_out/bench_group.json
TAG=line ARGS="--steps 200 --warmup 100 --no-cpu --c4-steps 3 --c4-warmup 1 --c5-steps 10 --c5-warmup 2 --c4a-steps 2 --c4a-warmup 1 --sparse-steps 10" bash scripts/gpu_prof.sh
