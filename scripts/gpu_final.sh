# Round-end check: GPU suite, smoke, default bench, sharded-path bench; stdout of
# each bench must be exactly one JSON line.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
echo smoke-ok
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
wc -l < gpurun_out/bench.json
cat gpurun_out/bench.json
timeout -k 10 300 python bench.py --group --no-cpu --sparse-steps 0 > gpurun_out/bench_group.json 2> gpurun_out/bench_group.err
wc -l < gpurun_out/bench_group.json
cat gpurun_out/bench_group.json
