# One GPU call: parity tests, smoke, default bench (with CPU baseline), rocprof
# kernel stats (dense and sparse) and separate FETCH_SIZE / WRITE_SIZE passes.
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stats -o run --output-format csv -- python3 bench.py --steps 200 --warmup 100 --no-cpu --sparse-steps 0 > gpurun_out/prof_stats.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sparse -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --sparse-steps 10 > gpurun_out/prof_sparse.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch -o run --output-format csv -- python3 bench.py --steps 10 --warmup 20 --no-cpu --sparse-steps 0 > gpurun_out/prof_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_write -o run --output-format csv -- python3 bench.py --steps 10 --warmup 20 --no-cpu --sparse-steps 0 > gpurun_out/prof_write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cfg5 -o run --output-format csv -- python3 bench.py --config 5 --cpu-seconds 2 > gpurun_out/prof_cfg5.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cfg4 -o run --output-format csv -- python3 bench.py --config 4 --cpu-seconds 2 > gpurun_out/prof_cfg4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cfg4-ada -o run --output-format csv -- python3 bench.py --config 4-ada --cpu-seconds 2 > gpurun_out/prof_cfg4-ada.log 2>&1
tail -1 gpurun_out/prof_cfg5.log
tail -1 gpurun_out/prof_cfg4.log
tail -1 gpurun_out/prof_cfg4-ada.log
echo all-done
