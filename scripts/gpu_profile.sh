# rocprofv3 evidence for profiles/: kernel-trace stats of the default bench and
# separate FETCH_SIZE / WRITE_SIZE counter passes (never combined with tracing).
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python bench.py > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
cat gpurun_out/bench_prof.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stats -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --sparse-steps 0 > gpurun_out/prof_stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --sparse-steps 0 > gpurun_out/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_write -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --sparse-steps 0 > gpurun_out/prof_write.log 2>&1

timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sparse -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --sparse-steps 5 > gpurun_out/prof_sparse.log 2>&1
echo sparse-profile-done
