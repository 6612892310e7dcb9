set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/gap_timing -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --sparse-steps 0 > gpurun_out/gap_timing.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/gap_notiming -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --sparse-steps 0 --no-timing > gpurun_out/gap_notiming.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 --no-timing
