set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "group or prereduce" > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]); print('single', d['ms_per_step'], d['value'], d['roofline']['avg_kernel_us'])"
for P in 1 2 4; do
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 --group --pieces $P > gpurun_out/bench_group.json 2> gpurun_out/bench_group.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench_group.json').read().strip().splitlines()[-1]); print('group P=$P', d['ms_per_step'], d['value'])"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tg -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu --sparse-steps 0 --group > gpurun_out/tg.log 2>&1
