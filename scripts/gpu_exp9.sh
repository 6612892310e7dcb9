set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
for rep in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]); print('single', d['ms_per_step'], d['value'], d['roofline']['avg_kernel_us'])"
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 --group > gpurun_out/bench_group.json 2> gpurun_out/bench_group.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench_group.json').read().strip().splitlines()[-1]); print('group', d['ms_per_step'], d['value'])"
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 > gpurun_out/bench4.json 2> gpurun_out/bench4.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench4.json').read().strip().splitlines()[-1]); print('single q4', d['ms_per_step'], d['value'], d['roofline']['avg_kernel_us'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tg -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu --sparse-steps 0 --group > gpurun_out/tg.log 2>&1
