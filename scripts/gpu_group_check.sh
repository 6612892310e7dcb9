set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "sampled_timing or oneshot or sharded_speculation or shard_group or headline" > gpurun_out/gpu_sel.log 2>&1 || { tail -30 gpurun_out/gpu_sel.log; exit 1; }
tail -1 gpurun_out/gpu_sel.log
timeout -k 10 200 python bench.py --group --no-cpu --sparse-steps 0 --legs x > gpurun_out/bench_group.json 2> gpurun_out/bench_group.err
python -c "import json;g=json.load(open('gpurun_out/bench_group.json'));print(g['ms_per_step'], g['roofline']['avg_kernel_us'])"
TAG=group ARGS='--group --legs x --no-cpu --sparse-steps 0 --steps 200 --warmup 100' bash scripts/gpu_trace.sh
