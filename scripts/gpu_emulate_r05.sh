# Scaling evidence on one GPU: the sharded config-2 path at world 1 with
# one rank's RING reduce-scatter footprint of N ranks (dml_diag_ring_rs) beside the
# real pre-reduce, N = 4 and 8, 32 and 64 channel blocks, pieces 1 and 2.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/emu_r05.jsonl
: > $O
for ARGS in "--emulate-rs 0" "--emulate-rs 4" "--emulate-rs 8" "--emulate-rs 4 --emulate-channels 64" "--emulate-rs 8 --emulate-channels 64" "--emulate-rs 4 --pieces 2" "--emulate-rs 8 --pieces 2" "--emulate-rs -1"; do
  timeout -k 10 200 python bench.py --group $ARGS --no-cpu --sparse-steps 0 --legs "" --steps 300 --warmup 50 > gpurun_out/emu_one.json 2> gpurun_out/emu_one.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/emu_one.json')); print(json.dumps({'args': sys.argv[1], 'ms_per_step': d['ms_per_step'], 'pre_us': d['roofline'].get('avg_kernel_us')}))" "$ARGS" >> $O
done
cat $O
