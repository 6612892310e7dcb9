# Scaling emulation, channel sweep (see scripts/gpu_emulate_r05.sh)
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/emu_r05b.jsonl
: > $O
for ARGS in "--emulate-rs -1" "--emulate-rs 4 --emulate-channels 128" "--emulate-rs 8 --emulate-channels 128" "--emulate-rs 4 --emulate-channels 256" "--emulate-rs 8 --emulate-channels 256" "--emulate-rs 8 --emulate-channels 64 --pieces 4"; do
  timeout -k 10 200 python bench.py --group $ARGS --no-cpu --sparse-steps 0 --legs "" --steps 300 --warmup 50 > gpurun_out/emu_one.json 2> gpurun_out/emu_one.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/emu_one.json')); print(json.dumps({'args': sys.argv[1], 'ms_per_step': d['ms_per_step'], 'pre_us': d['roofline'].get('avg_kernel_us')}))" "$ARGS" >> $O
done
cat $O
