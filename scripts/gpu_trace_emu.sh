# Kernel trace of the world-1 sharded line with the emulated 4-rank ring reduce-scatter
# (pieces 1 and 2): which kernels run beside each k_ring_rs launch and beside each
# pre-reduce piece (scripts/trace_overlap.py), DESIGN.md §6.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/emu_overlap.txt; : > $O
for P in 1 2; do
  T=emu4p$P
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/gpurun_out/trace_$T" -o run --output-format csv -- python3 bench.py --group --emulate-rs 4 --emulate-channels 64 --pieces $P --no-cpu --sparse-steps 0 --legs none --steps 100 --warmup 20 > gpurun_out/trace_$T.log 2>&1
  F=$(find gpurun_out/trace_$T -name "*kernel_trace.csv" | head -1)
  echo "## pieces $P: $(tail -1 gpurun_out/trace_$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ms_per_step", d["ms_per_step"])')" >> $O
  python3 scripts/trace_overlap.py $F k_ring_rs >> $O
  python3 scripts/trace_overlap.py $F k_reduce_rows >> $O
done
cat $O
