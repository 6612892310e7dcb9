# k_ada_flat block size with the write-burst barrier: 4 / 12 waves against the old (4, no barrier)
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
for V in ada4b ada12b adaold ada4b ada12b adaold; do
  cp scripts/ab/libdistml_ps_$V.so distml_amd/libdistml_ps.so
  timeout -k 10 300 python bench.py --legs 4a --sparse-steps 0 --no-cpu --steps 5 --warmup 2 > gpurun_out/ab2_$V.json 2> gpurun_out/ab2_$V.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); x=d['config4_ada']; print(sys.argv[2], x['ms_per_step'], x['roofline']['frac'], x['roofline']['avg_kernel_us'], x['roofline']['kernel'])" gpurun_out/ab2_$V.json $V
done
