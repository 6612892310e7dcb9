# k_ada_ident block shapes (256-thread blocks reducing maxDelta per block; per-wave
# candidates; 128 / 512-thread blocks), alternating builds on one box.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 1000 bash -c 'VARIANTS="adabase adawave ada128 ada512" ARGS="--legs 4a --sparse-steps 0 --no-cpu --steps 20 --warmup 5 --c4a-steps 4" LEG=config4_ada ROUNDS=2 bash scripts/ab_multi.sh' > gpurun_out/ab_ada_blocks.txt 2>&1; rc=$?
cp /tmp/ab_new.so distml_amd/libdistml_ps.so 2>/dev/null
echo "ab rc=$rc"; grep -v "^$" gpurun_out/ab_ada_blocks.txt
for v in adabase adawave ada128 ada512; do for r in 1 2; do python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['config4_ada']['roofline'];print(sys.argv[1].split('/')[-1], r['kernel'], r['avg_kernel_us'], r.get('measured_stream_floor_us'), r.get('frac_of_measured_floor'))" gpurun_out/abm_${v}_$r.json; done; done
