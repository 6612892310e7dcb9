# k_flat_ident shapes against the current one on one box (config-4 leg), alternating builds.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 1100 bash -c 'VARIANTS="base fij10d2 fij12d2 finoxcd" ARGS="--legs 4 --sparse-steps 0 --no-cpu --steps 20 --warmup 5 --c4-steps 4" LEG=config4 ROUNDS=2 bash scripts/ab_multi.sh' > gpurun_out/ab_flat_ident.txt 2>&1; rc=$?
cp /tmp/ab_new.so distml_amd/libdistml_ps.so 2>/dev/null
echo "ab rc=$rc"; cat gpurun_out/ab_flat_ident.txt | grep -v "^$"
for v in base fij10d2 fij12d2 finoxcd; do for r in 1 2; do python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['config4']['roofline'];print(sys.argv[1].split('/')[-1], r['kernel'], r['avg_kernel_us'], r.get('measured_stream_floor_us'), r.get('frac_of_measured_floor'))" gpurun_out/abm_${v}_$r.json; done; done
timeout -k 10 300 python bench.py --legs 4w --sparse-steps 0 --no-cpu --steps 20 --warmup 5 > gpurun_out/r06d_w.json 2> gpurun_out/r06d_w.err; rc=$?; echo "w legs rc=$rc"
python3 -c "
import json
d=json.load(open('gpurun_out/r06d_w.json'))
for k in ('config4_w8','config4_w32'):
    x=d[k]; r=x['roofline']; print(k, x['workload'][:60], x['ms_per_step'], r['frac'], r['avg_kernel_us'], r.get('frac_of_measured_floor'))
"
