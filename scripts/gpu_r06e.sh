# Config 2's record alignment against the flat stream (scripts/ubench_geom.hip rec), then
# the config-4 W = 8 / W = 32 legs.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 scripts/ubench_geom rec 3 > gpurun_out/ubench_geom_rec.jsonl; rc=$?; echo "rec rc=$rc"
cat gpurun_out/ubench_geom_rec.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['case'][:60], d['round'], d['best_us'], d['frac_best'])
"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python bench.py --legs 4w --sparse-steps 0 --no-cpu --steps 20 --warmup 5 > gpurun_out/r06e_w.json 2> gpurun_out/r06e_w.err; rc=$?; echo "w legs rc=$rc"
python3 -c "
import json
d=json.load(open('gpurun_out/r06e_w.json'))
for k in ('config4_w8','config4_w32'):
    x=d[k]; r=x['roofline']; print(k, x['workload'][:60], x['ms_per_step'], r['frac'], r['kernel'], r['avg_kernel_us'], r.get('frac_of_measured_floor'))
"
