# Config 3 with the partition's stream on part of the CUs (DML_KNOB_INDEX_CUS,
# VERDICT r5 #5): alternating splits in one box, 2 rounds, each its own process.
set -e
mkdir -p gpurun_out
O=gpurun_out/sparse_cu.jsonl
: > $O
for R in 1 2; do
for K in 0 16 32 48 64 65568 96; do
  timeout -k 10 120 python bench.py --legs "" --no-cpu --steps 50 --warmup 20 --sparse-steps 40 --sparse-cu-split $K > gpurun_out/sc.json 2> gpurun_out/sc.err
  python3 -c "import json;d=json.load(open('gpurun_out/sc.json'));s=d['sparse'];r=s['roofline'];print(json.dumps({'round':$R,'cu_split':$K,'ms_per_step':s['ms_per_step'],'leaf_us':r['avg_kernel_us'],'floor_us':r.get('measured_rmw_floor_us'),'headline_ms':d['ms_per_step']}))" >> $O
done
done
cat $O
