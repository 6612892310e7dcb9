# Round 6, third GPU call: AdaGrad parity on the new k_ada_ident, the default line,
# config 3 with the partition on part of the CUs (A/B), the geometry pair (third box).
export TMPDIR=/tmp; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fault/timeout rc=$1, stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "adagrad or ada or dense_floor" > gpurun_out/r06c_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; fatal $rc
grep -E "passed|failed" gpurun_out/r06c_tests.log | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/r06c_tests.log | head
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06c_bench.json 2> gpurun_out/r06c_bench.err; rc=$?; echo "bench rc=$rc"; fatal $rc
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r06c_bench.json"))
print("line", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["avg_kernel_us"])
for k in ("config4", "config5", "config4_ada", "sparse"):
    x = d.get(k, {}); r = x.get("roofline", {})
    print(k, x.get("ms_per_step"), r.get("frac"), r.get("kernel"), r.get("avg_kernel_us"), {kk: v for kk, v in r.items() if "floor" in kk})
PY
timeout -k 10 900 bash scripts/gpu_sparse_cu.sh > gpurun_out/sparse_cu.log 2>&1; rc=$?; echo "sparse cu rc=$rc"; fatal $rc
cat gpurun_out/sparse_cu.jsonl
timeout -k 10 200 scripts/ubench_geom alt 3 > gpurun_out/ubench_geom_alt_c.jsonl; rc=$?; echo "alt rc=$rc"; fatal $rc
python3 -c "
import json
for l in open('gpurun_out/ubench_geom_alt_c.jsonl'):
    d=json.loads(l); print(d['case'], d['round'], 'U', d['U_KiB_per_wave'], d['mode'], d['best_us'], d['frac_best'])
"
