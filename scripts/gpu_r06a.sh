# Round 6, first GPU call: the geometry sweep, the new GPU tests, the default line.
# A step that times out or faults ends the call; an ordinary test failure does not.
export TMPDIR=/tmp; mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@"; local rc=$?
  echo "[step] $n rc=$rc"
  case $rc in 124|134|137|139) echo "[step] $n: fault/timeout, stopping"; exit $rc;; esac
  return 0
}
step geom 300 bash scripts/gpu_geom.sh > gpurun_out/geom.log 2>&1
tail -60 gpurun_out/geom.log
step tests 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "floor or int32_negative or config5_model or flat_kernel or adagrad_ident" \
  tests/test_native_group.py tests/test_jni_shim.py > gpurun_out/r06a_tests.log 2>&1
tail -5 gpurun_out/r06a_tests.log; grep -E "FAILED|Error" gpurun_out/r06a_tests.log | head -20
step bench 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.err
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r06a_bench.json"))
print("line", d["value"], d["ms_per_step"], d["roofline"]["frac"])
for k in ("config4", "config5", "config4_ada", "sparse"):
    x = d.get(k, {}); r = x.get("roofline", {})
    print(k, x.get("ms_per_step"), r.get("frac"), r.get("avg_kernel_us"), {kk: v for kk, v in r.items() if "floor" in kk})
PY
