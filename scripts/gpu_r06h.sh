# The default line and the world-1 group lines (plain, emulated 4 / 8 ranks on the pinned
# 128 channels, native binding) on the current sources.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
for E in 0 4 8; do
timeout -k 10 200 python bench.py --group --emulate-rs $E --no-cpu --sparse-steps 0 --legs "" --steps 300 --warmup 50 > gpurun_out/bench_group_e$E.json 2> gpurun_out/bench_group_e$E.err
done
timeout -k 10 200 python bench.py --native-group --no-cpu --sparse-steps 0 --legs "" --steps 300 --warmup 50 > gpurun_out/bench_native.json 2> gpurun_out/bench_native.err
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench.json"))
print("line", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["launches"], d["roofline"]["avg_kernel_us"])
for k in ("config4", "config4_w8", "config4_w32", "config5", "config4_ada", "sparse"):
    x = d.get(k, {}); r = x.get("roofline", {})
    print(k, x.get("ms_per_step"), r.get("frac"), r.get("avg_kernel_us"), {kk: v for kk, v in r.items() if "floor" in kk})
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["all_cores"]["value"])
for E in (0, 4, 8):
    g = json.load(open(f"gpurun_out/bench_group_e{E}.json")); print("group e", E, g["ms_per_step"], g["roofline"]["avg_kernel_us"], g["config"]["rccl_channels"])
n = json.load(open("gpurun_out/bench_native.json"))["native_group"]; print("native", n["ms_per_step"], n["roofline"]["avg_kernel_us"])
PY
