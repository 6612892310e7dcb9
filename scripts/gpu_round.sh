# Round evidence, in two GPU calls (each under gpurun's 20-minute limit):
#   PART=a: the -m gpu suite, smoke, the default bench line, the sharded path at world 1
#           (torch binding: plain, emulated 4- and 8-rank ring footprint on the pinned 128 channels;
#           native binding)
#   PART=b: the line profile (kernel stats + separate FETCH_SIZE / WRITE_SIZE passes,
#           scripts/gpu_prof.sh), the N = 2 legs rehearsed on one GPU (gloo), e2e rates
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
if [ "${PART:-a}" = a ]; then
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
for E in 0 4 8; do
timeout -k 10 200 python bench.py --group --emulate-rs $E --no-cpu --sparse-steps 0 --legs "" --steps 300 --warmup 50 > gpurun_out/bench_group_e$E.json 2> gpurun_out/bench_group_e$E.err
done
timeout -k 10 200 python bench.py --native-group --no-cpu --sparse-steps 0 --legs "" --steps 300 --warmup 50 > gpurun_out/bench_native.json 2> gpurun_out/bench_native.err
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench.json"))
print("line", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["launches"], d["roofline"]["avg_kernel_us"])
for k in ("config4", "config5", "config4_ada", "sparse"):
    x = d.get(k, {}); r = x.get("roofline", {})
    print(k, x.get("ms_per_step"), r.get("frac"), r.get("avg_kernel_us"))
for E in (0, 4, 8):
    g = json.load(open(f"gpurun_out/bench_group_e{E}.json")); print("group e", E, g["ms_per_step"], g["roofline"]["avg_kernel_us"])
n = json.load(open("gpurun_out/bench_native.json"))["native_group"]; print("native", n["ms_per_step"], n["roofline"]["avg_kernel_us"])
PY
else
TAG=line ARGS="--steps 200 --warmup 100 --no-cpu --legs 4,5,4a --c4-steps 3 --c4-warmup 1 --c5-steps 10 --c5-warmup 2 --c4a-steps 2 --c4a-warmup 1 --sparse-steps 10" bash scripts/gpu_prof.sh
timeout -k 10 400 python bench.py --gpus 2 --rehearse-gloo --legs 4,5,4a --c4-pushes 4 --no-cpu --steps 50 --warmup 20 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
python3 -c "import json;d=json.load(open('gpurun_out/rehearse2.json'));print('rehearse N=2', d['n_gpus'], d['ms_per_step'], sorted(k for k in d if k.startswith('config')))"
timeout -k 10 300 python scripts/e2e.py > gpurun_out/e2e.log 2>&1
tail -12 gpurun_out/e2e.log
fi
