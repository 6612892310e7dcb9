# sparse path: parity tests + rocprof kernel stats of the config-3 leg
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider -k "array or config3 or kat" > gpurun_out/sparse_tests.log 2>&1 || { tail -40 gpurun_out/sparse_tests.log; exit 1; }
tail -2 gpurun_out/sparse_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sp${TAG:-} -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --sparse-steps 5 > gpurun_out/prof_sp${TAG:-}.log 2>&1
grep -E '^\{' gpurun_out/prof_sp${TAG:-}.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['sparse'])"
python3 - <<'PY'
import csv
for r in csv.DictReader(open(__import__("os").environ.get("STATS","gpurun_out/prof_sp/run_kernel_stats.csv"))):
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
