# rocprofv3 evidence for one bench workload (profiles/): a --kernel-trace --stats
# pass, then separate FETCH_SIZE and WRITE_SIZE counter passes (never combined
# with tracing; each pass its own time limit, MI355X_MICROARCH.md rocprofv3 PMC).
#   TAG=cfg5 ARGS="--config 5 --no-cpu" bash scripts/gpu_prof.sh
# Outputs gpurun_out/prof_<TAG>_{stats,fetch,write}/ ; scripts/summarize_profiles.py
# turns them into profiles/<round>_<TAG>_* and the pmc_traffic.json entry.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:?TAG required}
A=${ARGS:-}
O=$PWD/gpurun_out
# the device sources these counters stand for (bench.py's traffic_for checks it)
python3 -c "import bench, json; print(json.dumps(bench.device_src_hashes()))" > "$O/prof_${T}_src.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_${T}_stats" -o run --output-format csv -- python3 bench.py $A > "$O/prof_${T}_stats.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/prof_${T}_fetch" -o run --output-format csv -- python3 bench.py $A > "$O/prof_${T}_fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/prof_${T}_write" -o run --output-format csv -- python3 bench.py $A > "$O/prof_${T}_write.log" 2>&1
echo "prof $T done"
