# HBM traffic of the sparse leaf kernel (separate counter passes, no tracing)
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_sp_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --sparse-steps 3 > gpurun_out/pmc_sp_$c.log 2>&1
done
python3 - <<'PY'
import csv
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = {}
    for r in csv.DictReader(open(f"gpurun_out/pmc_sp_{c}/run_counter_collection.csv")):
        n = r["Kernel_Name"]
        if "k_sp_" in n or "k_array" in n:
            k = n.split("(")[0][-40:]
            acc.setdefault(k, []).append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(c, k, len(v), "avg KiB", round(sum(v) / len(v)))
PY
