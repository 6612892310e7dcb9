"""Summarize rocprofv3 output (gpurun_out/prof_*) into profiles/<tag>_*.

- <tag>_kernel_stats.csv : rocprofv3 --kernel-trace --stats summary (verbatim)
- <tag>_summary.md       : per-kernel table + HBM traffic of the dominant kernel
- pmc_traffic.json       : HBM bytes per k_reduce launch, read by bench.py

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE
are in KiB, collected in separate --pmc passes; on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read, so it is doubled.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
ALGO = 32 * 67_174_400 + 2 * 67_108_864


def counter_avg(path, name_part):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if name_part in r["Kernel_Name"]]
    return sum(vals) / len(vals), len(vals)


def main(tag):
    os.makedirs(PROF, exist_ok=True)
    stats = os.path.join(OUT, "prof_stats", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    fetch_kib, nf = counter_avg(os.path.join(OUT, "prof_fetch", "run_counter_collection.csv"), "k_reduce")
    write_kib, nw = counter_avg(os.path.join(OUT, "prof_write", "run_counter_collection.csv"), "k_reduce")
    read_b = fetch_kib * 1024 * 2
    write_b = write_kib * 1024
    traffic = read_b + write_b
    red = [r for r in rows if "k_reduce" in r["Name"]][0]
    avg_ns = float(red["AverageNs"])
    json.dump({"kernel": red["Name"], "hbm_bytes_per_launch": round(traffic),
               "fetch_bytes_corrected": round(read_b), "write_bytes": round(write_b),
               "algorithmic_bytes_per_launch": ALGO, "traffic_over_algorithmic": round(traffic / ALGO, 4),
               "rocprof_avg_ns": avg_ns, "source": f"profiles/{tag}_kernel_stats.csv + FETCH_SIZE/WRITE_SIZE passes"},
              open(os.path.join(PROF, "pmc_traffic.json"), "w"), indent=1)
    bench = ""
    bp = os.path.join(OUT, "bench_prof.json")
    if os.path.exists(bp):
        bench = open(bp).read().strip()
    with open(os.path.join(PROF, f"{tag}_summary.md"), "w") as f:
        f.write(f"# {tag}: rocprofv3 summary (MI355X, config 2 bench, 200 timed steps)\n\n")
        f.write("Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 200 --warmup 100 "
                "--no-cpu --sparse-steps 0`; counters: separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes.\n\n")
        f.write("| kernel | calls | avg µs | min µs | max µs | % time |\n|---|---|---|---|---|---|\n")
        for r in rows:
            f.write(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                    f"{float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |\n")
        f.write(f"\n## Dominant kernel HBM traffic (k_reduce, per launch, {nf}/{nw} launches sampled)\n\n")
        f.write(f"- FETCH_SIZE {fetch_kib:.0f} KiB x 1024 x 2 (gfx950 correction) = {read_b/1e9:.4f} GB read\n")
        f.write(f"- WRITE_SIZE {write_kib:.0f} KiB x 1024 = {write_b/1e9:.4f} GB written\n")
        f.write(f"- total {traffic/1e9:.4f} GB vs algorithmic {ALGO/1e9:.4f} GB "
                f"(x{traffic/ALGO:.3f}); rocprof avg {avg_ns/1e3:.1f} µs -> "
                f"{ALGO/avg_ns:.1f} GB/s algorithmic, {traffic/avg_ns:.1f} GB/s measured traffic\n")
        if bench:
            f.write(f"\n## bench.py line of the same box\n\n```\n{bench}\n```\n")
    sp = os.path.join(OUT, "prof_sparse", "run_kernel_stats.csv")
    if os.path.exists(sp):
        shutil.copy(sp, os.path.join(PROF, f"{tag}_sparse_kernel_stats.csv"))
        with open(os.path.join(PROF, f"{tag}_summary.md"), "a") as f:
            f.write("\n## Sparse leg (config 3), `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 2 "
                    "--warmup 1 --no-cpu --sparse-steps 10`\n\n| kernel | calls | avg µs | % time |\n|---|---|---|---|\n")
            for r in csv.DictReader(open(sp)):
                f.write(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                        f"{float(r['Percentage']):.1f} |\n")
    for cfg in ("5", "4", "4-ada"):
        cs = os.path.join(OUT, f"prof_cfg{cfg}", "run_kernel_stats.csv")
        if not os.path.exists(cs):
            continue
        shutil.copy(cs, os.path.join(PROF, f"{tag}_cfg{cfg}_kernel_stats.csv"))
        lines = [l for l in open(os.path.join(OUT, f"prof_cfg{cfg}.log")) if l.startswith("{")]
        with open(os.path.join(PROF, f"{tag}_summary.md"), "a") as f:
            f.write(f"\n## Config {cfg}, one GPU's shard (`rocprofv3 --kernel-trace --stats -- python3 bench.py "
                    f"--config {cfg} --cpu-seconds 2`)\n\n| kernel | calls | avg µs | % time |\n|---|---|---|---|\n")
            for r in csv.DictReader(open(cs)):
                f.write(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                        f"{float(r['Percentage']):.1f} |\n")
            if lines:
                f.write("\nbench line of the same run (under the profiler):\n\n```\n" + lines[-1] + "```\n")
    print(open(os.path.join(PROF, f"{tag}_summary.md")).read())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
