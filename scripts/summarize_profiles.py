"""Summarize scripts/gpu_prof.sh output (gpurun_out/prof_<tag>_*) into profiles/.

  python scripts/summarize_profiles.py <round> <tag> <kernel-substring> <algorithmic-bytes-per-launch> [cmd]

- profiles/<round>_<tag>_kernel_stats.csv : the --kernel-trace --stats summary (verbatim)
- profiles/<round>_<tag>_summary.md       : per-kernel table + HBM traffic of the dominant kernel
- profiles/pmc_traffic.json               : per_config[<tag>] (config2 also at the top level),
                                            read by bench.py as roofline.traffic

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE
are KiB, collected in separate --pmc passes; on gfx950 FETCH_SIZE reports half
the bytes of a wide coalesced streaming read (16 B/lane), so it is doubled.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def counter_avg(path, name_part):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if name_part in r["Kernel_Name"]]
    return sum(vals) / len(vals), len(vals)


def main(rnd, tag, kpart, algo, cmd=""):
    os.makedirs(PROF, exist_ok=True)
    algo = int(float(algo))
    stats = os.path.join(OUT, f"prof_{tag}_stats", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(PROF, f"{rnd}_{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    fetch_kib, nf = counter_avg(os.path.join(OUT, f"prof_{tag}_fetch", "run_counter_collection.csv"), kpart)
    write_kib, nw = counter_avg(os.path.join(OUT, f"prof_{tag}_write", "run_counter_collection.csv"), kpart)
    read_b, write_b = fetch_kib * 1024 * 2, write_kib * 1024
    traffic = read_b + write_b
    dom = [r for r in rows if kpart in r["Name"]][0]
    avg_ns = float(dom["AverageNs"])
    entry = {"kernel": dom["Name"], "hbm_bytes_per_launch": round(traffic), "fetch_bytes_corrected": round(read_b),
             "write_bytes": round(write_b), "algorithmic_bytes_per_launch": algo,
             "traffic_over_algorithmic": round(traffic / algo, 4), "rocprof_avg_ns": avg_ns,
             "achieved_algorithmic_GBps": round(algo / avg_ns, 1),
             "source": f"profiles/{rnd}_{tag}_kernel_stats.csv + FETCH_SIZE/WRITE_SIZE passes ({cmd})"}
    pj = os.path.join(PROF, "pmc_traffic.json")
    d = json.load(open(pj)) if os.path.exists(pj) else {}
    d.setdefault("per_config", {})[tag] = entry
    if tag == "config2":
        d.update({k: v for k, v in entry.items()})
    json.dump(d, open(pj, "w"), indent=1)
    with open(os.path.join(PROF, f"{rnd}_{tag}_summary.md"), "w") as f:
        f.write(f"# {rnd} {tag}: rocprofv3 summary (MI355X)\n\n")
        f.write(f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py {cmd}`; counters: separate "
                "`--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes of the same command (scripts/gpu_prof.sh).\n\n")
        f.write("| kernel | calls | avg µs | min µs | max µs | % time |\n|---|---|---|---|---|---|\n")
        for r in rows:
            f.write(f"| `{r['Name'][:100]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                    f"{float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |\n")
        f.write(f"\n## Dominant kernel HBM traffic (`{kpart}`, per launch, {nf}/{nw} launches sampled)\n\n")
        f.write(f"- FETCH_SIZE {fetch_kib:.0f} KiB x 1024 x 2 (gfx950 correction) = {read_b/1e9:.4f} GB read\n")
        f.write(f"- WRITE_SIZE {write_kib:.0f} KiB x 1024 = {write_b/1e9:.4f} GB written\n")
        f.write(f"- total {traffic/1e9:.4f} GB vs algorithmic {algo/1e9:.4f} GB (x{traffic/algo:.3f})\n")
        f.write(f"- rocprof average {avg_ns/1e3:.1f} µs -> {algo/avg_ns:.1f} GB/s algorithmic, "
                f"{algo/avg_ns/8000:.3f} of 8 TB/s; {traffic/avg_ns:.1f} GB/s of counted traffic\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
