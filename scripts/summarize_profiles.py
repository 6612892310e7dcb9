"""Summarize scripts/gpu_prof.sh output (gpurun_out/prof_<tag>_*) into profiles/.

  python scripts/summarize_profiles.py <round> <tag> "<bench args>" <key>=<kernel-substring>=<algo-bytes>[=<stream-bytes>] ...

One profiled run can hold several measured kernels (the default bench line runs
config 2, the config-4/5 legs and the sparse leg); each <key> names one of them
by a substring of its full kernel name and its algorithmic bytes per dispatch.
<stream-bytes>: for a kernel whose reads are only partly wide coalesced streams,
the algorithmic bytes of that streamed part (default: all reads streamed).

- profiles/<round>_<tag>_kernel_stats.csv : the --kernel-trace --stats summary (verbatim)
- profiles/<round>_<tag>_summary.md       : per-kernel table + HBM traffic per key
- profiles/pmc_traffic.json               : per_config[<key>], read by bench.py as roofline.traffic
                                            only for the same kernel instantiation and device
                                            sources (src_sha, written on the box by gpu_prof.sh)

HBM bytes per dispatch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE
are KiB, collected in separate --pmc passes. On gfx950 FETCH_SIZE reports half
the bytes of a wide coalesced streaming read, so the read side of the streaming
reduce kernels is doubled. The sparse kernels mix such streams (their 8-B key and
4-B value arrays: the partition passes' raw FETCH_SIZE is half their streamed
bytes, i.e. the same rule holds at 8 B/lane) with scattered line reads that are
counted whole; their read bytes are raw + stream/2.
"""
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def counter_avg(path, name_part):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if name_part in r["Kernel_Name"]]
    assert vals, (path, name_part)
    return sum(vals) / len(vals), len(vals)


def main(rnd, tag, cmd, *specs):
    os.makedirs(PROF, exist_ok=True)
    stats = os.path.join(OUT, f"prof_{tag}_stats", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(PROF, f"{rnd}_{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    pj = os.path.join(PROF, "pmc_traffic.json")
    d = json.load(open(pj)) if os.path.exists(pj) else {}
    d = {"per_config": d.get("per_config", {})}
    src_txt = open(os.path.join(OUT, f"prof_{tag}_src.txt")).read().strip()
    # gpu_prof.sh writes bench.device_src_hashes() (per kernel group + "all"); older
    # runs wrote the one all-sources hash
    by_group = json.loads(src_txt) if src_txt.startswith("{") else {}
    src_sha = by_group.pop("all", src_txt) if by_group else src_txt
    try:
        commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                                text=True, check=True).stdout.strip()
        if subprocess.run(["git", "-C", ROOT, "diff", "--quiet", "HEAD", "--", "distml_amd/csrc"]).returncode:
            commit += "+uncommitted"
    except Exception:
        commit = "?"
    md = [f"# {rnd} {tag}: rocprofv3 summary (MI355X)\n",
          f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py {cmd}`; counters: separate "
          "`--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes of the same command (scripts/gpu_prof.sh).\n",
          "| kernel | calls | avg µs | min µs | max µs | % time |", "|---|---|---|---|---|---|"]
    for r in rows:
        md.append(f"| `{r['Name'][:110]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                  f"{float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
    for spec in specs:
        f = spec.split("=")
        key, kpart, algo = f[0], f[1], int(float(f[2]))
        stream = int(float(f[3])) if len(f) > 3 else None
        fetch_kib, nf = counter_avg(os.path.join(OUT, f"prof_{tag}_fetch", "run_counter_collection.csv"), kpart)
        write_kib, nw = counter_avg(os.path.join(OUT, f"prof_{tag}_write", "run_counter_collection.csv"), kpart)
        raw = fetch_kib * 1024
        read_b = 2 * raw if stream is None else raw + stream / 2
        corr = round(read_b / raw, 4)
        write_b = write_kib * 1024
        traffic = read_b + write_b
        dom = [r for r in rows if kpart in r["Name"]]
        assert len(dom) == 1, (kpart, [r["Name"] for r in dom])
        dom = dom[0]
        avg_ns = float(dom["AverageNs"])
        entry = {"kernel": dom["Name"], "hbm_bytes_per_launch": round(traffic), "fetch_bytes_corrected": round(read_b),
                 "fetch_correction": corr, "fetch_bytes_raw": round(fetch_kib * 1024), "write_bytes": round(write_b),
                 "algorithmic_bytes_per_launch": algo, "traffic_over_algorithmic": round(traffic / algo, 4),
                 "rocprof_avg_ns": avg_ns, "achieved_algorithmic_GBps": round(algo / avg_ns, 1),
                 "source": f"profiles/{rnd}_{tag}_kernel_stats.csv + FETCH_SIZE/WRITE_SIZE passes ({cmd})",
                 "src_sha": src_sha, "commit": commit}
        if by_group:
            entry["src_sha_by_group"] = by_group
        d["per_config"][key] = entry
        md += ["", f"## {key}: `{kpart}` ({nf}/{nw} dispatches sampled)", "",
               (f"- FETCH_SIZE {fetch_kib:.0f} KiB x 1024 x 2 = {read_b/1e9:.4f} GB read (gfx950 wide-read correction)"
                if stream is None else
                f"- FETCH_SIZE {fetch_kib:.0f} KiB x 1024 = {raw/1e9:.4f} GB + half of the {stream/1e9:.3f} GB "
                f"streamed = {read_b/1e9:.4f} GB read"),
               f"- WRITE_SIZE {write_kib:.0f} KiB x 1024 = {write_b/1e9:.4f} GB written",
               f"- total {traffic/1e9:.4f} GB vs algorithmic {algo/1e9:.4f} GB (x{traffic/algo:.3f})",
               f"- rocprof average {avg_ns/1e3:.1f} µs -> {algo/avg_ns:.1f} GB/s algorithmic, "
               f"{algo/avg_ns/8000:.3f} of 8 TB/s; {traffic/avg_ns:.1f} GB/s of counted traffic"]
    json.dump(d, open(pj, "w"), indent=1)
    with open(os.path.join(PROF, f"{rnd}_{tag}_summary.md"), "w") as f:
        f.write("\n".join(md) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
