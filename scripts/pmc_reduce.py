"""Reduce rocprofv3 --pmc CSV output to per-kernel means per dispatch (diagnostic).
  python3 scripts/pmc_reduce.py OUT.json DIR [DIR ...] --match k_ada_flat k_flat_ident ...
Reads DIR/**/​*counter_collection.csv, keeps kernels whose name contains a --match
substring, and writes {kernel: {counter: mean per dispatch, "dispatches": n, "vgpr": v}}."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    out = args[0]
    i = args.index("--match")
    dirs, pats = args[1:i], args[i + 1:]
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f, newline="") as fh:
                for r in csv.DictReader(fh):
                    k = r["Kernel_Name"]
                    if not any(p in k for p in pats):
                        continue
                    key = k.split("(")[0]
                    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
                    disp[key].add((f, r["Dispatch_Id"]))
                    meta[key] = {"vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]),
                                 "wg": int(r["Workgroup_Size"]), "grid": int(r["Grid_Size"])}
    res = {}
    for k, cs in acc.items():
        n = len(disp[k])
        # every counter appears once per dispatch and pass directory
        res[k] = {c: v / n * len(dirs) for c, v in sorted(cs.items())}
        res[k].update(meta[k])
        res[k]["dispatches_per_pass"] = n / len(dirs)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
