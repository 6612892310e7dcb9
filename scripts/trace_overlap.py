"""Per-launch durations of one kernel and the kernels that overlap each launch
(rocprofv3 --kernel-trace CSV): median duration, the launches split by whether
another queue's kernel ran beside them, and the overlapping kernels' total time.

  python scripts/trace_overlap.py gpurun_out/trace_grp/run_kernel_trace.csv k_reduce_rows
"""
import collections
import csv
import statistics as st
import sys


def main(path, name):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows]
    main_k = [k for k in ks if name in k[2]]
    main_k = main_k[len(main_k) // 4: 3 * len(main_k) // 4]
    durs = [(e - s) / 1e3 for s, e, _, _ in main_k]
    print(f"{name}: {len(main_k)} launches (middle half), median {st.median(durs):.2f} us, "
          f"p10 {sorted(durs)[len(durs) // 10]:.2f} p90 {sorted(durs)[9 * len(durs) // 10]:.2f}")
    over = collections.Counter()
    for s, e, _, q in main_k:
        for s2, e2, n2, q2 in ks:
            if s2 >= e or e2 <= s or name in n2:
                continue
            over[n2.split("(")[0][:60]] += (min(e, e2) - max(s, s2)) / 1e3
    for n, t in over.most_common(12):
        print(f"  overlapping {n}: {t / len(main_k):.2f} us per launch")


if __name__ == "__main__":
    main(*sys.argv[1:3])
