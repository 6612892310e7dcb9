"""Gaps between consecutive dispatches of one kernel (rocprofv3 --kernel-trace CSV,
scripts/gpu_trace.sh): median / mean idle time from one launch's end to the next
one's start, and the kernels that ran inside a sample gap.

  python scripts/trace_gaps.py gpurun_out/trace_cfg2/run_kernel_trace.csv k_reduce_rows
"""
import csv
import statistics as st
import sys


def main(path, name, show=2):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if name in r["Kernel_Name"]]
    s = [int(rows[i]["Start_Timestamp"]) for i in idx]
    e = [int(rows[i]["End_Timestamp"]) for i in idx]
    gaps = [s[k + 1] - e[k] for k in range(len(idx) - 1)]
    mid = gaps[len(gaps) // 4: 3 * len(gaps) // 4] or gaps
    dur = [e[k] - s[k] for k in range(len(idx))]
    print(f"{name}: {len(idx)} launches, duration median {st.median(dur) / 1e3:.2f} us, "
          f"gap median {st.median(mid) / 1e3:.2f} us mean {st.mean(mid) / 1e3:.2f} us (middle half)")
    for k in range(len(idx) // 2, len(idx) // 2 + show):
        a, b = idx[k], idx[k + 1]
        t0 = e[k]
        print("--- one gap")
        for r in rows[max(0, a - 3): b + 1]:
            print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:10.2f} {(int(r['End_Timestamp']) - t0) / 1e3:10.2f} "
                  f"q{r['Queue_Id']} {r['Kernel_Name'][:60]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2)
