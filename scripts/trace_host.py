"""Host enqueue against the GPU timeline for one kernel (rocprofv3 --kernel-trace
--hip-runtime-trace CSVs): for each dispatch, the gap from the previous dispatch's end
to its start, and when its launch call returned on the host relative to that end
(negative: enqueued while the previous one still ran). Medians over the middle half.

  python scripts/trace_host.py gpurun_out/trace_host k_reduce_rows
"""
import csv
import glob
import os
import statistics as st
import sys


def main(d, name):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ht = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0]
    api = {r["Correlation_Id"]: r for r in csv.DictReader(open(ht))}
    ks = sorted((r for r in csv.DictReader(open(kt)) if name in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    gap, late, dur = [], [], []
    for a, b in zip(ks, ks[1:]):
        e0, s1 = int(a["End_Timestamp"]), int(b["Start_Timestamp"])
        gap.append((s1 - e0) / 1e3)
        dur.append((int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3)
        c = api.get(b["Correlation_Id"])
        if c:
            late.append((int(c["End_Timestamp"]) - e0) / 1e3)
    m = slice(len(gap) // 4, 3 * len(gap) // 4)
    print(f"{name}: {len(ks)} dispatches; duration median {st.median(dur[m]):.2f} us; gap median {st.median(gap[m]):.2f} "
          f"p10 {sorted(gap[m])[len(gap[m]) // 10]:.2f} p90 {sorted(gap[m])[9 * len(gap[m]) // 10]:.2f} us")
    if late:
        lm = late[len(late) // 4: 3 * len(late) // 4]
        print(f"  launch call returned {st.median(lm):.2f} us after the previous dispatch ended (median; "
              f"p10 {sorted(lm)[len(lm) // 10]:.2f}, p90 {sorted(lm)[9 * len(lm) // 10]:.2f}); "
              f"{sum(1 for x in lm if x > 0)} of {len(lm)} enqueued after it ended")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
