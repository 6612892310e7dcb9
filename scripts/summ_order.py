"""Print one line per exp_order.py log: row_order=median_us ..."""
import json
import sys

for path in sys.argv[1:]:
    parts = []
    for line in open(path):
        if line.startswith('{"row_order"'):
            d = json.loads(line)
            parts.append("%s=%.1f" % (d["row_order"], d["reduce_us_median"]))
    print(path, " ".join(parts))
