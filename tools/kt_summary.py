#!/usr/bin/env python3
"""Median / min kernel durations (us) by kernel name from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = re.sub(r"\(lamm::GemvArgs.*", "", r["Kernel_Name"]).replace("lamm::(anonymous namespace)::", "")
    d[n[:90]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in d.items():
    print(f"{k:90s} n={len(v):4d} median={statistics.median(v):8.2f} min={min(v):8.2f}")
