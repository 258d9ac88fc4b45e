#!/usr/bin/env python3
"""Per-launch HBM traffic of the config-2 single-call GEMV from tools/pmc_gemv_single.sh.

The counter CSVs hold two groups of gemv_rpw_kernel dispatches: 20 single 4096x4096 calls and
5 calibration launches over 33 slices (different grids).  FETCH_SIZE's
scale for this access pattern = algorithmic bytes / raw FETCH of the calibration launches (312 MB
read once: no over-fetch, no cache hits possible); WRITE_SIZE counted as is (KiB).
usage: pmc_traffic_rpw.py FETCH.csv WRITE.csv OUT.json"""
import csv
import json
import statistics
import sys

SINGLE = 9437184 + 4352 + 16384            # A + B + C of one 4096x4096 q4_0 GEMV
STACKED = 33 * SINGLE


def groups(path, counter):
    """(single-call values, calibration values): the two Grid_Size buckets of gemv_rpw_kernel
    dispatches, told apart by count (tools/pmc_rpw.py: 20 single calls, 5 calibration launches)."""
    by = {}
    for r in csv.DictReader(open(path)):
        if "gemv_rpw_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            by.setdefault(r["Grid_Size"], []).append(float(r["Counter_Value"]))
    b = sorted(by.values(), key=len)
    return b[-1], b[0]


fs, fk = groups(sys.argv[1], "FETCH_SIZE")
ws, wk = groups(sys.argv[2], "WRITE_SIZE")
scale = STACKED / (statistics.median(fk) * 1024)
fetch = statistics.median(fs) * 1024 * scale
write = statistics.median(ws) * 1024
out = {"kernel": "gemv_rpw_kernel", "workload": "q4_0 4096x4096 GEMV, one call (BASELINE config 2)",
       "fetch_size_kib_raw": statistics.median(fs), "write_size_kib": statistics.median(ws),
       "launches": [len(fs), len(ws)],
       "fetch_scale": round(scale, 4),
       "calibration": f"33-slice launch of the same kernel: raw FETCH {statistics.median(fk):.0f} KiB for {STACKED} "
                      "algorithmic bytes (read once, > MALL)",
       "bytes_per_launch": int(fetch + write),
       "algorithmic_bytes_per_launch": SINGLE,
       "traffic_over_algorithmic": round((fetch + write) / SINGLE, 4)}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))
