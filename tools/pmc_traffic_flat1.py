#!/usr/bin/env python3
"""Per-launch HBM traffic of config 2's kernel (gemv_flat1_kernel) from tools/pmc_flat1.sh.

FETCH_SIZE's scale for this access pattern = algorithmic bytes / raw FETCH of the calibration
launches (gemv_flat_kernel over 33 slices: the same body, 312 MB read once -- no over-fetch, no
cache hits possible; MI355X_MICROARCH.md: other access widths than 16-B streaming reads are
uncalibrated, calibrate on a known byte count); WRITE_SIZE counted as is (KiB).
usage: pmc_traffic_flat1.py FETCH.csv WRITE.csv OUT.json"""
import csv
import json
import statistics
import sys

SINGLE = 9437184 + 4352 + 16384            # A + B + C of one 4096x4096 q4_0 GEMV
STACKED = 33 * SINGLE


def vals(path, counter, kernel):
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]


fs, fk = vals(sys.argv[1], "FETCH_SIZE", "gemv_flat1_kernel"), vals(sys.argv[1], "FETCH_SIZE", "gemv_flat_kernel")
ws = vals(sys.argv[2], "WRITE_SIZE", "gemv_flat1_kernel")
scale = STACKED / (statistics.median(fk) * 1024)
fetch = statistics.median(fs) * 1024 * scale
write = statistics.median(ws) * 1024
out = {"kernel": "gemv_flat1_kernel", "workload": "q4_0 4096x4096 GEMV, one call (BASELINE config 2)",
       "fetch_size_kib_raw": statistics.median(fs), "write_size_kib": statistics.median(ws),
       "launches": [len(fs), len(ws)],
       "fetch_scale": round(scale, 4),
       "calibration": f"gemv_flat_kernel over 33 slices (the same body): raw FETCH {statistics.median(fk):.0f} KiB for "
                      f"{STACKED} algorithmic bytes (read once, > MALL)",
       "bytes_per_launch": int(fetch + write),
       "algorithmic_bytes_per_launch": SINGLE,
       "traffic_over_algorithmic": round((fetch + write) / SINGLE, 4)}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))
