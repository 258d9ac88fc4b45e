#!/usr/bin/env python3
"""kt_roofline.py TRACE.csv OUT.json [kernel-substring] -- per-dispatch durations of the config-2
kernel from a rocprofv3 kernel trace of tools/roofline_trace.py (paced launches), with the
start-to-start gaps that show the dispatches did not queue behind each other."""
import csv
import json
import statistics as st
import sys

ALG = 9437184 + 4352 + 16384   # A + B + C of one q4_0 4096x4096 GEMV (BASELINE config 2)
name = sys.argv[3] if len(sys.argv) > 3 else "gemv_flat1_kernel<2, false>"
rows = [r for r in csv.DictReader(open(sys.argv[1])) if name in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
s = sorted(int(r["Start_Timestamp"]) for r in rows)
gaps = [(s[i + 1] - s[i]) / 1e3 for i in range(len(s) - 1)]
out = {"kernel": rows[0]["Kernel_Name"] if rows else name, "dispatches": len(d),
       "duration_us": {"median": round(st.median(d), 3), "mean": round(st.mean(d), 3), "min": round(min(d), 3),
                       "max": round(max(d), 3)},
       "start_to_start_us_median": round(st.median(gaps), 3) if gaps else None,
       "algorithmic_bytes_per_launch": ALG,
       "frac_of_8TBs_at_median": round(ALG / (st.median(d) * 1e-6) / 8e12, 4),
       "frac_of_8TBs_at_mean": round(ALG / (st.mean(d) * 1e-6) / 8e12, 4),
       "source": "rocprofv3 --kernel-trace --stats of tools/roofline_trace.py (tools/roofline_trace.sh)"}
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out))
