"""Kernel statistics from a rocprofv3 SQLite output (run_results.db): name, calls, average /
median / min duration in us -- what `--stats` prints, for runs written in the rocpd format.
usage: python tools/rocpd_stats.py path/to/run_results.db [top]"""
import sqlite3
import statistics
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    cols = [r[1] for r in db.execute("pragma table_info(rocpd_kernel_dispatch)")]
    sym = [r[1] for r in db.execute("pragma table_info(rocpd_info_kernel_symbol)")]
    name_col = "display_name" if "display_name" in sym else "kernel_name"
    q = (f"select s.{name_col}, d.end - d.start from rocpd_kernel_dispatch d "
         f"join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    per = {}
    for name, dur in db.execute(q):
        per.setdefault(name, []).append(dur / 1000.0)
    rows = sorted(per.items(), key=lambda kv: -sum(kv[1]))[:top]
    print(f"{'calls':>7} {'avg_us':>9} {'med_us':>9} {'min_us':>9}  kernel")
    for name, d in rows:
        print(f"{len(d):7d} {sum(d) / len(d):9.2f} {statistics.median(d):9.2f} {min(d):9.2f}  {name[:110]}")
    _ = cols


if __name__ == "__main__":
    main()
