"""Per-kernel duration summary (rocprofv3 --stats layout) from a rocprofv3 rocpd database.

rocprofv3 on this image writes `<name>_results.db` (SQLite) by default; this reads its `kernels`
view and writes Name/Calls/TotalDurationNs/AverageNs/Percentage/MinNs/MaxNs as CSV.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db profiles/r01_kernel_stats_bench_full.csv
"""
import csv
import sqlite3
import sys


def main(db_path: str, out_path: str) -> None:
    con = sqlite3.connect(db_path)
    rows = con.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out_path, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, calls, tot, avg, mn, mx in rows:
            w.writerow([name, calls, tot, round(avg, 3), round(100.0 * tot / total, 3), mn, mx])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
