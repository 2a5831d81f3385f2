"""Per-kernel statistics from a rocprofv3 results database (rocpd SQLite, the default
output of `rocprofv3 --kernel-trace` on this image), as `--stats` would print them:

  python3 profiles/kstats_db.py gpurun_out/<dir>/<name>_results.db [--csv out.csv] [--match substr]
"""
import argparse
import csv
import sqlite3
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default="")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    by = {}
    for name, st, en in rows:
        if a.match and a.match not in name:
            continue
        by.setdefault(name, []).append((en - st) / 1e3)  # us
    out = []
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        out.append({"kernel": name[:160], "calls": len(v), "total_us": round(sum(v), 2),
                    "avg_us": round(statistics.mean(v), 2), "median_us": round(statistics.median(v), 2),
                    "min_us": round(min(v), 2), "max_us": round(max(v), 2)})
    w = csv.DictWriter(open(a.csv, "w") if a.csv else sys.stdout, fieldnames=list(out[0]) if out else ["kernel"])
    w.writeheader()
    w.writerows(out)


if __name__ == "__main__":
    main()
