"""Convert a rocprofv3 .db (rocpd sqlite) into the kernel-stats CSV layout of
`rocprofv3 --stats --output-format csv` (Name, Calls, TotalDurationNs, AverageNs,
Percentage).  Usage: python tools/rocpd_stats.py <results.db> <out.csv>"""
import csv
import sqlite3
import sys


def main(db, out):
    con = sqlite3.connect(db)
    rows = con.execute('select name, total_calls, total_duration, average, percentage '
                       'from top_kernels order by total_duration desc').fetchall()
    with open(out, 'w', newline='') as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage'])
        for name, calls, tot_us, avg_us, pct in rows:
            # top_kernels reports microseconds
            w.writerow([name, int(calls), round(tot_us * 1e3), round(avg_us * 1e3, 3), round(pct, 3)])


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
