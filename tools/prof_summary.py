"""Per-kernel summary of a rocprofv3 run database (``-d DIR -o run``):
calls, total / mean microseconds and share of GPU time, largest first.

usage: python tools/prof_summary.py gpurun_out/prof_x/run_results.db [top]
"""
import sqlite3
import sys


def summary(path, top=25):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = db.execute("select {n}, count(*), sum(end - start) from kernels group by {n}".format(n=name)).fetchall()
    tot = sum(r[2] for r in rows) or 1
    rows.sort(key=lambda r: -r[2])
    out = ["{:>6} {:>10} {:>9} {:>6}  {}".format("calls", "total_us", "mean_us", "pct", "kernel")]
    for n, c, t in rows[:top]:
        out.append("{:>6} {:>10.0f} {:>9.1f} {:>6.2f}  {}".format(c, t / 1e3, t / 1e3 / c, 100.0 * t / tot, n[:110]))
    out.append("total GPU kernel time {:.1f} ms over {} kernels".format(tot / 1e6, sum(r[1] for r in rows)))
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25))
