"""Per-kernel summary (calls, avg/min/max/total duration) from a rocprofv3 rocpd SQLite database.

With --phases (the bench run under `rocprofv3 --kernel-trace --marker-trace`), kernels are grouped by
the roctx range they ran in: bench.py wraps each leg in `fdbench:<leg>` (class phase), so e.g. the
k_corner launches that bench.py's roofline timed are the rows of phase `fdbench:roofline_kernel`.
"""
import sqlite3
import sys


def summary(path, phases=False):
    c = sqlite3.connect(path)
    if phases:
        q = ("select coalesce(region, ''), name, count(*), avg(duration), min(duration), max(duration), sum(duration) "
             "from kernels group by region, name order by region, 7 desc")
        out = ["phase,name,calls,avg_us,min_us,max_us,total_ms"]
        for r, n, k, a, lo, hi, t in c.execute(q).fetchall():
            out.append('"%s","%s",%d,%.2f,%.2f,%.2f,%.3f' % (r, n.replace('"', "'"), k, a / 1e3, lo / 1e3, hi / 1e3,
                                                             t / 1e6))
        return "\n".join(out)
    rows = c.execute("select name, count(*), avg(duration), min(duration), max(duration), sum(duration) "
                     "from kernels group by name order by 6 desc").fetchall()
    out = ["name,calls,avg_us,min_us,max_us,total_ms"]
    for n, k, a, lo, hi, t in rows:
        out.append('"%s",%d,%.2f,%.2f,%.2f,%.3f' % (n.replace('"', "'"), k, a / 1e3, lo / 1e3, hi / 1e3, t / 1e6))
    return "\n".join(out)


if __name__ == "__main__":
    args = sys.argv[1:]
    ph = "--phases" in args
    for p in [a for a in args if a != "--phases"]:
        print("#", p)
        print(summary(p, ph))
