"""Per-kernel summary (calls, avg/min/max/total duration) from a rocprofv3 rocpd SQLite database."""
import sqlite3
import sys


def summary(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), avg(duration), min(duration), max(duration), sum(duration) "
                     "from kernels group by name order by 6 desc").fetchall()
    out = ["name,calls,avg_us,min_us,max_us,total_ms"]
    for n, k, a, lo, hi, t in rows:
        out.append('"%s",%d,%.2f,%.2f,%.2f,%.3f' % (n.replace('"', "'"), k, a / 1e3, lo / 1e3, hi / 1e3, t / 1e6))
    return "\n".join(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print("#", p)
        print(summary(p))
