"""Kernel timeline from a rocprofv3 rocpd database: per-kernel durations and the idle gaps between
consecutive dispatches (e.g. inside a graph replay), for the last N dispatches."""
import sqlite3
import sys


def main(path, last=60):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    rows = rows[-last:]
    prev_end = None
    for n, s, e in rows:
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        print("%9.2f us  gap %8.2f us  %s" % ((e - s) / 1e3, gap, n[:90]))
        prev_end = e


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 60)
