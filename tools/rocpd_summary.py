"""Kernel summary (total, calls, average, share) from a rocprofv3 results database (its `top_kernels` view),
for runs made without --output-format csv. Usage: python tools/rocpd_summary.py results.db [top N]"""
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = name.split("(")[0] if not name.startswith("void at::") else name[:110]
    return name.replace("void ", "")


def main():
    db = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    for name, calls, tot, avg, pct in rows[:top]:   # the view's durations are in microseconds
        print(f"{tot / 1e3:10.3f} ms  calls={calls:5d}  avg={avg:10.2f} us  {pct:5.1f}%  {short(name)}")


if __name__ == "__main__":
    main()
