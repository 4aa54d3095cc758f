"""Per-kernel duration summary of a rocprofv3 results database (.db):
   python3 tools/db_kstats.py RUN_results.db [NAME_FILTER]
Prints n, median, min and max (us) per kernel name, largest total first.
Under bench.py the serial-schedule proofs run each kernel alone, so for
kernels that also run overlapped the min is the closer serial figure."""
import collections
import sqlite3
import statistics
import sys

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for name, start, end in c.execute("select name, start, end from kernels"):
    d[name.split("(")[0]].append((end - start) / 1000.0)
for nm, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if flt in nm:
        print(f"{nm[:64]:64s} n={len(v):4d} med={statistics.median(v):8.1f} min={min(v):8.1f} max={max(v):8.1f}")
