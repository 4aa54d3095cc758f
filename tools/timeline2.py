"""Per-stream phase timeline of one prove step from a rocprofv3 kernel-trace
database (rocprofv3 --kernel-trace -d DIR -o run -- python bench.py ...):
the step is the window between two consecutive k_csr_eval starts, shifted to
start at the step's first kernel.  Usage: timeline2.py run_results.db"""
import re
import sqlite3
import sys


def short(n):
    m = re.search(r"zk\d+(k_\w+?)(I|E)", n)
    s = m.group(1) if m else ("sort" if "rocprim" in n else n.split("(")[0][-25:])
    return s + ("<G2>" if "G2" in n else "")


def main(db):
    rows = sqlite3.connect(db).execute("select name, stream_id, start, end from kernels order by start").fetchall()
    evals = [r[2] for r in rows if "k_csr_eval" in r[0]]
    print("steps (csr_eval to csr_eval, ms):", [round((b - a) / 1e6, 3) for a, b in zip(evals, evals[1:])])
    # the last complete step: kernels launched after the previous step's last copy
    lo, hi = evals[-3], evals[-2]
    sel = [r for r in rows if lo - 4e6 <= r[2] < hi + 8e6]
    t0 = min(r[2] for r in sel if r[2] >= lo - 4e6)
    by = {}
    for n, sid, s, e in sel:
        by.setdefault(sid, []).append((short(n), (s - t0) / 1e6, (e - t0) / 1e6))
    for sid, ks in by.items():
        print("-- stream", sid)
        cur = None
        for n, s, e in ks + [(None, 0, 0)]:
            if n != cur:
                if cur:
                    print(f"   {cur:28s} {cs:8.3f} -> {ce:8.3f}  busy {busy:.3f}")
                cur, cs, busy = n, s, 0.0
            ce = e
            busy += e - s


if __name__ == "__main__":
    main(sys.argv[1])
