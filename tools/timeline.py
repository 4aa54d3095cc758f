"""Timeline of the last prove step from a rocprofv3 kernel-trace database:
per stream, the phases (consecutive kernels of one kind) with start/end in
ms relative to the step's first kernel.  Usage: timeline.py run_results.db"""
import re
import sqlite3
import sys


def short(name):
    m = re.search(r"zk\d+(k_\w+?)(I|E)", name)
    s = m.group(1) if m else name.split("(")[0][-30:]
    if "G2" in name:
        s += "<G2>"
    return s


def main(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, stream_id, queue_id, start, end from kernels order by start").fetchall()
    # step boundaries: k_csr_eval starts each prove
    starts = [r[3] for r in rows if "k_csr_eval" in r[0]]
    t0 = starts[-1]
    t_end = max(r[4] for r in rows)
    rows = [r for r in rows if r[3] >= t0]
    print(f"step span {(t_end - t0) / 1e6:.3f} ms")
    by_q = {}
    for name, sid, qid, s, e in rows:
        by_q.setdefault((sid, qid), []).append((short(name), (s - t0) / 1e6, (e - t0) / 1e6))
    for q, ks in sorted(by_q.items(), key=lambda kv: kv[1][0][1]):
        print(f"-- stream {q[0]} queue {q[1]}")
        cur, cs, ce, busy = None, 0, 0, 0.0
        for n, s, e in ks:
            grp = n.split("<")[0]
            if grp != cur:
                if cur:
                    print(f"   {cur:22s} {cs:8.3f} -> {ce:8.3f}  (busy {busy:.3f})")
                cur, cs, busy = grp, s, 0.0
            ce = e
            busy += e - s
        print(f"   {cur:22s} {cs:8.3f} -> {ce:8.3f}  (busy {busy:.3f})")


if __name__ == "__main__":
    main(sys.argv[1])
