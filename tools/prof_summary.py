"""Summarise rocprofv3 SQLite output (kernel trace and PMC passes) into the
files committed under profiles/.

  python tools/prof_summary.py trace <run_results.db> <out.md>
  python tools/prof_summary.py stats <run_kernel_stats.csv> <out.md>
  python tools/prof_summary.py pmc <fetch.db> <write.db> <out.json>

PMC correction (MI355X_MICROARCH.md, HBM): on gfx950 FETCH_SIZE reports half
the bytes of wide coalesced reads, so traffic = 2*FETCH_SIZE + WRITE_SIZE
(both in KiB per dispatch).  Our gathers of 96/192-byte points are not the
calibrated access shape; the doubled figure is an upper estimate.
"""
import json
import re
import sqlite3
import sys


def short(name):
    n = name.replace(".kd", "")
    for pre in ("_ZN2zk", "_Z"):
        if n.startswith(pre):
            n = n[len(pre):]
    i = 0
    while i < len(n) and n[i].isdigit():
        i += 1
    ln = int(n[:i]) if i else 0
    base = n[i:i + ln] if ln else n
    rest = n[i + ln:]
    tag = ""
    if "G1" in rest:
        tag = "<G1>"
    elif "G2" in rest:
        tag = "<G2>"
    elif rest.startswith("ILb1") or rest.startswith("ILi1ELb1") or rest.startswith("ILi4ELb1"):
        tag = "<scatter>" if "digits" in base else "<dit>"
    elif rest.startswith("ILb0") or rest.startswith("ILi1ELb0") or rest.startswith("ILi4ELb0"):
        tag = "<count>" if "digits" in base else "<dif>"
    return base + tag


def trace(db, out):
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("""select s.kernel_name, count(*), sum(d.end-d.start), avg(d.end-d.start),
                          min(d.end-d.start), max(d.end-d.start)
                          from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
                          group by s.kernel_name order by 3 desc""").fetchall()
    total = sum(r[2] for r in rows)
    lines = ["| kernel | calls | total ms | avg us | min us | max us | % |", "|---|---|---|---|---|---|---|"]
    for name, n, tot, avg, mn, mx in rows:
        lines.append("| %s | %d | %.3f | %.1f | %.1f | %.1f | %.1f |" % (
            short(name), n, tot / 1e6, avg / 1e3, mn / 1e3, mx / 1e3, 100.0 * tot / total))
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:20]))


def pmc_per_kernel(db, counter):
    cur = sqlite3.connect(db).cursor()
    q = f"""select s.kernel_name, count(*), avg(e.value)
            from rocpd_pmc_event e
            join rocpd_info_pmc p on e.pmc_id = p.id
            join rocpd_kernel_dispatch d on d.event_id = e.event_id
            join rocpd_info_kernel_symbol s on d.kernel_id = s.id
            where p.name = '{counter}' group by s.kernel_name"""
    return {short(r[0]): (r[1], r[2]) for r in cur.execute(q).fetchall()}


def pmc(fetch_db, write_db, out):
    f = pmc_per_kernel(fetch_db, "FETCH_SIZE")
    w = pmc_per_kernel(write_db, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        fk = f.get(k, (0, 0.0))[1]
        wk = w.get(k, (0, 0.0))[1]
        kernels[k] = {"fetch_kib": round(fk, 1), "write_kib": round(wk, 1),
                      "traffic_bytes_per_launch": int((2 * fk + wk) * 1024)}
    res = {"note": "traffic = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch (gfx950 FETCH correction); "
                   "averages over every dispatch of bench.py --no-msm (prove steps only)",
           "kernels": kernels}
    for k in kernels:
        if k.startswith("k_msm_accum"):
            tag = "g2" if ("G2" in k or "pair" in k) else "g1"   # k_msm_accum_pair: G2
            res[f"msm_accum_{tag}_bytes_per_launch"] = kernels[k]["traffic_bytes_per_launch"]
    json.dump(res, open(out, "w"), indent=1)
    for k, v in kernels.items():
        print(k, v)


def stats(csv_path, out):
    """rocprofv3 --stats CSV -> markdown table with short kernel names."""
    import csv
    rows = list(csv.DictReader(open(csv_path)))
    lines = ["| kernel | calls | total ms | avg us | min us | max us | % |", "|---|---|---|---|---|---|---|"]
    for r in rows:
        name = r["Name"]
        m = re.search(r"zk::(k_\w+)(<zk::(G1|G2)>|<(\w+)>)?", name)
        if m:
            short_name = m.group(1) + (f"<{m.group(3)}>" if m.group(3) else (f"<{m.group(4)}>" if m.group(4) else ""))
        elif "rocprim" in name:
            short_name = "rocprim radix_sort_onesweep " + ("histogram" if "histogram" in name else "iteration")
        else:
            short_name = name[:40]
        lines.append(f"| {short_name} | {r['Calls']} | {int(r['TotalDurationNs']) / 1e6:.3f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {int(r['MinNs']) / 1e3:.1f} | {int(r['MaxNs']) / 1e3:.1f} | "
                     f"{float(r['Percentage']):.2f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:12]))


def dispatches(db, counter):
    """[(dispatch id, full kernel name, value KiB)] in dispatch order."""
    cur = sqlite3.connect(db).cursor()
    q = f"""select d.id, s.kernel_name, e.value from rocpd_pmc_event e
            join rocpd_info_pmc p on e.pmc_id = p.id
            join rocpd_kernel_dispatch d on d.event_id = e.event_id
            join rocpd_info_kernel_symbol s on d.kernel_id = s.id
            where p.name = '{counter}' order by d.id"""
    return cur.execute(q).fetchall()


def calib(fetch_db, write_db, out, log_path):
    """FETCH_SIZE calibration of tools/gather_calib: counter bytes vs the
    distinct 128-byte lines each kernel touches (printed by the program)."""
    lines = {}
    for ln in open(log_path):
        m = re.match(r"(k_\w+(?:<[\d,]+>)?):\s+records (\d+) algorithmic_bytes (\d+) distinct_128B_lines (\d+)", ln)
        if m:
            lines[m.group(1)] = (int(m.group(2)), int(m.group(3)), int(m.group(4)))
        m = re.match(r"k_stream: algorithmic_bytes (\d+)", ln)
        if m:
            lines["k_stream"] = (0, int(m.group(1)), int(m.group(1)) // 128)
    names = {"_Z8k_gatherILi6ELi6E": "k_gather<6,6>", "_Z8k_gatherILi6ELi8E": "k_gather<6,8>",
             "_Z8k_gatherILi8ELi8E": "k_gather<8,8>", "_Z8k_stream": "k_stream"}
    f = {}
    for _, k, v in dispatches(fetch_db, "FETCH_SIZE"):
        for pre, nm in names.items():
            if k.startswith(pre):
                f.setdefault(nm, []).append(v * 1024)
    w = {}
    for _, k, v in dispatches(write_db, "WRITE_SIZE"):
        for pre, nm in names.items():
            if k.startswith(pre):
                w.setdefault(nm, []).append(v * 1024)
    res = {"note": "FETCH_SIZE (bytes) per dispatch vs the bytes of the distinct 128-B lines the kernel reads "
                   "(+ its 4-byte index stream for the gathers); true_over_fetch = line bytes / FETCH_SIZE",
           "kernels": {}}
    for nm, (recs, algo, nl) in lines.items():
        fv = sum(f.get(nm, [0])) / max(len(f.get(nm, [1])), 1)
        line_bytes = nl * 128 + recs * 4
        res["kernels"][nm] = {"records": recs, "algorithmic_bytes": algo, "line_bytes": line_bytes,
                              "fetch_size_bytes": int(fv), "write_size_bytes": int(sum(w.get(nm, [0])) / max(len(w.get(nm, [1])), 1)),
                              "true_over_fetch": round(line_bytes / fv, 3) if fv else None}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


def pmc_prove(fetch_db, write_db, out, factor):
    """Per-dispatch FETCH/WRITE of a serial prove run; the accumulate
    dispatches are split by their place in the prove (B2 G2, the A+B1 batch, IC+H)."""
    fd, wd = dispatches(fetch_db, "FETCH_SIZE"), dispatches(write_db, "WRITE_SIZE")
    agg = {}
    for (_, k, fv), (_, k2, wv) in zip(fd, wd):
        assert k == k2
        a = agg.setdefault(short(k), [0, 0.0, 0.0])
        a[0] += 1
        a[1] += fv * 1024
        a[2] += wv * 1024
    kernels = {k: {"dispatches": n, "fetch_bytes": int(fb / n), "write_bytes": int(wb / n),
                   "traffic_guide_2x": int((2 * fb + wb) / n), "traffic_calibrated": int((factor * fb + wb) / n)}
               for k, (n, fb, wb) in sorted(agg.items())}
    acc = [(fv * 1024, wv * 1024) for (_, k, fv), (_, _, wv) in zip(fd, wd) if short(k) == "k_msm_accum<G1>"]
    res = {"note": f"serial prove (zk_ctx_set_schedule 3); traffic_calibrated = {factor} x FETCH_SIZE + WRITE_SIZE "
                   "(FETCH factor from tools/gather_calib for the accumulate's gather shape -- 1.779 for 96-byte "
                   "points read at a 128-byte stride (k_gather<6,8>), 1.585 for packed 96-byte points -- "
                   "profiles/r02_fetch_calibration.json); traffic_guide_2x = the guide's streaming correction",
           "kernels": kernels}
    if acc:
        # round 6: the IC+H launch (4n points) vs the A+B1 batch launch (2n)
        # of each prove (rounds 1-5: the A+B1+IC batch vs H)
        cut = max(f for f, _ in acc) / 1.5
        big = [a for a in acc if a[0] > cut]
        small = [a for a in acc if a[0] <= cut]
        per = lambda L: int(sum(factor * f + w for f, w in L) / len(L)) if L else None
        res["msm_accum_g1_ich_bytes_per_launch"] = per(big)
        res["msm_accum_g1_ab_bytes_per_launch"] = per(small)
        res["msm_accum_g1_bytes_per_launch"] = per(acc)
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        if k != "kernels":
            print(k, v)


def part(fetch_db, write_db, out, kind, calls, factor):
    """HBM traffic of one standalone workload (tools/msm_only.py or
    tools/ntt_only.py ... fwd) from its FETCH_SIZE and WRITE_SIZE passes.
    msm: bytes per k_msm_accum<G1> launch (FETCH x `factor`, the gather
    calibration); ntt: bytes per forward transform = every dispatch of the
    run / `calls` (FETCH x 2, the guide's streaming correction)."""
    fd, wd = dispatches(fetch_db, "FETCH_SIZE"), dispatches(write_db, "WRITE_SIZE")
    assert len(fd) == len(wd), (len(fd), len(wd))
    agg = {}
    for (_, k, fv), (_, k2, wv) in zip(fd, wd):
        assert k == k2
        a = agg.setdefault(short(k), [0, 0.0, 0.0])
        a[0] += 1
        a[1] += fv * 1024
        a[2] += wv * 1024
    f = factor if kind == "msm" else 2.0
    kernels = {k: {"dispatches": n, "fetch_bytes": int(fb / n), "write_bytes": int(wb / n),
                   "traffic_bytes": int((f * fb + wb) / n)} for k, (n, fb, wb) in sorted(agg.items())}
    res = {"kind": kind, "calls": calls, "fetch_factor": f, "kernels": kernels}
    if kind == "msm":
        acc = [(fv * 1024, wv * 1024) for (_, k, fv), (_, _, wv) in zip(fd, wd)
               if short(k) == "k_msm_accum<G1>"]
        res["bytes_per_launch"] = int(sum(f * a + b for a, b in acc) / len(acc))
        per_call = [(fv * 1024, wv * 1024) for (_, k, fv), (_, _, wv) in zip(fd, wd)
                    if "k_msm" in k or "rocprim" in k]   # not the setup / base upload kernels
        res["whole_msm_bytes_per_call"] = int(sum(f * a + b for a, b in per_call) / calls)
        res["note"] = ("tools/msm_only.py: 2^20 bases x 13 window copies (c = 20), 255-bit scalars; "
                       f"bytes_per_launch = {f} x FETCH_SIZE + WRITE_SIZE of k_msm_accum<G1> "
                       "(FETCH factor from tools/gather_calib, profiles/r02_fetch_calibration.json)")
    else:
        res["bytes_per_launch"] = int(sum(f * v[1] + v[2] for v in agg.values()) / calls)
        res["note"] = ("tools/ntt_only.py ... fwd: forward zk_ntt_fr_dev calls only; bytes_per_launch = "
                       "2 x FETCH_SIZE + WRITE_SIZE over every dispatch / calls, i.e. per transform")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "part":
        part(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5], int(sys.argv[6]), float(sys.argv[7]))
        sys.exit(0)
    if sys.argv[1] == "calib":
        calib(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5])
        sys.exit(0)
    if sys.argv[1] == "pmc_prove":
        pmc_prove(sys.argv[2], sys.argv[3], sys.argv[4], float(sys.argv[5]))
        sys.exit(0)
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "trace":
        trace(sys.argv[2], sys.argv[3])
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4])
