"""Per-kernel stats of the serial-schedule proves in a rocprofv3 kernel trace
(run_kernel_trace.csv of `tools/r6_prof.sh`): the bench runs the overlapped
proves first and the serial ones (zk_ctx_set_schedule 3, one stream) last, so
the serial proves are the trailing block of consecutive non-overlapping
dispatches.  Usage: serial_cut.py TRACE.csv OUT.md [LINE.json]"""
import csv
import json
import sys


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Dispatch_Id"])))
    rows.sort()
    # trailing non-overlapping block
    i = len(rows) - 1
    while i > 0 and rows[i - 1][1] <= rows[i][0] + 1000:   # 1 us of timestamp slack between back-to-back kernels
        i -= 1
    block = rows[i:]
    # from the first prove on (a prove starts with its witness check): setup kernels precede it
    first = next((j for j, r in enumerate(block) if "k_check_canonical" in r[2]), 0)
    block = block[first:]
    agg = {}
    for s, e, k, _ in block:
        agg.setdefault(k.split("(")[0].replace("void ", "").replace("zk::", ""), []).append((e - s) / 1e3)
    accum = agg.get("k_msm_accum<G1>", [])
    lines = [f"# Serial-schedule proves only: the trailing block of consecutive non-overlapping dispatches "
             f"({len(block)} dispatches, ids {block[0][3]}-{block[-1][3]}) of `{sys.argv[1].split('gpurun_out/')[-1]}`. "
             "Per-kernel durations (us).", ""]
    if len(sys.argv) > 3:
        rf = json.load(open(sys.argv[3]))["roofline"]
        # the bench's HIP-event launches are the accumulates of its timed serial proves
        n = rf["launches"]
        last = accum[-n:]   # the bench's roofline proves are the run's last serial proves
        avg, lavg = sum(accum) / max(len(accum), 1), sum(last) / max(len(last), 1)
        lines.append(f"Roofline cross-check: `k_msm_accum<G1>` averages {avg:.1f} us over the {len(accum)} launches "
                     f"of this block and {lavg:.1f} us over its last {len(last)}; the same run's bench line reports "
                     f"{rf['avg_launch_ms'] * 1e3:.1f} us over its {n} roofline launches (HIP events), "
                     f"{abs(lavg / (rf['avg_launch_ms'] * 1e3) - 1) * 100:.1f} % apart.")
        lines.append("")
    lines += ["| kernel | calls | total ms | avg us | min us | max us |", "|---|---|---|---|---|---|"]
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| {k} | {len(v)} | {sum(v) / 1e3:.3f} | {sum(v) / len(v):.1f} | {min(v):.1f} | {max(v):.1f} |")
    open(sys.argv[2], "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
