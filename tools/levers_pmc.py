"""VALU instructions per lane per add for the tools/levers.hip kernels, from a
rocprofv3 --pmc pass (SQ_INSTS_VALU counts wave instructions: x 64 lanes /
adds).  Usage: levers_pmc.py PMC_DIR ADDS_FILE"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d, adds_file = sys.argv[1], sys.argv[2]
    adds = [ln.rsplit(" ", 1) for ln in open(adds_file).read().splitlines() if ln.strip()]
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = defaultdict(dict)
    names = {}
    for r in rows:
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    order = [did for did in sorted(per) if names[did].startswith(("k_chain_", "void k_chain_", "k_inv_chain", "void k_inv_chain"))]
    print(f"{'kernel':<48} {'adds':>12} {'VALU/lane/add':>14} {'SALU/lane/add':>14}")
    for did, (label, n) in zip(order, adds):
        c = per[did]
        n = float(n)
        print(f"{label:<48} {n:12.0f} {c.get('SQ_INSTS_VALU', 0) * 64 / n:14.0f} {c.get('SQ_INSTS_SALU', 0) * 64 / n:14.0f}")
    if len(order) != len(adds):
        print(f"note: {len(order)} chain dispatches, {len(adds)} labels")


if __name__ == "__main__":
    main()
