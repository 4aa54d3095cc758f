"""VALU issue rate of the MSM reduction kernels against the issue-bound
accumulate, from one SQ pass over serial-schedule proves (tools/pmc_prove_valu.sh:
every kernel alone on one stream).  Per kernel: SQ_INSTS_VALU wave
instructions per SIMD-cycle over its dispatch durations (1024 SIMDs, 2.4 GHz),
the fraction of that rate the G1 accumulate reaches in the same pass, and the
stalled share of wave cycles (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES).

  python tools/pmc_reductions.py PMC_DIR > profiles/r04_reductions_valu.json"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

SIMDS, CLK = 1024, 2.4e9


def short(name):
    m = re.match(r"(?:void )?(?:zk::)?([A-Za-z0-9_]+(?:<[^()]*?>)?)", name)
    return (m.group(1) if m else name[:40]).replace("zk::", "")


def main():
    d = sys.argv[1]
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    names = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(r["Dispatch_Id"])
            per[did][r["Counter_Name"]] += float(r["Counter_Value"])
            names[did] = short(r["Kernel_Name"])
            dur[did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = defaultdict(lambda: defaultdict(float))
    for did, c in per.items():
        a = agg[names[did]]
        a["dispatches"] += 1
        a["seconds"] += dur[did]
        for k, v in c.items():
            a[k] += v
    out = {}
    for k, a in agg.items():
        rate = a["SQ_INSTS_VALU"] / (a["seconds"] * SIMDS * CLK) if a["seconds"] else 0.0
        out[k] = {
            "dispatches": int(a["dispatches"]),
            "ms_total": round(a["seconds"] * 1e3, 3),
            "valu_insts_per_simd_cycle": round(rate, 4),
            "wait_inst_any_over_wave_cycles": round(a["SQ_WAIT_INST_ANY"] / a["SQ_WAVE_CYCLES"], 3) if a["SQ_WAVE_CYCLES"] else None,
        }
    ref = out.get("k_msm_accum<G1>", {}).get("valu_insts_per_simd_cycle")
    sel = {k: v for k, v in out.items() if re.match(r"k_msm_(accum|rowcol|quant|fixup|merge|combine)", k)}
    for v in sel.values():
        v["frac_of_g1_accumulate_rate"] = round(v["valu_insts_per_simd_cycle"] / ref, 3) if ref else None
    print(json.dumps({
        "source": "rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES "
                  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU over bench.py --schedule 3 (tools/pmc_prove_valu.sh)",
        "method": "valu_insts_per_simd_cycle = SQ_INSTS_VALU / (dispatch seconds x 1024 SIMDs x 2.4 GHz); "
                  "the G1 accumulate is VALU-issue bound (one wave instruction per ~4.7 SIMD cycles, "
                  "profiles/r03_valu_rates.txt), so frac_of_g1_accumulate_rate is each kernel's VALU fraction "
                  "against that roof",
        "kernels": dict(sorted(sel.items())),
    }, indent=1))


if __name__ == "__main__":
    main()
