"""Print the headline numbers and the serial phase table of a bench.py JSON line."""
import json
import sys


def main(path):
    p = json.load(open(path))
    print("prove %.3f ms  %s  bit_exact %s  pcie +%s" % (p["ms_per_step"], p["value"], p.get("bit_exact_vs_oracle"),
                                                        (p.get("pcie_inclusive") or {}).get("over_resident_ms")))
    ss = p.get("serial_schedule")
    if ss and "phases_ms_total" in ss:
        print("serial %.3f ms" % ss["ms_per_step"])
        tot = {"merge": 0.0, "bucket_sum": 0.0}
        for k, v in sorted(ss["phases_ms_total"].items()):
            ms = v["ms"] / ss["steps"]
            print("  %-28s %.3f" % (k, ms))
            for t in tot:
                if k.endswith("msm_" + t):
                    tot[t] += ms
        print("  merge + bucket_sum = %.3f (merge %.3f, bucket_sum %.3f)" % (sum(tot.values()), tot["merge"],
                                                                           tot["bucket_sum"]))
    roof = p.get("roofline") or {}
    print("roofline frac %s avg_launch %s valu %s" % (roof.get("frac"), roof.get("avg_launch_ms"),
                                                     (roof.get("valu") or {}).get("frac")))
    for k in ("msm_g1", "ntt"):
        if k in p:
            print(k, p[k].get("ms_per_msm", p[k].get("ms_per_ntt")), p[k].get("kernel_ms_per_ntt", ""))
    a = p.get("strong_scaling_anchor")
    if a:
        print("anchor %.3f ms msm_only %.3f bit_exact %s" % (a["ms_per_step"], a["msm_only"]["ms_per_step"],
                                                             a["bit_exact_vs_oracle"]))


if __name__ == "__main__":
    main(sys.argv[1])
