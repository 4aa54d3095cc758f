# Shared-bucket window sweep of the prove MSMs (ZK_PROVE_WIN_C: 16 -> 4
# windows over 2^16 buckets, 22 -> 3 windows over 2^21), at 2^20 (with the
# oracle check of the timed proof) and 2^24:
#   bash tools/sweep_winc.sh
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
for c in 22 16; do
  ZK_PROVE_WIN_C=$c timeout -k 10 300 python -u $R/bench.py --no-msm --steps 10 --cpu-log-n 10 > $O/winc_20_$c.json 2> $O/winc_20_$c.log
done
for c in 22 16; do
  ZK_PROVE_WIN_C=$c timeout -k 10 400 python -u $R/bench.py --no-msm --no-cpu-baseline --log-n 24 --steps 4 --warmup 1 > $O/winc_24_$c.json 2> $O/winc_24_$c.log
done
for f in $O/winc_*.json; do
  python3 - $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ph = d["serial_schedule"]["phases_ms_total"]; k = d["serial_schedule"]["steps"]
acc = sum(v["ms"] for n, v in ph.items() if n.endswith("msm_accum_g1")) / k
red = sum(v["ms"] for n, v in ph.items() if n.endswith(("msm_bucket_sum", "msm_merge"))) / k
srt = sum(v["ms"] for n, v in ph.items() if n.endswith("msm_sort")) / k
print(sys.argv[1].split("/")[-1], "prove_ms", d["ms_per_step"], "serial_ms", d["serial_schedule"]["ms_per_step"],
      "g1_accum", round(acc, 3), "merge+bucket_sum", round(red, 3), "sort", round(srt, 3),
      "exact", d.get("bit_exact_vs_oracle"))
PY
done
