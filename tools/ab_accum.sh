# Alternating A/B of an environment switch, reporting the overlapped prove and
# the serial k_msm_accum<G1> launch average (bench.py roofline.avg_launch_ms):
#   bash tools/ab_accum.sh ROUNDS VAR VAL_A VAL_B
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
rounds=$1; var=$2; shift 2
out=$O/ab_accum.txt
: > $out
for i in $(seq $rounds); do
  for v in "$@"; do
    env $var=$v timeout -k 10 200 python -u $R/bench.py --no-cpu-baseline --steps 20 > $O/ab_accum_$v.json 2>/dev/null
    python3 - $var=$v $O/ab_accum_$v.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], "prove_ms", d["ms_per_step"], "serial_ms", d["serial_schedule"]["ms_per_step"],
      "accum_g1_ms", r["avg_launch_ms"], "valu", r["valu"]["frac"], "msm_g1_ms", d["msm_g1"]["ms_per_msm"])
PY
  done
done
cat $out
