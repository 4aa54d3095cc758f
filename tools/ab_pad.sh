# A/B of line-padded MSM bases (ZK_BASE_PAD=1, default) against packed ones
# (=0) on one box, alternating, then the FETCH/WRITE passes of the padded
# serial prove (run from the repo root via gpurun):
#   bash tools/ab_pad.sh ROUNDS [LOG_N]
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
rounds=$1; logn=${2:-20}
out=$O/ab_pad_$logn.txt
: > $out
for i in $(seq $rounds); do
  for v in 0 1; do
    ZK_BASE_PAD=$v timeout -k 10 300 python -u $R/bench.py --no-cpu-baseline --log-n $logn --steps 10 \
      $([ $logn != 20 ] && echo --no-msm) > $O/ab_pad_${logn}_$v.json 2>/dev/null
    python3 - $v $O/ab_pad_${logn}_$v.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
m = d.get("msm_g1", {})
print(f"pad={sys.argv[1]} prove_ms {d['ms_per_step']} serial_ms {d['serial_schedule']['ms_per_step']} "
      f"accum_g1_ms {r['avg_launch_ms']} overlapped_accum_ms {r.get('overlapped_avg_launch_ms')} "
      f"msm_g1_ms {m.get('ms_per_msm')} msm_plain_ms {m.get('plain', {}).get('ms_per_msm')}")
PY
  done
done
cat $out
cd /tmp && export TMPDIR=/tmp
ZK_PROVE_SCHED=3 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$logn -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --no-serial --log-n $logn --steps 3 --warmup 1 > $O/pmc_fetch_$logn.log 2>&1
ZK_PROVE_SCHED=3 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$logn -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --no-serial --log-n $logn --steps 3 --warmup 1 > $O/pmc_write_$logn.log 2>&1
