# Alternating prove-schedule sweep with accumulate-chain orders on one box:
#   bash tools/sweep_order.sh ROUNDS SPEC...   SPEC = SCHED or SCHED:ORDER (ZK_ACCUM_ORDER)
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
rounds=$1; shift
: > $O/order.txt
for i in $(seq $rounds); do
  for spec in "$@"; do
    s=${spec%%:*}; o=${spec#*:}; [ "$o" = "$spec" ] && o=H2A
    ms=$(ZK_PROVE_SCHED=$s ZK_ACCUM_ORDER=$o timeout -k 10 120 python -u $R/bench.py --no-cpu-baseline --no-msm --no-serial --steps 20 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "$spec $ms" | tee -a $O/order.txt
  done
done
python3 - $O/order.txt <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    v, ms = line.split()
    d[v].append(float(ms))
for v, xs in d.items():
    print(f"{v:10s} median {statistics.median(xs):.3f}  min {min(xs):.3f}  n={len(xs)}  {xs}")
PY
