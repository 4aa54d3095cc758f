# Alternating prove-schedule sweep (ZK_PROVE_SCHED, prove.hip) on one box,
# then the live stream timeline of each schedule (tools/timeline_live.py):
#   bash tools/sweep_sched.sh ROUNDS SCHED...
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
rounds=$1; shift
: > $O/sched.txt
for i in $(seq $rounds); do
  for s in "$@"; do
    echo "sched=$s $(ZK_PROVE_SCHED=$s timeout -k 10 120 python -u $R/bench.py --no-cpu-baseline --no-msm --no-serial --steps 20 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $O/sched.txt
  done
done
python3 - $O/sched.txt <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    v, ms = line.split()
    d[v].append(float(ms))
for v, xs in d.items():
    print(f"{v:10s} median {statistics.median(xs):.3f}  min {min(xs):.3f}  n={len(xs)}  {xs}")
PY
for s in "$@"; do
  timeout -k 10 120 python -u $R/tools/timeline_live.py 20 $s > $O/timeline_s$s.txt 2>&1
done
