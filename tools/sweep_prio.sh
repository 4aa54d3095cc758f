# Alternating stream-priority sweep (ZK_SIDE_PRIO: h/l for side[0] = G2,
# side[1] = A+B1+IC, side[2]) under schedule 0:  bash tools/sweep_prio.sh ROUNDS SPEC...
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
rounds=$1; shift
: > $O/prio.txt
for i in $(seq $rounds); do
  for p in "$@"; do
    ms=$(ZK_SIDE_PRIO=$p timeout -k 10 120 python -u $R/bench.py --no-cpu-baseline --no-msm --no-serial --steps 20 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "$p $ms" | tee -a $O/prio.txt
  done
done
python3 - $O/prio.txt <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    v, ms = line.split()
    d[v].append(float(ms))
for v, xs in d.items():
    print(f"{v:6s} median {statistics.median(xs):.3f}  min {min(xs):.3f}  n={len(xs)}  {xs}")
PY
