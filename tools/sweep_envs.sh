# Alternating A/B/... of environment configurations on one box:
#   bash tools/sweep_envs.sh ROUNDS LABEL=VAR:VAL,VAR:VAL ...   (LABEL= alone: the defaults)
# prints the median / min prove ms per configuration (bench.py, 20 steps, 2^20).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
rounds=$1; shift
: > $O/envs.txt
for i in $(seq $rounds); do
  for cfg in "$@"; do
    label=${cfg%%=*}; spec=${cfg#*=}
    envs=$(echo "$spec" | tr ',' '\n' | sed -n 's/^\([A-Z0-9_]*\):\(.*\)$/\1=\2/p' | tr '\n' ' ')
    ms=$(env $envs timeout -k 10 120 python -u $R/bench.py --no-cpu-baseline --no-msm --no-serial --steps 20 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])')
    echo "$label $ms" >> $O/envs.txt
  done
done
python3 - $O/envs.txt <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    v, ms = line.split()
    d[v].append(float(ms))
for v, xs in d.items():
    print(f"{v:16s} median {statistics.median(xs):.3f}  min {min(xs):.3f}  n={len(xs)}  {xs}")
PY
