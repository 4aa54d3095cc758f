# Alternating prove A/B over environment settings on one build:
#   bash tools/ab_multi.sh ROUNDS SETTING...   (SETTING: "VAR=v,VAR2=w" or "base")
set -e
mkdir -p gpurun_out
out=gpurun_out/ab_multi.txt
: > $out
rounds=$1; shift
for i in $(seq $rounds); do
  for v in "$@"; do
    envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
    echo "prove $v $(env $envs timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-msm --steps 20 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $out
  done
done
python3 - $out <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    _, v, ms = line.split()
    d[v].append(float(ms))
for v, xs in d.items():
    print(f"{v:36s} median {statistics.median(xs):.3f}  min {min(xs):.3f}  n={len(xs)}  {xs}")
PY
