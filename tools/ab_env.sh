# Alternating prove A/B of an environment switch on one build:
#   bash tools/ab_env.sh ROUNDS VAR VALUE_A VALUE_B   (e.g. ZK_G2_PAIR 0 1)
set -e
mkdir -p gpurun_out
out=gpurun_out/ab_env.txt
: > $out
rounds=$1; var=$2; shift 2
for i in $(seq $rounds); do
  for v in "$@"; do
    echo "prove $var=$v $(env $var=$v timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-msm --steps 20 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $out
  done
done
python3 - $out <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    _, v, ms = line.split()
    d[v].append(float(ms))
for v, xs in d.items():
    print(f"{v:14s} median {statistics.median(xs):.3f}  min {min(xs):.3f}  n={len(xs)}  {xs}")
PY
