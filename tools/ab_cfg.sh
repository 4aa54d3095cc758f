# Alternating prove A/B over environment settings ("-" = defaults):
#   bash tools/ab_cfg.sh ROUNDS "-" "ZK_PROVE_SCHED=1" "ZK_G1_GROUPS=ABIH ZK_PROVE_SCHED=1" ...
set -e
mkdir -p gpurun_out
out=gpurun_out/ab_cfg.txt
: > $out
rounds=$1; shift
for i in $(seq $rounds); do
  for cfg in "$@"; do
    envs=""; [ "$cfg" != "-" ] && envs="$cfg"
    ms=$(env $envs timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-msm --steps 20 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "${cfg// /,} $ms" >> $out
  done
done
python3 - $out <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    v, ms = line.split()
    d[v].append(float(ms))
for v, xs in d.items():
    print(f"{v:40s} median {statistics.median(xs):.3f}  min {min(xs):.3f}  n={len(xs)}  {xs}")
PY
