# Alternating prove A/B between the default build and variant libraries:
#   bash tools/ab_prove.sh ROUNDS VARIANT...   (variants: zero-knowledge-proofs_amd/var_<name>/libzkp_amd.so)
# Each measurement is its own process: 10 warmup + 100 timed overlapped
# proves (~1 s), no serial roofline proves, no baselines, no 2^24 anchor.
set -e
mkdir -p gpurun_out
out=gpurun_out/ab_prove.txt
: > $out
rounds=$1; shift
for i in $(seq $rounds); do
  for v in base "$@"; do
    lib=""; [ $v != base ] && lib=$PWD/zero-knowledge-proofs_amd/var_$v/libzkp_amd.so
    echo "prove $v $(ZK_AMD_LIB=$lib timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-msm --no-serial --no-pcie --anchor-log-n 0 --steps 100 --warmup 10 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $out
  done
done
python3 - $out <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    _, v, ms = line.split()
    d[v].append(float(ms))
for v, xs in d.items():
    print(f"{v:8s} median {statistics.median(xs):.3f}  min {min(xs):.3f}  n={len(xs)}  {xs}")
PY
