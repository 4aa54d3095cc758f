# Alternating A/B of the quotient build (base vs var_old = the element-wise
# bit-reversed gathers) x ZK_NTT_FUSE at 2^24, then base vs var_old at 2^20.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
out=$O/ab_quot.txt
: > $out
run() {  # lib fuse log_n steps
  ZK_AMD_LIB=$1 ZK_NTT_FUSE=$2 timeout -k 10 240 python3 -u $R/bench.py --log-n $3 --no-cpu-baseline --no-msm --no-serial --steps $4 --warmup 1 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])'
}
for i in 1 2 3; do
  for v in base old; do
    lib=""; [ $v != base ] && lib=$R/zero-knowledge-proofs_amd/var_$v/libzkp_amd.so
    for f in 1 0; do echo "2p24 $v-fuse$f $(run "$lib" $f 24 5)" | tee -a $out; done
  done
done
for i in 1 2 3 4; do
  for v in base old; do
    lib=""; [ $v != base ] && lib=$R/zero-knowledge-proofs_amd/var_$v/libzkp_amd.so
    echo "2p20 $v-fuse1 $(run "$lib" 1 20 20)" | tee -a $out
  done
done
python3 - $out <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    sz, v, ms = line.split()
    d[sz + " " + v].append(float(ms))
for v, xs in d.items():
    print(f"{v:16s} median {statistics.median(xs):.3f}  min {min(xs):.3f}  n={len(xs)}  {xs}")
PY
