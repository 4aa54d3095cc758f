# Alternating API-NTT A/B (tools/ntt_only.py, host-timed) between the default
# build and variant libraries:
#   bash tools/ab_ntt.sh ROUNDS "LOGN..." VARIANT...   (zero-knowledge-proofs_amd/var_<name>/libzkp_amd.so)
set -e
mkdir -p gpurun_out
out=gpurun_out/ab_ntt.txt
: > $out
rounds=$1; sizes=$2; shift; shift
for i in $(seq $rounds); do
  for v in base "$@"; do
    lib=""; [ $v != base ] && lib=$PWD/zero-knowledge-proofs_amd/var_$v/libzkp_amd.so
    for ln in $sizes; do
      ms=$(ZK_AMD_LIB=$lib timeout -k 10 120 python -u tools/ntt_only.py $ln 30 2>/dev/null | sed -n 's/.*: \([0-9.]*\) ms host-timed/\1/p')
      echo "$v/2^$ln $ms" >> $out
    done
  done
done
python3 - $out <<'PY'
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    v, ms = line.split()
    d[v].append(float(ms))
for v, xs in sorted(d.items()):
    print(f"{v:16s} median {statistics.median(xs):.3f}  min {min(xs):.3f}  n={len(xs)}")
PY
