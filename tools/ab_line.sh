# Whole-line A/B (tuning): bench.py's 2^20 line WITH the configs[1] MSM and
# configs[2] NTT legs (no 2^24 anchor, no CPU baseline, no host witness) for
# the default library and each variant (zero-knowledge-proofs_amd/var_<name>),
# ROUNDS alternating rounds; prints tools/r6_cmp.py's summary of each run.
#   bash tools/ab_line.sh ROUNDS VARIANT...
set -e
mkdir -p gpurun_out
rounds=$1; shift
for i in $(seq $rounds); do
  for v in base "$@"; do
    lib=""; [ $v != base ] && lib=$PWD/zero-knowledge-proofs_amd/var_$v/libzkp_amd.so
    ZK_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-pcie --anchor-log-n 0 \
      --steps 20 --warmup 5 --details gpurun_out/abl_${v}_$i.json > /dev/null 2>&1
    echo "== $v round $i"
    python3 tools/r6_cmp.py gpurun_out/abl_${v}_$i.json
  done
done
