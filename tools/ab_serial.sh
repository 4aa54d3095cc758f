# Serial-schedule phase A/B (tuning): bench.py's 2^20 line (no anchor, no CPU
# baseline, no configs[1]/[2]) with the default library and each variant
# (zero-knowledge-proofs_amd/var_<name>/libzkp_amd.so), ROUNDS alternating
# rounds; prints the serial phase table of each run (tools/bench_summary.py).
#   bash tools/ab_serial.sh ROUNDS VARIANT...
set -e
mkdir -p gpurun_out
rounds=$1; shift
for i in $(seq $rounds); do
  for v in base "$@"; do
    lib=""; [ $v != base ] && lib=$PWD/zero-knowledge-proofs_amd/var_$v/libzkp_amd.so
    ZK_AMD_LIB=$lib timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-msm --no-pcie --anchor-log-n 0 \
      --steps 20 --warmup 5 --details gpurun_out/abs_${v}_$i.json > /dev/null 2>&1
    echo "== $v round $i"
    python3 tools/bench_summary.py gpurun_out/abs_${v}_$i.json
  done
done
