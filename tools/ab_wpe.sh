# A/B of accumulate register caps: default build vs ZK_ACCUM_WPE variants (isolated MSM phases + prove).
set -e
mkdir -p gpurun_out
out=gpurun_out/ab_wpe.txt
: > $out
for v in base wpe2 wpe4; do
  lib=""; [ $v != base ] && lib=$PWD/zero-knowledge-proofs_amd/var_$v/libzkp_amd.so
  echo "== $v phases" >> $out
  ZK_AMD_LIB=$lib timeout -k 10 150 python -u tools/phase_bench.py --no-ntt --steps 5 2>/dev/null >> $out
done
for i in 1 2; do
  for v in base wpe2; do
    lib=""; [ $v != base ] && lib=$PWD/zero-knowledge-proofs_amd/var_$v/libzkp_amd.so
    echo "prove $v $(ZK_AMD_LIB=$lib timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-msm --steps 12 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $out
  done
done
