# Prove-step time per G1 grouping / schedule (run on the GPU box from the repo root).
set -e
mkdir -p gpurun_out
for g in "ABI,H" "ABIH" "AB,I,H" "A,B,I,H" "ABI,H" "ABIH"; do
  for s in 0 1; do
    echo "groups=$g sched=$s $(ZK_G1_GROUPS=$g ZK_PROVE_SCHED=$s timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-msm --steps 8 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> gpurun_out/groups.txt
  done
done
