# A/B: per-slot MSMs (ZK_MSM_BATCH=0) vs batched G1 groups, alternating on one box.
set -e
mkdir -p gpurun_out
for i in 1 2 3; do
  for b in 0 1; do
    echo "batch=$b $(ZK_MSM_BATCH=$b timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-msm --steps 12 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> gpurun_out/ab.txt
  done
done
