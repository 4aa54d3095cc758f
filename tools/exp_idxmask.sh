set -e
for m in 0x7fffffff 0x3ff 0xfffff 0x7fffffff 0x3ff; do
  echo "mask=$m $(ZK_MSM_IDXMASK=$m ZK_PROVE_SCHED=3 timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-msm --steps 5 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], {k: round(v["ms"]/5,3) for k,v in d["phases_ms_total"].items() if "accum" in k})')" >> gpurun_out/mask.txt
done
