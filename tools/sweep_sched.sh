for s in 0 5 0 5; do
  echo "sched=$s" >> gpurun_out/sched.txt
  ZK_PROVE_SCHED=$s timeout -k 10 300 python bench.py --no-cpu-baseline --no-msm --steps 8 2>/dev/null >> gpurun_out/sched.txt || exit 1
done
