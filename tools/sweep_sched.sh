for s in 0 1 2; do
  echo "sched=$s" >> gpurun_out/sched.txt
  ZK_PROVE_SCHED=$s timeout -k 10 300 python bench.py --no-cpu-baseline --no-msm 2>/dev/null >> gpurun_out/sched.txt || exit 1
done
