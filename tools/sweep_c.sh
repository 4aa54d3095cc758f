# Tuning sweep of the isolated MSMs (tools/phase_bench.py), one process per setting.
for r in 1 2; do for f in 4 8 16; do
  echo "rounds=$r fix=$f" >> gpurun_out/sweep.txt
  ZK_MSM_ROUNDS=$r ZK_MSM_FIX=$f timeout -k 10 120 python tools/phase_bench.py --no-ntt --steps 3 2>/dev/null >> gpurun_out/sweep.txt || exit 1
done; done
