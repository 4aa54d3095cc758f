# Window-size sweep of the isolated MSMs (tools/phase_bench.py), one process per setting.
for c in 12 13 14 15 16 17; do
  echo "c=$c" >> gpurun_out/sweep.txt
  ZK_MSM_C=$c timeout -k 10 120 python tools/phase_bench.py --no-ntt --steps 3 2>/dev/null >> gpurun_out/sweep.txt || exit 1
done
