set -e
for c in 11 12 13 14 15 16; do
  echo "c=$c" >> gpurun_out/sweep.txt
  ZK_MSM_C=$c timeout -k 10 120 python tools/phase_bench.py --no-ntt --steps 3 2>/dev/null >> gpurun_out/sweep.txt
done
for k in 8 16 64; do
  echo "K=$k" >> gpurun_out/sweep.txt
  ZK_MSM_K=$k timeout -k 10 120 python tools/phase_bench.py --no-ntt --steps 3 2>/dev/null >> gpurun_out/sweep.txt
done
