set -e
mkdir -p gpurun_out
timeout -k 10 600 bash tools/ab_kernels.sh "tools/ntt_only.py 22 20" $1 > gpurun_out/ntt_abk.txt 2>&1
timeout -k 10 600 bash tools/ab_ntt.sh 4 "22" $1 > gpurun_out/ntt_abn.txt 2>&1 || true
timeout -k 10 400 bash tools/ab_prove.sh 4 $1 > gpurun_out/ntt_abp.txt 2>&1
