set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_prove.py -x -q --timeout 300 --timeout-method thread > gpurun_out/g2_tests.log 2>&1
timeout -k 10 600 bash tools/ab_kernels.sh "bench.py --no-cpu-baseline --no-msm --anchor-log-n 0 --no-pcie --no-serial --schedule 3 --steps 10" $1 > gpurun_out/g2_abk.txt 2>&1
timeout -k 10 400 bash tools/ab_prove.sh 4 $1 > gpurun_out/g2_abp.txt 2>&1
