set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t5_tests.log 2>&1
timeout -k 10 600 bash tools/ab_fuse_2p24.sh
timeout -k 10 600 bash tools/sweep_order.sh 4 0 9 > gpurun_out/sched9_sweep.txt 2>&1
