# GPU tests of the MSM/prove paths on the ILP-tail build, then an alternating
# prove A/B: default (ZK_TAIL_ILP=1) vs var_noilp (barriers kept).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_prove.py tests/test_gpu_headline.py -x -q --timeout 280 --timeout-method thread > gpurun_out/t11_tests.log 2>&1
timeout -k 10 900 bash tools/ab_prove.sh 5 noilp
cat gpurun_out/ab_prove.txt
