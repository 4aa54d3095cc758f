# MSM/prove GPU tests on the default build and on var_g2ilp (ZK_TAIL_ILP_G2=1),
# then an alternating prove A/B between them.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_prove.py -x -q --timeout 280 --timeout-method thread > gpurun_out/t12_tests.log 2>&1
ZK_AMD_LIB=$R/zero-knowledge-proofs_amd/var_g2ilp/libzkp_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_prove.py -x -q --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/t12_tests_g2.log 2>&1 || echo "variant tests failed (see log)"
timeout -k 10 900 bash tools/ab_prove.sh 5 g2ilp
cat gpurun_out/ab_prove.txt
