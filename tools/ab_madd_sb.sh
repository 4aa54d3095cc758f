# MSM tests on var_madd (ZK_MADD_SB=0: no scheduling barriers in the
# accumulate's mixed add), then an alternating prove A/B against the default.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
ZK_AMD_LIB=$R/zero-knowledge-proofs_amd/var_madd/libzkp_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_prove.py -x -q --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/t14_tests_madd.log 2>&1 || echo "variant tests failed"
timeout -k 10 900 bash tools/ab_prove.sh 5 madd
cat gpurun_out/ab_prove.txt
