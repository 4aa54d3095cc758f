# MSM/prove tests on var_quad (the G1 lane-quad adds with the doubling inlined: no
# scratch), then an alternating prove A/B against the default build.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
ZK_AMD_LIB=$R/zero-knowledge-proofs_amd/var_quad/libzkp_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_prove.py -x -q --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/t17_tests_quad.log 2>&1 || echo "variant tests failed"
timeout -k 10 900 bash tools/ab_prove.sh 5 quad
cat gpurun_out/ab_prove.txt
