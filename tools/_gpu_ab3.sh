set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_msm.py tests/test_gpu_prove.py tests/test_gpu_api.py tests/test_gpu_setup_size.py > gpurun_out/r6_t5.log 2>&1
ZK_AMD_LIB=$PWD/zero-knowledge-proofs_amd/var_t512/libzkp_amd.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_group.py > gpurun_out/r6_t5b.log 2>&1
timeout -k 10 400 bash tools/ab_serial.sh 1 preich t512 rocprim g2split > gpurun_out/r6_abs3.txt 2>&1
timeout -k 10 500 bash tools/ab_prove.sh 4 preich t512 rocprim g2split > gpurun_out/r6_abp3.txt 2>&1
