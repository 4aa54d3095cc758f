# GPU tests, then the 2^24 prove against the oracle on the new large-domain
# quotient path, then default-build vs var_old A/B at 2^24 and 2^20.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t7_tests.log 2>&1
timeout -k 10 400 python3 -u tools/check_2p24.py 24 > gpurun_out/check_2p24.json 2> gpurun_out/check_2p24.log
out=gpurun_out/ab_quot2.txt
: > $out
run() {  # lib log_n steps
  ZK_AMD_LIB=$1 timeout -k 10 240 python3 -u bench.py --log-n $2 --no-cpu-baseline --no-msm --no-serial --steps $3 --warmup 1 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])'
}
for i in 1 2 3; do
  echo "2p24 base $(run '' 24 5)" >> $out
  echo "2p24 old $(run $R/zero-knowledge-proofs_amd/var_old/libzkp_amd.so 24 5)" >> $out
done
for i in 1 2 3 4; do
  echo "2p20 base $(run '' 20 20)" >> $out
  echo "2p20 old $(run $R/zero-knowledge-proofs_amd/var_old/libzkp_amd.so 20 20)" >> $out
done
cat $out
