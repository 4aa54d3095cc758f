set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_unfused.py -x -q --timeout 280 --timeout-method thread > gpurun_out/t10_tests.log 2>&1
timeout -k 10 900 bash tools/sweep_prio.sh 3 hll hhl lhl hhh > gpurun_out/prio_sweep.txt 2>&1
out=gpurun_out/fixup2.txt
: > $out
for i in 1 2 3 4; do
  for f in 0 1; do
    echo "fixup2=$f $(ZK_MSM_FIXUP2=$f timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-msm --no-serial --steps 20 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $out
  done
done
cat $out
