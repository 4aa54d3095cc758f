# Same-box A/B of the fused quotient round trip (ZK_NTT_FUSE=1, default) against
# the unfused one (=0) at 2^24 constraints, alternating, 5 timed proves each.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
: > $O/ab_fuse_2p24.txt
for i in 1 2; do
  for f in 1 0; do
    ms=$(ZK_NTT_FUSE=$f timeout -k 10 240 python3 -u $R/bench.py --log-n 24 --no-cpu-baseline --no-msm --no-serial --steps 5 --warmup 1 2>>$O/ab_fuse_2p24.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "fuse=$f $ms" | tee -a $O/ab_fuse_2p24.txt
  done
done
