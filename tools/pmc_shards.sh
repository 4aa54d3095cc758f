# FETCH_SIZE / WRITE_SIZE of one configs[4] shard's serial proves for N = 2,
# 4, 8 (separate passes: TCC slots), summarised per k_msm_accum<G1> launch
# into gpurun_out/pmc_traffic_2p24_shardN.json (bench.py reads the copies
# under profiles/ for the N > 1 lines' roofline.traffic).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for N in 2 4 8; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/shard${N}_fetch -o run -- python3 $R/tools/shard_prove.py 24 $N 2 > $O/shard${N}_fetch.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/shard${N}_write -o run -- python3 $R/tools/shard_prove.py 24 $N 2 > $O/shard${N}_write.log 2>&1
  python3 $R/tools/prof_summary.py pmc_prove $O/shard${N}_fetch/run_results.db $O/shard${N}_write/run_results.db $O/pmc_traffic_2p24_shard${N}.json 1.779 > $O/shard${N}_summary.txt
done
# the counter databases are large; keep the summaries and logs only
rm -rf $O/shard*_fetch $O/shard*_write
