# Standalone NTT (zk_ntt_fr_dev) host-timed at 2^22 / 2^24 for strided-pass
# depths ZK_NTT_MAXSTRIDED (9: 3 passes at 2^22, 11: 2 passes), then a
# kernel trace of the default:   bash tools/ntt_sweep.sh
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
: > $O/ntt_sweep.txt
for ms in 9 10 11; do
  for ln in 22 24; do
    echo "maxstrided=$ms $(ZK_NTT_MAXSTRIDED=$ms timeout -k 10 120 python -u $R/tools/ntt_only.py $ln 20 | tr '\n' ' ')" >> $O/ntt_sweep.txt
  done
done
cat $O/ntt_sweep.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ntt_stats -o run -- python3 $R/tools/ntt_only.py 22 20 > $O/ntt_stats.log 2>&1
