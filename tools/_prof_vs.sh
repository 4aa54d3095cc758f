set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vs -o run -- python3 $R/tools/virtual_shards.py 24 8 2 > $O/prof_vs.log 2>&1
