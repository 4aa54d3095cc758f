set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 120 python3 -u tools/h2d_rates.py 20 > $O/h2d.txt 2>&1
timeout -k 10 120 python3 -u tools/timeline_live.py 20 0 > $O/timeline0.txt 2>&1
timeout -k 10 120 python3 -u tools/timeline_live.py 20 3 > $O/timeline3.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_serial -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --anchor-log-n 0 --schedule 3 --steps 5 > $O/prof_serial.log 2>&1
