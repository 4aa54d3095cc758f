# Round-end evidence (run on the GPU box from the repo root via gpurun):
#   1. the default bench line (with the CPU baseline and oracle check)
#   2. rocprofv3 kernel trace + stats of the bench (overlapped timed region,
#      serial roofline proves, MSM and NTT lines)
#   3. the same with every prove kernel serial (ZK_PROVE_SCHED=3)
#   4. FETCH_SIZE and WRITE_SIZE passes (separate: TCC slots) of 3.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u $R/bench.py > $O/final_bench.json 2> $O/final_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/final_stats -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 > $O/final_stats.log 2>&1
ZK_PROVE_SCHED=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/final_serial -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --steps 5 > $O/final_serial.log 2>&1
ZK_PROVE_SCHED=3 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/final_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --no-serial --steps 3 --warmup 1 > $O/final_fetch.log 2>&1
ZK_PROVE_SCHED=3 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/final_write -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --no-serial --steps 3 --warmup 1 > $O/final_write.log 2>&1
