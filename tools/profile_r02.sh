# Round-2 profiles (run on the GPU box from the repo root via gpurun):
#   1. kernel trace + stats of the default bench (overlapped timed region,
#      serial roofline proves, MSM and NTT lines)
#   2. the same prove with every kernel serial (ZK_PROVE_SCHED=3): per-kernel
#      averages comparable with roofline.avg_launch_ms
#   3. FETCH_SIZE and WRITE_SIZE passes (separate: TCC slots) of 2., for HBM traffic
#   4. FETCH_SIZE calibration of the accumulate's gather shape (tools/gather_calib)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 > $O/prof_stats.log 2>&1
ZK_PROVE_SCHED=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_serial -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --steps 5 > $O/prof_serial.log 2>&1
ZK_PROVE_SCHED=3 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --no-serial --steps 3 --warmup 1 > $O/pmc_fetch.log 2>&1
ZK_PROVE_SCHED=3 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --no-serial --steps 3 --warmup 1 > $O/pmc_write.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_calib -o run -- $R/tools/gather_calib > $O/calib.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_calib_w -o run -- $R/tools/gather_calib > $O/calib_w.log 2>&1
timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/calib_trace -o run -- $R/tools/gather_calib > $O/calib_trace.log 2>&1
