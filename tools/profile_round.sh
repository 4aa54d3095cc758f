# Profiles committed under profiles/ (run on the GPU box from the repo root):
#   1. kernel trace + stats of the default bench (CSV summary + SQLite)
#   2. FETCH_SIZE and WRITE_SIZE passes (separate: TCC slots), for HBM traffic
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --steps 5 > $R/gpurun_out/prof_stats.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_db -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 > $R/gpurun_out/prof_db.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --steps 3 --warmup 1 > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --steps 3 --warmup 1 > $R/gpurun_out/pmc_write.log 2>&1
