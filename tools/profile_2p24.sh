# 2^24 on one GPU (configs[4]'s size): oracle parity of the default build
# (c = 22 windows from 2^24), the bench line, and the FETCH/WRITE passes of
# the serial prove for profiles/pmc_traffic_2p24.json:  bash tools/profile_2p24.sh
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u $R/tools/check_2p24.py 24 > $O/check_2p24.json 2> $O/check_2p24.log
timeout -k 10 300 python -u $R/bench.py --log-n 24 --no-msm --no-cpu-baseline --steps 5 --warmup 1 > $O/bench_2p24.json 2> $O/bench_2p24.log
cd /tmp && export TMPDIR=/tmp
ZK_PROVE_SCHED=3 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_24 -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --no-serial --log-n 24 --steps 2 --warmup 1 > $O/pmc_fetch_24.log 2>&1
ZK_PROVE_SCHED=3 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_24 -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --no-serial --log-n 24 --steps 2 --warmup 1 > $O/pmc_write_24.log 2>&1
