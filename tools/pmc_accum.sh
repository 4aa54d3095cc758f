# PMC passes over tools/phase_bench.py (MSM kernels): issue/stall and I-cache counters.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $R/gpurun_out/pmc_sq -o run -- python3 $R/tools/phase_bench.py --no-ntt --steps 2 --warmup 1 > $R/gpurun_out/pmc_sq.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQC_ICACHE_MISSES_DUPLICATE -d $R/gpurun_out/pmc_ic -o run -- python3 $R/tools/phase_bench.py --no-ntt --steps 2 --warmup 1 > $R/gpurun_out/pmc_ic.log 2>&1
