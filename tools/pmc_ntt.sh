# PMC passes over the configs[2] NTT alone: VALU / LDS / wait counters.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ntt_trace -o run -- python3 $R/tools/ntt_only.py 22 5 > $O/ntt_trace.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $O/ntt_pmc1 -o run -- python3 $R/tools/ntt_only.py 22 2 > $O/ntt_pmc1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAVES -d $O/ntt_pmc2 -o run -- python3 $R/tools/ntt_only.py 22 2 > $O/ntt_pmc2.log 2>&1
ZK_PROVE_SCHED=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY -d $O/prove_pmc1 -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --no-serial --steps 2 --warmup 1 > $O/prove_pmc1.log 2>&1
ZK_PROVE_SCHED=3 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM -d $O/prove_pmc2 -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --no-serial --steps 2 --warmup 1 > $O/prove_pmc2.log 2>&1
