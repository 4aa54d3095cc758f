# configs[2] NTT alone: kernel trace + VALU / LDS / wait counters + HBM traffic, one pass each.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ntt_trace -o run -- python3 $R/tools/ntt_only.py 22 5 > $O/ntt_trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/ntt_pmc1 -o run -- python3 $R/tools/ntt_only.py 22 2 > $O/ntt_pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES --output-format csv -d $O/ntt_pmc2 -o run -- python3 $R/tools/ntt_only.py 22 2 > $O/ntt_pmc2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/ntt_fetch -o run -- python3 $R/tools/ntt_only.py 22 2 > $O/ntt_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/ntt_write -o run -- python3 $R/tools/ntt_only.py 22 2 > $O/ntt_write.log 2>&1
