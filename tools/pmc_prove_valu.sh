# One SQ counter pass over serial-schedule 2^20 proves (every kernel alone on
# one stream): VALU instructions and cycles per kernel, for the G2 (lane-pair)
# and G1 accumulates.  Run on the GPU box from the repo root.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc_prove_valu -o run -- python3 $R/bench.py --no-msm --no-cpu-baseline --anchor-log-n 0 --no-serial --schedule 3 --steps 2 --warmup 1 > $R/gpurun_out/pmc_prove_valu.log 2>&1
