# Round-6 profiles (run on the GPU box from the repo root via gpurun):
#   1. rocprofv3 kernel trace + stats of the serial-schedule 2^20 prove whose
#      HIP-event roofline the bench line reports (same launches)
#   2. FETCH_SIZE and WRITE_SIZE passes of the same serial proves (separate
#      runs: TCC counter slots) -> per-launch HBM traffic of k_msm_accum<G1>
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-msm --anchor-log-n 0 --no-pcie --schedule 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r6_prof_serial -o run -- python3 $R/bench.py $ARGS --steps 5 --details $O/r6_prof_serial_details.json > $O/r6_prof_serial.json 2> $O/r6_prof_serial.log
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/r6_pmc_fetch -o run -- python3 $R/bench.py $ARGS --no-serial --steps 3 --warmup 1 --details $O/r6_pmc_f_details.json > $O/r6_pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/r6_pmc_write -o run -- python3 $R/bench.py $ARGS --no-serial --steps 3 --warmup 1 --details $O/r6_pmc_w_details.json > $O/r6_pmc_write.log 2>&1
cd $R
python3 tools/serial_cut.py $O/r6_prof_serial/run_kernel_trace.csv $O/r6_kernel_stats_serial.md $O/r6_prof_serial.json
python3 tools/prof_summary.py pmc_prove $(ls $O/r6_pmc_fetch/*/run_results.db $O/r6_pmc_fetch/run_results.db 2>/dev/null | head -1) $(ls $O/r6_pmc_write/*/run_results.db $O/r6_pmc_write/run_results.db 2>/dev/null | head -1) $O/pmc_traffic_2p20.json 1.779 > $O/r6_pmc_summary.txt
rm -rf $O/r6_pmc_fetch $O/r6_pmc_write
