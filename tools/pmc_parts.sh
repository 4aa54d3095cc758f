# configs[1] MSM and configs[2] NTT alone: kernel stats, then FETCH_SIZE and
# WRITE_SIZE in separate passes (TCC slots), summarised into
# gpurun_out/pmc_msm_2p20.json and gpurun_out/pmc_ntt_2p22.json (bench.py reads
# the copies under profiles/).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/msm_stats -o run -- python3 $R/tools/msm_only.py 20 10 > $O/msm_stats.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ntt_stats -o run -- python3 $R/tools/ntt_only.py 22 20 > $O/ntt_stats.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/msm_fetch -o run -- python3 $R/tools/msm_only.py 20 2 > $O/msm_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/msm_write -o run -- python3 $R/tools/msm_only.py 20 2 > $O/msm_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/ntt_fetch -o run -- python3 $R/tools/ntt_only.py 22 4 fwd > $O/ntt_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/ntt_write -o run -- python3 $R/tools/ntt_only.py 22 4 fwd > $O/ntt_write.log 2>&1
cd $R
python3 tools/prof_summary.py part $O/msm_fetch/run_results.db $O/msm_write/run_results.db $O/pmc_msm_2p20.json msm 3 1.779
python3 tools/prof_summary.py part $O/ntt_fetch/run_results.db $O/ntt_write/run_results.db $O/pmc_ntt_2p22.json ntt 4 2
python3 tools/prof_summary.py stats $O/msm_stats/run_kernel_stats.csv $O/msm_stats.md
python3 tools/prof_summary.py stats $O/ntt_stats/run_kernel_stats.csv $O/ntt_stats.md
