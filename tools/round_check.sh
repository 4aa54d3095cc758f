# Round check on the GPU box (from the repo root via gpurun):
#   GPU tests (one process), smoke(), the default bench line, then the
#   rocprofv3 kernel stats of the serial-schedule prove whose HIP-event
#   roofline the bench line reports (same kernel launches: resident proves
#   only), and a stream timeline of the overlapped prove.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/check_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/check_smoke.log 2>&1
timeout -k 10 400 python3 -u bench.py > $O/check_bench.json 2> $O/check_bench.log
timeout -k 10 120 python3 -u tools/timeline_live.py 20 0 > $O/check_timeline.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/check_prof_serial -o run -- python3 $R/bench.py --no-cpu-baseline --no-msm --anchor-log-n 0 --no-pcie --schedule 3 --steps 5 > $O/check_prof_serial.json 2> $O/check_prof_serial.log
