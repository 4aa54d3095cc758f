# Round check on the GPU box (from the repo root via gpurun):
#   GPU tests (one process), smoke(), the default bench line.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/check_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/check_smoke.log 2>&1
timeout -k 10 400 python3 -u bench.py > $O/check_bench.json 2> $O/check_bench.log
