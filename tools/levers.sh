# The accumulate-lever prototypes (tools/levers.hip) on the GPU box, from the
# repo root: timing + correctness, then one SQ counter pass for VALU
# instructions per add (tools/levers_pmc.py).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
# the binary is gpurun-ignored (4 MB): build it on the box when absent
[ -x $R/tools/levers ] || hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -pragma-unroll-threshold=2000000 \
  $R/tools/levers.hip -o $R/tools/levers
timeout -k 10 180 $R/tools/levers > $O/levers.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/levers_pmc -o run -- $R/tools/levers --pmc $O/levers_adds.txt > $O/levers_pmc.log 2>&1
python3 $R/tools/levers_pmc.py $O/levers_pmc $O/levers_adds.txt > $O/levers_valu.txt
