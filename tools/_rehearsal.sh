# bench.py's N>1 path at configs[4]'s full size with N ranks sharing ONE GPU
# (gloo, host-staged all-to-alls): every field of the N>1 line, the folded
# proof against the pinned oracle bytes.
#   bash tools/_rehearsal.sh [N] [torchrun|bench]
# bench (default): `python bench.py --gpus N` starts its own ranks, as the
# driver's plain command would; torchrun: under torch.distributed.run.
set -e
N=${1:-2}
L=${2:-bench}
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
export ZK_BENCH_DIST_BACKEND=gloo ZK_BENCH_DEVICE=0
if [ "$L" = torchrun ]; then
  timeout -k 10 1000 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus $N --total-log-n 24 > $O/rehearsal_${N}rank_2p24.json 2> $O/rehearsal_${N}rank_2p24.log
else
  timeout -k 10 1000 python3 bench.py --gpus $N --total-log-n 24 > $O/rehearsal_${N}rank_2p24.json 2> $O/rehearsal_${N}rank_2p24.log
fi
