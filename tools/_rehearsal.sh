set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
export ZK_BENCH_DIST_BACKEND=gloo ZK_BENCH_DEVICE=0
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --total-log-n 24 > $O/rehearsal_2rank_2p24.json 2> $O/rehearsal_2rank_2p24.log
