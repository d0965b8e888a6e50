set -o pipefail
cd $GRAFT_REPO_ROOT
echo skip-n1
echo n1-ok
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --grid 128 --steps 5 --warmup 1 --converge-max 20 > gpurun_out/b128_n2.json 2> gpurun_out/b128_n2.err || { echo n2 failed; tail -40 gpurun_out/b128_n2.err; exit 1; }
echo n2-ok
