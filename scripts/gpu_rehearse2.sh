# Rehearse the N=2 bench path on one GPU: two ranks share cuda:0, gloo for the collectives.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --dist-backend gloo > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.log
