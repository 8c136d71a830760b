#!/bin/bash
# N=2 rehearsal of the bench contract on a 1-GPU box: two torchrun ranks on
# cuda:0, gloo for the barrier / max-time reduce (RCCL refuses duplicate GPUs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/n2
mkdir -p $O
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  $R/bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu --no-latency --same-device --dist-backend gloo > $O/bench.json 2> $O/bench.err || { echo "n2 bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
