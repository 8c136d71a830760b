set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 --dist-backend gloo --same-device > gpurun_out/b2.json 2> gpurun_out/b2.err; echo "torchrun rc=$?"; cat gpurun_out/b2.json | cut -c1-400
