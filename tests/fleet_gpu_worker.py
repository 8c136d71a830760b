"""Worker for tests/test_gpu_fleet.py: one rank of a sharded fleet step.
Env: RANK, WORLD_SIZE, MASTER_ADDR/PORT, FLEET_BATCH, FLEET_MODEL, FLEET_OUT."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    from go2_onnx_controller_amd import Engine
    from go2_onnx_controller_amd.fleet import FleetShard, gather_actions
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    batch = int(os.environ["FLEET_BATCH"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        obs = np.random.default_rng(77).standard_normal((batch, 48)).astype(np.float32)
        with Engine(os.environ["FLEET_MODEL"], device=0, max_batch=batch) as e:
            shard = FleetShard(e, batch, rank, world)
            x = torch.from_numpy(obs[shard.start:shard.stop]).to("cuda:0")
            y = shard.step(x)
            torch.cuda.synchronize()
            full = gather_actions(y.cpu(), batch)
        np.save(os.path.join(os.environ["FLEET_OUT"], f"rank{rank}.npy"), full.numpy())
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
