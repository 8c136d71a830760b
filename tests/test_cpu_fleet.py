"""CPU: many-robot sharding — contiguous row shards per rank, no
collective in the step, optional all-gather of actions; world_size 2 over gloo.
Each rank's per-row compute here is the oracle's fp32 path (row-independent,
like the GPU kernel), so the gathered result must equal the unsharded one
bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from go2_onnx_controller_amd.fleet import shard_range, shard_sizes


@pytest.mark.parametrize("batch,world", [(0, 1), (1, 2), (7, 2), (32768, 8), (4097, 8), (10, 3), (3, 8)])
def test_shard_ranges_partition(batch, world):
    spans = [shard_range(batch, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == batch
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c
    sizes = shard_sizes(batch, world)
    assert sum(sizes) == batch and max(sizes) - min(sizes) <= 1


def test_shard_range_errors():
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)
    with pytest.raises(ValueError):
        shard_range(-1, 0, 1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, batch, model_path, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from go2_onnx_controller_amd.fleet import FleetShard, gather_actions
    from oracle import mlp_ref
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ref = mlp_ref.MlpRef.from_onnx(model_path)
        obs = np.random.default_rng(123).standard_normal((batch, ref.in_dim)).astype(np.float32)
        shard = FleetShard(engine=None, batch=batch, rank=rank, world=world)
        local = torch.from_numpy(ref.f32(obs[shard.start:shard.stop], nthreads=1))
        full = gather_actions(local, batch)
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), full.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("batch", [4096, 1001])
def test_gloo_world2_gather_bitwise(tmp_path, synth_path, batch):
    from oracle import mlp_ref
    path = synth_path("go2_mlp_512")
    mp.spawn(_worker, args=(2, _free_port(), batch, path, str(tmp_path)), nprocs=2, join=True)
    ref = mlp_ref.MlpRef.from_onnx(path)
    obs = np.random.default_rng(123).standard_normal((batch, ref.in_dim)).astype(np.float32)
    want = ref.f32(obs, nthreads=1)
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"rank{r}.npy"), want)
