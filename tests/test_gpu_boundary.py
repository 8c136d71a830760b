"""GPU: the boundary end to end — the drop-in C++ ONNXActor in the reference
controller's call pattern, the Python mirrors, loader breadth through the
kernels, and the sharded fleet step (2 ranks, one GPU, gloo gather)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import graphs
from conftest import GOLDEN, ROOT, SHIPPED, abs_err, rel_err
from test_cpu_boundary import build_controller_shape

pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.mark.parametrize("resident", ["100", "0"])
@pytest.mark.parametrize("mode", ["zeros", "twos"])
def test_cpp_onnx_actor_known_answers(mode, resident):
    """tests/cpp/controller_shape.cpp: make_unique<ONNXActor>(path, std::array<float,98>&,
    std::array<float,12>&), print_model_info(), act() — as controller.cpp:25,49,215.
    The shim's resident kernel (default) and one launch per call (GO2PI_RESIDENT_MS=0)."""
    exe = build_controller_shape()
    r = subprocess.run([exe, SHIPPED, mode], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, GO2PI_RESIDENT_MS=resident))
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    assert lines[:5] == ["Input dimension: 98", "Output dimension: 12", "Input name: observation",
                         "Output name: action", "check_dims: 1"]
    act = np.array([float(v) for v in next(l for l in lines if l.startswith("Action:")).split()[1:]])
    want = np.load(os.path.join(GOLDEN, "golden_shipped.npz"))[f"{mode}_y"][0]
    assert rel_err(act, want) <= TOL


@pytest.mark.parametrize("resident", ["100", "0"])
def test_cpp_onnx_actor_ticks(resident, tmp_path):
    """500 ticks of the C++ shim with the observation rewritten in place before each
    act() (controller.cpp:200-215 at 50 Hz): every tick's action against the fp64
    oracle on the same observation sequence, in the resident and launch-per-call forms."""
    from oracle import mlp_ref
    exe = build_controller_shape()
    dump, ticks = tmp_path / "actions.bin", 500
    r = subprocess.run([exe, SHIPPED, "ticks", str(ticks), str(dump)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, GO2PI_RESIDENT_MS=resident))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "best_us:" in r.stdout
    got = np.fromfile(dump, np.float32).reshape(ticks, 12)
    obs, seq = np.zeros(98, np.float32), np.empty((ticks, 98), np.float32)
    for t in range(ticks):  # the same float32 in-place updates as the C++ loop
        obs[t % 98] += np.float32(0.001)
        seq[t] = obs
    want = mlp_ref.MlpRef.from_onnx(SHIPPED).f64(seq)
    assert abs_err(got, want) <= TOL
    assert len(np.unique(got[:, 0])) > ticks // 2  # the actions follow the changing observation


def test_python_onnx_actor_aliasing(capsys):
    from go2_onnx_controller_amd import ONNXActor
    from oracle import mlp_ref
    obs = np.zeros(98, np.float32)
    act = np.zeros(12, np.float32)
    actor = ONNXActor(SHIPPED, obs, act)
    actor.print_model_info()
    assert capsys.readouterr().out.splitlines() == ["Input dimension: 98", "Output dimension: 12",
                                                    "Input name: observation", "Output name: action"]
    assert actor.check_dims()
    ref = mlp_ref.MlpRef.from_onnx(SHIPPED)
    rng = np.random.default_rng(1)
    for _ in range(5):
        obs[:] = rng.standard_normal(98)   # caller writes in place, like populate_buffer
        actor.act()
        assert abs_err(act, ref.f64(obs)[0]) <= TOL
    assert not ONNXActor(SHIPPED, np.zeros(100, np.float32), np.zeros(12, np.float32)).check_dims()


def test_inference_session_mirror():
    """The reference Python driver's calls (src/python/main.py:8-27)."""
    from go2_onnx_controller_amd import InferenceSession
    sess = InferenceSession(SHIPPED)
    inp, out = sess.get_inputs()[0], sess.get_outputs()[0]
    assert (inp.name, inp.shape, out.name, out.shape) == ("observation", [1, 98], "action", [1, 12])
    y = sess.run([out.name], {inp.name: np.ones(inp.shape, dtype=np.float32) * 2})[0]
    want = np.load(os.path.join(GOLDEN, "golden_shipped.npz"))["twos_y"]
    assert rel_err(y, want) <= TOL


# (batch, resident_ms): batch <= 8 runs the single-launch latency kernel (0) or the
# resident kernel (100); 300 the batched kernel (the 4-wave pipeline where it applies)
PATHS = [(1, 0), (1, 100), (5, 0), (5, 100), (300, 0)]


@pytest.mark.parametrize("kind", graphs.VARIANTS)
@pytest.mark.parametrize("B,res", PATHS)
def test_graph_variants_on_gpu(tmp_path, kind, B, res):
    from go2_onnx_controller_amd import Engine
    from oracle import onnx_ref
    p = graphs.write(tmp_path, kind, seed=B)
    g = onnx_ref.load(p)
    x = np.random.default_rng(B).standard_normal((B, g.inputs[0][1][1])).astype(np.float32) * 2
    want = onnx_ref.act(g, x.astype(np.float64))
    # These graphs have unnormalised N(0, 0.3^2) weights: relu_deep's activations
    # reach |600| and small outputs arise by cancellation, where even the CPU fp32
    # path (oracle in float32) is 4.9e-5 off element-wise. The fp32 rounding scale
    # is the activations' magnitude, so the bound is normwise:
    # max|y - ref| / max(1, max|ref|) <= 1e-5.
    with Engine(p, max_batch=512, resident_ms=res) as e:
        y = e.run(x)
        y2 = e.run(x)  # a second call (the resident kernel: the live one answers)
    assert abs_err(y, want) / max(1.0, float(np.abs(want).max())) <= TOL
    np.testing.assert_array_equal(y2, y)
    assert abs_err(onnx_ref.act(g, x, dtype=np.float32), want) / max(1.0, float(np.abs(want).max())) <= TOL


@pytest.mark.parametrize("kind", graphs.NAN_VARIANTS)
@pytest.mark.parametrize("B,res", PATHS)
def test_graph_nan_propagates(tmp_path, kind, B, res):
    """ONNX Clip / Elu / Tanh propagate a NaN (onnxruntime's Clip is
    std::min(std::max(x, lo), hi)): a NaN in an observation row makes that row's
    actions NaN on every kernel path, never the clip bound, and leaves the other
    rows untouched."""
    from go2_onnx_controller_amd import Engine
    from oracle import onnx_ref
    p = graphs.write(tmp_path, kind, seed=B)
    g = onnx_ref.load(p)
    x = np.random.default_rng(B).standard_normal((B, g.inputs[0][1][1])).astype(np.float32)
    x[0, 3] = np.nan
    if B > 2:
        x[B - 1, 0] = np.nan
    want = onnx_ref.act(g, x.astype(np.float64))
    assert np.isnan(want[0]).all()
    with Engine(p, max_batch=512, resident_ms=res) as e:
        y = e.run(x)
    np.testing.assert_array_equal(np.isnan(y), np.isnan(want))
    ok = ~np.isnan(want)
    if ok.any():
        assert abs_err(y[ok], want[ok]) / max(1.0, float(np.abs(want[ok]).max())) <= TOL


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_fleet_two_ranks_bitwise(tmp_path, synth_path):
    """Two processes each run their contiguous shard on the GPU and all-gather the
    actions (gloo); the result equals the unsharded batch bit for bit."""
    from go2_onnx_controller_amd import Engine
    batch, path = 4096, synth_path("go2_mlp_512")
    env = dict(os.environ, WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               FLEET_BATCH=str(batch), FLEET_MODEL=path, FLEET_OUT=str(tmp_path))
    worker = os.path.join(ROOT, "tests", "fleet_gpu_worker.py")
    procs = [subprocess.Popen([sys.executable, worker], env=dict(env, RANK=str(r))) for r in range(2)]
    assert [p.wait(timeout=300) for p in procs] == [0, 0]
    obs = np.random.default_rng(77).standard_normal((batch, 48)).astype(np.float32)
    with Engine(path, max_batch=batch) as e:
        want = e.run(obs)
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"rank{r}.npy"), want)


def test_configs3_fleet_at_size(synth_path):
    """BASELINE configs[3] at its size on the HIP path: 32,768 robots of the
    48->512^3->12 policy, seed-1 observations. The full batch in
    one launch is bitwise equal to the eight contiguous 4,096-row shards
    fleet.shard_range gives the eight ranks (each robot's row runs the same
    instruction sequence wherever it sits), and 256 sampled rows —
    the first and last 16-row tile of every shard among them — are within 1e-5 of
    the fp64 oracle."""
    import torch
    from go2_onnx_controller_amd import Engine, fleet
    from oracle import mlp_ref
    B, world, path = 32768, 8, synth_path("go2_mlp_512")
    obs = np.random.default_rng(1).standard_normal((B, 48)).astype(np.float32)
    x = torch.from_numpy(obs).to("cuda:0")
    with Engine(path, max_batch=B) as e:
        full = e.run_torch(x)
        shards = torch.empty_like(full)
        for r in range(world):
            a, b = fleet.shard_range(B, r, world)
            assert b - a == 4096
            e.run_torch(x[a:b], out=shards[a:b])
        torch.cuda.synchronize()
    full, shards = full.cpu().numpy(), shards.cpu().numpy()
    np.testing.assert_array_equal(full, shards)
    rows = set()
    for r in range(world):
        a, b = fleet.shard_range(B, r, world)
        rows.update(range(a, a + 16))
        rows.update(range(b - 16, b))
    rng = np.random.default_rng(3)
    while len(rows) < 256:
        rows.add(int(rng.integers(0, B)))
    rows = np.array(sorted(rows))
    ref = mlp_ref.MlpRef.from_onnx(path).f64(obs[rows])
    assert abs_err(full[rows], ref) <= TOL
