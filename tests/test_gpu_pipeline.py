"""GPU parity of the 4-wave uniform-MLP pipeline (kernels.hip, w4_step / w4_gru)
in every shape it is instantiated for, against the fp64 oracle and against the
generic 8-wave body on the same inputs.

Shapes (tiles per wave x head tiles): 8 x 1 with a 128-wide input (two 64-column
input chunks, register hand-off between layers), 4 x 2 (hand-off, two head
tiles), 2 x 2 (epilogue + barrier between layers, Tanh), a single hidden layer
(the head fetched before layer 0), and GRU front stages with H = 256 and 128.
Batches cover a partial tile, a partial last workgroup and several workgroups.
Tolerance: 1e-5 absolute against fp64 (the synthetic models' outputs are
O(0.1-1)); the generic body is held to the same bound, not to bitwise equality,
because the pipeline consumes each layer's k-chunks in a rotated order.
"""
import numpy as np
import pytest

from conftest import abs_err

pytestmark = pytest.mark.gpu

TOL = 1e-5

# instantiation names: policy_mlp_kernel<tiles per wave, head tiles, layer-0 chunks mod 4, hidden
# activation (1 Elu compile-time, -1 runtime), hidden layers (3 compile-time, 0 runtime), waves> (the lean body) or policy_fused_kernel<waves, tiles per wave, head tiles, layer-0 chunks mod 4,
# recurrent cell (0 none / GRU, 1 LSTM), act, hidden layers>
# (a 33-, 40- or 48-wide observation is padded to 48 columns: 3 chunks; 70 to 128)
SHAPES = {
    "pipe_512_relu": "policy_mlp_kernel<8, 1, 0, -1, 0, 4>",
    "pipe_256_h2": "policy_mlp_kernel<4, 2, 3, 1, 0, 4>",
    "pipe_128_tanh_h2": "policy_mlp_kernel<2, 2, 3, -1, 0, 4>",
    "pipe_one_hidden": "policy_mlp_kernel<4, 1, 3, 1, 0, 4>",
    "go2_mlp_512": "policy_mlp_kernel<8, 1, 3, 1, 3, 4>",
}


@pytest.mark.parametrize("name", sorted(SHAPES))
def test_pipeline_shapes(synth_path, name):
    from go2_onnx_controller_amd import Engine
    from oracle import onnx_ref
    p = synth_path(name)
    g = onnx_ref.load(p)
    in_dim = g.inputs[0][1][1]
    x = np.random.default_rng(7).standard_normal((300, in_dim)).astype(np.float32)
    with Engine(p, max_batch=512, small_batch=-1) as e, Engine(p, max_batch=512, waves=8, small_batch=-1) as gen:
        assert e.batched_kernel == SHAPES[name]
        assert gen.batched_kernel == "policy_fused_kernel<8, 0, 0, 0, 0, -1, 0>"
        for B in (1, 16, 17, 300):
            want = onnx_ref.act(g, x[:B])
            assert abs_err(e.run(x[:B]), want) <= TOL, (name, B)
            assert abs_err(gen.run(x[:B]), want) <= TOL, (name, B)


@pytest.mark.parametrize("name,kernel,env", [("go2_gru_256", "policy_gru_kernel<8, 1, 4>", {}),
                                             ("go2_gru_256", "policy_fused_kernel<4, 8, 1, 0, 0, 1, 3>",
                                              {"GO2PI_GRU_GENERAL": "1"}),
                                             ("go2_gru_256", "policy_fused_kernel<4, 8, 1, 0, 0, -1, 0>",
                                              {"GO2PI_LEAN_RT_NH": "1"}),
                                             ("gru_128", "policy_fused_kernel<4, 4, 1, 0, 0, -1, 0>", {}),
                                             ("gru_128_deep", "policy_gru_kernel<4, 1, 2>", {}),
                                             ("gru_128_deep", "policy_fused_kernel<4, 4, 1, 0, 0, 1, 3>",
                                              {"GO2PI_GRU_GENERAL": "1"})])
def test_pipeline_gru_ticks(synth_path, monkeypatch, name, kernel, env):
    """GRU front stage + MLP pipeline over several ticks (hidden state carried by
    the engine), against the fp64 ONNX GRU oracle, actions and hidden state; the
    lean GRU tick (policy_gru_kernel), the general body with the compile-time Elu and
    layer count, and the runtime forms."""
    from go2_onnx_controller_amd import Engine
    from oracle import onnx_ref
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    p = synth_path(name)
    g = onnx_ref.load(p)
    I, H = g.inputs[0][1][1], g.inputs[1][1][2]
    B, T = 37, 4
    xs = np.random.default_rng(3).standard_normal((T, B, I)).astype(np.float32)
    h = np.zeros((1, B, H))
    with Engine(p, max_batch=64, small_batch=-1) as e:
        assert e.batched_kernel == kernel
        e.reset_hidden()
        for t in range(T):
            r = onnx_ref.run(g, {"observation": xs[t].astype(np.float64), "h_in": h})
            h = r["h_out"]
            assert abs_err(e.run(xs[t]), r["action"]) <= TOL, t
            assert abs_err(e.get_hidden(B), h[0]) <= TOL, t


@pytest.mark.parametrize("env,kname,c0m", [({}, "policy_mlp_kernel", "3"),
                                           ({"GO2PI_NO_PLAIN": "1"}, "policy_fused_kernel", "3"),
                                           ({"GO2PI_K0_PAD64": "1"}, "policy_mlp_kernel", "0"),
                                           ({"GO2PI_NO_PLAIN": "1", "GO2PI_K0_PAD64": "1"}, "policy_fused_kernel", "0"),
                                           ({"GO2PI_LEAN_RT_ACT": "1"}, "policy_mlp_kernel", "3"),
                                           ({"GO2PI_LEAN_RT_NH": "1"}, "policy_mlp_kernel", "3")])
@pytest.mark.parametrize("name", ["go2_mlp_512", "pipe_128_tanh_h2", "pipe_256_h2"])
def test_pipeline_body_and_layer0_variants(synth_path, monkeypatch, name, env, kname, c0m):
    """The lean body (no prologue / epilogue) and the general one, each with layer 0
    padded to 3 chunks (48 columns) or 4 (64), and the lean body with the runtime
    activation dispatch: all against the fp64 oracle (the engine reads the GO2PI_*
    switches at create; A/B diagnostics)."""
    from go2_onnx_controller_amd import Engine
    from oracle import onnx_ref
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    p = synth_path(name)
    g = onnx_ref.load(p)
    x = np.random.default_rng(11).standard_normal((4096, g.inputs[0][1][1])).astype(np.float32)
    with Engine(p, max_batch=4096, small_batch=-1) as e:
        k = e.batched_kernel
        args = k[k.index("<") + 1:-1].split(", ")  # mlp: <tpw, ht, c0m, act, nh>; fused: <waves, tpw, ht, c0m, rnn>
        assert k.startswith(kname) and args[2 if kname == "policy_mlp_kernel" else 3] == c0m, k
        if "GO2PI_LEAN_RT_ACT" in env:
            assert args[3] == "-1", k
        if kname == "policy_mlp_kernel":  # the compile-time layer count only with Elu, 3 hidden layers
            nhc = "3" if name == "go2_mlp_512" and not {"GO2PI_LEAN_RT_ACT", "GO2PI_LEAN_RT_NH"} & set(env) else "0"
            assert args[4] == nhc, k
        for B in (5, 16, 4096):
            assert abs_err(e.run(x[:B]), onnx_ref.act(g, x[:B])) <= TOL, (B, env)


@pytest.mark.parametrize("env", [{"GO2PI_NO_W4": "1"}, {"GO2PI_NO_HEAD_FUSE": "1"}])
@pytest.mark.parametrize("name", ["go2_mlp_512", "pipe_256_h2"])
def test_generic_body_switches(synth_path, monkeypatch, env, name):
    """The generic 8-wave body the engine falls back to when the pipeline is switched off
    (GO2PI_NO_W4=1), and without the head fused into the last hidden layer
    (GO2PI_NO_HEAD_FUSE=1, which also keeps the pipeline off): A/B switches read at
    create, each against the fp64 oracle."""
    from go2_onnx_controller_amd import Engine
    from oracle import onnx_ref
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    p = synth_path(name)
    g = onnx_ref.load(p)
    x = np.random.default_rng(13).standard_normal((4096, g.inputs[0][1][1])).astype(np.float32)
    with Engine(p, max_batch=4096, small_batch=-1) as e:
        assert e.batched_kernel.startswith("policy_fused_kernel<8, 0, 0,"), e.batched_kernel
        for B in (5, 16, 300, 4096):
            assert abs_err(e.run(x[:B]), onnx_ref.act(g, x[:B])) <= TOL, (B, env)


def test_small_chain_switch(synth_path, monkeypatch):
    """GO2PI_SMALL_CHAIN=1 at create: batches <= 8 by the GEMV chain (one launch per layer,
    replayed as a hipGraph) instead of the single-launch latency kernel, against the fp64
    oracle; larger batches are unaffected."""
    from go2_onnx_controller_amd import Engine
    from oracle import onnx_ref
    monkeypatch.setenv("GO2PI_SMALL_CHAIN", "1")
    for name in ("go2_mlp_512", "pipe_one_hidden"):
        p = synth_path(name)
        g = onnx_ref.load(p)
        x = np.random.default_rng(17).standard_normal((64, g.inputs[0][1][1])).astype(np.float32)
        with Engine(p, max_batch=64, small_batch=8) as e:
            for B in (1, 2, 8, 9, 64, 1):
                assert abs_err(e.run(x[:B]), onnx_ref.act(g, x[:B])) <= TOL, (name, B)
