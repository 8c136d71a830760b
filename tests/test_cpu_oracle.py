"""CPU: the oracle pinned against the committed golden fixtures and cross-checked
between its independent restatements (numpy fp64 decoder+evaluator, C fp64,
C fp32). Parity vs onnxruntime is unpinned (absent) — the pins here
are the survey's independently computed known answers for the reference
drivers' inputs (zeros: src/cpp/main.cpp:32, 2*ones: src/python/main.py:20)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, SHIPPED, abs_err, rel_err

# SURVEY.md §8(c), computed independently during the survey with numpy fp64
SURVEY_ZEROS = [-0.795116175, 0.495336666, -0.280416397, 0.764204133, -0.693019657, -0.392156917,
                0.180990518, -0.362693726, 1.064260258, 0.517744812, 0.418805890, 0.866443300]
SURVEY_TWOS = [5.640298546, 0.859931734, 8.819978564, -3.643365861, -19.413944458, -7.316530415,
               0.820267543, 1.408699122, -1.644512823, -5.953271685, -2.744231396, -3.518555660]


@pytest.fixture(scope="module")
def shipped():
    from oracle import onnx_ref
    return onnx_ref.load(SHIPPED)


def test_shipped_model_structure(shipped):
    assert shipped.ir_version == 8 and shipped.opset == 17 and shipped.producer == "pytorch"
    assert shipped.inputs == [("observation", [1, 98])]
    assert shipped.outputs == [("action", [1, 12])]
    assert [n.op_type for n in shipped.nodes] == ["Gemm", "Elu", "Gemm", "Elu", "Gemm", "Elu", "Gemm"]
    assert sum(v.size for v in shipped.inits.values()) == 47244


def test_survey_known_answers(shipped):
    from oracle import onnx_ref
    np.testing.assert_allclose(onnx_ref.act(shipped, np.zeros((1, 98)))[0], SURVEY_ZEROS, atol=5e-9)
    np.testing.assert_allclose(onnx_ref.act(shipped, np.full((1, 98), 2.0))[0], SURVEY_TWOS, atol=5e-9)


def test_golden_shipped_fixture(shipped):
    from oracle import onnx_ref
    g = np.load(os.path.join(GOLDEN, "golden_shipped.npz"))
    for k in ("zeros", "twos", "normal", "realistic"):
        np.testing.assert_allclose(onnx_ref.act(shipped, g[f"{k}_x"].astype(np.float64)), g[f"{k}_y"],
                                   rtol=0, atol=1e-12)


def test_c_oracle_matches_numpy(shipped):
    from oracle import mlp_ref, onnx_ref
    ref = mlp_ref.MlpRef.from_onnx(SHIPPED)
    x = np.random.default_rng(0).standard_normal((257, 98)).astype(np.float32)
    want = onnx_ref.act(shipped, x.astype(np.float64))
    assert abs_err(ref.f64(x), want) < 1e-12
    assert abs_err(ref.f64(x, nthreads=1), want) < 1e-12
    # the fp32 CPU path (bench cpu_baseline) is within the fp32 drift SURVEY §8c measured
    assert rel_err(ref.f32(x), want) < 1e-5


def test_synth_hashes_pinned():
    from go2_onnx_controller_amd import synth
    pinned = json.load(open(os.path.join(GOLDEN, "synth_hashes.json")))
    for name, h in pinned.items():
        assert synth.sha256(name) == h, name


def test_golden_mlp512_fixture(synth_path):
    from oracle import mlp_ref, onnx_ref
    g = np.load(os.path.join(GOLDEN, "golden_mlp512.npz"))
    p = synth_path("go2_mlp_512")
    np.testing.assert_allclose(onnx_ref.act(onnx_ref.load(p), g["x"].astype(np.float64)), g["y"], atol=1e-12)
    assert abs_err(mlp_ref.MlpRef.from_onnx(p).f32(g["x"]), g["y"]) < 1e-6


@pytest.mark.parametrize("name", ["gru_small", "go2_gru_256"])
def test_gru_oracles_agree_with_fixture(synth_path, name):
    """numpy ONNX-GRU evaluator vs the C gruref_step_f64 + MLP head, vs the fixture."""
    from oracle import mlp_ref, onnx_ref
    p = synth_path(name)
    g = onnx_ref.load(p)
    fx = np.load(os.path.join(GOLDEN, f"golden_{name}.npz"))
    gru = next(n for n in g.nodes if n.op_type == "GRU")
    W, R, B = (g.inits[gru.inputs[i]] for i in (1, 2, 3))
    H = R.shape[2]
    head = mlp_ref.MlpRef(mlp_ref_head_layers(g))
    h = np.zeros((fx["x"].shape[1], H))
    for t in range(fx["x"].shape[0]):
        h = mlp_ref.gru_step_f64(W[0], R[0], B[0, :3 * H], B[0, 3 * H:], fx["x"][t], h, lbr=1)
        y = head.f64(h.astype(np.float32))   # head input rounded to fp32 like the graph's f32 tensors
        assert abs_err(y, fx["y"][t]) < 1e-6
    assert abs_err(h, fx["h"]) < 1e-12


def mlp_ref_head_layers(g):
    """Dense layers after the GRU (Squeeze output onward)."""
    layers = []
    for n in g.nodes:
        if n.op_type == "Gemm":
            W = g.inits[n.inputs[1]]
            layers.append([W if n.attrs.get("transB", 0) else W.T, g.inits[n.inputs[2]], "none", 0.0])
        elif n.op_type == "Elu":
            layers[-1][2], layers[-1][3] = "Elu", float(n.attrs.get("alpha", 1.0))
    return [tuple(l) for l in layers]


def test_gru_lbr0_oracle_semantics():
    """linear_before_reset=0 (the ONNX default) differs from lbr=1; the oracle implements both."""
    from oracle import mlp_ref
    r = np.random.default_rng(2)
    I, H, B = 5, 8, 3
    W, R = r.standard_normal((3 * H, I)) * 0.3, r.standard_normal((3 * H, H)) * 0.3
    Wb, Rb = r.standard_normal(3 * H) * 0.3, r.standard_normal(3 * H) * 0.3
    x, h = r.standard_normal((B, I)).astype(np.float32), r.standard_normal((B, H))
    h1 = mlp_ref.gru_step_f64(W, R, Wb, Rb, x, h, lbr=1)
    h0 = mlp_ref.gru_step_f64(W, R, Wb, Rb, x, h, lbr=0)
    sig = lambda v: 1 / (1 + np.exp(-v))  # noqa: E731
    W, R, Wb, Rb = (np.asarray(a, np.float32).astype(np.float64) for a in (W, R, Wb, Rb))
    z = sig(x @ W[:H].T + h @ R[:H].T + Wb[:H] + Rb[:H])
    rg = sig(x @ W[H:2 * H].T + h @ R[H:2 * H].T + Wb[H:2 * H] + Rb[H:2 * H])
    n1 = np.tanh(x @ W[2 * H:].T + Wb[2 * H:] + rg * (h @ R[2 * H:].T + Rb[2 * H:]))
    n0 = np.tanh(x @ W[2 * H:].T + Wb[2 * H:] + (rg * h) @ R[2 * H:].T + Rb[2 * H:])
    np.testing.assert_allclose(h1, (1 - z) * n1 + z * h, atol=1e-12)
    np.testing.assert_allclose(h0, (1 - z) * n0 + z * h, atol=1e-12)
    assert np.abs(h1 - h0).max() > 1e-3


def _torch_gate_reorder(M, order, H):
    """ONNX gate blocks (rows of H) reordered into torch's order."""
    return np.concatenate([M[g * H:(g + 1) * H] for g in order], axis=0)


@pytest.mark.parametrize("name", ["lstm_small", "lstm_128"])
def test_lstm_oracle_matches_torch_lstm(synth_path, name):
    """Pin the oracle's ONNX LSTM against PyTorch's own nn.LSTM (an independent
    implementation, present in this image): ONNX gates i, o, f, c are torch's
    i, f, g, o reordered; biases b_ih / b_hh are ONNX Wb / Rb. 6 ticks, random
    initial (h, c), fp64."""
    import torch
    from oracle import onnx_ref
    g = onnx_ref.load(synth_path(name))
    node = next(n for n in g.nodes if n.op_type == "LSTM")
    W, R, Bb = (g.inits[node.inputs[i]].astype(np.float64)[0] for i in (1, 2, 3))
    H, I = R.shape[1], W.shape[1]
    order = [0, 2, 3, 1]  # torch i, f, g, o from ONNX i, o, f, c
    lstm = torch.nn.LSTM(I, H).double()
    with torch.no_grad():
        lstm.weight_ih_l0.copy_(torch.from_numpy(_torch_gate_reorder(W, order, H)))
        lstm.weight_hh_l0.copy_(torch.from_numpy(_torch_gate_reorder(R, order, H)))
        lstm.bias_ih_l0.copy_(torch.from_numpy(_torch_gate_reorder(Bb[:4 * H], order, H)))
        lstm.bias_hh_l0.copy_(torch.from_numpy(_torch_gate_reorder(Bb[4 * H:], order, H)))
    rng = np.random.default_rng(8)
    B, T = 5, 6
    xs = rng.standard_normal((T, B, I))
    h = rng.standard_normal((1, B, H))
    c = rng.standard_normal((1, B, H))
    with torch.no_grad():
        y_t, (h_t, c_t) = lstm(torch.from_numpy(xs), (torch.from_numpy(h), torch.from_numpy(c)))
    env = {"x_seq": xs, node.inputs[1]: g.inits[node.inputs[1]], node.inputs[2]: g.inits[node.inputs[2]],
           node.inputs[3]: g.inits[node.inputs[3]], "h_in": h, "c_in": c}
    res = onnx_ref._lstm(node, env, np.float64)
    np.testing.assert_allclose(res[node.outputs[0]][:, 0], y_t.numpy(), rtol=0, atol=1e-12)
    np.testing.assert_allclose(res[node.outputs[1]], h_t.numpy(), rtol=0, atol=1e-12)
    np.testing.assert_allclose(res[node.outputs[2]], c_t.numpy(), rtol=0, atol=1e-12)


@pytest.mark.parametrize("name", ["gru_small", "gru_128"])
def test_gru_oracle_matches_torch_gru(synth_path, name):
    """Pin the oracle's ONNX GRU (linear_before_reset = 1) against PyTorch's nn.GRU,
    whose n-gate formula is lbr = 1: ONNX gates z, r, h are torch's r, z, n
    reordered. 6 ticks, random initial h, fp64."""
    import torch
    from oracle import onnx_ref
    g = onnx_ref.load(synth_path(name))
    node = next(n for n in g.nodes if n.op_type == "GRU")
    W, R, Bb = (g.inits[node.inputs[i]].astype(np.float64)[0] for i in (1, 2, 3))
    H, I = R.shape[1], W.shape[1]
    order = [1, 0, 2]  # torch r, z, n from ONNX z, r, h
    gru = torch.nn.GRU(I, H).double()
    with torch.no_grad():
        gru.weight_ih_l0.copy_(torch.from_numpy(_torch_gate_reorder(W, order, H)))
        gru.weight_hh_l0.copy_(torch.from_numpy(_torch_gate_reorder(R, order, H)))
        gru.bias_ih_l0.copy_(torch.from_numpy(_torch_gate_reorder(Bb[:3 * H], order, H)))
        gru.bias_hh_l0.copy_(torch.from_numpy(_torch_gate_reorder(Bb[3 * H:], order, H)))
    rng = np.random.default_rng(9)
    B, T = 5, 6
    xs = rng.standard_normal((T, B, I))
    h = rng.standard_normal((1, B, H))
    with torch.no_grad():
        y_t, h_t = gru(torch.from_numpy(xs), torch.from_numpy(h))
    env = {"x_seq": xs, node.inputs[1]: g.inits[node.inputs[1]], node.inputs[2]: g.inits[node.inputs[2]],
           node.inputs[3]: g.inits[node.inputs[3]], "h_in": h}
    res = onnx_ref._gru(node, env, np.float64)
    np.testing.assert_allclose(res[node.outputs[0]][:, 0], y_t.numpy(), rtol=0, atol=1e-12)
    np.testing.assert_allclose(res[node.outputs[1]], h_t.numpy(), rtol=0, atol=1e-12)
