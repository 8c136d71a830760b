"""GPU parity for the recurrent (GRU) policy path — BASELINE configs[4].

Build-defined model: ONNX GRU, gate order z,r,h,
linear_before_reset=1, hidden state carried per robot by the engine. The
oracle is oracle/onnx_ref.py (numpy fp64, ONNX GRU spec) / oracle/mlp_ref.c
(gruref_step_f64). Tolerance: 1e-5 absolute on actions and hidden state per
tick (SURVEY §8c measured fp32 drift 2.3e-7 over 100 ticks).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, abs_err

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _oracle_rollout(path, xs, h0=None):
    from oracle import onnx_ref
    g = onnx_ref.load(path)
    H = g.inputs[1][1][2]
    T, B = xs.shape[:2]
    h = np.zeros((1, B, H)) if h0 is None else h0[None].astype(np.float64)
    ys = []
    for t in range(T):
        r = onnx_ref.run(g, {"observation": xs[t].astype(np.float64), "h_in": h})
        ys.append(r["action"])
        h = r["h_out"]
    return np.stack(ys), h[0]


@pytest.mark.parametrize("name", ["gru_small", "go2_gru_256"])
def test_gru_golden_ticks(synth_path, name):
    from go2_onnx_controller_amd import Engine
    g = np.load(os.path.join(GOLDEN, f"golden_{name}.npz"))
    xs, ys, hT = g["x"], g["y"], g["h"]
    with Engine(synth_path(name), max_batch=64) as e:
        assert e.hidden_dim == hT.shape[1]
        e.reset_hidden()
        for t in range(xs.shape[0]):
            assert abs_err(e.run(xs[t]), ys[t]) <= TOL, t
        assert abs_err(e.get_hidden(xs.shape[1]), hT) <= TOL


@pytest.mark.parametrize("waves", [4, 8, 16])
def test_gru256_batch_4096_ticks(synth_path, waves):
    from go2_onnx_controller_amd import Engine
    p = synth_path("go2_gru_256")
    rng = np.random.default_rng(waves)
    T, B = 4, 4096
    xs = rng.standard_normal((T, B, 48)).astype(np.float32)
    want_y, want_h = _oracle_rollout(p, xs)
    with Engine(p, max_batch=B, waves=waves) as e:
        for t in range(T):
            assert abs_err(e.run(xs[t]), want_y[t]) <= TOL
        assert abs_err(e.get_hidden(B), want_h) <= TOL


# linear_before_reset = 0 (n = tanh(Wh x + Wbh + Rh (r . h) + Rbh)): the generic body's
# two-pass cell on every path the graph-variant tests cover — batch 1 and 5 with a launch
# per call or the resident option (which serves lbr = 0 by a launch too), and batch 300
@pytest.mark.parametrize("name", ["gru_lbr0_small", "gru_lbr0_128", "go2_gru_256_lbr0"])
@pytest.mark.parametrize("B,res", [(1, 0), (1, 100), (5, 0), (5, 100), (300, 0)])
def test_gru_lbr0_rollout(synth_path, name, B, res):
    from go2_onnx_controller_amd import Engine
    p = synth_path(name)
    with Engine(p, max_batch=512, resident_ms=res) as e:
        rng = np.random.default_rng(B + res)
        T = 5
        xs = rng.standard_normal((T, B, e.in_dim)).astype(np.float32)
        want_y, want_h = _oracle_rollout(p, xs)
        e.reset_hidden()
        for t in range(T):
            assert abs_err(e.run(xs[t]), want_y[t]) <= TOL, t
        assert abs_err(e.get_hidden(B), want_h) <= TOL


def test_gru_lbr0_differs_from_lbr1(synth_path):
    """The two GRU forms are different functions of the same weights: the oracle's lbr=0
    rollout is not the lbr=1 one (so the test above pins the lbr=0 cell itself)."""
    from oracle import onnx_ref
    g = onnx_ref.load(synth_path("gru_lbr0_small"))
    x = np.random.default_rng(3).standard_normal((2, 4, 10))
    y0, _ = _oracle_rollout(synth_path("gru_lbr0_small"), x)
    cell = next(n for n in g.nodes if n.op_type == "GRU")
    cell.attrs["linear_before_reset"] = 1
    h = np.zeros((1, 4, 32))
    y1 = onnx_ref.run(g, {"observation": x[0], "h_in": h})["action"]
    assert np.abs(y1 - y0[0]).max() > 1e-4


def test_gru_lbr0_sequence_matches_ticks(synth_path):
    """run_sequence (h in LDS across ticks) with the two-pass lbr = 0 cell."""
    import torch
    from go2_onnx_controller_amd import Engine
    p = synth_path("gru_lbr0_128")
    T, B = 6, 300
    x = torch.randn(T, B, 30, device="cuda:0")
    with Engine(p, max_batch=B) as a:
        ya = a.run_sequence_torch(x)
        torch.cuda.synchronize()
        ha = a.get_hidden(B)
    want_y, want_h = _oracle_rollout(p, x.cpu().numpy())
    assert abs_err(ya.cpu().numpy(), want_y) <= TOL
    assert abs_err(ha, want_h) <= TOL


def test_gru_sequence_lds_carry_matches_ticks(synth_path):
    """run_sequence keeps h in LDS across ticks; identical math to per-tick calls."""
    import torch
    from go2_onnx_controller_amd import Engine
    p = synth_path("go2_gru_256")
    T, B = 8, 1000
    x = torch.randn(T, B, 48, device="cuda:0")
    with Engine(p, max_batch=B) as a, Engine(p, max_batch=B) as b:
        ya = a.run_sequence_torch(x)
        torch.cuda.synchronize()
        yb = torch.stack([b.run_torch(x[t].contiguous()) for t in range(T)])
        torch.cuda.synchronize()
        assert torch.equal(ya, yb)
        np.testing.assert_array_equal(a.get_hidden(B), b.get_hidden(B))
    want_y, want_h = _oracle_rollout(p, x.cpu().numpy())
    assert abs_err(ya.cpu().numpy(), want_y) <= TOL


def test_gru_reset_mask_and_set_hidden(synth_path):
    from go2_onnx_controller_amd import Engine
    p = synth_path("gru_small")
    rng = np.random.default_rng(3)
    B = 40
    with Engine(p, max_batch=B) as e:
        h0 = rng.standard_normal((B, e.hidden_dim)).astype(np.float32)
        e.set_hidden(h0)
        np.testing.assert_array_equal(e.get_hidden(B), h0)
        mask = np.zeros(B, np.uint8)
        mask[[0, 5, 6, 7, 39]] = 1
        e.reset_hidden(mask)
        h1 = e.get_hidden(B)
        np.testing.assert_array_equal(h1[mask == 1], 0)
        np.testing.assert_array_equal(h1[mask == 0], h0[mask == 0])
        x = rng.standard_normal((1, B, 10)).astype(np.float32)
        want_y, want_h = _oracle_rollout(p, x, h0=h1)
        assert abs_err(e.run(x[0]), want_y[0]) <= TOL
        assert abs_err(e.get_hidden(B), want_h) <= TOL


def test_gru_small_batches_use_graph(synth_path):
    """Batch 1..8 host path (hipGraph over host-mapped staging) carries h too."""
    from go2_onnx_controller_amd import Engine
    p = synth_path("gru_small")
    rng = np.random.default_rng(4)
    xs = rng.standard_normal((5, 3, 10)).astype(np.float32)
    want_y, want_h = _oracle_rollout(p, xs)
    with Engine(p, max_batch=16) as e:
        for t in range(5):
            assert abs_err(e.run(xs[t]), want_y[t]) <= TOL
        assert abs_err(e.get_hidden(3), want_h) <= TOL


def test_gru_inference_session_explicit_hidden(synth_path):
    """InferenceSession mirror with the graph's explicit (h_in -> h_out) I/O."""
    from go2_onnx_controller_amd import InferenceSession
    p = synth_path("gru_small")
    rng = np.random.default_rng(5)
    sess = InferenceSession(p, max_batch=8)
    names = [o.name for o in sess.get_outputs()]
    assert names == ["action", "h_out"]
    x = rng.standard_normal((1, 4, 10)).astype(np.float32)
    h = rng.standard_normal((1, 4, 32)).astype(np.float32)
    act, h_out = sess.run(None, {"observation": x[0], "h_in": h})
    want_y, want_h = _oracle_rollout(p, x, h0=h[0])
    assert abs_err(act, want_y[0]) <= TOL
    assert abs_err(h_out[0], want_h) <= TOL


def test_gru256_sequence_100_ticks_b4096(synth_path):
    """BASELINE configs[4] as specified: 4096 robots, T = 100 ticks through the
    sequence path (go2pi_run_sequence_device: h0 = 0, hidden rows carried in LDS
    between ticks), checked against the fp64 ONNX-GRU oracle on the actions of every
    tick and on h at t = 100, on 256 sampled robots (rows are independent; the sample
    covers the first and last 16-robot tiles). The per-tick device path over the same
    100 ticks must be bitwise identical to the sequence."""
    import torch
    from go2_onnx_controller_amd import Engine
    p = synth_path("go2_gru_256")
    T, B = 100, 4096
    g = torch.Generator().manual_seed(100)
    x = torch.randn((T, B, 48), generator=g)
    rng = np.random.default_rng(100)
    rows = np.unique(np.concatenate([np.arange(16), np.arange(B - 16, B), rng.choice(B, 224, replace=False)]))
    want_y, want_h = _oracle_rollout(p, x[:, rows].numpy())
    xd = x.to("cuda:0")
    with Engine(p, max_batch=B) as a, Engine(p, max_batch=B) as b:
        a.reset_hidden()
        ya = a.run_sequence_torch(xd)
        torch.cuda.synchronize()
        ha = a.get_hidden(B)
        y = ya.cpu().numpy()
        for t in range(T):
            assert abs_err(y[t, rows], want_y[t]) <= TOL, f"tick {t}"
        assert abs_err(ha[rows], want_h) <= TOL
        b.reset_hidden()
        yb = torch.stack([b.run_torch(xd[t].contiguous()) for t in range(T)])
        torch.cuda.synchronize()
        assert torch.equal(ya, yb)
        np.testing.assert_array_equal(ha, b.get_hidden(B))
