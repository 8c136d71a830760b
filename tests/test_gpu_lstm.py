"""GPU parity for LSTM policies (SURVEY §8f.3 loader breadth: recurrent rsl_rl /
Isaac exports commonly use an LSTM cell; the reference's ORT session loads any
exported policy, onnx_inference/src/cpp/onnx_actor.cpp:16,23-28).

ONNX LSTM (opset 14): gates i, o, f, c, default activations, no peepholes; the
engine keeps h | c per robot (hidden_dim = 2H). Oracle: oracle/onnx_ref.py
(_lstm, numpy fp64), itself pinned against PyTorch's nn.LSTM
(tests/test_cpu_oracle.py::test_lstm_oracle_matches_torch_lstm). Paths: the
4-wave pipeline's LSTM stage (H = 128, 256: c in registers across the ticks of a
sequence), and the generic body (H = 32, or waves = 8: c read and written per tick
by the lane that owns it). Tolerance 1e-5 absolute on actions, h and c per tick.
"""
import numpy as np
import pytest

from conftest import abs_err

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _rollout(path, xs, h0=None, c0=None):
    from oracle import onnx_ref
    g = onnx_ref.load(path)
    H = g.inputs[1][1][2]
    T, B = xs.shape[:2]
    h = np.zeros((1, B, H)) if h0 is None else h0[None].astype(np.float64)
    c = np.zeros((1, B, H)) if c0 is None else c0[None].astype(np.float64)
    ys = []
    for t in range(T):
        r = onnx_ref.run(g, {"observation": xs[t].astype(np.float64), "h_in": h, "c_in": c})
        ys.append(r["action"])
        h, c = r["h_out"], r["c_out"]
    return np.stack(ys), h[0], c[0]


# go2_lstm_256 (LSTM-256 + 512^3 Elu head) takes the lean LSTM tick (policy_lstm_kernel,
# r06); GO2PI_GRU_GENERAL=1 keeps the general body's pipelined LSTM stage
@pytest.mark.parametrize("name,waves,kernel,general", [
    ("lstm_small", 0, "policy_fused_kernel<8, 0, 0, 0, 1, -1, 0>", False),
    ("lstm_128", 0, "policy_fused_kernel<4, 4, 1, 0, 1, -1, 0>", False),
    ("go2_lstm_256", 0, "policy_lstm_kernel<8, 1, 4>", False),
    ("go2_lstm_256", 0, "policy_fused_kernel<4, 8, 1, 0, 1, 1, 3>", True),
    ("go2_lstm_256", 8, "policy_fused_kernel<8, 0, 0, 0, 1, -1, 0>", False)])
@pytest.mark.parametrize("B", [1, 37, 4096])
def test_lstm_ticks(synth_path, monkeypatch, name, waves, kernel, general, B):
    from go2_onnx_controller_amd import Engine
    if general:
        monkeypatch.setenv("GO2PI_GRU_GENERAL", "1")  # read at engine creation
    p = synth_path(name)
    rng = np.random.default_rng(B + waves)
    with Engine(p, max_batch=max(B, 64), waves=waves) as e:
        assert e.batched_kernel == kernel
        H = e.hidden_dim // 2
        T = 4 if B == 4096 else 6
        xs = rng.standard_normal((T, B, e.in_dim)).astype(np.float32)
        rows = np.arange(B) if B < 4096 else np.unique(np.r_[0:16, B - 16:B, rng.choice(B, 96, replace=False)])
        want_y, want_h, want_c = _rollout(p, xs[:, rows])
        e.reset_hidden()
        for t in range(T):
            assert abs_err(e.run(xs[t])[rows], want_y[t]) <= TOL, t
        st = e.get_hidden(B)[rows]
        assert abs_err(st[:, :H], want_h) <= TOL
        assert abs_err(st[:, H:], want_c) <= TOL


@pytest.mark.parametrize("name", ["go2_lstm_256", "lstm_128", "lstm_small"])
def test_lstm_sequence_matches_ticks(synth_path, name):
    """run_sequence carries h in LDS and c in registers across the ticks (pipeline),
    bitwise equal to per-tick launches; actions and (h, c) at t = T against fp64."""
    import torch
    from go2_onnx_controller_amd import Engine
    p = synth_path(name)
    T, B = 20, 1000
    g = torch.Generator().manual_seed(7)
    with Engine(p, max_batch=B) as a, Engine(p, max_batch=B) as b:
        x = torch.randn((T, B, a.in_dim), generator=g)
        xd = x.to("cuda:0")
        ya = a.run_sequence_torch(xd)
        torch.cuda.synchronize()
        yb = torch.stack([b.run_torch(xd[t].contiguous()) for t in range(T)])
        torch.cuda.synchronize()
        assert torch.equal(ya, yb)
        np.testing.assert_array_equal(a.get_hidden(B), b.get_hidden(B))
        H = a.hidden_dim // 2
        rows = np.r_[0:16, 500:516, B - 8:B]
        want_y, want_h, want_c = _rollout(p, x[:, rows].numpy())
        assert abs_err(ya.cpu().numpy()[:, rows], want_y) <= TOL
        st = a.get_hidden(B)[rows]
        assert abs_err(st[:, :H], want_h) <= TOL and abs_err(st[:, H:], want_c) <= TOL


def test_lstm_state_set_reset_and_session_io(synth_path):
    """set_hidden / masked reset of (h, c), and the InferenceSession mirror with the
    graph's explicit (h_in, c_in) -> (h_out, c_out) I/O."""
    from go2_onnx_controller_amd import Engine, InferenceSession
    p = synth_path("lstm_128")
    rng = np.random.default_rng(5)
    B = 40
    with Engine(p, max_batch=B) as e:
        H = e.hidden_dim // 2
        s0 = rng.standard_normal((B, 2 * H)).astype(np.float32)
        e.set_hidden(s0)
        np.testing.assert_array_equal(e.get_hidden(B), s0)
        mask = np.zeros(B, np.uint8)
        mask[[1, 2, 30]] = 1
        e.reset_hidden(mask)
        s1 = e.get_hidden(B)
        np.testing.assert_array_equal(s1[mask == 1], 0)
        np.testing.assert_array_equal(s1[mask == 0], s0[mask == 0])
        x = rng.standard_normal((1, B, e.in_dim)).astype(np.float32)
        want_y, want_h, want_c = _rollout(p, x, h0=s1[:, :H], c0=s1[:, H:])
        assert abs_err(e.run(x[0]), want_y[0]) <= TOL
        st = e.get_hidden(B)
        assert abs_err(st[:, :H], want_h) <= TOL and abs_err(st[:, H:], want_c) <= TOL
    sess = InferenceSession(p, max_batch=8)
    assert [o.name for o in sess.get_outputs()] == ["action", "h_out", "c_out"]
    x = rng.standard_normal((1, 4, 30)).astype(np.float32)
    h = rng.standard_normal((1, 4, 128)).astype(np.float32)
    c = rng.standard_normal((1, 4, 128)).astype(np.float32)
    act, h_out, c_out = sess.run(None, {"observation": x[0], "h_in": h, "c_in": c})
    want_y, want_h, want_c = _rollout(p, x, h0=h[0], c0=c[0])
    assert abs_err(act, want_y[0]) <= TOL
    assert abs_err(h_out[0], want_h) <= TOL and abs_err(c_out[0], want_c) <= TOL
