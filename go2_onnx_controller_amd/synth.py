"""Deterministic synthetic policies named by BASELINE.json's configs.

BASELINE.json quotes its metric on a "48-obs -> 3x512 MLP -> 12 actions" Go2
policy and a "GRU hidden 256" recurrent policy; neither ships with the
reference (which only has the 98->128^3->12 model). They are
generated here from a counter-based hash (splitmix64 of seed/tensor/element),
PyTorch-style U(-1/sqrt(fan_in), 1/sqrt(fan_in)) init, and written as .onnx
with our own writer. Same seed -> same bytes on any machine (sha256 pinned in
tests/golden/synth_hashes.json).

Model specs:
  go2_mlp_512 : observation[batch,48] -> Gemm(512)+Elu -> Gemm(512)+Elu ->
                Gemm(512)+Elu -> Gemm(12) -> action[batch,12]
  go2_gru_256 : observation[batch,48], h_in[1,batch,256] ->
                Unsqueeze -> GRU(H=256, linear_before_reset=1) -> Squeeze ->
                256->512^3->12 Elu head -> action[batch,12], h_out[1,batch,256]
  go2_lstm_256: observation[batch,48], h_in, c_in[1,batch,256] ->
                Unsqueeze -> LSTM(H=256) -> Squeeze -> 256->512^3->12 Elu head
                -> action[batch,12], h_out, c_out[1,batch,256]
"""
from __future__ import annotations

import hashlib
import os

import numpy as np

from . import onnx_writer as ow

_M1 = np.uint64(0x9E3779B97F4A7C15)
_M2 = np.uint64(0xBF58476D1CE4E5B9)
_M3 = np.uint64(0x94D049BB133111EB)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _M1
        z = (z ^ (z >> np.uint64(30))) * _M2
        z = (z ^ (z >> np.uint64(27))) * _M3
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, tensor_id: int, shape, bound: float) -> np.ndarray:
    """U(-bound, bound) float32, element i = f(splitmix64(seed, tensor_id, i))."""
    n = int(np.prod(shape)) if len(shape) else 1
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * np.uint64(0xD1B54A32D192ED03) + np.uint64(tensor_id) * np.uint64(0x8CB92BA72F3D8DD7)
        key = base + np.arange(n, dtype=np.uint64)
    u = (_splitmix64(key) >> np.uint64(40)).astype(np.float64) / float(1 << 24)  # [0,1)
    return ((2.0 * u - 1.0) * bound).astype(np.float32).reshape(shape)


def mlp_layers(dims, seed=0, first_tid=0):
    layers = []
    tid = first_tid
    for k, n in zip(dims[:-1], dims[1:]):
        bound = 1.0 / np.sqrt(k)
        W = uniform(seed, tid, (n, k), bound)
        b = uniform(seed, tid + 1, (n,), bound)
        tid += 2
        layers.append((W, b))
    return layers


def mlp_model_bytes(dims=(48, 512, 512, 512, 12), seed=0, act="Elu", batch="batch") -> bytes:
    layers = mlp_layers(dims, seed)
    nodes, inits = [], []
    cur = "observation"
    for i, (W, b) in enumerate(layers):
        wn, bn = f"{2 * i}.weight", f"{2 * i}.bias"
        inits += [(wn, W), (bn, b)]
        last = i == len(layers) - 1
        out = "action" if last else f"/{2 * i}/Gemm_output_0"
        nodes.append(ow.node("Gemm", [cur, wn, bn], [out], f"/{2 * i}/Gemm",
                             [ow.attr_float("alpha", 1.0), ow.attr_float("beta", 1.0), ow.attr_int("transB", 1)]))
        cur = out
        if not last:
            aout = f"/{2 * i + 1}/{act}_output_0"
            attrs = [ow.attr_float("alpha", 1.0)] if act == "Elu" else []
            nodes.append(ow.node(act, [cur], [aout], f"/{2 * i + 1}/{act}", attrs))
            cur = aout
    return ow.model(nodes, inits, [("observation", [batch, dims[0]])], [("action", [batch, dims[-1]])])


def gru_params(I=48, H=256, seed=0):
    bound = 1.0 / np.sqrt(H)
    W = uniform(seed, 100, (1, 3 * H, I), bound)
    R = uniform(seed, 101, (1, 3 * H, H), bound)
    B = uniform(seed, 102, (1, 6 * H), bound)
    return W, R, B


def gru_model_bytes(I=48, H=256, head=(512, 512, 512, 12), seed=0, batch="batch", lbr=1) -> bytes:
    """lbr: linear_before_reset (1: torch.onnx.export's nn.GRU and Keras' default
    reset_after=True; 0: Keras reset_after=False and the ONNX default)."""
    W, R, B = gru_params(I, H, seed)
    layers = mlp_layers((H,) + tuple(head), seed, first_tid=200)
    axes = np.array([0], np.int64)
    inits = [("gru.W", W), ("gru.R", R), ("gru.B", B), ("axes0", axes)]
    nodes = [
        ow.node("Unsqueeze", ["observation", "axes0"], ["x_seq"], "/gru/Unsqueeze"),
        ow.node("GRU", ["x_seq", "gru.W", "gru.R", "gru.B", "", "h_in"], ["gru_Y", "h_out"], "/gru/GRU",
                [ow.attr_int("hidden_size", H)] + ([ow.attr_int("linear_before_reset", 1)] if lbr else [])),
        ow.node("Squeeze", ["h_out", "axes0"], ["h_t"], "/gru/Squeeze"),
    ]
    cur = "h_t"
    for i, (Wl, bl) in enumerate(layers):
        wn, bn = f"head.{i}.weight", f"head.{i}.bias"
        inits += [(wn, Wl), (bn, bl)]
        last = i == len(layers) - 1
        out = "action" if last else f"/head/{i}/Gemm_output_0"
        nodes.append(ow.node("Gemm", [cur, wn, bn], [out], f"/head/{i}/Gemm",
                             [ow.attr_float("alpha", 1.0), ow.attr_float("beta", 1.0), ow.attr_int("transB", 1)]))
        cur = out
        if not last:
            aout = f"/head/{i}/Elu_output_0"
            nodes.append(ow.node("Elu", [cur], [aout], f"/head/{i}/Elu", [ow.attr_float("alpha", 1.0)]))
            cur = aout
    return ow.model(nodes, inits,
                    [("observation", [batch, I]), ("h_in", [1, batch, H])],
                    [("action", [batch, head[-1]]), ("h_out", [1, batch, H])])


def lstm_params(I=48, H=256, seed=0):
    bound = 1.0 / np.sqrt(H)
    W = uniform(seed, 110, (1, 4 * H, I), bound)
    R = uniform(seed, 111, (1, 4 * H, H), bound)
    B = uniform(seed, 112, (1, 8 * H), bound)
    return W, R, B


def _head(cur, head, H, seed, nodes, inits):
    layers = mlp_layers((H,) + tuple(head), seed, first_tid=200)
    for i, (Wl, bl) in enumerate(layers):
        wn, bn = f"head.{i}.weight", f"head.{i}.bias"
        inits += [(wn, Wl), (bn, bl)]
        last = i == len(layers) - 1
        out = "action" if last else f"/head/{i}/Gemm_output_0"
        nodes.append(ow.node("Gemm", [cur, wn, bn], [out], f"/head/{i}/Gemm",
                             [ow.attr_float("alpha", 1.0), ow.attr_float("beta", 1.0), ow.attr_int("transB", 1)]))
        cur = out
        if not last:
            aout = f"/head/{i}/Elu_output_0"
            nodes.append(ow.node("Elu", [cur], [aout], f"/head/{i}/Elu", [ow.attr_float("alpha", 1.0)]))
            cur = aout


def lstm_model_bytes(I=48, H=256, head=(512, 512, 512, 12), seed=0, batch="batch") -> bytes:
    """ONNX LSTM (gates i, o, f, c) as torch.onnx.export writes an nn.LSTM policy: the
    observation unsqueezed to a 1-step sequence, (h, c) explicit graph I/O."""
    W, R, B = lstm_params(I, H, seed)
    axes = np.array([0], np.int64)
    inits = [("lstm.W", W), ("lstm.R", R), ("lstm.B", B), ("axes0", axes)]
    nodes = [
        ow.node("Unsqueeze", ["observation", "axes0"], ["x_seq"], "/lstm/Unsqueeze"),
        ow.node("LSTM", ["x_seq", "lstm.W", "lstm.R", "lstm.B", "", "h_in", "c_in"], ["lstm_Y", "h_out", "c_out"],
                "/lstm/LSTM", [ow.attr_int("hidden_size", H)]),
        ow.node("Squeeze", ["h_out", "axes0"], ["h_t"], "/lstm/Squeeze"),
    ]
    _head("h_t", head, H, seed, nodes, inits)
    return ow.model(nodes, inits,
                    [("observation", [batch, I]), ("h_in", [1, batch, H]), ("c_in", [1, batch, H])],
                    [("action", [batch, head[-1]]), ("h_out", [1, batch, H]), ("c_out", [1, batch, H])])


MODELS = {
    "go2_mlp_512": lambda: mlp_model_bytes(),
    "go2_gru_256": lambda: gru_model_bytes(),
    # small variants for fast tests
    "mlp_small_relu": lambda: mlp_model_bytes((20, 64, 40, 5), seed=3, act="Relu"),
    "mlp_small_tanh": lambda: mlp_model_bytes((33, 48, 7), seed=4, act="Tanh"),
    "gru_small": lambda: gru_model_bytes(I=10, H=32, head=(64, 6), seed=5),
    # launch/sync floor probe (tools/latency_probe.py)
    "tiny": lambda: mlp_model_bytes((4, 16, 4), seed=6),
    # controller-tick policies (49 * kHistory observations, 12 actions) besides the shipped 98 -> 12
    "ctl_h1": lambda: mlp_model_bytes((49, 64, 64, 12), seed=7),
    "ctl_h3": lambda: mlp_model_bytes((147, 128, 128, 12), seed=8),
    "ctl_h16": lambda: mlp_model_bytes((784, 128, 128, 12), seed=17),  # the longest history (16 x 49)
    # three hidden layers (the lean controller tick) at histories whose layer-0 K pads to 64
    # (147 -> 10 chunks of 16, padded to 12; 196 -> 13, padded to 16)
    "ctl_h3_deep": lambda: mlp_model_bytes((147, 128, 128, 128, 12), seed=9),
    "ctl_h4_deep": lambda: mlp_model_bytes((196, 128, 128, 128, 12), seed=10),
    "gru_ctl": lambda: gru_model_bytes(I=98, H=64, head=(128, 12), seed=9),
    # shapes of the 4-wave pipeline (kernels.hip w4_step): tiles per wave x head tiles
    "pipe_256_h2": lambda: mlp_model_bytes((40, 256, 256, 20), seed=10),                      # 4 x 2, hand-off
    "pipe_128_tanh_h2": lambda: mlp_model_bytes((33, 128, 128, 128, 30), seed=11, act="Tanh"),  # 2 x 2, barrier
    "pipe_512_relu": lambda: mlp_model_bytes((70, 512, 512, 7), seed=12, act="Relu"),         # 8 x 1, K0 = 128
    "pipe_one_hidden": lambda: mlp_model_bytes((48, 256, 12), seed=13),                       # one hidden layer
    # the resident wide-policy kernel's other shapes (resident_wide.hip): hidden width 256
    # (four compute waves) with one and two sliced layers, 512 with one; a 16-output head
    "wide_256_3": lambda: mlp_model_bytes((45, 256, 256, 16), seed=21),
    "wide_256_4": lambda: mlp_model_bytes((60, 256, 256, 256, 12), seed=22, act="Tanh"),
    "wide_512_3": lambda: mlp_model_bytes((33, 512, 512, 10), seed=23, act="Relu"),
    "gru_128": lambda: gru_model_bytes(I=30, H=128, head=(256, 256, 12), seed=14),            # 2-tile GRU stage
    "gru_128_deep": lambda: gru_model_bytes(I=30, H=128, head=(256, 256, 256, 12), seed=15),  # lean GRU tick, H = 128
    # GRU with linear_before_reset = 0 (the attribute left at its ONNX default): the
    # generic body's two-pass cell (fused_impl.hpp gru0_cell)
    "gru_lbr0_small": lambda: gru_model_bytes(I=10, H=32, head=(64, 6), seed=18, lbr=0),
    "gru_lbr0_128": lambda: gru_model_bytes(I=30, H=128, head=(256, 256, 12), seed=19, lbr=0),
    "go2_gru_256_lbr0": lambda: gru_model_bytes(seed=20, lbr=0),
    # LSTM policies (the other recurrent cell of exported rsl_rl / Isaac policies)
    "go2_lstm_256": lambda: lstm_model_bytes(),
    "lstm_128": lambda: lstm_model_bytes(I=30, H=128, head=(256, 256, 12), seed=15),           # 2-tile LSTM stage
    "lstm_small": lambda: lstm_model_bytes(I=10, H=32, head=(64, 6), seed=16),                 # generic body
}

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODEL_DIR = os.path.join(_REPO, "build", "models")


def ensure_model(name: str, directory: str | None = None) -> str:
    """Write (if absent or stale) and return the path of synthetic model `name`."""
    directory = directory or MODEL_DIR
    os.makedirs(directory, exist_ok=True)
    data = MODELS[name]()
    path = os.path.join(directory, name + ".onnx")
    if not os.path.exists(path) or open(path, "rb").read() != data:
        tmp = path + f".tmp{os.getpid()}"
        with open(tmp, "wb") as fh:
            fh.write(data)
        os.replace(tmp, path)
    return path


def sha256(name: str) -> str:
    return hashlib.sha256(MODELS[name]()).hexdigest()
