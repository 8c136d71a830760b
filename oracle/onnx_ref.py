"""ORACLE — test infrastructure only. NOT part of the product path.

Parity status: **parity unpinned** by the reference. The reference's arithmetic
lives in the third-party prebuilt onnxruntime v1.20.1 binary
(`onnx_inference/cmake/dependencies.cmake:14-31`), which is fetched by URL at
configure time and is absent from this container and from the GPU box; the
reference ships no tests and no expected outputs. This
module is therefore a CPU restatement of the published ONNX operator semantics
the reference's graph uses, evaluated on the reference's own weights
(`onnx_inference/data/model.onnx`, copied byte-identical to
`tests/golden/model.onnx`, sha256 9bdcb0f4…8eae):

* `Gemm` (opset 13): Y = alpha * A' @ B' + beta * C, A' = A^T if transA,
  B' = B^T if transB. The shipped graph uses transB=1, alpha=beta=1
  (nodes /0/Gemm, /2/Gemm, /4/Gemm, /6/Gemm).
* `Elu` (opset 6): y = x if x > 0 else alpha * (exp(x) - 1).
* `Relu`, `Tanh`, `Sigmoid`, `LeakyRelu`, `Selu`, `Softplus`, `HardSigmoid`,
  `HardSwish`, `Softsign`, `MatMul`, `Add`, `Clip` (opset 6 attributes or opset
  11 inputs; NaN passes through, as onnxruntime's std::min(std::max(x, lo), hi)),
  `Sub`, `Div`, `Mul`, `Constant` for the other exported-policy graph shapes
  (SURVEY §8f.3), each as the ONNX operator specification states it.
* `GRU` (opset 14), build-defined recurrent policy:
  gate order z, r, h; f = sigmoid, g = tanh;
  linear_before_reset=1:  h~ = tanh(Wh x + Wbh + r * (Rh h + Rbh))
  linear_before_reset=0:  h~ = tanh(Wh x + Wbh + Rh (r * h) + Rbh)
  H' = (1 - z) * h~ + z * H.
* `Slice` (opset 13; opset 1 attributes) and `Concat` (opset 13), the per-block
  observation front-end (Slice the observation, normalise each block, Concat) an
  exported policy may carry (numpy slicing semantics: negative indices count from
  the end, out-of-range ones clamp, as the operator specification states).
* `LSTM` (opset 14), the other recurrent cell exported policies use (SURVEY
  §8f.3): gate order i, o, f, c; f = sigmoid, g = h = tanh; no peepholes,
  input_forget = 0:
  i = f(Wi x + Ri H + Wbi + Rbi), o = f(Wo x + Ro H + Wbo + Rbo),
  f = f(Wf x + Rf H + Wbf + Rbf), c~ = g(Wc x + Rc H + Wbc + Rbc),
  C' = f * C + i * c~, H' = o * h(C').

The I/O contract mirrors `ONNXActor` (`onnx_inference/src/cpp/onnx_actor.cpp:23-35`):
input 0 -> output 0, row-major float32, element count = shape[1].

The protobuf decoder below is an independent re-implementation of the proto3
wire format (varint / 64-bit / length-delimited / 32-bit) with the ONNX field
numbers of onnx.proto (ModelProto.graph=7, GraphProto.node=1, initializer=5,
input=11, output=12; NodeProto input=1, output=2, name=3, op_type=4,
attribute=5; AttributeProto name=1, f=2, i=3, floats=7, ints=8, type=20;
TensorProto dims=1, data_type=2, float_data=4, name=8, raw_data=9). It shares
no code with the product's C++ loader (go2_onnx_controller_amd/csrc/onnx_model.cpp),
so a decoding bug in one is caught by the other.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

import numpy as np

# ----------------------------------------------------------------- wire format


def _varint(buf: bytes, pos: int) -> tuple[int, int]:
    shift = 0
    out = 0
    while True:
        b = buf[pos]
        pos += 1
        out |= (b & 0x7F) << shift
        if not b & 0x80:
            return out, pos
        shift += 7


def _fields(buf: bytes):
    """Yield (field_number, wire_type, value) for one message body."""
    pos = 0
    n = len(buf)
    while pos < n:
        key, pos = _varint(buf, pos)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            val, pos = _varint(buf, pos)
        elif wt == 1:
            val = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            val = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            val = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fno, wt, val


def _packed_varints(val, wt) -> list[int]:
    if wt == 0:
        return [val]
    out, p = [], 0
    while p < len(val):
        v, p = _varint(val, p)
        out.append(v)
    return out


def _signed64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


@dataclass
class Node:
    op_type: str
    name: str
    inputs: list
    outputs: list
    attrs: dict = field(default_factory=dict)


@dataclass
class Graph:
    nodes: list
    inits: dict          # name -> np.ndarray (float64 copy of the stored float32)
    inputs: list         # [(name, shape)]
    outputs: list        # [(name, shape)]
    opset: int = 0
    producer: str = ""
    ir_version: int = 0


def _tensor(buf: bytes):
    dims, dtype, name, raw, fdata, idata = [], 1, "", None, [], []
    for fno, wt, val in _fields(buf):
        if fno == 1:
            dims.extend(_signed64(v) for v in _packed_varints(val, wt))
        elif fno == 2:
            dtype = val
        elif fno == 4:
            if wt == 2:
                fdata.extend(struct.unpack(f"<{len(val) // 4}f", val))
            else:
                fdata.append(struct.unpack("<f", val)[0])
        elif fno == 7:
            idata.extend(_signed64(v) for v in _packed_varints(val, wt))
        elif fno == 8:
            name = val.decode()
        elif fno == 9:
            raw = bytes(val)
    if dtype == 7:                           # INT64 (e.g. Unsqueeze/Squeeze axes, opset 13+)
        arr = np.frombuffer(raw, dtype="<i8").copy() if raw is not None else np.asarray(idata, np.int64)
        return name, arr.reshape(dims) if dims else arr.reshape(())
    if dtype != 1:
        raise ValueError(f"initializer {name}: only FLOAT/INT64 tensors supported (got {dtype})")
    if raw is not None:
        arr = np.frombuffer(raw, dtype="<f4").copy()
    else:
        arr = np.asarray(fdata, dtype=np.float32)
    return name, arr.reshape(dims) if dims else arr.reshape(())


def _attr(buf: bytes):
    name, kind, f, i, s, t, floats, ints = "", 0, None, None, None, None, [], []
    for fno, wt, val in _fields(buf):
        if fno == 1:
            name = val.decode()
        elif fno == 2:
            f = struct.unpack("<f", val)[0]
        elif fno == 3:
            i = _signed64(val)
        elif fno == 4:
            s = val.decode()
        elif fno == 7:
            if wt == 2:
                floats.extend(struct.unpack(f"<{len(val) // 4}f", val))
            else:
                floats.append(struct.unpack("<f", val)[0])
        elif fno == 8:
            ints.extend(_signed64(v) for v in _packed_varints(val, wt))
        elif fno == 5:                       # t: TensorProto (Constant's value)
            t = _tensor(val)[1]
        elif fno == 20:
            kind = val
    # AttributeProto.AttributeType: FLOAT=1 INT=2 STRING=3 TENSOR=4 FLOATS=6 INTS=7
    value = {1: f, 2: i, 3: s, 4: t, 6: floats, 7: ints}.get(kind)
    if value is None:
        value = f if f is not None else (i if i is not None else (t if t is not None else (floats or ints or s)))
    return name, value


def _node(buf: bytes) -> Node:
    n = Node("", "", [], [])
    for fno, _, val in _fields(buf):
        if fno == 1:
            n.inputs.append(val.decode())
        elif fno == 2:
            n.outputs.append(val.decode())
        elif fno == 3:
            n.name = val.decode()
        elif fno == 4:
            n.op_type = val.decode()
        elif fno == 5:
            k, v = _attr(val)
            n.attrs[k] = v
    return n


def _value_info(buf: bytes):
    name, shape = "", []
    for fno, _, val in _fields(buf):
        if fno == 1:
            name = val.decode()
        elif fno == 2:                       # TypeProto
            for f2, _, v2 in _fields(val):
                if f2 == 1:                  # tensor_type
                    for f3, _, v3 in _fields(v2):
                        if f3 == 2:          # TensorShapeProto
                            for f4, _, v4 in _fields(v3):
                                if f4 == 1:  # Dimension
                                    d = None
                                    for f5, _, v5 in _fields(v4):
                                        if f5 == 1:
                                            d = _signed64(v5)
                                        elif f5 == 2:
                                            d = v5.decode()
                                    shape.append(d)
    return name, shape


def load(path_or_bytes) -> Graph:
    """Decode an ONNX ModelProto (ref: onnx_actor.cpp:16 opens the same file)."""
    if isinstance(path_or_bytes, (bytes, bytearray)):
        data = bytes(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as fh:
            data = fh.read()
    g = Graph([], {}, [], [])
    graph_buf = None
    for fno, _, val in _fields(data):
        if fno == 1:
            g.ir_version = val
        elif fno == 2:
            g.producer = val.decode()
        elif fno == 7:
            graph_buf = val
        elif fno == 8:                       # opset_import
            for f2, _, v2 in _fields(val):
                if f2 == 2:
                    g.opset = max(g.opset, v2)
    if graph_buf is None:
        raise ValueError("no graph in model")
    raw_inputs = []
    for fno, _, val in _fields(graph_buf):
        if fno == 1:
            g.nodes.append(_node(val))
        elif fno == 5:
            name, arr = _tensor(val)
            g.inits[name] = arr
        elif fno == 11:
            raw_inputs.append(_value_info(val))
        elif fno == 12:
            g.outputs.append(_value_info(val))
    # graph inputs that are also initializers are not runtime inputs
    g.inputs = [(n, s) for n, s in raw_inputs if n not in g.inits]
    return g


# ------------------------------------------------------------------ evaluation


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def _gru(node: Node, env: dict, dt):
    """ONNX GRU, layout=0, forward direction, one or more time steps."""
    X = env[node.inputs[0]].astype(dt)              # [T, B, I]
    W = env[node.inputs[1]].astype(dt)[0]           # [3H, I]  (z, r, h)
    R = env[node.inputs[2]].astype(dt)[0]           # [3H, H]
    H = R.shape[1]
    B = X.shape[1]
    if len(node.inputs) > 3 and node.inputs[3]:
        bias = env[node.inputs[3]].astype(dt)[0]    # [6H] = Wb(z,r,h) | Rb(z,r,h)
    else:
        bias = np.zeros(6 * H, dt)
    h = np.zeros((B, H), dt)
    if len(node.inputs) > 5 and node.inputs[5]:
        h = env[node.inputs[5]].astype(dt)[0].copy()
    lbr = int(node.attrs.get("linear_before_reset", 0))
    Wz, Wr, Wh = W[:H], W[H:2 * H], W[2 * H:]
    Rz, Rr, Rh = R[:H], R[H:2 * H], R[2 * H:]
    Wbz, Wbr, Wbh = bias[:H], bias[H:2 * H], bias[2 * H:3 * H]
    Rbz, Rbr, Rbh = bias[3 * H:4 * H], bias[4 * H:5 * H], bias[5 * H:]
    Y = []
    for t in range(X.shape[0]):
        x = X[t]
        z = _sigmoid(x @ Wz.T + h @ Rz.T + Wbz + Rbz)
        r = _sigmoid(x @ Wr.T + h @ Rr.T + Wbr + Rbr)
        if lbr:
            hh = np.tanh(x @ Wh.T + Wbh + r * (h @ Rh.T + Rbh))
        else:
            hh = np.tanh(x @ Wh.T + Wbh + (r * h) @ Rh.T + Rbh)
        h = (1.0 - z) * hh + z * h
        Y.append(h)
    Yarr = np.stack(Y)[:, None]                      # [T, 1, B, H]
    outs = node.outputs
    res = {}
    if len(outs) > 0 and outs[0]:
        res[outs[0]] = Yarr
    if len(outs) > 1 and outs[1]:
        res[outs[1]] = h[None]                       # [1, B, H]
    return res


def _lstm(node: Node, env: dict, dt):
    """ONNX LSTM, layout=0, forward direction, no peepholes, one or more time steps."""
    if int(node.attrs.get("input_forget", 0)) != 0:
        raise NotImplementedError("oracle: LSTM input_forget=1")
    if len(node.inputs) > 7 and node.inputs[7]:
        raise NotImplementedError("oracle: LSTM peepholes")
    X = env[node.inputs[0]].astype(dt)              # [T, B, I]
    W = env[node.inputs[1]].astype(dt)[0]           # [4H, I]  (i, o, f, c)
    R = env[node.inputs[2]].astype(dt)[0]           # [4H, H]
    H = R.shape[1]
    B = X.shape[1]
    if len(node.inputs) > 3 and node.inputs[3]:
        bias = env[node.inputs[3]].astype(dt)[0]    # [8H] = Wb(i,o,f,c) | Rb(i,o,f,c)
    else:
        bias = np.zeros(8 * H, dt)
    h = np.zeros((B, H), dt)
    c = np.zeros((B, H), dt)
    if len(node.inputs) > 5 and node.inputs[5]:
        h = env[node.inputs[5]].astype(dt)[0].copy()
    if len(node.inputs) > 6 and node.inputs[6]:
        c = env[node.inputs[6]].astype(dt)[0].copy()
    b = bias[:4 * H] + bias[4 * H:]
    Y = []
    for t in range(X.shape[0]):
        gates = X[t] @ W.T + h @ R.T + b             # [B, 4H]
        i = _sigmoid(gates[:, :H])
        o = _sigmoid(gates[:, H:2 * H])
        f = _sigmoid(gates[:, 2 * H:3 * H])
        cc = np.tanh(gates[:, 3 * H:])
        c = f * c + i * cc
        h = o * np.tanh(c)
        Y.append(h)
    outs = node.outputs
    res = {}
    if len(outs) > 0 and outs[0]:
        res[outs[0]] = np.stack(Y)[:, None]          # [T, 1, B, H]
    if len(outs) > 1 and outs[1]:
        res[outs[1]] = h[None]                       # [1, B, H]
    if len(outs) > 2 and outs[2]:
        res[outs[2]] = c[None]
    return res


def _slice(node: Node, env: dict, x):
    """ONNX Slice: opset >= 10 takes starts / ends / axes / steps as inputs, opset 1-9
    as attributes; negative starts / ends count from the end and out-of-range ones clamp
    (numpy slicing does both). The loader's Slice -> ... -> Concat front-end
    (onnx_model.cpp) is checked against this."""
    ins = node.inputs
    if len(ins) > 1:
        starts, ends = (env[ins[i]].astype(np.int64).ravel() for i in (1, 2))
        axes = env[ins[3]].astype(np.int64).ravel() if len(ins) > 3 and ins[3] else np.arange(len(starts))
        steps = env[ins[4]].astype(np.int64).ravel() if len(ins) > 4 and ins[4] else np.ones(len(starts), np.int64)
    else:
        starts, ends = np.asarray(node.attrs["starts"]), np.asarray(node.attrs["ends"])
        axes = np.asarray(node.attrs.get("axes", list(range(len(starts)))))
        steps = np.ones(len(starts), np.int64)
    sl = [slice(None)] * x.ndim
    for s0, e0, ax, st in zip(starts, ends, axes, steps):
        sl[int(ax) % x.ndim] = slice(int(s0), int(e0), int(st))
    return x[tuple(sl)]


def run(g: Graph, feeds: dict, dtype=np.float64) -> dict:
    """Evaluate the graph in node order with numpy in `dtype` arithmetic."""
    dt = np.dtype(dtype)
    env = {k: (v.astype(dt) if v.dtype != np.int64 else v) for k, v in g.inits.items()}
    env.update({k: np.asarray(v, dtype=dt) for k, v in feeds.items()})
    for nd in g.nodes:
        op, a = nd.op_type, nd.attrs
        ins = [env[i] if i else None for i in nd.inputs]
        if op == "Gemm":
            A, B = ins[0], ins[1]
            if a.get("transA", 0):
                A = A.T
            if a.get("transB", 0):
                B = B.T
            y = dt.type(a.get("alpha", 1.0)) * (A @ B)
            if len(ins) > 2 and ins[2] is not None:
                y = y + dt.type(a.get("beta", 1.0)) * ins[2]
            out = {nd.outputs[0]: y}
        elif op == "MatMul":
            out = {nd.outputs[0]: ins[0] @ ins[1]}
        elif op == "Add":
            out = {nd.outputs[0]: ins[0] + ins[1]}
        elif op == "Sub":
            out = {nd.outputs[0]: ins[0] - ins[1]}
        elif op == "Mul":
            out = {nd.outputs[0]: ins[0] * ins[1]}
        elif op == "Div":
            out = {nd.outputs[0]: ins[0] / ins[1]}
        elif op == "Elu":
            al = dt.type(a.get("alpha", 1.0))
            x = ins[0]
            out = {nd.outputs[0]: np.where(x > 0, x, al * np.expm1(np.minimum(x, 0)))}
        elif op == "Relu":
            out = {nd.outputs[0]: np.maximum(ins[0], 0)}
        elif op == "LeakyRelu":
            al = dt.type(a.get("alpha", 0.01))
            out = {nd.outputs[0]: np.where(ins[0] >= 0, ins[0], al * ins[0])}
        elif op == "Tanh":
            out = {nd.outputs[0]: np.tanh(ins[0])}
        elif op == "Sigmoid":
            out = {nd.outputs[0]: _sigmoid(ins[0])}
        elif op == "Clip":
            lo = ins[1] if len(ins) > 1 and ins[1] is not None else a.get("min", -np.inf)
            hi = ins[2] if len(ins) > 2 and ins[2] is not None else a.get("max", np.inf)
            x = ins[0]
            out = {nd.outputs[0]: np.where(x < lo, lo, np.where(x > hi, hi, x)).astype(dt)}
        elif op == "Selu":
            al, ga = dt.type(a.get("alpha", 1.67326319217681884765625)), dt.type(a.get("gamma", 1.05070102214813232421875))
            x = ins[0]
            out = {nd.outputs[0]: ga * np.where(x > 0, x, al * np.expm1(np.minimum(x, 0)))}
        elif op == "Softplus":
            x = ins[0]
            out = {nd.outputs[0]: np.maximum(x, 0) + np.log1p(np.exp(-np.abs(x)))}
        elif op in ("HardSigmoid", "HardSwish"):
            if op == "HardSigmoid":
                al, be = dt.type(a.get("alpha", 0.2)), dt.type(a.get("beta", 0.5))
            else:
                al, be = dt.type(1.0 / 6.0), dt.type(0.5)
            x = ins[0]
            hs = np.clip(al * x + be, 0, 1)
            out = {nd.outputs[0]: hs if op == "HardSigmoid" else x * hs}
        elif op == "Softsign":
            out = {nd.outputs[0]: ins[0] / (1 + np.abs(ins[0]))}
        elif op == "Constant":
            v = a.get("value")
            if v is None:
                v = a.get("value_float", a.get("value_floats"))
            out = {nd.outputs[0]: np.asarray(v, dtype=dt)}
        elif op == "Slice":
            out = {nd.outputs[0]: _slice(nd, env, ins[0])}
        elif op == "Concat":
            out = {nd.outputs[0]: np.concatenate(ins, axis=int(a["axis"]))}
        elif op == "GRU":
            out = _gru(nd, env, dt)
        elif op == "LSTM":
            out = _lstm(nd, env, dt)
        elif op in ("Squeeze", "Unsqueeze", "Identity", "Flatten", "Reshape"):
            x = ins[0]
            if op == "Squeeze":
                axes = a.get("axes") or (list(env[nd.inputs[1]].astype(int)) if len(nd.inputs) > 1 else None)
                x = np.squeeze(x, axis=tuple(axes)) if axes else np.squeeze(x)
            elif op == "Unsqueeze":
                axes = a.get("axes") or list(env[nd.inputs[1]].astype(int))
                for ax in sorted(axes):
                    x = np.expand_dims(x, ax)
            elif op == "Flatten":
                x = x.reshape(x.shape[0], -1)
            elif op == "Reshape":
                x = x.reshape([int(s) for s in env[nd.inputs[1]]])
            out = {nd.outputs[0]: x}
        else:
            raise NotImplementedError(f"oracle: op {op}")
        env.update(out)
    return {name: env[name] for name, _ in g.outputs}


def act(g: Graph, obs: np.ndarray, dtype=np.float64) -> np.ndarray:
    """Single-input/single-output policy call, like ONNXActor::act()
    (onnx_actor.cpp:38-48): obs [B, in] -> action [B, out]. The batch dim of
    the shipped graph is static 1, so evaluation runs the graph row-agnostic
    (Gemm broadcasts over rows; ONNX static shapes are not enforced here)."""
    (in_name, _), = g.inputs[:1]
    out_name = g.outputs[0][0]
    return run(g, {in_name: obs}, dtype)[out_name]
