"""ORACLE — test infrastructure only (tests/, smoke(), bench.py cpu_baseline).

ctypes front-end for oracle/mlp_ref.c plus a layer-list extraction from the
oracle's own decoded graph (oracle/onnx_ref.py). Parity status: parity
unpinned — see oracle/onnx_ref.py.

`mlp_layers(graph)` recognises the reference graph pattern
(`onnx_inference/data/model.onnx`: Gemm(transB=1) -> Elu -> ... -> Gemm) and
the MatMul+Add / Relu / Tanh / Sigmoid / LeakyRelu / Clip / Selu / Softplus /
HardSigmoid / HardSwish / Softsign / constant-Mul variants, independently of
the product's C++ pattern matcher.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from . import onnx_ref

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libmlpref.so")
_lib = None

ACT = {"none": 0, "Elu": 1, "Relu": 2, "Tanh": 3, "Sigmoid": 4, "LeakyRelu": 5}


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.mlpref_create.restype = P
        L.mlpref_create.argtypes = [ctypes.c_int, P, P, P, P, P, P]
        L.mlpref_run_f32.argtypes = [P, P, P, ctypes.c_long, ctypes.c_int]
        L.mlpref_run_f64.argtypes = [P, P, P, ctypes.c_long, ctypes.c_int]
        L.mlpref_destroy.argtypes = [P]
        L.mlpref_time_b1.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, P]
        L.gruref_step_f64.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P, ctypes.c_int, P, P,
                                      ctypes.c_long, ctypes.c_int]
        _lib = L
    return _lib


ACT_DEFAULTS = {  # ONNX attribute defaults (alpha, beta) per activation
    "Elu": (1.0, 0.0), "LeakyRelu": (0.01, 0.0), "Selu": (1.67326319217681884765625, 1.05070102214813232421875),
    "HardSigmoid": (0.2, 0.5), "HardSwish": (1.0 / 6.0, 0.5), "Relu": (0.0, 0.0), "Tanh": (0.0, 0.0),
    "Sigmoid": (0.0, 0.0), "Softplus": (0.0, 0.0), "Softsign": (0.0, 0.0)}


def mlp_layers(g: onnx_ref.Graph, strict: bool = False):
    """Return [(W[N,K] f32, b[N] f32, act_name, alpha, beta)] for a Linear/act chain.

    Lowering rules (the ONNX semantics, restated independently of the product's
    C++ matcher): a Clip right after a Gemm is that layer's activation (alpha =
    min, beta = max); a constant Mul / Div right after a Gemm scales the layer's
    rows and bias; one after an activation scales the next layer's input columns
    (fp32 products in graph order). Prologue / output elementwise ops are not
    layers (onnx_ref.act evaluates them); a Slice -> ... -> Concat observation
    front-end is prologue too (the walk follows its first block to the Concat).
    strict: raise NotImplementedError when the graph has output-side work the
    returned layers do not carry (a Mul / Div or a Clip after the final activation),
    so that MlpRef.from_onnx never returns a silently different policy."""
    layers = []
    cur = g.inputs[0][0]
    producers = {}
    consts = dict(g.inits)
    for nd in g.nodes:
        if nd.op_type == "Constant":
            v = nd.attrs.get("value")
            consts[nd.outputs[0]] = np.asarray(v if v is not None else nd.attrs.get("value_float",
                                                                                   nd.attrs.get("value_floats")),
                                               np.float32)
        for i in nd.inputs:
            producers.setdefault(i, []).append(nd)
    consumed = set()
    last_act = True
    col_scale = None

    def const_of(name):
        return np.asarray(consts[name], np.float32)

    while True:
        nds = [n for n in producers.get(cur, []) if id(n) not in consumed]
        if not nds:
            break
        nd = nds[0]
        consumed.add(id(nd))
        op = nd.op_type
        if op in ("Gemm", "MatMul"):
            if op == "Gemm":
                W = g.inits[nd.inputs[1]].astype(np.float32)
                if not nd.attrs.get("transB", 0):
                    W = W.T
                W = W * np.float32(nd.attrs.get("alpha", 1.0))
                b = g.inits[nd.inputs[2]].astype(np.float32) * np.float32(nd.attrs.get("beta", 1.0)) \
                    if len(nd.inputs) > 2 else np.zeros(W.shape[0], np.float32)
                b = np.broadcast_to(b, (W.shape[0],)).astype(np.float32)
            else:
                W = g.inits[nd.inputs[1]].astype(np.float32).T
                b = np.zeros(W.shape[0], np.float32)
            if col_scale is not None:
                W = W * np.broadcast_to(col_scale, (W.shape[1],))[None, :]
                col_scale = None
            layers.append([np.ascontiguousarray(W, np.float32), np.ascontiguousarray(b), "none", 0.0, 0.0])
            last_act = False
        elif op == "Add":
            other = nd.inputs[1] if nd.inputs[0] == cur else nd.inputs[0]
            layers[-1][1] = layers[-1][1] + const_of(other)
        elif op in ("Mul", "Div") and layers:
            other = nd.inputs[1] if nd.inputs[0] == cur else nd.inputs[0]
            f = const_of(other).reshape(-1)
            if op == "Div":
                f = np.float32(1.0) / f
            if not last_act:
                f = np.broadcast_to(f, (layers[-1][0].shape[0],))
                layers[-1][0] = layers[-1][0] * f[:, None]
                layers[-1][1] = layers[-1][1] * f
            else:
                col_scale = f if col_scale is None else col_scale * f
        elif op == "Clip" and layers and not last_act:
            lo = float(const_of(nd.inputs[1]).reshape(-1)[0]) if len(nd.inputs) > 1 and nd.inputs[1] else nd.attrs.get("min", -np.inf)
            hi = float(const_of(nd.inputs[2]).reshape(-1)[0]) if len(nd.inputs) > 2 and nd.inputs[2] else nd.attrs.get("max", np.inf)
            layers[-1][2:5] = ["Clip", float(np.float32(lo)), float(np.float32(hi))]
            last_act = True
        elif op in ACT_DEFAULTS:
            da, db = ACT_DEFAULTS[op]
            if op == "Selu":
                al, be = nd.attrs.get("alpha", da), nd.attrs.get("gamma", db)
            elif op == "HardSwish":
                al, be = da, db
            else:
                al, be = nd.attrs.get("alpha", da), nd.attrs.get("beta", db)
            layers[-1][2:5] = [op, float(np.float32(al)), float(np.float32(be))]
            last_act = True
        elif op in ("Sub", "Div", "Mul", "Clip", "Identity", "Flatten") or (op in ("Slice", "Concat") and not layers):
            # prologue / epilogue elementwise ops: not dense layers (onnx_ref.act evaluates them)
            if strict and layers and op in ("Mul", "Div", "Clip"):
                raise NotImplementedError(f"{op} after the final activation: MlpRef would not apply it")
        else:
            raise NotImplementedError(op)
        cur = nd.outputs[0]
    if strict and col_scale is not None:
        raise NotImplementedError("a Mul / Div after the final activation: MlpRef would not apply it")
    return [tuple(l) for l in layers]


class MlpRef:
    """fp32 / fp64 CPU restatement of the MLP policy forward."""

    def __init__(self, layers):
        self.layers = layers
        L = lib()
        nl = len(layers)
        self._W = [np.ascontiguousarray(l[0], np.float32) for l in layers]
        self._b = [np.ascontiguousarray(l[1], np.float32) for l in layers]
        K = (ctypes.c_int * nl)(*[w.shape[1] for w in self._W])
        N = (ctypes.c_int * nl)(*[w.shape[0] for w in self._W])
        Wp = (ctypes.c_void_p * nl)(*[w.ctypes.data for w in self._W])
        bp = (ctypes.c_void_p * nl)(*[b.ctypes.data for b in self._b])
        act = (ctypes.c_int * nl)(*[ACT[l[2]] for l in layers])
        al = (ctypes.c_float * nl)(*[l[3] for l in layers])
        self.in_dim = self._W[0].shape[1]
        self.out_dim = self._W[-1].shape[0]
        self._h = L.mlpref_create(nl, K, N, Wp, bp, act, al)
        if not self._h:
            raise RuntimeError("mlpref_create failed")

    @classmethod
    def from_onnx(cls, path):
        return cls(mlp_layers(onnx_ref.load(path), strict=True))

    def f32(self, x, nthreads=0):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, self.in_dim)
        y = np.empty((x.shape[0], self.out_dim), np.float32)
        lib().mlpref_run_f32(self._h, x.ctypes.data, y.ctypes.data, x.shape[0], nthreads)
        return y

    def f64(self, x, nthreads=0):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, self.in_dim)
        y = np.empty((x.shape[0], self.out_dim), np.float64)
        lib().mlpref_run_f64(self._h, x.ctypes.data, y.ctypes.data, x.shape[0], nthreads)
        return y

    def time_b1(self, x, warm=1000, iters=10000):
        """Per-call microseconds of `iters` single-robot fp32 forwards of row x (after
        `warm` untimed ones), timed inside C on the calling thread (bench.py cpu_baseline)."""
        x = np.ascontiguousarray(x, np.float32).reshape(-1)[: self.in_dim]
        y = np.empty(self.out_dim, np.float32)
        out = np.empty(iters, np.float64)
        if lib().mlpref_time_b1(self._h, x.ctypes.data, y.ctypes.data, int(warm), int(iters), out.ctypes.data):
            raise RuntimeError("mlpref_time_b1 failed")
        return out

    def __del__(self):
        try:
            if self._h:
                lib().mlpref_destroy(self._h)
                self._h = None
        except Exception:
            pass


def gru_step_f64(W, R, Wb, Rb, x, h, lbr=1, nthreads=0):
    """One ONNX GRU step in fp64. W [3H,I], R [3H,H], Wb/Rb [3H], x [B,I] f32,
    h [B,H] f64 (updated copy returned)."""
    W = np.ascontiguousarray(W, np.float32)
    R = np.ascontiguousarray(R, np.float32)
    Wb = np.ascontiguousarray(Wb, np.float32)
    Rb = np.ascontiguousarray(Rb, np.float32)
    x = np.ascontiguousarray(x, np.float32)
    h = np.array(h, np.float64, copy=True, order="C")
    I, H = W.shape[1], R.shape[1]
    lib().gruref_step_f64(I, H, W.ctypes.data, R.ctypes.data, Wb.ctypes.data, Rb.ctypes.data, int(lbr),
                          x.ctypes.data, h.ctypes.data, x.shape[0], nthreads)
    return h
