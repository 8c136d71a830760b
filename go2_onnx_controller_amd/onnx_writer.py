"""Minimal ONNX (protobuf) writer for the build-defined synthetic policies.

`onnx` and `torch.onnx.export` are unavailable in this image, so
the synthetic 48->512^3->12 MLP and GRU-256 policies that BASELINE.json's
configs name are serialised here directly in the ModelProto wire format
(field numbers as documented in go2_onnx_controller_amd/csrc/onnx_model.cpp).
The output is deterministic byte for byte.
"""
from __future__ import annotations

import struct

import numpy as np


def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(fno: int, wt: int) -> bytes:
    return _varint((fno << 3) | wt)


def f_varint(fno: int, v: int) -> bytes:
    return _key(fno, 0) + _varint(v)


def f_bytes(fno: int, b: bytes) -> bytes:
    return _key(fno, 2) + _varint(len(b)) + b


def f_str(fno: int, s: str) -> bytes:
    return f_bytes(fno, s.encode())


def f_float(fno: int, x: float) -> bytes:
    return _key(fno, 5) + struct.pack("<f", x)


def attr_float(name: str, x: float) -> bytes:
    return f_str(1, name) + f_float(2, x) + f_varint(20, 1)


def attr_int(name: str, i: int) -> bytes:
    return f_str(1, name) + f_varint(3, i) + f_varint(20, 2)


def attr_ints(name: str, ints) -> bytes:
    return f_str(1, name) + b"".join(f_varint(8, int(i)) for i in ints) + f_varint(20, 7)


def attr_tensor(name: str, arr: np.ndarray) -> bytes:
    """A TENSOR attribute (e.g. a Constant node's value)."""
    return f_str(1, name) + f_bytes(5, tensor("", arr)) + f_varint(20, 4)


def node(op: str, inputs, outputs, name: str = "", attrs=()) -> bytes:
    body = b"".join(f_str(1, i) for i in inputs)
    body += b"".join(f_str(2, o) for o in outputs)
    if name:
        body += f_str(3, name)
    body += f_str(4, op)
    body += b"".join(f_bytes(5, a) for a in attrs)
    return body


def tensor(name: str, arr: np.ndarray) -> bytes:
    arr = np.ascontiguousarray(arr)
    if arr.dtype == np.float32:
        dt = 1
    elif arr.dtype == np.int64:
        dt = 7
    else:
        raise TypeError(arr.dtype)
    body = b"".join(f_varint(1, d) for d in arr.shape)
    body += f_varint(2, dt) + f_str(8, name) + f_bytes(9, arr.astype(arr.dtype.newbyteorder("<")).tobytes())
    return body


def value_info(name: str, shape, elem_type: int = 1) -> bytes:
    dims = b""
    for d in shape:
        if isinstance(d, str):
            dims += f_bytes(1, f_str(2, d))
        else:
            dims += f_bytes(1, f_varint(1, int(d)))
    tensor_type = f_varint(1, elem_type) + f_bytes(2, dims)
    return f_str(1, name) + f_bytes(2, f_bytes(1, tensor_type))


def model(nodes, initializers, inputs, outputs, graph_name="main_graph", opset=17, producer="go2pi-synth",
          ir_version=8) -> bytes:
    g = b"".join(f_bytes(1, n) for n in nodes)
    g += f_str(2, graph_name)
    g += b"".join(f_bytes(5, tensor(k, v)) for k, v in initializers)
    g += b"".join(f_bytes(11, value_info(n, s)) for n, s in inputs)
    g += b"".join(f_bytes(12, value_info(n, s)) for n, s in outputs)
    m = f_varint(1, ir_version) + f_str(2, producer) + f_str(3, "0.1")
    m += f_bytes(7, g)
    m += f_bytes(8, f_str(1, "") + f_varint(2, opset))
    return m
