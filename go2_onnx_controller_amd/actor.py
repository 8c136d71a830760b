"""Host-side mirrors of the reference's operator interface for this path.

* `ONNXActor` mirrors the C++ class of onnx_inference/include/onnx_actor.hpp:14-76
  (ctor(model_path, observation, action, log_level), act(), print_model_info(),
  check_dims()): the caller's float32 arrays are aliased, not copied — act()
  reads `observation` at call time and overwrites `action` in place
  (onnx_actor.cpp:31-35, :47).
* `InferenceSession` mirrors the slice of onnxruntime's Python API the
  reference's Python driver uses (onnx_inference/src/python/main.py:8-27:
  InferenceSession(path), get_inputs()/get_outputs() -> .name/.shape,
  run([output_name], {input_name: array})).

Both run on the GPU through libgo2pi.so; there is no CPU fallback.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from .engine import Engine

ORT_LOGGING_LEVEL_VERBOSE = 0
ORT_LOGGING_LEVEL_INFO = 1
ORT_LOGGING_LEVEL_WARNING = 2
ORT_LOGGING_LEVEL_ERROR = 3
ORT_LOGGING_LEVEL_FATAL = 4


class ONNXActor:
    def __init__(self, model_path, observation: np.ndarray, action: np.ndarray,
                 log_level: int = ORT_LOGGING_LEVEL_WARNING, **engine_kwargs):
        for name, a in (("observation", observation), ("action", action)):
            if not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous):
                raise TypeError(f"{name} must be a C-contiguous float32 numpy array (it is aliased)")
        self._obs = observation
        self._act = action
        engine_kwargs.setdefault("max_batch", 64)
        # as the C++ shim: a resident kernel serves act() (no launch per tick), leaving
        # after 100 ms without one; GO2PI_RESIDENT_MS=0 -> one launch per call
        engine_kwargs.setdefault("resident_ms", int(os.environ.get("GO2PI_RESIDENT_MS", "100")))
        self._engine = Engine(model_path, log_level=log_level, **engine_kwargs)
        self.model_path = model_path
        self.input_name, self.input_shape = self._engine.inputs[0]
        self.output_name, self.output_shape = self._engine.outputs[0]
        if len(self.input_shape) < 2 or len(self.output_shape) < 2:
            raise RuntimeError("ONNXActor: model input/output must be 2-D [batch, features]")
        if observation.size < self._engine.in_dim or action.size < self._engine.out_dim:
            raise RuntimeError("ONNXActor: observation/action buffer smaller than the model's feature dims")

    def act(self) -> None:
        self._engine.run_ptr(self._obs.ctypes.data, self._act.ctypes.data, 1)

    def check_dims(self) -> bool:
        return self._obs.size == self.input_shape[1] and self._act.size == self.output_shape[1]

    def print_model_info(self) -> None:
        print(f"Input dimension: {self.input_shape[1]}")
        print(f"Output dimension: {self.output_shape[1]}")
        print(f"Input name: {self.input_name}")
        print(f"Output name: {self.output_name}")

    @property
    def engine(self) -> Engine:
        return self._engine


@dataclass
class NodeArg:
    name: str
    shape: list
    type: str = "tensor(float)"


class InferenceSession:
    """GPU-backed stand-in for onnxruntime.InferenceSession on policy graphs."""

    def __init__(self, path_or_bytes, providers=None, **engine_kwargs):
        self._engine = Engine(path_or_bytes, **engine_kwargs)

    def get_inputs(self):
        return [NodeArg(n, [("batch" if d < 0 else d) for d in s]) for n, s in self._engine.inputs]

    def get_outputs(self):
        return [NodeArg(n, [("batch" if d < 0 else d) for d in s]) for n, s in self._engine.outputs]

    def run(self, output_names, input_feed, run_options=None):
        e = self._engine
        in_name = e.inputs[0][0]
        if in_name not in input_feed:
            raise ValueError(f"missing input '{in_name}'")
        x = np.asarray(input_feed[in_name], dtype=np.float32).reshape(-1, e.in_dim)
        B = x.shape[0]
        # recurrent state: GRU h [H]; LSTM h [H] | c [H] (the engine keeps both per robot).
        # The loader lists the state inputs / outputs as (h, c), whatever their order in the
        # graph (traced to the cell's initial_h / initial_c and Y_h / Y_c by name); the
        # split follows from the cell, not from how many of them the graph exports.
        nparts = 2 if e.cost["cell"] == "LSTM" else 1
        parts = [n for n, _ in e.inputs[1:1 + nparts]]  # h_in (, c_in), possibly none
        width = e.hidden_dim // nparts if e.hidden_dim else 0
        if e.hidden_dim:
            # explicit recurrent I/O when the caller feeds/asks for it; otherwise engine-resident
            fed = [n in input_feed for n in parts]
            if any(fed):
                cur = e.get_hidden(B).reshape(B, nparts, width) if not all(fed) or len(parts) < nparts else \
                    np.empty((B, nparts, width), np.float32)
                for k, n in enumerate(parts):
                    if n in input_feed:
                        cur[:, k] = np.asarray(input_feed[n], np.float32).reshape(B, width)
                e.set_hidden(cur.reshape(B, e.hidden_dim))
        y = e.run(x)
        results = {e.outputs[0][0]: y}
        if e.hidden_dim and len(e.outputs) > 1:
            st = e.get_hidden(B).reshape(B, nparts, width)
            for k, (n, _) in enumerate(e.outputs[1:1 + nparts]):
                results[n] = np.ascontiguousarray(st[:, k]).reshape(1, B, width)
        names = output_names or [n for n, _ in e.outputs]
        return [results[n] for n in names]

    @property
    def engine(self) -> Engine:
        return self._engine
