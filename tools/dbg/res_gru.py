"""Diagnostics: one resident GRU request (GO2PI_LIB -> a GO2PI_DIAG_RESDBG build prints the stages)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from go2_onnx_controller_amd import Engine, synth
p = synth.ensure_model(sys.argv[1] if len(sys.argv) > 1 else "gru_128")
with Engine(p, max_batch=8, resident_ms=300) as e:
    x = np.ones((1, e.in_dim), np.float32)
    try:
        print("y", e.run(x), flush=True)
        print("y2", e.run(x), flush=True)
    except Exception as ex:
        print("error", ex, flush=True)
