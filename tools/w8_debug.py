"""Diagnostics (r05): where the 8-wave lean kernel's actions differ from the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from go2_onnx_controller_amd import Engine, synth  # noqa: E402
from oracle import mlp_ref  # noqa: E402

path = synth.ensure_model("go2_mlp_512")
ref = mlp_ref.MlpRef.from_onnx(path)
with Engine(path, device=0, max_batch=4096) as e:
    print("kernel", e.batched_kernel)
    for B in (4096, 256, 64):
        x = np.random.default_rng(B).standard_normal((B, 48)).astype(np.float32)
        y = e.run(x)
        want = ref.f64(x)
        bad = ~(np.abs(y - want) <= 1e-5)
        rows = np.nonzero(bad.any(1))[0]
        cols = np.nonzero(bad.any(0))[0]
        print(f"B={B}: bad {bad.sum()} of {bad.size}; rows {len(rows)} (first {rows[:20].tolist()}, mod16 "
              f"{sorted(set((rows % 16).tolist()))}); cols {cols.tolist()}; nan {np.isnan(y).sum()}")
        if len(rows):
            r = rows[0]
            print("  row", r, "got", y[r, :4], "want", want[r, :4])
