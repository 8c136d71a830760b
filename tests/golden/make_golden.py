"""Generate the committed golden fixtures (run from the repo root:
`python tests/golden/make_golden.py`).

Expected outputs come from the fp64 oracle (oracle/onnx_ref.py, numpy) on the
reference's own weights (tests/golden/model.onnx = onnx_inference/data/model.onnx)
and on the deterministic synthetic policies (go2_onnx_controller_amd/synth.py).
They are the oracle's outputs, not onnxruntime's (absent: parity unpinned,
SURVEY §8c); the shipped-model zeros/twos vectors agree with the survey's
independent numpy computation to <1e-8.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import realistic_obs  # noqa: E402
from go2_onnx_controller_amd import synth  # noqa: E402
from oracle import onnx_ref  # noqa: E402


def main():
    g = onnx_ref.load(os.path.join(HERE, "model.onnx"))
    out = {}
    out["zeros_x"] = np.zeros((1, 98), np.float32)                       # src/cpp/main.cpp:32
    out["twos_x"] = np.full((1, 98), 2.0, np.float32)                    # src/python/main.py:20
    out["normal_x"] = np.random.default_rng(1).standard_normal((64, 98)).astype(np.float32)
    out["realistic_x"] = realistic_obs(64, seed=2025)
    for k in ("zeros", "twos", "normal", "realistic"):
        out[f"{k}_y"] = onnx_ref.act(g, out[f"{k}_x"].astype(np.float64))
    np.savez(os.path.join(HERE, "golden_shipped.npz"), **out)

    gm = onnx_ref.load(synth.ensure_model("go2_mlp_512"))
    x = np.random.default_rng(1).standard_normal((64, 48)).astype(np.float32)
    np.savez(os.path.join(HERE, "golden_mlp512.npz"), x=x, y=onnx_ref.act(gm, x.astype(np.float64)))

    for name, T, B in (("go2_gru_256", 6, 16), ("gru_small", 6, 16)):
        gg = onnx_ref.load(synth.ensure_model(name))
        I = gg.inputs[0][1][1]
        H = gg.inputs[1][1][2]
        xs = np.random.default_rng(5).standard_normal((T, B, I)).astype(np.float32)
        h = np.zeros((1, B, H))
        ys = []
        for t in range(T):
            r = onnx_ref.run(gg, {"observation": xs[t].astype(np.float64), "h_in": h})
            ys.append(r["action"])
            h = r["h_out"]
        np.savez(os.path.join(HERE, f"golden_{name}.npz"), x=xs, y=np.stack(ys), h=h[0])

    hashes = {n: synth.sha256(n) for n in synth.MODELS}
    with open(os.path.join(HERE, "synth_hashes.json"), "w") as fh:
        json.dump(hashes, fh, indent=1, sort_keys=True)
    print("golden fixtures written")


if __name__ == "__main__":
    main()
