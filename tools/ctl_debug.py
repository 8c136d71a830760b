"""Diagnostics: one batch-1 controller tick through each resident form against the
launch-per-tick path (prints which outputs differ)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from go2_onnx_controller_amd import Engine  # noqa: E402
from oracle import controller_ref as cr  # noqa: E402

SHIPPED = os.path.join(ROOT, "tests", "golden", "model.onnx")
rng = np.random.default_rng(21)
st, joy = cr.synthetic_states(rng, 1), cr.synthetic_joy(rng, 1)
obs0 = rng.standard_normal((1, 98)).astype(np.float32)
act0 = rng.standard_normal((1, 12)).astype(np.float32)
want_obs, _ = cr.assemble_obs(obs0, act0, st, joy, 2)
outs = {}
for name, res, env in (("launch", 0, {}), ("a1", 500, {}), ("r1w", 500, {"GO2PI_RES_R1W": "1"})):
    os.environ.pop("GO2PI_RES_R1W", None)
    os.environ.update(env)
    with Engine(SHIPPED, max_batch=8, resident_ms=res) as e:
        for rep in range(2):
            o, a = obs0.copy(), act0.copy()
            q = e.controller_step(st, o, a, joy=joy)
            print(name, rep, "obs==want", np.array_equal(o, want_obs), "obs==input", np.array_equal(o, obs0),
                  "act", a[0, :4], "q_des", q[0][0, :2], "status", q[3])
        outs[name] = (o, a)
print("a1 vs launch act max diff", float(np.abs(outs["a1"][1] - outs["launch"][1]).max()))
