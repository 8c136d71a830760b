"""Replay the recorded /observation_action log (rosbag2 fixture) through the
GPU engine: every logged action that the stop button did not zero is
reproduced within the policy tolerance (1e-5, max(1,|ref|)-relative), through
both the batched kernel (all 80 ticks in one launch) and the single-launch
small-batch kernel (8 rows per call)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, SHIPPED

pytestmark = pytest.mark.gpu

BAG = os.path.join(GOLDEN, "replay_bag")


@pytest.mark.parametrize("max_batch", [4096, 8])
def test_replay_fixture_bag(max_batch):
    from go2_onnx_controller_amd import Engine, replay
    log = replay.read_log(BAG)
    with Engine(SHIPPED, max_batch=max_batch) as e:
        r = replay.replay(e, log)
    assert r.n == 80
    assert r.stopped.tolist() == list(range(40, 46))
    assert r.max_rel_err <= 1e-5
    assert r.history_breaks.size == 0


def test_replay_cli():
    out = subprocess.run([sys.executable, "-m", "go2_onnx_controller_amd.replay", BAG], cwd=ROOT,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    import json
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["ticks"] == 80 and d["max_rel_err"] <= 1e-5 and d["history_breaks"] == []
