import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
SHIPPED = os.path.join(GOLDEN, "model.onnx")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (runs on the MI355X box)")
    # the product libraries are built in-tree (git-ignored); build them once if a
    # fresh checkout runs the tests before __graft_entry__.build()
    lib = os.path.join(ROOT, "go2_onnx_controller_amd", "lib", "libonnx_actor.so")
    if not os.path.exists(lib):
        import subprocess
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "go2_onnx_controller_amd", "csrc")],
                       check=True)


@pytest.fixture(scope="session")
def shipped_path():
    return SHIPPED


@pytest.fixture(scope="session")
def synth_path():
    from go2_onnx_controller_amd import synth
    return synth.ensure_model


def realistic_obs(n, seed=2025):
    """'Realistic' observations in the controller's 98-float layout
    (controller.cpp:200-212, controller.hpp:45-68): per history
    step gravity_b (~(0,0,-1)), base_ang_vel, vel_cmd, q - q0, dq, previous
    action, foot contacts — two steps [t-1, t] concatenated per block."""
    rng = np.random.default_rng(seed)
    blocks = []
    g = np.tile(np.array([0, 0, -1.0]), (n, 2)) + rng.normal(0, 0.05, (n, 6))
    blocks.append(g)
    blocks.append(rng.normal(0, 0.5, (n, 6)))
    blocks.append(rng.uniform(-1, 1, (n, 6)))
    blocks.append(rng.normal(0, 0.2, (n, 24)))
    blocks.append(rng.normal(0, 2.0, (n, 24)))
    blocks.append(rng.normal(0, 1.0, (n, 24)))
    blocks.append(rng.integers(0, 2, (n, 8)).astype(np.float64))
    return np.concatenate(blocks, axis=1).astype(np.float32)


def rel_err(y, ref):
    y = np.asarray(y, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(y - ref) / np.maximum(1.0, np.abs(ref)))) if ref.size else 0.0


def abs_err(y, ref):
    return float(np.max(np.abs(np.asarray(y, np.float64) - np.asarray(ref, np.float64)))) if np.size(ref) else 0.0
