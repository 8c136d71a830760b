"""ORACLE — test infrastructure only. NOT part of the product path.

CPU restatement (numpy) of the Go2 controller's per-tick work around
`ONNXActor::act()` — SURVEY.md §8f rows 1-2 — that go2pi fuses into the
policy launch (go2pi_controller_step*, kernels.hip ctl_*):

* observation assembly, `onnx_controller/src/controller.cpp:173-212`, with the
  members and helpers of `onnx_controller/include/onnx_controller/controller.hpp`:
  - `lowstate_cb_` (:93-110): quaternion (w,x,y,z), foot contacts
    `foot_force >= 22` with the FL/FR and RL/RR swap, gyroscope;
  - joystick velocity command (controller.cpp:173-179), kept when no axes;
  - `gravity_b = quaternion_.inverse() * gravity_w_` (controller.cpp:182-184);
  - `q_[i] -= q0_[i]` with a double `q0_` (controller.cpp:194-197, hpp:165);
  - `populate_buffer` (hpp:45-68): each history block shifts left by its
    width and appends the current value; the observation is the
    concatenation of the seven blocks (controller.cpp:200-212). A NaN among
    the appended values makes the reference `exit(1)` (hpp:57-64): reported
    here as status bit 0 instead.
* action post-processing, controller.cpp:217-223 (std::clamp to
  +-kActionLimit, `a *= buttons[0] == 0`) and 240-248 (q_des = q0 + 0.25 a,
  kp = buttons[0] == 0 ? kp_ : 5, kd = kd_), in double as send_command takes.

`quaternion_.inverse() * v` follows Eigen 3.4 (the ROS 2 Humble / Ubuntu 22.04
libeigen3-dev 3.4.0 the reference builds against; Eigen is a third-party
dependency absent here): `inverse()` = conjugate coefficients / squaredNorm
(zero quaternion if squaredNorm <= 0), squaredNorm = (x²+z²)+(y²+w²) (SSE
predux of the 4-float coefficient packet), `q * v` = `_transformVector`:
uv = 2 (q.vec × v); result = (v + w·uv) + q.vec × uv. Every operation is one
float32 rounding in that order, as on the reference's x86-64 build (no FMA).

Parity status: the reference has no tests or recorded data for this code
(SURVEY §4), and Eigen/ROS are absent, so this restatement is pinned only by
analytic identities (tests/test_cpu_controller.py: identity / axis rotations
against a float64 rotation matrix, the history layout of SURVEY §8a, sticky
command, stop button, clamp, NaN exit condition) — "parity unpinned" against
the reference binary itself.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32

# (name, width) of the observation blocks, in concatenation order (controller.cpp:210-212)
BLOCKS = (("gravity_b", 3), ("base_ang_vel", 3), ("vel_cmd", 3), ("q", 12), ("dq", 12), ("action", 12),
          ("foot_contact", 4))
STEP_DIM = 49  # kDimObs, controller.hpp:14
DOF = 12
STATE_DIM = 36
JOY_DIM = 5
# state row: quaternion 0:4, gyro 4:7, q 7:19, dq 19:31, foot_force 31:35
Q0 = np.array([0.1, -0.1, 0.1, -0.1, 0.8, 0.8, 1.0, 1.0, -1.5, -1.5, -1.5, -1.5], np.float64)  # hpp:165


def default_params() -> dict:
    return {"kp": 28.0, "kd": 0.5, "kp_stop": 5.0, "action_limit": 1000.0, "contact_threshold": 22.0,
            "gravity_w": (0.0, 0.0, -1.0), "action_scale": 0.25, "q0": Q0.copy()}


def gravity_b(quat: np.ndarray, gravity_w=(0.0, 0.0, -1.0)) -> np.ndarray:
    """quat [B,4] float32 (w,x,y,z) -> quaternion.inverse() * gravity_w, [B,3] float32."""
    q = np.asarray(quat, f32)
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        n2 = (x * x + z * z) + (y * y + w * w)
        ok = n2 > f32(0)
        safe = np.where(ok, n2, f32(1))
        zero = f32(0)
        qx = np.where(ok, -x / safe, zero)
        qy = np.where(ok, -y / safe, zero)
        qz = np.where(ok, -z / safe, zero)
        qw = np.where(ok, w / safe, zero)
        v0, v1, v2 = (f32(c) for c in gravity_w)
        u0 = qy * v2 - qz * v1
        u1 = qz * v0 - qx * v2
        u2 = qx * v1 - qy * v0
        u0, u1, u2 = u0 + u0, u1 + u1, u2 + u2
        c0 = qy * u2 - qz * u1
        c1 = qz * u0 - qx * u2
        c2 = qx * u1 - qy * u0
        r = np.stack([(v0 + qw * u0) + c0, (v1 + qw * u1) + c1, (v2 + qw * u2) + c2], axis=1)
    return r.astype(f32)


def vel_cmd(joy: np.ndarray | None, prev: np.ndarray) -> np.ndarray:
    """controller.cpp:173-179 per robot; joy row {has_axes, axes0, axes1, axes3, button0}."""
    if joy is None:
        return prev.copy()
    j = np.asarray(joy, f32)
    a0 = j[:, 1].astype(np.float64)
    sign = np.where(j[:, 1] > 0, 1.0, -1.0)
    cmd = np.stack([j[:, 2], ((a0 * a0) * sign * 0.8).astype(f32), j[:, 3] * j[:, 2]], axis=1).astype(f32)
    return np.where((j[:, 0] != 0)[:, None], cmd, prev).astype(f32)


def current_signals(state, joy, prev_obs, prev_action, hist: int, params=None) -> list[np.ndarray]:
    """The seven values appended this tick (BLOCKS order), each [B, width] float32."""
    p = params or default_params()
    st = np.asarray(state, f32)
    H = hist
    # the previous vel_cmd_ is the newest slot of the command history block
    c0 = H * 6 + (H - 1) * 3
    prev_cmd = np.asarray(prev_obs, f32)[:, c0:c0 + 3]
    q = (st[:, 7:19].astype(np.float64) - np.asarray(p["q0"], np.float64)).astype(f32)
    ff = st[:, 31:35][:, [1, 0, 3, 2]]
    contact = (ff >= f32(p["contact_threshold"])).astype(f32)
    return [gravity_b(st[:, 0:4], p["gravity_w"]), st[:, 4:7].copy(), vel_cmd(joy, prev_cmd), q,
            st[:, 19:31].copy(), np.asarray(prev_action, f32).copy(), contact]


def assemble_obs(prev_obs, prev_action, state, joy, hist: int, params=None):
    """(new observation [B, 49*hist] float32, status [B] uint32) for this tick."""
    prev_obs = np.asarray(prev_obs, f32)
    cur = current_signals(state, joy, prev_obs, prev_action, hist, params)
    new = np.empty_like(prev_obs)
    status = np.zeros(prev_obs.shape[0], np.uint32)
    cum = 0
    for bi, ((_, d), c) in enumerate(zip(BLOCKS, cur)):
        s = hist * cum
        new[:, s:s + (hist - 1) * d] = prev_obs[:, s + d:s + hist * d]  # std::shift_left by d
        new[:, s + (hist - 1) * d:s + hist * d] = c                        # std::copy of the head
        if bi < 6:  # populate_buffer's tail check (exit(1) on NaN), the single-signal calls
            status |= np.isnan(c).any(axis=1).astype(np.uint32)
        cum += d
    return new, status


def post_process(y, joy, params=None):
    """Policy output y [B,12] float32 -> (action f32, q_des f64, kp f64, kd f64)."""
    p = params or default_params()
    a = np.asarray(y, f32).copy()
    lim = f32(p["action_limit"])
    with np.errstate(invalid="ignore"):
        a = np.where(a < -lim, -lim, np.where(lim < a, lim, a)).astype(f32)  # std::clamp
    stop = np.zeros(a.shape[0], bool) if joy is None else (np.asarray(joy, f32)[:, 4] != 0)
    a = (a * np.where(stop, f32(0), f32(1))[:, None]).astype(f32)
    q_des = np.asarray(p["q0"], np.float64)[None, :] + a.astype(np.float64) * float(p["action_scale"])
    kp = np.where(stop, float(np.float32(p["kp_stop"])), float(np.float32(p["kp"])))[:, None] * np.ones((1, DOF))
    kd = np.full(a.shape, float(np.float32(p["kd"])))
    return a, q_des, kp, kd


def tick(policy, state, joy, obs, action, hist: int, params=None):
    """One full controller tick. policy: obs [B, in] float32 -> y [B, 12].
    Returns (obs', action', q_des, kp, kd, status)."""
    new_obs, status = assemble_obs(obs, action, state, joy, hist, params)
    y = np.asarray(policy(new_obs), f32)
    a, q_des, kp, kd = post_process(y, joy, params)
    return new_obs, a, q_des, kp, kd, status


def synthetic_states(rng: np.random.Generator, B: int, upright=True) -> np.ndarray:
    """Plausible raw robot state rows [B, 36] float32 (test inputs)."""
    st = np.zeros((B, STATE_DIM), f32)
    if upright:
        q = np.concatenate([np.ones((B, 1)), rng.normal(0, 0.08, (B, 3))], axis=1)
    else:
        q = rng.normal(0, 1, (B, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    st[:, 0:4] = q
    st[:, 4:7] = rng.normal(0, 0.5, (B, 3))
    st[:, 7:19] = Q0 + rng.normal(0, 0.2, (B, 12))
    st[:, 19:31] = rng.normal(0, 2.0, (B, 12))
    st[:, 31:35] = rng.integers(0, 60, (B, 4))  # int16 foot_force values
    return st


def synthetic_joy(rng: np.random.Generator, B: int, p_axes=0.8, p_stop=0.1) -> np.ndarray:
    j = np.zeros((B, JOY_DIM), f32)
    j[:, 0] = rng.random(B) < p_axes
    j[:, 1:4] = rng.uniform(-1, 1, (B, 3))
    j[:, 4] = rng.random(B) < p_stop
    return j
