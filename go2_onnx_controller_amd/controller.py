"""The Go2 controller tick for a fleet of robots, fused on the GPU.

Mirrors the per-tick state of the reference's `ONNXController`
(onnx_controller/include/onnx_controller/controller.hpp:147-148: the
`observation_` history and the `action_` fed back into it) and its `publish()`
tick (onnx_controller/src/controller.cpp:155-252) minus ROS: one call takes the
raw robot state rows (IMU quaternion + gyro, joint q / dq, foot forces — what
`lowstate_cb_` and `robot_interface_->get_q/get_dq` supply) and the joystick
rows, and returns what `send_command` receives (q_des, kp, kd) plus the
ObservationAction log row (onnx_interfaces/msg/ObservationAction.msg). The
observation assembly, the policy and the action post-processing run in ONE
launch (go2pi_controller_step_device).
"""
from __future__ import annotations

from dataclasses import dataclass

from .engine import CTL_DOF, CTL_JOY_DIM, CTL_STATE_DIM, Engine


@dataclass
class TickOutput:
    action: object   # [B, 12] float32, post-processed (also the next tick's history)
    q_des: object    # [B, 12] float64
    kp: object       # [B, 12] float64
    kd: object       # [B, 12] float64
    status: object   # [B] int32, bit 0: NaN entered the observation (the reference exit(1)s)


class Go2ControllerFleet:
    """B robots' controller state resident in HBM; `step()` is one 50 Hz tick."""

    def __init__(self, engine: Engine, batch: int, device="cuda:0"):
        import torch
        self.engine = engine
        self.history = engine.ctl_history()  # raises for a non-controller policy
        self.batch = int(batch)
        self.device = torch.device(device)
        B = self.batch
        f32, f64 = torch.float32, torch.float64
        self.observation = torch.zeros((B, engine.in_dim), dtype=f32, device=self.device)
        self.action = torch.zeros((B, CTL_DOF), dtype=f32, device=self.device)
        self.q_des = torch.empty((B, CTL_DOF), dtype=f64, device=self.device)
        self.kp = torch.empty_like(self.q_des)
        self.kd = torch.empty_like(self.q_des)
        self.status = torch.zeros((B,), dtype=torch.int32, device=self.device)

    def reset(self, mask=None):
        """Zero the history (and recurrent state) of all robots, or those in `mask` [B] bool."""
        if mask is None:
            self.observation.zero_()
            self.action.zero_()
            self.engine.reset_hidden()
        else:
            import numpy as np
            import torch
            m = torch.as_tensor(mask, device=self.device, dtype=torch.bool)
            self.observation[m] = 0
            self.action[m] = 0
            self.engine.reset_hidden(np.asarray(m.cpu(), np.uint8), self.batch)

    def step(self, state, joy=None, stream=None) -> TickOutput:
        """state [B, 36] float32 device tensor, joy [B, 5] float32 or None."""
        if state.shape != (self.batch, CTL_STATE_DIM):
            raise ValueError(f"state must be [{self.batch}, {CTL_STATE_DIM}]")
        if joy is not None and joy.shape != (self.batch, CTL_JOY_DIM):
            raise ValueError(f"joy must be [{self.batch}, {CTL_JOY_DIM}]")
        self.engine.controller_step_torch(state, self.observation, self.action, joy=joy, q_des=self.q_des,
                                          kp=self.kp, kd=self.kd, status=self.status, stream=stream)
        return TickOutput(self.action, self.q_des, self.kp, self.kd, self.status)
