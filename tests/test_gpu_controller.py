"""GPU parity of the fused controller tick against
oracle/controller_ref.py (controller.cpp:173-248 restated) + the policy oracle.

Per tick, with the GPU's previous observation / action as the state:
* the new observation (history shift, gravity projection, q - q0, joystick
  command, contacts) is BIT-IDENTICAL to the oracle's (integer-exact layout
  work and the same float32 operation order);
* the action equals post_process(policy(obs)) within the policy tolerance
  (1e-5, max(1, |ref|)-relative as in test_gpu_parity);
* q_des = q0 + 0.25 a (double) and kp / kd are exact given the GPU's action;
* status flags exactly the robots the reference would exit(1) on.
"""
import numpy as np
import pytest

from conftest import SHIPPED, rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _mlp_policy(path):
    from oracle import mlp_ref
    ref = mlp_ref.MlpRef.from_onnx(path)
    return lambda x: ref.f64(np.asarray(x, np.float32))


def _check(st, joy, obs_prev, act_prev, obs, act, outs, hist, policy_y, params=None):
    from oracle import controller_ref as cr
    want_obs, want_status = cr.assemble_obs(obs_prev, act_prev, st, joy, hist, params)
    assert np.array_equal(obs, want_obs, equal_nan=True), np.argwhere(obs != want_obs)[:5]
    a_ref, _, kp_ref, kd_ref = cr.post_process(policy_y(obs), joy, params)
    assert rel_err(act, a_ref) <= TOL
    if outs is not None:
        q_des, kp, kd, status = outs
        p = params or cr.default_params()
        assert np.array_equal(q_des, np.asarray(p["q0"])[None] + act.astype(np.float64) * p["action_scale"])
        assert np.array_equal(kp, kp_ref) and np.array_equal(kd, kd_ref)
        assert np.array_equal(status, want_status)


def _run_ticks(e, policy_y, B, T, seed, hist=2, joy_mode="random", params=None):
    from oracle import controller_ref as cr
    rng = np.random.default_rng(seed)
    obs = np.zeros((B, e.in_dim), np.float32)
    act = np.zeros((B, 12), np.float32)
    for t in range(T):
        st = cr.synthetic_states(rng, B, upright=t % 2 == 0)
        joy = None if joy_mode == "none" else cr.synthetic_joy(rng, B)
        o0, a0 = obs.copy(), act.copy()
        outs = e.controller_step(st, obs, act, joy=joy)
        _check(st, joy, o0, a0, obs, act, outs, hist, policy_y, params)
    return obs, act


@pytest.mark.parametrize("B", [1, 3, 8, 37, 4096])
def test_controller_ticks_shipped(B):
    """Shipped 98 -> 12 policy: B <= 8 runs the single-launch kernel, larger the fused batched one."""
    from go2_onnx_controller_amd import Engine
    with Engine(SHIPPED, max_batch=max(B, 8)) as e:
        assert e.ctl_history() == 2
        _run_ticks(e, _mlp_policy(SHIPPED), B, 4, seed=B)


def test_controller_long_closed_loop_no_joystick():
    from go2_onnx_controller_amd import Engine
    with Engine(SHIPPED, max_batch=16) as e:
        _run_ticks(e, _mlp_policy(SHIPPED), 16, 50, seed=11, joy_mode="none")


@pytest.mark.parametrize("name,hist", [("ctl_h1", 1), ("ctl_h3", 3), ("ctl_h16", 16), ("ctl_h3_deep", 3),
                                       ("ctl_h4_deep", 4)])
@pytest.mark.parametrize("B,res", [(5, 0), (5, 500), (300, 0)])
def test_controller_history_lengths(synth_path, name, hist, B, res):
    """Other history lengths (49 x kHistory observations): B = 5 by one launch per tick or
    by the resident kernel's controller form (the generic policy_act1_kernel shapes for
    ctl_h1 and ctl_h3, the multi-workgroup form for ctl_h16), and the batched kernel.
    The _deep variants (three hidden layers) take the lean tick kernel at B = 300 with a
    layer 0 whose K pads to 64 (147 -> 192, 196 -> 256 columns): its chunk count is not
    ceil(in_dim / 16)."""
    from go2_onnx_controller_amd import Engine
    p = synth_path(name)
    with Engine(p, max_batch=B, resident_ms=res) as e:
        assert e.ctl_history() == hist
        _run_ticks(e, _mlp_policy(p), B, 3, seed=B + hist, hist=hist)


@pytest.mark.parametrize("env", [{}, {"GO2PI_CTL_GENERAL": "1"}])
@pytest.mark.parametrize("name,hist", [("shipped", 2), ("ctl_h3_deep", 3)])
def test_controller_tick_bodies(synth_path, monkeypatch, env, name, hist):
    """The batched controller tick in both bodies: the lean tick kernel (policy_mlp_ctl_kernel,
    the default for Elu policies with three hidden layers) and the general body
    (GO2PI_CTL_GENERAL=1 at create, A/B), bit-exact observations and oracle actions."""
    from go2_onnx_controller_amd import Engine
    for k, v in env.items():
        monkeypatch.setenv(k, v)  # read at engine creation
    p = SHIPPED if name == "shipped" else synth_path(name)
    with Engine(p, max_batch=300) as e:
        _run_ticks(e, _mlp_policy(p), 300, 3, seed=hist + len(env), hist=hist)


@pytest.mark.parametrize("waves", [4, 16])
def test_controller_waves(waves):
    from go2_onnx_controller_amd import Engine
    with Engine(SHIPPED, max_batch=512, waves=waves) as e:
        _run_ticks(e, _mlp_policy(SHIPPED), 512, 3, seed=waves)


def test_controller_gru_policy(synth_path):
    """A recurrent controller policy: the hidden rows advance once per tick."""
    from go2_onnx_controller_amd import Engine
    from oracle import onnx_ref
    p = synth_path("gru_ctl")
    g = onnx_ref.load(p)
    B, H = 40, 64
    state = {"h": np.zeros((1, B, H))}

    def policy_y(obs):
        r = onnx_ref.run(g, {"observation": obs.astype(np.float64), "h_in": state["h"]})
        state["h"] = r["h_out"]
        return r["action"]
    with Engine(p, max_batch=B) as e:
        e.reset_hidden()
        _run_ticks(e, policy_y, B, 3, seed=4)
        assert float(np.max(np.abs(e.get_hidden(B) - state["h"][0]))) <= TOL


def test_controller_params():
    from go2_onnx_controller_amd import Engine
    from oracle import controller_ref as cr
    params = cr.default_params()
    params.update(kp=40.0, kd=1.25, kp_stop=3.0, action_limit=0.05, contact_threshold=30.0,
                  gravity_w=(0.1, 0.0, -9.81), action_scale=0.3,  # not a power of two: q_des rounds twice
                  q0=np.linspace(-1, 1, 12))
    for B in (2, 64):
        with Engine(SHIPPED, max_batch=B) as e:
            e.ctl_set_params(**params)
            obs, act = _run_ticks(e, _mlp_policy(SHIPPED), B, 3, seed=B, params=params)
            assert np.max(np.abs(act)) <= 0.05


@pytest.mark.parametrize("B", [8, 64])
def test_controller_nan_status(B):
    from go2_onnx_controller_amd import Engine
    from oracle import controller_ref as cr
    rng = np.random.default_rng(B)
    st = cr.synthetic_states(rng, B)
    obs = np.zeros((B, 98), np.float32)
    act = np.zeros((B, 12), np.float32)
    st[1, 5] = np.nan   # gyro
    act[2, 3] = np.nan  # previous action
    st[3, 33] = np.nan  # foot force (a comparison, never NaN in the observation)
    with Engine(SHIPPED, max_batch=B) as e:
        o0, a0 = obs.copy(), act.copy()
        q_des, kp, kd, status = e.controller_step(st, obs, act)
        want_obs, want_status = cr.assemble_obs(o0, a0, st, None, 2)
        assert np.array_equal(obs, want_obs, equal_nan=True)
        assert status.tolist() == want_status.tolist()
        assert status[:4].tolist() == [0, 1, 1, 0]


def test_controller_device_path_matches_host():
    """go2pi_controller_step_device on torch tensors == the host path, bitwise."""
    import torch
    from go2_onnx_controller_amd import Engine
    from oracle import controller_ref as cr
    for B in (4, 96):
        rng = np.random.default_rng(B)
        with Engine(SHIPPED, max_batch=B) as e:
            obs = rng.normal(size=(B, 98)).astype(np.float32)
            act = rng.normal(size=(B, 12)).astype(np.float32)
            st, joy = cr.synthetic_states(rng, B), cr.synthetic_joy(rng, B)
            dev = torch.device("cuda:0")
            t_obs, t_act = torch.from_numpy(obs).to(dev), torch.from_numpy(act).to(dev)
            t_st, t_joy = torch.from_numpy(st).to(dev), torch.from_numpy(joy).to(dev)
            q = torch.empty((B, 12), dtype=torch.float64, device=dev)
            kp = torch.empty_like(q)
            kd = torch.empty_like(q)
            status = torch.full((B,), 7, dtype=torch.int32, device=dev)
            e.controller_step_torch(t_st, t_obs, t_act, joy=t_joy, q_des=q, kp=kp, kd=kd, status=status)
            torch.cuda.synchronize()
            outs = e.controller_step(st, obs, act, joy=joy)
            assert np.array_equal(t_obs.cpu().numpy(), obs)
            assert np.array_equal(t_act.cpu().numpy(), act)
            assert np.array_equal(q.cpu().numpy(), outs[0])
            assert np.array_equal(kp.cpu().numpy(), outs[1]) and np.array_equal(kd.cpu().numpy(), outs[2])
            assert np.array_equal(status.cpu().numpy().astype(np.uint32), outs[3])


def test_controller_rejects_non_controller_policy(synth_path):
    from go2_onnx_controller_amd import Engine, Go2piError
    with Engine(synth_path("go2_mlp_512"), max_batch=8) as e:
        with pytest.raises(Go2piError) as ex:
            e.ctl_history()
        assert ex.value.code == -2
        with pytest.raises(Go2piError):
            e.controller_step(np.zeros((1, 36), np.float32), np.zeros((1, 48), np.float32),
                              np.zeros((1, 12), np.float32))


@pytest.mark.parametrize("form", ["one", "one_r1w", "multi"])
@pytest.mark.parametrize("B", [1, 3, 8])
def test_controller_ticks_resident(B, form, monkeypatch):
    """The resident kernel's controller form (go2pi_opts.resident_ms > 0, batch <= 8):
    same bit-exact observation / action contract, with and without joystick rows,
    with and without the optional outputs, and switching to and from the act() form.
    form: the single-workgroup kernel (the shipped model's default: r05's polling-wave
    policy_act1_kernel, or r04's 512-thread form with GO2PI_RES_R1W=1) or the
    multi-workgroup one (GO2PI_RES_MULTI=1)."""
    from go2_onnx_controller_amd import Engine
    from oracle import controller_ref as cr
    if form == "multi":
        monkeypatch.setenv("GO2PI_RES_MULTI", "1")
    elif form == "one_r1w":
        monkeypatch.setenv("GO2PI_RES_R1W", "1")
    pol = _mlp_policy(SHIPPED)
    with Engine(SHIPPED, max_batch=8, resident_ms=500) as e:
        obs, act = _run_ticks(e, pol, B, 6, seed=40 + B)
        _run_ticks(e, pol, B, 4, seed=50 + B, joy_mode="none")
        rng = np.random.default_rng(60 + B)
        for t in range(4):
            st, joy = cr.synthetic_states(rng, B), cr.synthetic_joy(rng, B)
            o0, a0 = obs.copy(), act.copy()
            assert e.controller_step(st, obs, act, joy=joy, outputs=False) is None
            _check(st, joy, o0, a0, obs, act, None, 2, pol)
            x = rng.standard_normal((B, 98)).astype(np.float32)  # the act() form in between
            assert rel_err(e.run(x), pol(x)) <= TOL


@pytest.mark.parametrize("form", ["one", "one_r1w", "multi"])
def test_controller_resident_nan_status(form, monkeypatch):
    from go2_onnx_controller_amd import Engine
    from oracle import controller_ref as cr
    if form == "multi":
        monkeypatch.setenv("GO2PI_RES_MULTI", "1")
    elif form == "one_r1w":
        monkeypatch.setenv("GO2PI_RES_R1W", "1")
    rng = np.random.default_rng(77)
    B = 4
    with Engine(SHIPPED, max_batch=8, resident_ms=500) as e:
        st = cr.synthetic_states(rng, B)
        st[1, 8] = np.nan  # q of robot 1
        obs = np.zeros((B, 98), np.float32)
        act = np.zeros((B, 12), np.float32)
        o0, a0 = obs.copy(), act.copy()
        _, _, _, status = e.controller_step(st, obs, act)
        _, want = cr.assemble_obs(o0, a0, st, None, 2)
        assert np.array_equal(status, want) and status[1] == 1 and status[0] == 0
