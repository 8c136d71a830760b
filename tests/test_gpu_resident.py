"""GPU: the resident batch <= 8 act() path (opts.resident_ms > 0, resident.hip).

One launch serves every go2pi_run at batch <= 8: the observation and the
request header travel as {epoch, value} granules in host-mapped memory. Layers
1.. are policy_latency_kernel's; layer 0 is computed by every workgroup for
itself (one fma chain per output), so the resident path matches the
one-launch-per-call path within the 1e-5 contract of the fp64 oracle, and is
bit-identical to it with GO2PI_RES_TILED0=1 (layer 0 tiled like the others). Also covered: the kernel leaving on idle (a request racing that exit is
served by a relaunch), another engine call in between (the kernel is stopped
and relaunched), and destroy while resident.
"""
import time

import numpy as np
import pytest

from conftest import SHIPPED, abs_err, realistic_obs, rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _models(synth_path):
    return {"shipped": SHIPPED, "mlp512": synth_path("go2_mlp_512"), "wide_256_3": synth_path("wide_256_3"),
            "wide_256_4": synth_path("wide_256_4"), "wide_512_3": synth_path("wide_512_3")}


# resident forms: "one" the single-workgroup kernel (the default where the weights fit
# one CU: the shipped model; r05 policy_act1_kernel, a polling wave + 8 compute waves,
# two poll sweeps in flight), "one_d1" the same with one sweep in flight, "one_c4" with
# four compute waves instead of eight, "one_r1w" the
# r04 1024-thread form (GO2PI_RES_R1W=1), "multi" the multi-workgroup kernel
# (GO2PI_RES_MULTI=1; for mlp512 the form without large BAR), "tiled0" multi with
# layer 0 tiled like every other layer (bit-identical to the launch path), "wide" the
# wide-policy kernel (r06 policy_wide_kernel, the default for 256- and 512-wide policies
# where the request ring is in device memory): mlp512 (BASELINE configs[1]), hidden width
# 256 with one and two sliced layers, 512 with one
@pytest.mark.parametrize("name,form", [("shipped", "one"), ("shipped", "one_d1"), ("shipped", "one_c4"),
                                       ("shipped", "one_r1w"),
                                       ("shipped", "multi"), ("shipped", "tiled0"),
                                       ("mlp512", "multi"), ("mlp512", "tiled0"),
                                       ("mlp512", "wide"), ("wide_256_3", "wide"), ("wide_256_4", "wide"),
                                       ("wide_512_3", "wide")])
def test_resident_vs_launch_per_call(synth_path, name, form, monkeypatch):
    from go2_onnx_controller_amd import Engine
    from oracle import mlp_ref
    tiled0 = form == "tiled0"
    if form == "one_d1":
        monkeypatch.setenv("GO2PI_A1_DEPTH", "1")  # read at each resident launch
    elif form == "one_c4":
        monkeypatch.setenv("GO2PI_A1_CW", "4")  # four compute waves (one per SIMD)
    elif form == "one_r1w":
        monkeypatch.setenv("GO2PI_RES_R1W", "1")
    elif form not in ("one", "wide"):
        monkeypatch.setenv("GO2PI_RES_MULTI", "1")  # read at engine creation
    if tiled0:
        monkeypatch.setenv("GO2PI_RES_TILED0", "1")  # read at each resident launch
    path = _models(synth_path)[name]
    ref = mlp_ref.MlpRef.from_onnx(path)
    with Engine(path, max_batch=64, resident_ms=500) as r, Engine(path, max_batch=64) as p:
        if form == "wide":  # (without large BAR the multi-workgroup kernel serves, ring in host memory)
            want = "policy_wide_kernel" if r.resident_kernel.endswith("ring=vram") else "policy_resident_kernel"
            assert r.resident_kernel.startswith(want), r.resident_kernel
        elif form == "multi" or tiled0:
            assert r.resident_kernel.startswith("policy_resident_kernel"), r.resident_kernel
        rng = np.random.default_rng(7)
        for i, B in enumerate([1, 1, 2, 3, 1, 8, 5, 1, 4, 1] * 3):
            x = (realistic_obs(B, seed=i) if name == "shipped"
                 else rng.standard_normal((B, r.in_dim)).astype(np.float32))
            y = r.run(x)
            assert y.shape == (B, r.out_dim)
            assert np.array_equal(y, r.run(x)), f"call {i} B={B}: resident path not deterministic"
            yp = p.run(x)
            if tiled0:
                assert np.array_equal(y, yp), f"call {i} B={B}: resident (tiled layer 0) != launch-per-call"
            else:
                assert abs_err(y, yp) <= TOL
            assert abs_err(y, ref.f64(x)) <= TOL


@pytest.mark.parametrize("name,form", [("shipped", "one"), ("shipped", "multi"), ("mlp512", "multi"),
                                       ("mlp512", "wide"), ("wide_256_3", "wide"), ("wide_256_4", "wide"),
                                       ("wide_512_3", "wide")])
def test_resident_kernel_stays_live(synth_path, name, form, monkeypatch):
    """One resident launch serves a run of requests at batch 1..8 (go2pi_resident_launches):
    a kernel that gives up on every request (a failed sweep, a clobbered LDS word) still
    answers correctly through a relaunch per call, so parity alone does not show it."""
    from go2_onnx_controller_amd import Engine
    from oracle import mlp_ref
    if form == "multi":
        monkeypatch.setenv("GO2PI_RES_MULTI", "1")  # read at engine creation
    path = _models(synth_path)[name]
    ref = mlp_ref.MlpRef.from_onnx(path)
    rng = np.random.default_rng(11)
    with Engine(path, max_batch=8, resident_ms=5000) as e:
        if e.resident_kernel == "none":
            pytest.skip("no resident form for this model")
        assert e.resident_launches == 0
        for i, B in enumerate([1, 8, 1, 1, 3, 1, 8, 1] * 25):
            x = (realistic_obs(B, seed=i) if name == "shipped"
                 else rng.standard_normal((B, e.in_dim)).astype(np.float32))
            y = e.run(x)
            if i % 20 == 0:
                assert abs_err(y, ref.f64(x)) <= TOL, f"call {i} B={B}"
        assert e.resident_launches == 1, f"{e.resident_kernel}: {e.resident_launches} launches for 200 requests"


def test_resident_known_answers():
    """The reference drivers' inputs (src/cpp/main.cpp:32 zeros, src/python/main.py:20 twos)."""
    import os
    from conftest import GOLDEN, rel_err
    from go2_onnx_controller_amd import Engine
    g = np.load(os.path.join(GOLDEN, "golden_shipped.npz"))
    with Engine(SHIPPED, max_batch=8, resident_ms=500) as e:
        for _ in range(3):
            for name in ("zeros", "twos"):
                assert rel_err(e.run(g[f"{name}_x"]), g[f"{name}_y"]) <= TOL, name


def test_resident_wide_known_answers(synth_path):
    """The wide-policy kernel on the committed mlp512 fixture (tests/golden/golden_mlp512.npz,
    fp64 ONNX oracle outputs), row by row at batch 1 and all rows at batch 8, over
    repeated requests; the answer is deterministic across requests."""
    import os
    from conftest import GOLDEN
    from go2_onnx_controller_amd import Engine
    g = np.load(os.path.join(GOLDEN, "golden_mlp512.npz"))
    x, want = g["x"].astype(np.float32), g["y"]
    with Engine(synth_path("go2_mlp_512"), max_batch=8, resident_ms=500) as e:
        first = None
        for rep in range(3):
            for i in range(min(len(x), 8)):
                assert abs_err(e.run(x[i:i + 1]), want[i:i + 1]) <= TOL, f"rep {rep} row {i}"
            y8 = e.run(x[:8])
            assert abs_err(y8, want[:8]) <= TOL
            first = y8 if first is None else first
            assert np.array_equal(y8, first), "the resident answer changed between requests"


@pytest.mark.parametrize("name", ["shipped", "mlp512"])
def test_resident_request_ring_in_host_memory(synth_path, name, monkeypatch):
    """GO2PI_REQ_HOST=1: the request ring in pinned host memory, as on a host without
    large BAR (the production path there; engine.cpp bar_take falls back to it). act() at
    batch 1 and 8 and the controller tick at batch 1 and 8 (shipped model) against the
    fp64 oracle."""
    from go2_onnx_controller_amd import Engine
    from oracle import controller_ref as cr
    from oracle import mlp_ref
    monkeypatch.setenv("GO2PI_REQ_HOST", "1")  # read at engine creation
    path = _models(synth_path)[name]
    ref = mlp_ref.MlpRef.from_onnx(path)
    rng = np.random.default_rng(37)
    with Engine(path, max_batch=8, resident_ms=500) as e:
        assert e.resident_kernel.endswith("ring=host"), e.resident_kernel
        for i, B in enumerate([1, 8, 1, 3, 8, 1] * 3):
            x = realistic_obs(B, seed=200 + i) if name == "shipped" else rng.standard_normal((B, 48)).astype(np.float32)
            assert abs_err(e.run(x), ref.f64(x)) <= TOL, f"call {i} B={B}"
        if name == "shipped":
            for i, B in enumerate([1, 8, 1, 8]):
                st, joy = cr.synthetic_states(rng, B), cr.synthetic_joy(rng, B)
                obs = rng.standard_normal((B, 98)).astype(np.float32)
                act = rng.standard_normal((B, 12)).astype(np.float32)
                want_obs, _ = cr.assemble_obs(obs, act, st, joy, 2)
                a_ref = cr.post_process(ref.f64(want_obs), joy)[0]
                e.controller_step(st, obs, act, joy=joy)
                assert np.array_equal(obs, want_obs), f"tick {i}: observation differs"
                assert rel_err(act, a_ref) <= TOL, f"tick {i}"


def test_resident_interleaved_with_batched_calls(synth_path):
    """A batched call parks the resident kernel; the next small call relaunches it."""
    from go2_onnx_controller_amd import Engine
    from oracle import mlp_ref
    path = synth_path("go2_mlp_512")
    ref = mlp_ref.MlpRef.from_onnx(path)
    rng = np.random.default_rng(3)
    with Engine(path, max_batch=4096, resident_ms=500) as e:
        for i in range(4):
            x1 = rng.standard_normal((1, 48)).astype(np.float32)
            assert abs_err(e.run(x1), ref.f64(x1)) <= TOL
            xb = rng.standard_normal((256 * (i + 1), 48)).astype(np.float32)
            assert abs_err(e.run(xb), ref.f64(xb)) <= TOL
            e.sync()
            x2 = rng.standard_normal((3, 48)).astype(np.float32)
            assert abs_err(e.run(x2), ref.f64(x2)) <= TOL


def test_resident_idle_exit_and_relaunch():
    """resident_ms = 4: requests after 0-12 ms pauses meet a live kernel, one near its
    idle deadline (the host relaunches past half of it) or one that has left."""
    from go2_onnx_controller_amd import Engine
    from oracle import mlp_ref
    ref = mlp_ref.MlpRef.from_onnx(SHIPPED)
    rng = np.random.default_rng(11)
    with Engine(SHIPPED, max_batch=8, resident_ms=4) as e:
        for i in range(60):
            x = realistic_obs(1 + i % 3, seed=100 + i)
            assert abs_err(e.run(x), ref.f64(x)) <= TOL, f"call {i}"
            time.sleep(float(rng.uniform(0.0, 0.012)))


def test_resident_destroy_while_live(synth_path):
    from go2_onnx_controller_amd import Engine
    path = synth_path("go2_mlp_512")
    x = np.ones((1, 48), np.float32)
    for _ in range(5):
        e = Engine(path, max_batch=8, resident_ms=10000)
        e.run(x)
        t0 = time.perf_counter()
        e.close()  # the kernel leaves on the LEAVE header, not on its 10 s idle bound
        assert time.perf_counter() - t0 < 1.0


def test_resident_two_engines(synth_path):
    """Two resident kernels on one device, served alternately."""
    from go2_onnx_controller_amd import Engine
    from oracle import mlp_ref
    pa, pb = SHIPPED, synth_path("go2_mlp_512")
    ra, rb = mlp_ref.MlpRef.from_onnx(pa), mlp_ref.MlpRef.from_onnx(pb)
    rng = np.random.default_rng(5)
    with Engine(pa, max_batch=8, resident_ms=500) as a, Engine(pb, max_batch=8, resident_ms=500) as b:
        for i in range(20):
            xa = realistic_obs(1, seed=i)
            xb = rng.standard_normal((2, 48)).astype(np.float32)
            assert abs_err(a.run(xa), ra.f64(xa)) <= TOL
            assert abs_err(b.run(xb), rb.f64(xb)) <= TOL


def test_resident_prologue_epilogue(synth_path):
    """The optional normalisation prologue and tanh/clip/scale epilogue (go2pi_opts) on the resident path."""
    from go2_onnx_controller_amd import Engine
    path = synth_path("go2_mlp_512")
    rng = np.random.default_rng(9)
    kw = dict(obs_mean=rng.normal(0, 0.3, 48).astype(np.float32), obs_std=rng.uniform(0.5, 2, 48).astype(np.float32),
              obs_clip=3.0, action_tanh=True, action_clip=0.8, action_scale=0.25, max_batch=8)
    with Engine(path, resident_ms=500, **kw) as r, Engine(path, **kw) as p:
        for B in (1, 2, 8, 1):
            x = rng.normal(0, 2, (B, 48)).astype(np.float32)
            assert abs_err(r.run(x), p.run(x)) <= TOL


def test_create_destroy_while_other_engine_resident(synth_path):
    """Engine B is created and destroyed while engine A's resident kernel is kept live
    by another thread (a 200 Hz act() loop, faster than A's idle bound): neither
    create nor destroy may wait on A's kernel (no device-wide synchronisation)."""
    import threading
    from go2_onnx_controller_amd import Engine
    from oracle import mlp_ref
    ref = mlp_ref.MlpRef.from_onnx(SHIPPED)
    stop, errs = threading.Event(), []
    with Engine(SHIPPED, max_batch=8, resident_ms=100) as a:
        x = realistic_obs(1, seed=1)
        a.run(x)

        def tick():
            try:
                while not stop.is_set():
                    if abs_err(a.run(x), ref.f64(x)) > TOL:
                        errs.append("A's output changed")
                    time.sleep(0.005)
            except Exception as ex:  # noqa: BLE001 - reported below
                errs.append(repr(ex))
        th = threading.Thread(target=tick)
        th.start()
        try:
            time.sleep(0.05)
            path = synth_path("go2_mlp_512")
            for _ in range(3):
                t0 = time.perf_counter()
                b = Engine(path, max_batch=64)
                y = b.run(np.ones((2, 48), np.float32))
                b.close()
                dt = time.perf_counter() - t0
                assert np.isfinite(y).all()
                assert dt < 1.0, f"create + run + destroy took {dt:.2f} s beside a live resident kernel"
        finally:
            stop.set()
            th.join(timeout=10)
    assert not errs, errs


def test_resident_controller_step_then_device_step():
    """go2pi_controller_step (served by the resident kernel at B <= 8) alternating with
    go2pi_controller_step_device on the same engine: the device call stops the resident
    kernel first (they share granules and the epoch), both match the oracle."""
    import torch
    from go2_onnx_controller_amd import Engine
    from oracle import controller_ref as cr
    from oracle import mlp_ref
    ref = mlp_ref.MlpRef.from_onnx(SHIPPED)
    rng = np.random.default_rng(21)
    dev = torch.device("cuda:0")
    with Engine(SHIPPED, max_batch=8, resident_ms=500) as e:
        for i in range(6):
            B = 1 + i % 4
            st, joy = cr.synthetic_states(rng, B), cr.synthetic_joy(rng, B)
            obs = rng.standard_normal((B, 98)).astype(np.float32)
            act = rng.standard_normal((B, 12)).astype(np.float32)
            want_obs, _ = cr.assemble_obs(obs, act, st, joy, 2)
            a_ref = cr.post_process(ref.f64(want_obs), joy)[0]
            if i % 2 == 0:
                e.controller_step(st, obs, act, joy=joy)
                o, a = obs, act
            else:
                t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
                     for k, v in (("st", st), ("joy", joy), ("obs", obs), ("act", act))}
                e.controller_step_torch(t["st"], t["obs"], t["act"], joy=t["joy"])
                torch.cuda.synchronize(dev)
                o, a = t["obs"].cpu().numpy(), t["act"].cpu().numpy()
            assert np.array_equal(o, want_obs), f"tick {i}: observation differs"
            assert rel_err(a, a_ref) <= TOL, f"tick {i}"


def test_entry_points_restore_current_device():
    """Every C-ABI call switches to the engine's device for its work and restores the
    caller's current device (with one GPU this checks the ordinal is left alone; with
    two or more, an engine on the last device is driven while the caller sits on 0)."""
    import torch
    from go2_onnx_controller_amd import Engine
    from oracle import controller_ref as cr
    n = torch.cuda.device_count()
    edev = n - 1
    torch.cuda.set_device(0)
    rng = np.random.default_rng(4)
    with Engine(SHIPPED, device=edev, max_batch=64, resident_ms=200) as e:
        assert torch.cuda.current_device() == 0
        x = realistic_obs(3)
        e.run(x)
        assert torch.cuda.current_device() == 0
        e.run(realistic_obs(1))  # resident path
        assert torch.cuda.current_device() == 0
        d = torch.device(f"cuda:{edev}")
        xo = torch.from_numpy(realistic_obs(64)).to(d)
        with torch.cuda.device(d):
            s = torch.cuda.Stream(d)
        torch.cuda.set_device(0)
        e.run_torch(xo, stream=s)
        assert torch.cuda.current_device() == 0
        st, joy = cr.synthetic_states(rng, 2), cr.synthetic_joy(rng, 2)
        obs, act = np.zeros((2, 98), np.float32), np.zeros((2, 12), np.float32)
        e.controller_step(st, obs, act, joy=joy)
        assert torch.cuda.current_device() == 0
        e.sync()
        assert torch.cuda.current_device() == 0
    assert torch.cuda.current_device() == 0


def _gru_oracle_step(path, x, h):
    from oracle import onnx_ref
    g = onnx_ref.load(path)
    r = onnx_ref.run(g, {"observation": x.astype(np.float64), "h_in": h[None]})
    return r["action"], r["h_out"][0]


@pytest.mark.parametrize("name", ["go2_gru_256", "gru_128"])
def test_resident_gru_rollout(synth_path, name):
    """The resident kernel's GRU form (resident.hip, RNN): the hidden rows are carried
    inside the live kernel between requests as tagged granules. 40 requests at batch
    1..8 (rows past a request's batch keep their state), with a masked reset, a
    set_hidden and get_hidden reads interleaved (each stops the kernel; the next
    request relaunches and resumes from the engine's state rows), against the fp64
    ONNX-GRU oracle rollout per row, and against the launch-per-call engine."""
    from go2_onnx_controller_amd import Engine
    p = synth_path(name)
    rng = np.random.default_rng(17)
    with Engine(p, max_batch=8, resident_ms=500) as r, Engine(p, max_batch=8) as q:
        H = r.hidden_dim
        h_ref = np.zeros((8, H))
        r.reset_hidden()
        q.reset_hidden()
        for i in range(40):
            B = [1, 1, 2, 8, 3, 1, 5, 8][i % 8]
            x = rng.standard_normal((B, r.in_dim)).astype(np.float32)
            want, h_new = _gru_oracle_step(p, x, h_ref[:B])
            h_ref[:B] = h_new
            y = r.run(x)
            assert abs_err(y, want) <= TOL, f"request {i} B={B}"
            assert abs_err(q.run(x), want) <= TOL, f"request {i} B={B} (launch path)"
            if i == 12:  # masked reset (stops the kernel; the next request relaunches)
                mask = np.array([1, 0, 1, 0, 0, 0, 0, 1], np.uint8)
                r.reset_hidden(mask)
                q.reset_hidden(mask)
                h_ref[mask == 1] = 0
            if i == 25:
                s = rng.standard_normal((8, H)).astype(np.float32) * 0.5
                r.set_hidden(s)
                q.set_hidden(s)
                h_ref[:] = s
            if i % 10 == 9:
                assert abs_err(r.get_hidden(8), h_ref) <= TOL, f"request {i}: hidden rows"


def test_resident_gru_idle_exit_keeps_state(synth_path):
    """resident_ms = 3: requests after pauses meet a kernel that has left (or is about
    to); its h' stores to the state rows carry the hidden state across relaunches."""
    from go2_onnx_controller_amd import Engine
    p = synth_path("gru_128")
    rng = np.random.default_rng(23)
    with Engine(p, max_batch=8, resident_ms=3) as r:
        h_ref = np.zeros((8, r.hidden_dim))
        for i in range(30):
            B = 1 + i % 3
            x = rng.standard_normal((B, r.in_dim)).astype(np.float32)
            want, h_new = _gru_oracle_step(p, x, h_ref[:B])
            h_ref[:B] = h_new
            assert abs_err(r.run(x), want) <= TOL, f"request {i}"
            time.sleep(float(rng.uniform(0.0, 0.008)))


def _lstm_oracle_step(path, x, hc):
    from oracle import onnx_ref
    g = onnx_ref.load(path)
    H = hc.shape[1] // 2
    r = onnx_ref.run(g, {"observation": x.astype(np.float64), "h_in": hc[None, :, :H], "c_in": hc[None, :, H:]})
    return r["action"], np.concatenate([r["h_out"][0], r["c_out"][0]], axis=1)


@pytest.mark.parametrize("name", ["go2_lstm_256", "lstm_128"])
def test_resident_lstm_rollout(synth_path, name):
    """The resident kernel's LSTM form (resident.hip, RNN = 2): h' carried between
    requests as tagged granules, the cell state c in the owning workgroups' LDS.
    40 requests at batch 1..8 with a masked reset, a set_hidden and get_hidden reads
    (h | c rows) interleaved, against the fp64 ONNX-LSTM oracle rollout per row and
    against the launch-per-call engine."""
    from go2_onnx_controller_amd import Engine
    p = synth_path(name)
    rng = np.random.default_rng(29)
    with Engine(p, max_batch=8, resident_ms=500) as r, Engine(p, max_batch=8) as q:
        S = r.hidden_dim  # 2H: h | c
        hc_ref = np.zeros((8, S))
        r.reset_hidden()
        q.reset_hidden()
        for i in range(40):
            B = [1, 1, 2, 8, 3, 1, 5, 8][i % 8]
            x = rng.standard_normal((B, r.in_dim)).astype(np.float32)
            want, hc_new = _lstm_oracle_step(p, x, hc_ref[:B])
            hc_ref[:B] = hc_new
            assert abs_err(r.run(x), want) <= TOL, f"request {i} B={B}"
            assert abs_err(q.run(x), want) <= TOL, f"request {i} B={B} (launch path)"
            if i == 12:
                mask = np.array([0, 1, 1, 0, 1, 0, 0, 0], np.uint8)
                r.reset_hidden(mask)
                q.reset_hidden(mask)
                hc_ref[mask == 1] = 0
            if i == 25:
                s = rng.standard_normal((8, S)).astype(np.float32) * 0.5
                r.set_hidden(s)
                q.set_hidden(s)
                hc_ref[:] = s
            if i % 10 == 9:
                assert abs_err(r.get_hidden(8), hc_ref) <= TOL, f"request {i}: h | c rows"


def test_resident_lstm_idle_exit_keeps_state(synth_path):
    """resident_ms = 3: the LSTM kernel leaves between requests; its h and c
    write-back to the state rows carries both across relaunches."""
    from go2_onnx_controller_amd import Engine
    p = synth_path("lstm_128")
    rng = np.random.default_rng(31)
    with Engine(p, max_batch=8, resident_ms=3) as r:
        hc_ref = np.zeros((8, r.hidden_dim))
        for i in range(30):
            B = 1 + i % 3
            x = rng.standard_normal((B, r.in_dim)).astype(np.float32)
            want, hc_new = _lstm_oracle_step(p, x, hc_ref[:B])
            hc_ref[:B] = hc_new
            assert abs_err(r.run(x), want) <= TOL, f"request {i}"
            time.sleep(float(rng.uniform(0.0, 0.008)))
        assert abs_err(r.get_hidden(8), hc_ref) <= TOL


def test_batched_launch_evicts_other_resident_kernels(synth_path):
    """A batched launch on the device tells other engines' live resident kernels to
    leave (they hold CUs the launch needs: DESIGN §4.2b); the evicted engine's act()
    keeps answering correctly from another thread throughout (a request met by the
    eviction is served by a relaunch or by a launch), and the batched results stay
    correct."""
    import threading
    import torch
    from go2_onnx_controller_amd import Engine
    from oracle import mlp_ref
    pb = synth_path("go2_mlp_512")
    ra, rb = mlp_ref.MlpRef.from_onnx(SHIPPED), mlp_ref.MlpRef.from_onnx(pb)
    errs, n_act = [], [0]
    stop = threading.Event()
    with Engine(SHIPPED, max_batch=8, resident_ms=1000) as a, Engine(pb, max_batch=4096) as b:
        x1 = realistic_obs(1, seed=3)
        want1 = ra.f64(x1)

        def tick():
            try:
                while not stop.is_set():
                    if abs_err(a.run(x1), want1) > TOL:
                        errs.append("act() output changed")
                    n_act[0] += 1
                    time.sleep(0.001)
            except Exception as ex:  # noqa: BLE001 - reported below
                errs.append(repr(ex))
        th = threading.Thread(target=tick)
        th.start()
        try:
            xb = torch.randn((4096, 48), device="cuda:0")
            s = torch.cuda.Stream()
            for _ in range(30):
                yb = b.run_torch(xb, stream=s)
                s.synchronize()
                time.sleep(0.002)
            assert abs_err(yb.cpu().numpy(), rb.f64(xb.cpu().numpy())) <= TOL
        finally:
            stop.set()
            th.join(timeout=10)
    assert not errs, errs
    assert n_act[0] > 10


def test_diag_stamps_switch(synth_path, monkeypatch):
    """GO2PI_DIAG_STAMPS=1 at create allocates the diagnostics stamp buffer the clock /
    timeline builds write; in the product build nothing writes it, and every path stays
    correct: batched, one launch per call and resident (wide policy and the shipped one)."""
    from go2_onnx_controller_amd import Engine
    from oracle import mlp_ref
    monkeypatch.setenv("GO2PI_DIAG_STAMPS", "1")
    rng = np.random.default_rng(8)
    for path in (synth_path("go2_mlp_512"), SHIPPED):
        ref = mlp_ref.MlpRef.from_onnx(path)
        with Engine(path, max_batch=512, resident_ms=200) as r, Engine(path, max_batch=512) as q:
            for B in (1, 8, 300):
                x = rng.standard_normal((B, r.in_dim)).astype(np.float32)
                assert abs_err(r.run(x), ref.f64(x)) <= TOL, (path, B)
                assert abs_err(q.run(x), ref.f64(x)) <= TOL, (path, B)
            st = r.diag_stamps(64)
            assert st.size == 64 and not st.any()


def test_small_batched_launch_beside_busy_resident_kernel(synth_path):
    """A batched launch of <= GO2PI_YIELD_MIN_GRID workgroups (1024 rows) evicts no
    resident kernel: it fits on the CUs the resident kernels leave free.
    While another engine's resident kernel answers act() at ~1 kHz from another thread,
    1024-row launches of the 48->512^3->12 policy stay correct and bounded: their median
    wall time stays within 3x the same launch with no resident kernel live."""
    import threading
    import torch
    from go2_onnx_controller_amd import Engine
    from oracle import mlp_ref
    pb = synth_path("go2_mlp_512")
    ra, rb = mlp_ref.MlpRef.from_onnx(SHIPPED), mlp_ref.MlpRef.from_onnx(pb)
    xb = torch.randn((1024, 48), device="cuda:0")
    s = torch.cuda.Stream()

    def timed(b, n=40, until=None):
        # n launches; with `until`, launches continue (within 3 s) until it holds
        ts, t_end = [], time.perf_counter() + 3.0
        while len(ts) < n or (until is not None and not until() and time.perf_counter() < t_end):
            t0 = time.perf_counter()
            yb = b.run_torch(xb, stream=s)
            s.synchronize()
            ts.append(time.perf_counter() - t0)
            time.sleep(0.0002)
        return sorted(ts)[len(ts) // 2], yb
    errs, n_act = [], [0]
    stop = threading.Event()
    with Engine(pb, max_batch=4096) as b:
        alone, _ = timed(b)
        with Engine(SHIPPED, max_batch=8, resident_ms=1000) as a:
            x1 = realistic_obs(1, seed=4)
            want1 = ra.f64(x1)
            a.run(x1)  # the resident kernel is live before the launches start

            def tick():
                try:
                    while not stop.is_set():
                        if abs_err(a.run(x1), want1) > TOL:
                            errs.append("act() output changed")
                        n_act[0] += 1
                        time.sleep(0.001)
                except Exception as ex:  # noqa: BLE001 - reported below
                    errs.append(repr(ex))
            th = threading.Thread(target=tick)
            th.start()
            try:
                busy, yb = timed(b, until=lambda: n_act[0] >= 20)
            finally:
                stop.set()
                th.join(timeout=10)
    assert not errs, errs
    assert n_act[0] > 10
    assert abs_err(yb.cpu().numpy(), rb.f64(xb.cpu().numpy())) <= TOL
    assert busy <= 3 * alone + 2e-4, (busy, alone)


@pytest.mark.parametrize("name", ["gru_128", "lstm_128"])
def test_batched_launch_evicts_recurrent_resident_kernel(synth_path, name):
    """The eviction race of ADVICE r03 on a recurrent policy: while another engine's
    4096-robot launches keep evicting it, the resident GRU / LSTM engine's act() runs
    a rollout from another thread. A request the kernel answered just before it left
    must not be served a second time (that would step the hidden state twice), so
    every action and the final hidden rows match the fp64 oracle rollout."""
    import threading
    import torch
    from go2_onnx_controller_amd import Engine
    p, pb = synth_path(name), synth_path("go2_mlp_512")
    step = _lstm_oracle_step if name.startswith("lstm") else _gru_oracle_step
    rng = np.random.default_rng(41)
    xs = [rng.standard_normal((1 + i % 2, 30)).astype(np.float32) for i in range(60)]
    errs, got = [], []
    stop = threading.Event()
    with Engine(p, max_batch=8, resident_ms=1000) as a, Engine(pb, max_batch=4096) as b:
        a.reset_hidden()

        def tick():
            try:
                for x in xs:
                    got.append(a.run(x).copy())
                    time.sleep(0.0005)
            except Exception as ex:  # noqa: BLE001 - reported below
                errs.append(repr(ex))
            finally:
                stop.set()
        xb = torch.randn((4096, 48), device="cuda:0")
        s = torch.cuda.Stream()
        b.run_torch(xb, stream=s)  # (warm: the first launch's one-time costs stay out of the race)
        s.synchronize()
        th = threading.Thread(target=tick)
        th.start()
        n = 0
        while not stop.is_set() and n < 2000:
            b.run_torch(xb, stream=s)
            s.synchronize()
            n += 1
        th.join(timeout=30)
        assert not errs, errs
        assert len(got) == len(xs) and n > 5
        h_ref = np.zeros((8, a.hidden_dim))
        for i, x in enumerate(xs):
            B = x.shape[0]
            want, h_new = step(p, x, h_ref[:B])
            h_ref[:B] = h_new
            assert abs_err(got[i], want) <= TOL, f"request {i}"
        assert abs_err(a.get_hidden(8), h_ref) <= TOL
