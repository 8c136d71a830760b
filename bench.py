#!/usr/bin/env python3
"""Benchmark: control steps/sec (whole node) + p50 single-step latency.

BASELINE.json metric: "control steps/sec (whole node) + p50 single-step
latency, Go2 48-obs MLP policy". A "control step" is one robot's policy
evaluation; a bench "step" is one pass of the hot path
(`go2pi_run_device`, the batched fused kernel) over one batch of synthetic
observations already resident in HBM.

Default workload (N=1): configs[2] of BASELINE.json — the 48->512^3->12 ELU
MLP (deterministic synthetic weights, go2_onnx_controller_amd/synth.py) at
batch 4096 robots per GPU, fp32. Beside it, on rank 0 at N=1:
  * configs[1] (batch 1): `latency_b1_p50_us` (host obs -> host action, PCIe
    included, the ONNXActor::act() contract), resident kernel and launch per call;
  * configs[4]: `gru256` — the GRU-256 policy at 4096 robots, the 100-tick
    sequence with the hidden rows carried in LDS beside the per-tick form;
  * configs[0]: `cpu_baseline` — the oracle's fp32 C restatement on the host
    cores (1 thread and all allowed threads at batch 4096, and the batch-1
    p50/p99 of the reference's own measurement, main.cpp:38-42).

Multi-GPU (configs[3]): `--gpus N` runs one process per GPU. Under
torch.distributed.run (WORLD_SIZE set) this process is one rank; otherwise this
script starts the N ranks itself (child processes, before anything touches a
GPU) and waits for them. Every rank runs its own 4096-robot shard (weak
scaling, no data-path collective: N=8 is 32768 robots); a barrier brackets the
timed region and the max time over ranks is reported.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 (MFMA = VALU rate), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec
METRIC = "control steps/sec (whole node) + p50 single-step latency, Go2 48-obs MLP policy"

WORKLOADS = {
    # name: (synthetic model, batch per GPU, ticks per launch, BASELINE config)
    "go2_mlp_512_b4096": ("go2_mlp_512", 4096, 1, "configs[2]: Go2 MLP 48->512x3->12, batch 4096/GPU, MFMA path"),
    "go2_gru_256_b4096": ("go2_gru_256", 4096, 1,
                          "configs[4]: Go2 GRU-256 + 512x3 head, batch 4096/GPU, one tick per launch (h in HBM)"),
    "go2_gru_256_b4096_seq100": ("go2_gru_256", 4096, 100,
                                 "configs[4]: Go2 GRU-256 + 512x3 head, batch 4096/GPU, 100 ticks per launch "
                                 "(hidden rows carried in LDS)"),
    "shipped_b4096": ("__shipped__", 4096, 1, "shipped model 98->128x3->12, batch 4096/GPU"),
    "go2_lstm_256_b4096": ("go2_lstm_256", 4096, 1, "LSTM-256 + 512x3 head, batch 4096/GPU, one tick per launch"),
    "go2_lstm_256_b4096_seq100": ("go2_lstm_256", 4096, 100,
                                  "LSTM-256 + 512x3 head, batch 4096/GPU, 100 ticks per launch "
                                  "(h in LDS, c in registers)"),
}


def cpu_model_name():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def host_threads():
    """Threads for the all-cores CPU leg: OMP_NUM_THREADS when set (the GPU box sets
    it to its CPU share, 16 per GPU, while nproc shows the whole machine), else the
    CPUs this process may run on."""
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = os.cpu_count() or 1
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (env or allowed), allowed


def _pct(ts, q):
    ts = sorted(ts)
    return ts[min(len(ts) - 1, int(len(ts) * q))]


def cpu_baseline(model_path, in_dim, batch, seconds=8.0):
    """The oracle's fp32 C restatement (oracle/mlp_ref.c, OpenMP over rows) on the
    host cores, on bounded samples: whole `batch`-row steps for ~`seconds` on 1
    thread and on all allowed threads; and configs[0], the batch-1 act() latency
    (1k warm-up + 10k timed single-robot forwards, timed inside C) for the shipped
    98->128^3->12 model and the synthetic 48->512^3->12 one."""
    import numpy as np
    from oracle import mlp_ref
    from go2_onnx_controller_amd import synth
    nthr, allowed = host_threads()
    ref = mlp_ref.MlpRef.from_onnx(model_path)
    x = np.random.default_rng(1).standard_normal((batch, in_dim)).astype(np.float32)

    def rate(threads):
        ref.f32(x, threads)  # warm
        n, t0 = 0, time.perf_counter()
        while True:
            ref.f32(x, threads)
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                return n * batch / el, n, el
    v1, n1, e1 = rate(1)
    vn, nn, en = rate(nthr)
    b1 = {}
    shipped = os.path.join(ROOT, "tests", "golden", "model.onnx")
    for key, path in (("shipped", shipped), ("mlp512", synth.ensure_model("go2_mlp_512"))):
        r = mlp_ref.MlpRef.from_onnx(path)
        row = np.random.default_rng(2).standard_normal(r.in_dim).astype(np.float32)
        ts = r.time_b1(row, warm=1000, iters=10000)
        b1[f"{key}_b1_p50_us"] = round(float(_pct(ts, 0.5)), 2)
        b1[f"{key}_b1_p99_us"] = round(float(_pct(ts, 0.99)), 2)
    return {"value": vn, "unit": "control steps/sec", "cores": nthr, "kind": "port",
            "sample": f"{nn} steps x {batch} robots ({en:.1f} s) of the fp32 C restatement "
                      f"(oracle/mlp_ref.c, -O3 x86-64-v3, OpenMP {nthr} threads) on {cpu_model_name()}",
            "single_thread": {"value": v1, "cores": 1, "sample": f"{n1} steps x {batch} robots ({e1:.1f} s)"},
            "cpu_model": cpu_model_name(), "host_cpus_allowed": allowed,
            "threads_leg": (f"{nthr} threads: OMP_NUM_THREADS, the GPU box's CPU share per GPU (host_cpus_allowed "
                            f"counts the whole machine's {allowed}, shared with other jobs)") if nthr != allowed
                           else f"{nthr} threads: every CPU this process may run on",
            "configs0_batch1": dict(b1, warmup=1000, iters=10000, threads=1,
                                    what="one single-robot fp32 forward per call, timed in C "
                                         "(the reference's main.cpp:38-42 measurement)")}


def latency_b1(model_path, device, iters=10000, warm=1000, resident_ms=0):
    """p50/p99 of one host->host batch-1 step (ONNXActor::act() path, pinned
    host-mapped staging). resident_ms > 0: the resident kernel the ONNXActor shim
    uses (no launch per call); 0: one launch of policy_latency_kernel per call."""
    import numpy as np
    from go2_onnx_controller_amd import Engine
    with Engine(model_path, device=device, max_batch=64, resident_ms=resident_ms) as e:
        x = np.random.default_rng(2).standard_normal((1, e.in_dim)).astype(np.float32)
        y = np.empty((1, e.out_dim), np.float32)
        for _ in range(warm):
            e.run_ptr(x.ctypes.data, y.ctypes.data, 1)
        ts = []
        for i in range(iters):
            x[0, i % e.in_dim] += 1e-3
            t0 = time.perf_counter_ns()
            e.run_ptr(x.ctypes.data, y.ctypes.data, 1)
            ts.append((time.perf_counter_ns() - t0) / 1e3)
    return _pct(ts, 0.5), _pct(ts, 0.99)


def latency_b1_cpp(model_path, in_dim, out_dim, iters=10000, warm=1000):
    """p50/p99 of ONNXActor::act() at batch 1 timed in C++ the way the reference's
    own driver times it (onnx_inference/src/cpp/main.cpp:38-42: steady_clock around
    one act()), through the drop-in shim (libonnx_actor.so, resident kernel by
    default): tests/cpp/controller_shape.cpp's `lat` mode, built here with g++ if
    absent. None when it cannot be built or run."""
    lib = os.path.join(ROOT, "go2_onnx_controller_amd", "lib")
    exe = os.path.join(ROOT, "build", "controller_shape")
    src = os.path.join(ROOT, "tests", "cpp", "controller_shape.cpp")
    try:
        if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(src):
            os.makedirs(os.path.dirname(exe), exist_ok=True)
            subprocess.run(["g++", "-std=c++20", "-O2", "-I" + os.path.join(ROOT, "include"), src, "-L" + lib,
                            "-lonnx_actor", "-Wl,-rpath," + lib, "-o", exe], check=True, capture_output=True)
        r = subprocess.run([exe, model_path, "lat", str(iters), str(warm), str(in_dim), str(out_dim)],
                           capture_output=True, text=True, timeout=120)
        vals = dict(ln.split(": ") for ln in r.stdout.splitlines() if ln.startswith("p"))
        return float(vals["p50_us"]), float(vals["p99_us"])
    except (OSError, subprocess.SubprocessError, KeyError, ValueError):
        return None


def timed_launches(call, stream, dev, n, warm):
    """Average microseconds per `call` from HIP events recorded on `stream` (the stream
    the kernels are launched on)."""
    import torch
    for _ in range(warm):
        call()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(n):
        call()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    return ev0.elapsed_time(ev1) / n * 1e3


def gru_leg(device, launches=20, seq_ticks=100):
    """BASELINE configs[4]: the GRU-256 policy (48 -> GRU 256 -> 512^3 -> 12) at
    4096 robots. `seq100`: go2pi_run_sequence_device over 100 ticks per launch, the
    hidden rows carried in LDS between ticks (HBM only at sequence start / end);
    `per_tick`: one go2pi_run_device per tick, the hidden rows round-trip HBM."""
    import torch
    from go2_onnx_controller_amd import Engine, synth
    dev = torch.device(f"cuda:{device}")
    B = 4096
    out = {}
    with Engine(synth.ensure_model("go2_gru_256"), device=device, max_batch=B) as e:
        g = torch.Generator().manual_seed(5)
        obs = torch.randn((seq_ticks, B, e.in_dim), generator=g).to(dev)
        act = torch.empty((seq_ticks, B, e.out_dim), device=dev)
        s = torch.cuda.Stream(dev)
        e.reset_hidden()  # h0 = 0 (the sequences continue the hidden state after that)
        fpr = e.cost["flops_per_row"]

        def seq():
            e.run_sequence_device(obs.data_ptr(), act.data_ptr(), seq_ticks, B, s.cuda_stream)
        tick = e.device_launcher(obs.data_ptr(), act.data_ptr(), B, s.cuda_stream)
        us_seq = timed_launches(seq, s, dev, launches, 2)
        us_tick = timed_launches(tick, s, dev, launches * 20, 20)
        for key, us, ticks, res in (("seq100", us_seq, seq_ticks, "lds"), ("per_tick", us_tick, 1, "hbm")):
            per_tick = us / ticks
            tf = fpr * B / (per_tick * 1e-6) / 1e12
            out[key] = {"us_per_launch": round(us, 3), "ticks_per_launch": ticks, "us_per_tick": round(per_tick, 3),
                        "robot_steps_per_s": round(B / (per_tick * 1e-6), 1), "achieved_tflops": round(tf, 3),
                        "frac_fp32_peak": round(tf / PEAK_FP32_TFLOPS, 4), "hidden_residency": res}
        out["kernel"] = e.batched_kernel
        out["robots"] = B
        # memory-side bytes of one 100-tick launch (committed rocprofv3 FETCH/WRITE passes)
        tr, note = load_pmc("go2_gru_256_b4096_seq100", e.batched_kernel)
        out["seq100"]["traffic_bytes_per_launch"] = round(tr) if tr else None
        out["seq100"]["traffic_source"] = note
    return out


def controller_leg(device, steps=200, warm=20, iters=10000):
    """The fused controller tick (go2pi_controller_step*: observation assembly +
    shipped policy + action post-processing in one launch):
    robot-ticks/s at 4096 robots (device path, HIP events on the launch stream)
    beside the policy-only launch, and the batch-1 host tick p50/p99 (the
    reference's publish() work around act(), host arrays in and out)."""
    import ctypes

    import numpy as np
    import torch
    from go2_onnx_controller_amd import Engine
    from go2_onnx_controller_amd.engine import lib
    path = os.path.join(ROOT, "tests", "golden", "model.onnx")
    dev = torch.device(f"cuda:{device}")
    B = 4096
    g = torch.Generator().manual_seed(3)
    q0 = torch.tensor([0.1, -0.1, 0.1, -0.1, 0.8, 0.8, 1.0, 1.0, -1.5, -1.5, -1.5, -1.5])

    def states(n):
        st = torch.zeros((n, 36))
        quat = torch.cat([torch.ones((n, 1)), 0.08 * torch.randn((n, 3), generator=g)], 1)
        st[:, 0:4] = quat / quat.norm(dim=1, keepdim=True)
        st[:, 4:7] = 0.5 * torch.randn((n, 3), generator=g)
        st[:, 7:19] = q0 + 0.2 * torch.randn((n, 12), generator=g)
        st[:, 19:31] = 2.0 * torch.randn((n, 12), generator=g)
        st[:, 31:35] = torch.randint(0, 60, (n, 4), generator=g).float()
        joy = torch.zeros((n, 5))
        joy[:, 0] = 1
        joy[:, 1:4] = torch.rand((n, 3), generator=g) * 2 - 1
        return st, joy
    out = {}
    with Engine(path, device=device, max_batch=B) as e:
        st, joy = (t.to(dev) for t in states(B))
        obs = torch.zeros((B, e.in_dim), device=dev)
        act = torch.zeros((B, 12), device=dev)
        qd = torch.empty((B, 12), dtype=torch.float64, device=dev)
        kp, kd = torch.empty_like(qd), torch.empty_like(qd)
        status = torch.empty((B,), dtype=torch.int32, device=dev)
        s = torch.cuda.Stream(dev)
        fn = lib().go2pi_controller_step_device
        P = ctypes.c_void_p
        args = (e._h, P(st.data_ptr()), P(joy.data_ptr()), P(obs.data_ptr()), P(act.data_ptr()),
                P(qd.data_ptr()), P(kp.data_ptr()), P(kd.data_ptr()), P(status.data_ptr()), ctypes.c_int64(B),
                P(s.cuda_stream))
        policy = e.device_launcher(obs.data_ptr(), act.data_ptr(), B, s.cuda_stream)

        def tick():
            if fn(*args):
                raise RuntimeError(lib().go2pi_last_error().decode())
        tick_us = timed_launches(tick, s, dev, steps, warm)
        policy_us = timed_launches(policy, s, dev, steps, warm)
        out["robots"] = B
        out["tick_us"] = round(tick_us, 3)
        out["policy_only_us"] = round(policy_us, 3)
        out["robot_ticks_per_s"] = round(B / (tick_us * 1e-6), 1)
    # batch-1 host tick: the resident kernel (go2pi_opts.resident_ms, as the ONNXActor shim
    # uses for act()), then one launch per tick
    for key, res_ms in (("b1_tick", 100), ("b1_tick_launch", 0)):
        with Engine(path, device=device, max_batch=8, resident_ms=res_ms) as e:
            st1, joy1 = (np.ascontiguousarray(t.numpy()) for t in states(1))
            obs1 = np.zeros((1, e.in_dim), np.float32)
            act1 = np.zeros((1, 12), np.float32)
            bufs = [np.empty((1, 12)), np.empty((1, 12)), np.empty((1, 12)), np.empty(1, np.uint32)]
            fn = lib().go2pi_controller_step
            args = (e._h, st1.ctypes.data, joy1.ctypes.data, obs1.ctypes.data, act1.ctypes.data,
                    *[b.ctypes.data for b in bufs], 1)
            ts = []
            for i in range(warm * 10 + iters):
                st1[0, 4 + i % 3] = 0.01 * (i % 7)
                t0 = time.perf_counter_ns()
                rc = fn(*args)
                t1 = time.perf_counter_ns()
                if rc:
                    raise RuntimeError(lib().go2pi_last_error().decode())
                if i >= warm * 10:
                    ts.append((t1 - t0) / 1e3)
            out[f"{key}_p50_us"] = round(_pct(ts, 0.5), 2)
            out[f"{key}_p99_us"] = round(_pct(ts, 0.99), 2)
    return out


def load_pmc(workload, kernel):
    """(bytes, note): memory-side bytes per launch of the batched kernel
    instantiation `kernel` (e.g. "policy_mlp_kernel<8, 1, 3, 1, 3, 4>",
    Engine.batched_kernel) from the committed rocprofv3 --pmc summary of this
    workload (tools/profile.sh + tools/summarize_prof.py: separate FETCH_SIZE /
    WRITE_SIZE passes, gfx950 read correction x2), and where it came from. bytes is
    None, with the reason in note, when no summary of this exact kernel is committed
    or the kernel sources changed after it was taken (provenance.kernel_source_digest)."""
    from go2_onnx_controller_amd.provenance import kernel_source_digest
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        for k, v in d.get("workloads", {}).get(workload, {}).items():
            if f"::{kernel}(" in k:
                src = v.get("source", "?")
                if v.get("src_digest") != kernel_source_digest():
                    return None, (f"stale: profiles/{src} was taken on other kernel sources "
                                  f"(digest {v.get('src_digest')}, now {kernel_source_digest()}); re-profile")
                return v.get("hbm_bytes_per_launch"), f"profiles/{src} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)"
    except (OSError, ValueError):
        pass
    return None, "no committed rocprofv3 --pmc summary of this kernel"



def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """Start `n` ranks of this script (one process per GPU, LOCAL_RANK = GPU ordinal)
    with the torch.distributed env contract, wait for all of them, and return the
    first non-zero exit code. Rank 0 prints the JSON line. This process never
    touches a GPU. If one rank fails, the others are stopped (they would wait at
    the barrier forever)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--settle-s", type=float, default=0.3, help="untimed clock-settle phase before the warmup")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="go2_mlp_512_b4096", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="override robots per GPU")
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-latency", action="store_true", help="skip the batch-1 latency leg")
    ap.add_argument("--no-ctl", action="store_true", help="skip the controller-tick leg")
    ap.add_argument("--no-gru", action="store_true", help="skip the configs[4] GRU leg")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for the barrier / max-time reduce (nccl = RCCL)")
    ap.add_argument("--same-device", action="store_true",
                    help="testing only: every rank on device 0 (rehearse N>1 on a 1-GPU box with gloo)")
    ap.add_argument("--dry-run", action="store_true",
                    help="testing only: no device work; exercises the rank launcher, the process group, "
                         "the barriers and the max-over-ranks reduce")
    args = ap.parse_args()

    if args.gpus < 1:
        sys.exit("--gpus must be >= 1")
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (one process per GPU)")
    elif args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    else:
        world = 1
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group("gloo")

    mname, batch, ticks, cfg_desc = WORKLOADS[args.workload]
    if args.batch:
        batch = args.batch
    if args.dry_run:
        dev = None

        def launch():
            pass
    else:
        if local >= torch.cuda.device_count():
            sys.exit(f"rank {rank}: LOCAL_RANK {local} but only {torch.cuda.device_count()} GPU(s) visible")
        from go2_onnx_controller_amd import Engine, synth
        torch.cuda.set_device(local)
        dev = torch.device(f"cuda:{local}")
        model_path = os.path.join(ROOT, "tests", "golden", "model.onnx") if mname == "__shipped__" \
            else synth.ensure_model(mname)
        eng = Engine(model_path, device=local, max_batch=batch, waves=args.waves)
        in_dim, out_dim = eng.in_dim, eng.out_dim
        gen = torch.Generator(device="cpu").manual_seed(1 + rank)
        obs = torch.randn((ticks, batch, eng.in_dim), generator=gen).to(dev)
        act = torch.empty((ticks, batch, eng.out_dim), device=dev)
        stream = torch.cuda.Stream(dev)  # the stream every timed launch goes to
        if ticks > 1:
            eng.reset_hidden()

            def launch():
                eng.run_sequence_device(obs.data_ptr(), act.data_ptr(), ticks, batch, stream.cuda_stream)
        else:
            launch = eng.device_launcher(obs.data_ptr(), act.data_ptr(), batch, stream.cuda_stream)
        # clock settle (untimed): an idle MI355X needs tens of ms of load before its
        # clocks reach steady state; without this a short default run times the ramp
        # (200 launches: 42.0 us each straight from idle vs 38.8 us settled)
        t_settle = time.perf_counter()
        while time.perf_counter() - t_settle < args.settle_s:
            for _ in range(max(1, 50 // ticks)):
                launch()
            torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        launch()
    if dev is not None:
        torch.cuda.synchronize(dev)
        # host enqueue cost per launch (must stay below the kernel time for the GPU to stay fed)
        h0 = time.perf_counter()
        for _ in range(args.steps):
            launch()
        host_us = (time.perf_counter() - h0) / args.steps * 1e6
        torch.cuda.synchronize(dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    # ---- the timed region: barrier + sync on both sides, max over ranks
    if world > 1:
        dist.barrier()
    if dev is not None:
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if dev is not None:
        ev0.record(stream)
    for _ in range(args.steps):
        launch()
    if dev is not None:
        ev1.record(stream)
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps if dev is not None else 0.0  # avg launch on the launching stream
    k_min = k_max = kernel_ms
    if world > 1:
        on = dev if (args.dist_backend == "nccl" and dev is not None) else "cpu"
        t = torch.tensor([elapsed, kernel_ms, -kernel_ms], device=on, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, k_max, k_min = float(t[0].item()), float(t[1].item()), -float(t[2].item())

    total_rows = batch * ticks * world * args.steps
    value = total_rows / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "control steps/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic obs N(0,1); deterministic synthetic weights (synth.py, seed 0)"
                 if mname != "__shipped__" else "synthetic obs N(0,1); shipped reference weights"),
        "config": {"workload": args.workload, "description": cfg_desc, "robots_per_gpu": batch,
                   "ticks_per_step": ticks, "global_batch": batch * world,
                   "parallelism": f"dp{world} (contiguous robot-row shards, no data-path collective)"},
    }
    if args.dry_run:
        out["dry_run"] = True
    else:
        cost = eng.cost
        flops_launch = cost["flops_per_row"] * batch * ticks
        bytes_launch = cost["weight_bytes"] + cost["io_bytes_per_row"] * batch * ticks
        achieved_tf = flops_launch / (kernel_ms * 1e-3) / 1e12
        kernel_name = eng.batched_kernel
        traffic, traffic_note = load_pmc(args.workload, kernel_name)
        eng.close()
        out.update({
            "kernel": kernel_name,
            "kernel_us": round(kernel_ms * 1e3, 3),
            "kernel_us_min_max_over_ranks": [round(k_min * 1e3, 3), round(k_max * 1e3, 3)],
            "host_enqueue_us": round(host_us, 3),
            "roofline": {"bound": "mfma", "achieved": round(achieved_tf, 3), "peak": PEAK_FP32_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_FP32_TFLOPS, 4),
                         "frac_per_gpu_min": round(flops_launch / (k_max * 1e-3) / 1e12 / PEAK_FP32_TFLOPS, 4),
                         "traffic": traffic,
                         "traffic_source": traffic_note,
                         "algorithmic_flops_per_launch": flops_launch,
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "hbm_frac": round(bytes_launch / (kernel_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 5)},
        })
        if ticks > 1:
            out["hidden_residency"] = "lds"
        elif cost["has_gru"]:
            out["hidden_residency"] = "hbm"
    if rank == 0 and world == 1 and not args.dry_run:
        if not args.no_latency:
            # the ONNXActor shim's default (resident kernel, 100 ms idle bound), then one launch per call
            p50, p99 = latency_b1(model_path, local, resident_ms=100)
            out["latency_b1_p50_us"] = round(p50, 2)
            out["latency_b1_p99_us"] = round(p99, 2)
            # configs[1] as an HBM fraction: weights + one robot's I/O per step over the p50
            b1_bytes = eng.cost["weight_bytes"] + eng.cost["io_bytes_per_row"]
            out["latency_b1_hbm_frac"] = round(b1_bytes / (p50 * 1e-6) / 1e9 / PEAK_HBM_GBS, 5)
            p50, p99 = latency_b1(model_path, local)
            out["latency_b1_launch_p50_us"] = round(p50, 2)
            out["latency_b1_launch_p99_us"] = round(p99, 2)
            # the same act() timed from C++ through the drop-in ONNXActor, as the
            # reference's main.cpp times it (the legs above call through Python ctypes)
            shipped = os.path.join(ROOT, "tests", "golden", "model.onnx")
            cpp = {}
            for name, path, i_d, o_d in (("go2_mlp_512", model_path, in_dim, out_dim),
                                         ("shipped", shipped, 98, 12)):
                r = latency_b1_cpp(path, i_d, o_d)
                if r:
                    cpp[name] = {"p50_us": round(r[0], 2), "p99_us": round(r[1], 2)}
            if cpp:
                cpp["what"] = ("ONNXActor::act() at batch 1 timed in C++ (steady_clock around one call, "
                               "main.cpp:38-42), resident kernel, 1,000 warm + 10,000 timed calls")
                from go2_onnx_controller_amd import Engine as _Engine
                for name, path in (("go2_mlp_512", model_path), ("shipped", shipped)):
                    if name in cpp:  # the resident form each model gets (no launch: the name only)
                        with _Engine(path, device=local, max_batch=8, resident_ms=100) as _e:
                            cpp[name]["resident_kernel"] = _e.resident_kernel
                out["latency_b1_act_cpp"] = cpp
            # the recurrent policy (configs[4]'s GRU-256) at batch 1: the resident kernel's GRU
            # form (hidden rows carried inside the live kernel), then one fused launch per call
            from go2_onnx_controller_amd import synth as _synth
            gru_path = _synth.ensure_model("go2_gru_256")
            p50, p99 = latency_b1(gru_path, local, resident_ms=100)
            out["latency_b1_gru_p50_us"] = round(p50, 2)
            out["latency_b1_gru_p99_us"] = round(p99, 2)
            p50, p99 = latency_b1(gru_path, local)
            out["latency_b1_gru_launch_p50_us"] = round(p50, 2)
            out["latency_b1_gru_launch_p99_us"] = round(p99, 2)
            # LSTM-256 (the same head): resident (h as granules, c in the owning
            # workgroups' LDS), then one fused launch per call
            lstm_path = _synth.ensure_model("go2_lstm_256")
            p50, p99 = latency_b1(lstm_path, local, resident_ms=100)
            out["latency_b1_lstm_p50_us"] = round(p50, 2)
            out["latency_b1_lstm_p99_us"] = round(p99, 2)
            p50, p99 = latency_b1(lstm_path, local)
            out["latency_b1_lstm_launch_p50_us"] = round(p50, 2)
            out["latency_b1_lstm_launch_p99_us"] = round(p99, 2)
        if not args.no_gru and mname == "go2_mlp_512":
            out["gru256"] = gru_leg(local)
        if not args.no_ctl:
            out["controller_tick"] = controller_leg(local)
        if not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(model_path, in_dim, batch, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
