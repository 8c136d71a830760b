#!/usr/bin/env python3
"""Benchmark: control steps/sec (whole node) + p50 single-step latency.

BASELINE.json metric: "control steps/sec (whole node) + p50 single-step
latency, Go2 48-obs MLP policy". A "control step" is one robot's policy
evaluation; a bench "step" is one pass of the hot path
(`go2pi_run_device`, the batched fused kernel) over one batch of synthetic
observations already resident in HBM.

Default workload (N=1): configs[2] of BASELINE.json — the 48->512^3->12 ELU
MLP (deterministic synthetic weights, go2_onnx_controller_amd/synth.py) at
batch 4096 robots per GPU, fp32. configs[1] (batch 1, hipGraph step) is
reported beside it as `latency_b1_p50_us` (host obs -> host action, PCIe
included, the ONNXActor::act() contract). With --gpus N (torchrun, one process
per GPU) every rank runs its own 4096-robot shard (weak scaling, no data-path
collective: configs[3] at N=8 is 32768 robots).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 (MFMA = VALU rate), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec

WORKLOADS = {
    # name: (synthetic model, batch per GPU, BASELINE config)
    "go2_mlp_512_b4096": ("go2_mlp_512", 4096, "configs[2]: Go2 MLP 48->512x3->12, batch 4096/GPU, MFMA path"),
    "go2_gru_256_b4096": ("go2_gru_256", 4096, "configs[4]: Go2 GRU-256 + 512x3 head, batch 4096/GPU"),
    "shipped_b4096": ("__shipped__", 4096, "shipped model 98->128x3->12, batch 4096/GPU"),
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


def cpu_baseline(model_path, in_dim, batch, seconds=10.0):
    """The oracle's fp32 C restatement (oracle/mlp_ref.c, OpenMP over rows) on the
    host cores, on a bounded sample: whole `batch`-row steps for ~`seconds`."""
    import numpy as np
    from oracle import mlp_ref
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    ref = mlp_ref.MlpRef.from_onnx(model_path)
    x = np.random.default_rng(1).standard_normal((batch, in_dim)).astype(np.float32)
    ref.f32(x, threads)  # warm
    n, t0 = 0, time.perf_counter()
    while True:
        ref.f32(x, threads)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": n * batch / el, "unit": "control steps/sec", "cores": threads, "kind": "port",
            "sample": f"{n} steps x {batch} robots ({el:.1f} s) of the fp32 C restatement "
                      f"(oracle/mlp_ref.c, -O3 x86-64-v3, OpenMP {threads} threads) on {cpu_model_name()}"}


def latency_b1(model_path, device, iters=3000, warm=300, resident_ms=0):
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
    ts.sort()
    return ts[len(ts) // 2], ts[int(len(ts) * 0.99)]


def controller_leg(device, steps=200, warm=20, iters=3000):
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

        def timed(call):
            for _ in range(warm):
                call()
            torch.cuda.synchronize(dev)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(s)
            for _ in range(steps):
                call()
            ev1.record(s)
            torch.cuda.synchronize(dev)
            return ev0.elapsed_time(ev1) / steps * 1e3

        def tick():
            if fn(*args):
                raise RuntimeError(lib().go2pi_last_error().decode())
        tick_us = timed(tick)
        policy_us = timed(policy)
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
            ts.sort()
            out[f"{key}_p50_us"] = round(ts[len(ts) // 2], 2)
            out[f"{key}_p99_us"] = round(ts[int(len(ts) * 0.99)], 2)
    return out


def load_pmc(workload, kernel):
    """Memory-side bytes per launch of the batched kernel instantiation `kernel`
    (e.g. "policy_fused_kernel<4, 8, 1>", Engine.batched_kernel) from the
    committed rocprofv3 --pmc summary of this workload (tools/profile.sh +
    tools/summarize_prof.py: separate FETCH_SIZE / WRITE_SIZE passes, gfx950 read
    correction x2). None when no summary of this exact kernel is committed."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        for k, v in d.get("workloads", {}).get(workload, {}).items():
            if f"::{kernel}(" in k:
                return v.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


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
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for the barrier / max-time reduce (nccl = RCCL)")
    ap.add_argument("--same-device", action="store_true",
                    help="testing only: every rank on device 0 (rehearse N>1 on a 1-GPU box with gloo)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from go2_onnx_controller_amd import Engine, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")

    mname, batch, cfg_desc = WORKLOADS[args.workload]
    if args.batch:
        batch = args.batch
    model_path = os.path.join(ROOT, "tests", "golden", "model.onnx") if mname == "__shipped__" \
        else synth.ensure_model(mname)

    eng = Engine(model_path, device=local, max_batch=batch, waves=args.waves)
    in_dim = eng.in_dim
    gen = torch.Generator(device="cpu").manual_seed(1 + rank)
    obs = torch.randn((batch, eng.in_dim), generator=gen).to(dev)
    act = torch.empty((batch, eng.out_dim), device=dev)
    stream = torch.cuda.Stream(dev)  # the stream every timed launch goes to

    launch = eng.device_launcher(obs.data_ptr(), act.data_ptr(), batch, stream.cuda_stream)
    # clock settle (untimed): an idle MI355X needs tens of ms of load before its
    # clocks reach steady state; without this a short default run times the ramp
    # (200 launches: 42.0 us each straight from idle vs 38.8 us settled)
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle_s:
        for _ in range(50):
            launch()
        torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        launch()
    torch.cuda.synchronize(dev)
    # host enqueue cost per launch (must stay below the kernel time for the GPU to stay fed)
    h0 = time.perf_counter()
    for _ in range(args.steps):
        launch()
    host_us = (time.perf_counter() - h0) / args.steps * 1e6
    torch.cuda.synchronize(dev)

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        launch()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # avg launch duration on the launching stream
    if world > 1:
        t = torch.tensor([elapsed], device=dev if args.dist_backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    cost = eng.cost
    total_rows = batch * world * args.steps
    value = total_rows / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    flops_launch = cost["flops_per_row"] * batch
    bytes_launch = cost["weight_bytes"] + cost["io_bytes_per_row"] * batch
    achieved_tf = flops_launch / (kernel_ms * 1e-3) / 1e12
    kernel_name = eng.batched_kernel
    traffic = load_pmc(args.workload, kernel_name)
    eng.close()

    out = {
        "metric": "control steps/sec (whole node) + p50 single-step latency, Go2 48-obs MLP policy",
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
        "data": "synthetic obs N(0,1); deterministic synthetic weights (synth.py, seed 0)"
                if mname != "__shipped__" else "synthetic obs N(0,1); shipped reference weights",
        "config": {"workload": args.workload, "description": cfg_desc, "robots_per_gpu": batch,
                   "global_batch": batch * world, "parallelism": f"fleet shards x{world} (no data-path collective)"},
        "kernel": kernel_name,
        "kernel_us": round(kernel_ms * 1e3, 3),
        "host_enqueue_us": round(host_us, 3),
        "roofline": {"bound": "mfma", "achieved": round(achieved_tf, 3), "peak": PEAK_FP32_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_FP32_TFLOPS, 4),
                     "traffic": traffic,
                     "algorithmic_flops_per_launch": flops_launch,
                     "algorithmic_bytes_per_launch": bytes_launch,
                     "hbm_frac": round(bytes_launch / (kernel_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 5)},
    }
    if rank == 0 and world == 1:
        if not args.no_latency:
            # the ONNXActor shim's default (resident kernel, 100 ms idle bound), then one launch per call
            p50, p99 = latency_b1(model_path, local, resident_ms=100)
            out["latency_b1_p50_us"] = round(p50, 2)
            out["latency_b1_p99_us"] = round(p99, 2)
            p50, p99 = latency_b1(model_path, local)
            out["latency_b1_launch_p50_us"] = round(p50, 2)
            out["latency_b1_launch_p99_us"] = round(p99, 2)
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
