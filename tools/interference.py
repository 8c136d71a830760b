#!/usr/bin/env python3
"""Diagnostics: what a live resident act() kernel costs a batched launch on the
same device.

Engine A (batch-1 act(), resident kernel, the ONNXActor shim's default) is kept
live by a host thread calling act() at a given rate; engine B times batches of
4096 robots (go2pi_run_device on its own stream, HIP events) at the same time.
Cases: no A at all; A live but idle (inside its idle bound, the kernel polls);
A ticking at 50 Hz (the reference's controller rate, controller.cpp:61) and
at 1 kHz. Prints one JSON object.
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--resident-model", default="go2_mlp_512")
    ap.add_argument("--batched-model", default="go2_mlp_512")
    ap.add_argument("--launches", type=int, default=2000)
    args = ap.parse_args()
    import numpy as np
    import torch
    from go2_onnx_controller_amd import Engine, synth
    rpath = synth.ensure_model(args.resident_model) if not args.resident_model.endswith(".onnx") \
        else args.resident_model
    bpath = synth.ensure_model(args.batched_model)
    dev = torch.device("cuda:0")
    b = Engine(bpath, max_batch=4096)
    x = torch.randn((4096, b.in_dim), device=dev)
    y = torch.empty((4096, b.out_dim), device=dev)
    torch.cuda.synchronize(dev)
    s = torch.cuda.Stream(dev)
    launch = b.device_launcher(x.data_ptr(), y.data_ptr(), 4096, s.cuda_stream)

    def timed():
        # (stream syncs only: a device-wide sync would wait for the live resident kernel)
        for _ in range(50):
            launch()
        s.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(s)
        for _ in range(args.launches):
            launch()
        ev1.record(s)
        s.synchronize()
        return ev0.elapsed_time(ev1) / args.launches * 1e3

    out = {"batched": b.batched_kernel, "resident_model": args.resident_model}
    out["no_resident_us"] = round(timed(), 3)
    a = Engine(rpath, max_batch=8, resident_ms=100000)
    obs = np.random.default_rng(0).standard_normal((1, a.in_dim)).astype(np.float32)
    for name, hz in (("resident_idle", 0), ("resident_50hz", 50), ("resident_1khz", 1000)):
        stop = threading.Event()
        lat = []

        def tick():
            while not stop.is_set():
                t0 = time.perf_counter()
                a.run(obs)
                lat.append((time.perf_counter() - t0) * 1e6)
                if hz:
                    time.sleep(max(0.0, 1.0 / hz - (time.perf_counter() - t0)))
                else:
                    stop.wait()
        th = threading.Thread(target=tick)
        th.start()
        time.sleep(0.05)
        us = timed()
        stop.set()
        th.join()
        lat.sort()
        out[f"{name}_us"] = round(us, 3)
        out[f"{name}_act_p50_us"] = round(lat[len(lat) // 2], 2) if lat else None
    a.close()
    out["after_resident_left_us"] = round(timed(), 3)
    b.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
