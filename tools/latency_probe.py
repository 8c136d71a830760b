#!/usr/bin/env python3
"""Batch-1 act() latency probe: p50/p99 host->host, optional mode knobs.
Usage: latency_probe.py [--model go2_mlp_512|shipped] [--iters N] [--no-graph] [--small-batch K]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="go2_mlp_512")
    ap.add_argument("--iters", type=int, default=3000)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--small-batch", type=int, default=0)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--resident-ms", type=int, default=0)
    args = ap.parse_args()
    import numpy as np
    from go2_onnx_controller_amd import Engine, synth
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                        "model.onnx") if args.model == "shipped" else synth.ensure_model(args.model)
    with Engine(path, max_batch=64, use_graph=not args.no_graph, small_batch=args.small_batch,
                resident_ms=args.resident_ms) as e:
        x = np.random.default_rng(2).standard_normal((args.batch, e.in_dim)).astype(np.float32)
        y = np.empty((args.batch, e.out_dim), np.float32)
        for _ in range(300):
            e.run_ptr(x.ctypes.data, y.ctypes.data, args.batch)
        ts = []
        for i in range(args.iters):
            x[0, i % e.in_dim] += 1e-3
            t0 = time.perf_counter_ns()
            e.run_ptr(x.ctypes.data, y.ctypes.data, args.batch)
            ts.append((time.perf_counter_ns() - t0) / 1e3)
    ts.sort()
    print(f"{args.model} B={args.batch} graph={not args.no_graph} small={args.small_batch}: "
          f"resident={args.resident_ms}: p50 {ts[len(ts)//2]:.2f} us  p99 {ts[int(len(ts)*0.99)]:.2f} us  min {ts[0]:.2f} us")


if __name__ == "__main__":
    main()
