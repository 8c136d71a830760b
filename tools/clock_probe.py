#!/usr/bin/env python3
"""Diagnostics: in-kernel clock and per-workgroup cycles of the batched kernel.

Run with GO2PI_LIB pointing at a GO2PI_DIAG_CLOCK build and GO2PI_DIAG_STAMPS=1:
each workgroup stamps s_memtime (shader clock) and s_memrealtime (100 MHz) at
start and end; clock = d(memtime) / d(realtime) * 100 MHz (MI355X_MICROARCH.md,
DVFS give-back item 6). Launches back to back for `--seconds` first so the chip
settles at the clock it holds under this load.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--waves", type=int, default=8)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--model", default="go2_mlp_512")
    ap.add_argument("--ctl", action="store_true", help="time the controller tick (shipped-layout policy)")
    args = ap.parse_args()
    os.environ.setdefault("GO2PI_DIAG_STAMPS", "1")
    import numpy as np
    import torch
    from go2_onnx_controller_amd import Engine, synth
    path = args.model if args.model.endswith(".onnx") else synth.ensure_model(args.model)
    e = Engine(path, max_batch=args.batch, waves=args.waves)
    x = torch.randn(args.batch, e.in_dim, device="cuda:0")
    y = torch.empty(args.batch, e.out_dim, device="cuda:0")
    s = torch.cuda.Stream()
    if args.ctl:
        st = torch.zeros(args.batch, 36, device="cuda:0")
        st[:, 0] = 1
        joy = torch.zeros(args.batch, 5, device="cuda:0")
        q = torch.empty(args.batch, 12, dtype=torch.float64, device="cuda:0")
        kp, kd = torch.empty_like(q), torch.empty_like(q)
        status = torch.empty(args.batch, dtype=torch.int32, device="cuda:0")

        def call():
            e.controller_step_torch(st, x, y, joy=joy, q_des=q, kp=kp, kd=kd, status=status, stream=s)
    else:
        def call():
            e.run_torch(x, out=y, stream=s)
    t0 = time.time()
    n = 0
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    per_launch = []
    while time.time() - t0 < args.seconds:
        ev0.record(s)
        for _ in range(50):
            call()
        ev1.record(s)
        n += 50
        s.synchronize()
        per_launch.append(ev0.elapsed_time(ev1) * 1e3 / 50)
    SPW = 64
    st = e.diag_stamps(SPW * ((args.batch + 15) // 16)).reshape(-1, SPW).astype(np.float64)
    nl = e.cost["n_layers"]
    # per-wave layer-1 marks (slots 16 + 3w + {0,1,2}), relative to the layer-0 barrier (slot 6)
    waves_l1 = {}
    for w in range(min(args.waves, 16)):
        s0, s1, s2 = st[:, 16 + 3 * w], st[:, 17 + 3 * w], st[:, 18 + 3 * w]
        if np.all(s0 > 0):
            waves_l1[w] = [float(np.median(s0 - st[:, 6])), float(np.median(s1 - st[:, 6])),
                           float(np.median(s2 - st[:, 6])), float(np.median(st[:, 7] - st[:, 6]))]
    # pipeline builds (4-wave uniform MLP): layer-1 sub-phases per wave, slots 28 + 3w +
    # {own phase done, flag wait done, LDS phase done}, relative to the wave's layer-0 end (16 + 3w)
    sub_l1 = {}
    for w in range(min(args.waves, 4)):
        a, b, c, z = st[:, 28 + 3 * w], st[:, 29 + 3 * w], st[:, 30 + 3 * w], st[:, 16 + 3 * w]
        if np.all(a > 0) and np.all(z > 0):
            sub_l1[w] = [float(np.median(a - z)), float(np.median(b - z)), float(np.median(c - z))]
            if np.all(st[:, 46 + w] > 0):  # epilogue issued (slot 46 + w), first in the list
                sub_l1[w].insert(0, float(np.median(st[:, 46 + w] - z)))
    init_sub = {}
    if np.all(st[:, 40] > 0):  # init sub-phases (slots 40-42) relative to the workgroup start
        for k, nm in ((40, "descriptors"), (41, "obs_issued"), (42, "barrier_reached")):
            if np.all(st[:, k] > 0):
                init_sub[nm] = float(np.median(st[:, k] - st[:, 0]))
    gru_sub = {}
    if np.all(st[:, 43] > 0):  # pipelined GRU stage (wave 0): entry, contraction done, epilogue done
        gru_sub = {"entry": float(np.median(st[:, 43] - st[:, 0])),
                   "contraction": float(np.median(st[:, 44] - st[:, 43])),
                   "epilogue": float(np.median(st[:, 45] - st[:, 44]))}
        for slot, name in ((56, "prologue_hidden_issued"), (57, "prologue_step_loop"), (58, "prologue_cell_call")):
            if np.all(st[:, slot] > 0):
                gru_sub[name] = float(np.median(st[:, slot] - st[:, 0]))
    blocks = {}
    if args.ctl and np.all(st[:, 51] > 0):  # the assembly's passes (slots 50-51, thread 0) from slot 5
        prev = st[:, 5]
        names = ("append", "shift") + (("append_again", "shift_again") if np.all(st[:, 53] > 0) else ())
        for b, name in enumerate(names):  # (the _again passes: GO2PI_DIAG_ASM2 builds)
            blocks[name] = float(np.median(st[:, 50 + b] - prev))
            prev = st[:, 50 + b]
    if np.all(st[:, 55] > 0):  # the pipeline's head tail (wave 0): partials summed, stored, from the head barrier
        hb = st[:, 6 + nl - 1]
        blocks["tail_partials"] = float(np.median(st[:, 54] - hb))
        blocks["tail_store"] = float(np.median(st[:, 55] - st[:, 54]))
        blocks["tail_end"] = float(np.median(st[:, 2] - st[:, 55]))
    if args.ctl:  # slot 5: inputs staged in LDS, 4: obs assembled, 15: obs published
        marks = [st[:, 0], st[:, 5], st[:, 4], st[:, 15]] + [st[:, 6 + l] for l in range(nl)] + [st[:, 2]]
        names = ["ctl_load", "assemble", "publish"] + [f"layer{l}" for l in range(nl)] + ["tail"]
    else:
        marks = [st[:, 0], st[:, 4]] + [st[:, 6 + l] for l in range(nl)] + [st[:, 2]]
        names = ["init"] + [f"layer{l}" for l in range(nl)] + ["tail"]
    phases = {n: float(np.median(b - a)) for n, a, b in zip(names, marks[:-1], marks[1:])}
    cyc = st[:, 2] - st[:, 0]
    rt = (st[:, 3] - st[:, 1]) / 100e6
    clk = cyc / rt
    # per XCD (workgroups are dispatched round-robin over the 8 XCDs: blockIdx % 8): where
    # the start and end spreads come from (late starts, slower clocks, longer lives)
    t0s = st[:, 1].min()
    per_xcd = {}
    for x in range(8):
        m = np.arange(st.shape[0]) % 8 == x
        if m.any():
            per_xcd[x] = {"start_us_med": float(np.median(st[m, 1] - t0s) / 100),
                          "start_us_max": float((st[m, 1] - t0s).max() / 100),
                          "end_us_med": float(np.median(st[m, 3] - t0s) / 100),
                          "end_us_max": float((st[m, 3] - t0s).max() / 100),
                          "cycles_med": float(np.median(cyc[m])), "clk_ghz_med": float(np.median(clk[m]) / 1e9)}
    out = {"lib": os.path.basename(os.environ.get("GO2PI_LIB", "default")), "waves": args.waves,
           "launches": n, "clock_ghz_median": float(np.median(clk) / 1e9),
           "clock_ghz_min": float(clk.min() / 1e9), "wg_cycles_median": float(np.median(cyc)),
           "wg_us_median": float(np.median(rt) * 1e6), "wg_us_max": float(rt.max() * 1e6),
           "launch_span_us": float((st[:, 3].max() - st[:, 1].min()) / 100),
           "event_us_per_launch": float(np.median(per_launch)),
           "wg_start_spread_us": float((st[:, 1].max() - st[:, 1].min()) / 100),
           "wg_end_spread_us": float((st[:, 3].max() - st[:, 3].min()) / 100),
           "phase_cycles_median": phases,
           "layer1_wave_marks": waves_l1,  # [entry, contraction done, epilogue done, barrier] cycles
           "pipeline_layer1_subphases": sub_l1, "init_subphases": init_sub, "gru_stage": gru_sub,
           "ctl_assembly_blocks": blocks, "per_xcd": per_xcd}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
