#!/usr/bin/env python3
"""Batch-1 resident act() timeline (diagnostics): where a request's time goes.

Needs a library whose resident kernel records wall-clock stamps
(GO2PI_DIAG_RESCLK), built beside the default one:

  cd go2_onnx_controller_amd/csrc && hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 \\
      -I../../include -DGO2PI_DIAG_RESCLK -c resident.hip -o ../lib/diag/resident_clk.o && \\
  hipcc -shared -fPIC --offload-arch=gfx950 -o ../lib/diag/libgo2pi_resclk.so ../lib/kernels.o \\
      ../lib/kernels_w4_t2.o ../lib/kernels_w4_t4.o ../lib/kernels_w4_t8.o ../lib/kernels_gen_w4.o \\
      ../lib/kernels_gen_w8.o ../lib/kernels_gen_w16.o ../lib/diag/resident_clk.o ../lib/engine.o ../lib/onnx_model.o

  GO2PI_LIB=$PWD/go2_onnx_controller_amd/lib/diag/libgo2pi_resclk.so python3 tools/res_timeline.py

Stamps (100 MHz wall clock, 10 ns) per request, relative to workgroup 0 seeing the
request on the host: workgroup 0 (0 seen, 1 mirror stored, 2 waves released,
3 layer 0 done, 2l+2 layer l input ready, 2l+3 layer l published / done written)
and workgroup 17 (another XCD; same slots + 16). Host p50 beside them.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = {0: "seen", 1: "mirror stored", 2: "waves released", 3: "layer0 done", 10: "layer1 fma done",
         12: "layer1 partials written",
         13: "layer1 partials visible", 14: "layer1 wave0 stored"}
for _l in range(1, 4):
    NAMES[2 * _l + 2] = f"layer{_l} input ready"
    NAMES[2 * _l + 3] = f"layer{_l} published"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="go2_mlp_512")
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "res_timeline.json"))
    ap.add_argument("--ctl", action="store_true",
                    help="time the controller tick (go2pi_controller_step, batch 1) instead of act()")
    ap.add_argument("--form", choices=["multi", "one", "wide"], default="multi",
                    help="the resident kernel the engine runs: multi-workgroup (policy_resident_kernel) or the "
                         "single-workgroup policy_resident1_kernel (r04; GO2PI_RES_MULTI=1 forces multi)")
    args = ap.parse_args()
    os.environ["GO2PI_DIAG_STAMPS"] = "1"
    import numpy as np
    from go2_onnx_controller_amd import Engine, synth
    path = os.path.join(ROOT, "tests", "golden", "model.onnx") if args.model == "shipped" \
        else synth.ensure_model(args.model)
    with Engine(path, device=0, max_batch=4096, resident_ms=100) as e:
        x = np.random.default_rng(2).standard_normal((1, e.in_dim)).astype(np.float32)
        y = np.empty((1, e.out_dim), np.float32)
        ts = []
        st = np.zeros((1, 36), np.float32)
        st[0, 0] = 1.0
        for i in range(args.iters):
            x[0, i % e.in_dim] += 1e-3
            t0 = time.perf_counter_ns()
            if args.ctl:
                st[0, 7 + i % 12] += 1e-3
                e.controller_step(st, x, y)
            else:
                e.run_ptr(x.ctypes.data, y.ctypes.data, 1)
            ts.append((time.perf_counter_ns() - t0) / 1e3)
        st = e.diag_stamps(512 * 32).astype(np.int64).reshape(512, 32)  # syncs: waits for the idle exit
    ts.sort()
    if args.form == "one":
        return one_workgroup(args, st, ts, np)
    if args.form == "wide":
        return wide(args, st, ts, np, e.resident_kernel)
    rows = st[(st[:, 0] > 0) & (st[:, 9] > 0)]
    base = rows[:, 0:1]
    rel = (rows - base) * 10.0 / 1e3  # us
    med = {}
    for s in range(32):
        col = rows[:, s]
        ok = col > 0
        if ok.sum() < len(rows) // 2:
            continue
        if s % 16 in (11, 15):  # shader-clock stamps, not wall clock
            continue
        name = ("wg0 " if s < 16 else "wg17 ") + NAMES.get(s % 16, str(s % 16))
        med[name] = round(float(np.median(rel[ok, s])), 3)
    # shader clock over waves released -> layer 2 published (slots 15 / 11: s_memtime)
    dt_us = (rows[:, 7] - rows[:, 2]) * 10.0 / 1e3
    ghz = (rows[:, 11] - rows[:, 15]) / np.maximum(dt_us, 1e-3) / 1e3
    med.pop("wg0 15", None)
    med.pop("wg0 11", None)
    # the gap between a request's done and the next one's seen = host side + PCIe
    gaps = (rows[1:, 0] - rows[:-1, 9]) * 10.0 / 1e3
    out = {"model": args.model, "requests_stamped": int(len(rows)), "host_p50_us": ts[len(ts) // 2],
           "host_p99_us": ts[int(len(ts) * 0.99)], "median_us_from_wg0_seen": med,
           "median_done_to_next_seen_us": round(float(np.median(gaps)), 3),
           "shader_clock_ghz_median": round(float(np.median(ghz)), 3)}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


def one_workgroup(args, st, ts, np):
    """policy_resident1_kernel stamps (100 MHz wall clock): 0 request seen by the
    polling wave, 1 layer 0's input staged, 2 + l layer l's outputs in LDS (hidden
    layers), 8 the answer's granule stores issued (wave 1's head output)."""
    rows = st[(st[:, 0] > 0) & (st[:, 8] > 0)]
    rel = (rows - rows[:, 0:1]) * 10.0 / 1e3
    names = {1: "input staged", 8: "answer issued", 9: "done word (controller form)",
             10: "request staged (controller form: before the assembly)"}
    for l in range(6):
        names[2 + l] = f"layer{l} done"
    med, prev, at = {}, 0.0, {}
    for s_ in names:
        ok = rows[:, s_] > 0
        if ok.sum() >= len(rows) // 2:
            at[s_] = float(np.median(rel[ok, s_]))
    for s_ in sorted(at, key=lambda k: at[k]):  # in time order
        med[names[s_]] = {"at_us": round(at[s_], 3), "step_us": round(at[s_] - prev, 3)}
        prev = at[s_]
    gaps = (rows[1:, 0] - rows[:-1, 8]) * 10.0 / 1e3
    # shader clock (s_memtime, slots 13..30) over the wall clock from seen (15) to answer (14)
    dwall = (rows[:, 8] - rows[:, 0]) * 10e-9
    ghz = (rows[:, 14] - rows[:, 15]) / np.maximum(dwall, 1e-9) / 1e9
    cyc = {}
    marks = [(11, "request staged (controller form)"), (19, "controller parameters loaded"),
             (20, "appended values stored"), (21, "shifted values stored"), (22, "appended again (GO2PI_DIAG_ASM2)"),
             (23, "shifted again (GO2PI_DIAG_ASM2)"), (13, "input staged")]
    act1_ctl = (rows[:, 11] > 0).sum() >= len(rows) // 2  # (its slots 19-21 are the assembly's)
    for l in range(3):
        if l == 0 or not act1_ctl:
            marks += [(16 + 3 * l, f"layer{l} fma done"), (17 + 3 * l, f"layer{l} group sums done"),
                      (18 + 3 * l, f"layer{l} outputs stored")]
        marks += [(25 + l, f"layer{l} barrier passed")]
    marks += [(14, "answer issued")]
    prev = rows[:, 15]
    for s_, nm in marks:
        ok = rows[:, s_] > 0
        if ok.sum() < len(rows) // 2:
            continue
        cyc[nm] = float(np.median((rows[ok, s_] - prev[ok])))
        prev = np.where(ok, rows[:, s_], prev)
    out = {"model": args.model, "kernel": ("policy_resident1_kernel (r04 form, GO2PI_RES_R1W=1)" if os.environ.get("GO2PI_RES_R1W") else "policy_act1_kernel (one workgroup, r05)"),
           "shader_clock_ghz_median": round(float(np.median(ghz)), 3),
           "wave0_cycles_since_previous_mark": cyc,
           "requests_stamped": int(len(rows)), "host_p50_us": ts[len(ts) // 2], "host_p99_us": ts[int(len(ts) * 0.99)],
           "median_from_request_seen": med,
           "median_answer_to_next_seen_us": round(float(np.median(gaps)), 3)}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


def wide(args, st, ts, np, kernel):
    """policy_wide_kernel stamps (r06, resident_wide.hip W_STAMP; 100 MHz wall clock) of
    workgroups 0 and 17 (another XCD), per request: 0 request seen by the workgroup's
    polling wave, 1 layer 0 done (first compute wave), 2 + l sliced layer l's input in
    registers (l >= 1: after the granule sweep), 6 the last sliced layer's outputs in
    LDS, 7 the head partials published, 8 every workgroup's partials gathered
    (workgroup 0), 9 the answer stored. Times relative to workgroup 0 seeing the request."""
    rows = st[(st[:, 0] > 0) & (st[:, 9] > 0)]
    rel = (rows - rows[:, 0:1]) * 10.0 / 1e3
    names = {0: "request seen", 1: "layer0 done", 3: "layer2 input swept", 4: "layer3 input swept",
             6: "last sliced layer stored", 7: "partials published", 8: "partials gathered", 9: "answer stored"}
    med = {}
    for base, wgn in ((0, "wg0"), (16, "wg17")):
        for s_, nm in names.items():
            ok = rows[:, base + s_] > 0
            if ok.sum() >= len(rows) // 2:
                med[f"{wgn} {nm}"] = round(float(np.median(rel[ok, base + s_])), 3)
    med = dict(sorted(med.items(), key=lambda kv: kv[1]))
    gaps = (rows[1:, 0] - rows[:-1, 9]) * 10.0 / 1e3
    out = {"model": args.model, "kernel": kernel, "requests_stamped": int(len(rows)),
           "host_p50_us": ts[len(ts) // 2], "host_p99_us": ts[int(len(ts) * 0.99)],
           "median_us_from_wg0_seen": med,
           "median_answer_to_next_seen_us": round(float(np.median(gaps)), 3)}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
