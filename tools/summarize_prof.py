#!/usr/bin/env python3
"""Condense rocprofv3 outputs of tools/profile.sh into profiles/ (committed).

Inputs (gpurun_out/prof_<tag>_{kt,fetch,write}/run_*.csv):
  kt    — kernel trace + stats: per-kernel average duration;
  fetch — FETCH_SIZE per dispatch (KiB), its own --pmc pass;
  write — WRITE_SIZE per dispatch (KiB), its own --pmc pass.
Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports exactly
half the bytes of a wide coalesced 16-B/lane read — the weight stream's shape —
so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B stores and
calibrated-enough for the 4-B action stores (their bytes are known: B x 12 x 4).
FETCH_SIZE counts L2 fabric requests, Infinity-Cache hits included: for this
kernel it is dominated by each XCD's L2 pulling the 2.2 MB weight set once.

Writes profiles/<round>_<tag>_kernel_stats.csv (verbatim copy),
profiles/<round>_<tag>_pmc.csv (per-kernel averages) and updates
profiles/pmc_summary.json {"workloads": {bench workload: {kernel: {...}}}}
that bench.py reads for roofline.traffic.
"""
import argparse
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def avg_counter(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="mlp")
    ap.add_argument("--round", default="r01")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--note", default="")
    ap.add_argument("--workload", required=True, help="bench.py workload the profile ran")
    args = ap.parse_args()
    src = lambda kind: os.path.join(args.src, f"prof_{args.tag}_{kind}")  # noqa: E731
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats_dst = os.path.join(prof, f"{args.round}_{args.tag}_kernel_stats.csv")
    shutil.copyfile(os.path.join(src("kt"), "run_kernel_stats.csv"), stats_dst)
    dur = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(stats_dst))}
    calls = {r["Name"]: int(r["Calls"]) for r in csv.DictReader(open(stats_dst))}
    fetch = avg_counter(os.path.join(src("fetch"), "run_counter_collection.csv"), "FETCH_SIZE")
    write = avg_counter(os.path.join(src("write"), "run_counter_collection.csv"), "WRITE_SIZE")
    rows = []
    summary_path = os.path.join(prof, "pmc_summary.json")
    try:
        summary = json.load(open(summary_path))
    except (OSError, ValueError):
        summary = {}
    summary.pop("kernels", None)
    import sys
    sys.path.insert(0, ROOT)
    from go2_onnx_controller_amd.provenance import kernel_source_digest
    digest = kernel_source_digest()  # the sources the profiled library was built from (bench.py checks it)
    wl = summary.setdefault("workloads", {}).setdefault(args.workload, {})
    for name in dur:
        if name.startswith("__amd"):
            continue
        f_kib, w_kib = fetch.get(name), write.get(name)
        hbm = None if f_kib is None or w_kib is None else (2.0 * f_kib + w_kib) * 1024.0
        rows.append([name, calls[name], round(dur[name], 1), f_kib, w_kib, hbm])
        wl[name] = {"avg_ns": dur[name], "fetch_size_kib": f_kib, "write_size_kib": w_kib,
                                    "hbm_bytes_per_launch": hbm, "source": os.path.basename(stats_dst),
                                    "correction": "read bytes = 2 x FETCH_SIZE (gfx950, 16-B/lane streams)",
                                    "note": args.note, "src_digest": digest}
    with open(os.path.join(prof, f"{args.round}_{args.tag}_pmc.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "calls", "avg_ns", "FETCH_SIZE_KiB", "WRITE_SIZE_KiB", "traffic_bytes_corrected"])
        w.writerows(rows)
    with open(summary_path, "w") as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)
    for r in rows:
        print(r)


if __name__ == "__main__":
    main()
