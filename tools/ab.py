#!/usr/bin/env python3
"""Same-box A/B of engine variants on the GPU box (diagnostics).

Each variant is NAME[=LIB][,ENV=VALUE...]: LIB 'default' (lib/libgo2pi.so) or a
name under lib/diag (libgo2pi_<LIB>.so); ENV settings are exported to that run
only (e.g. GO2PI_NO_PLAIN=1). Rounds alternate the variants so box drift hits
them all alike; per variant the bench's kernel_us (HIP events on the launching
stream) is printed per round and summarised as min / median.

  python3 tools/ab.py --rounds 3 --workload go2_mlp_512_b4096 \
      new r02=r02 noplain,GO2PI_NO_PLAIN=1
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse(spec):
    parts = spec.split(",")
    name, _, lib = parts[0].partition("=")
    env = dict(p.split("=", 1) for p in parts[1:])
    lib = lib or "default"
    path = os.path.join(ROOT, "go2_onnx_controller_amd", "lib",
                        "libgo2pi.so" if lib == "default" else os.path.join("diag", f"libgo2pi_{lib}.so"))
    return name, path, env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--workload", default="go2_mlp_512_b4096")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ab"))
    ap.add_argument("--ctl", action="store_true",
                    help="compare the controller tick (controller_tick.tick_us, 4096 robots) instead of kernel_us")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    vs = [parse(v) for v in args.variants]
    res = {v[0]: [] for v in vs}
    for r in range(args.rounds):
        for name, path, env in vs:
            e = dict(os.environ, GO2PI_LIB=path, **env)
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", args.workload, "--steps",
                   str(args.steps), "--no-cpu", "--no-latency", "--no-gru"] + ([] if args.ctl else ["--no-ctl"])
            p = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=300)
            if p.returncode:
                print(f"{name}: bench failed\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
            if args.ctl:
                res[name].append(d["controller_tick"]["tick_us"])
                print(f"round {r} {name:12s} tick {d['controller_tick']['tick_us']:8.3f} us", flush=True)
            else:
                res[name].append(d["kernel_us"])
                print(f"round {r} {name:12s} {d['kernel_us']:8.3f} us  frac {d['roofline']['frac']:.4f}  {d['kernel']}",
                      flush=True)
    summary = {n: {"min": min(v), "median": statistics.median(v), "all": v} for n, v in res.items()}
    for n, s in summary.items():
        print(f"{n:12s} min {s['min']:8.3f}  median {s['median']:8.3f}")
    with open(os.path.join(args.out, f"ab_{args.workload}{'_ctl' if args.ctl else ''}.json"), "w") as fh:
        json.dump(summary, fh, indent=1)


if __name__ == "__main__":
    main()
