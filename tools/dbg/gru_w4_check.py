"""Debug: GRU policy, one step from h0 = 0: pipeline (default) and generic body
(GO2PI_NO_W4=1, 4 waves) against the fp64 oracle; per-16-column-tile errors."""
import os, subprocess, sys
import numpy as np
sys.path.insert(0, os.getcwd())
mode = sys.argv[1] if len(sys.argv) > 1 else "parent"
B = int(os.environ.get("B", "16"))
x = np.random.default_rng(0).standard_normal((B, 48)).astype(np.float32)
if mode == "child":
    from go2_onnx_controller_amd import Engine, synth
    path = synth.ensure_model("go2_gru_256")
    with Engine(path, max_batch=B, waves=4) as e:
        e.reset_hidden()
        y = e.run(x)
        h = e.get_hidden(B)
        print(e.batched_kernel, file=sys.stderr)
    np.savez(sys.argv[2], y=y, h=h)
else:
    from go2_onnx_controller_amd import synth
    from oracle import onnx_ref
    path = synth.ensure_model("go2_gru_256")
    g = onnx_ref.load(path)
    r = onnx_ref.run(g, {"observation": x.astype(np.float64), "h_in": np.zeros((1, B, 256))})
    want_h, want_y = r["h_out"][0], r["action"]
    print("x", x[0, :2], x[0, 47], x[1, :2], x[1, 47])
    print("want h1", want_h[0, :2], want_h[0, 255], want_h[1, :2], want_h[1, 255])
    for tag, env in (("w4", {}), ("gen", {"GO2PI_NO_W4": "1"})):
        subprocess.run([sys.executable, __file__, "child", f"gpurun_out/gru_{tag}.npz"], env={**os.environ, **env}, check=True)
        a = np.load(f"gpurun_out/gru_{tag}.npz")
        eh = np.abs(a["h"] - want_h)
        print(tag, "h err", float(eh.max()), "y err", float(np.abs(a["y"] - want_y).max()))
        print("   per tile", np.round(eh.reshape(B, 16, 16).max(axis=(0, 2)), 4).tolist())
        print("   per row ", np.round(eh.max(1), 4).tolist())
