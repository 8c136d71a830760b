"""CPU: the drop-in boundary without a GPU.

* libgo2pi.so loads and exports every symbol include/go2pi.h declares;
* the product's C++ ONNX loader (go2pi_inspect_model, no device) lowers every
  supported graph form to the same program the oracle's independent decoder
  sees (dims, activations, weight/bias checksums) and rejects unsupported ones;
* without a HIP device go2pi_create fails loudly (GO2PI_E_DEVICE) — there is no
  CPU fallback in the product;
* include/onnx_actor.hpp compiles in the reference controller's call pattern
  and links against libonnx_actor.so (controller.cpp:25,49,215).
"""
import ctypes
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

import graphs
from conftest import ROOT, SHIPPED

HEADER = os.path.join(ROOT, "include", "go2pi.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(go2pi_[a-z_]+)\s*\(", src)))


def test_header_symbols_exported():
    from go2_onnx_controller_amd import engine
    L = engine.lib()
    declared = header_functions()
    assert set(declared) == set(engine.EXPORTS), "engine.EXPORTS out of sync with go2pi.h"
    for name in declared:
        assert hasattr(L, name), name
    assert engine.version().startswith("go2pi")


def test_actor_library_exports():
    from go2_onnx_controller_amd import ACTOR_LIB_PATH
    out = subprocess.run(["nm", "-DC", ACTOR_LIB_PATH], capture_output=True, text=True, check=True).stdout
    for sym in ("ONNXActor::ONNXActor(", "ONNXActor::act()", "ONNXActor::print_model_info()",
                "ONNXActor::check_dims()", "ONNXActor::~ONNXActor()"):
        assert sym in out, sym


def _oracle_layers(path):
    from oracle import mlp_ref, onnx_ref
    return mlp_ref.mlp_layers(onnx_ref.load(path))


ACT_CODE = {"none": 0, "Elu": 1, "Relu": 2, "Tanh": 3, "Sigmoid": 4, "LeakyRelu": 5, "Clip": 6, "Selu": 7,
            "Softplus": 8, "HardSigmoid": 9, "HardSwish": 10, "Softsign": 11}


def _check_layers(view, layers):
    assert len(view["layers"]) == len(layers)
    for v, (W, b, act, alpha, beta) in zip(view["layers"], layers):
        assert (v["N"], v["K"]) == W.shape
        assert v["act"] == ACT_CODE[act]
        assert v["alpha"] == pytest.approx(alpha, abs=1e-7)
        assert v["beta"] == pytest.approx(beta, abs=1e-7)
        assert v["w_sum"] == pytest.approx(float(W.astype(np.float64).sum()), rel=1e-9, abs=1e-9)
        assert v["b_sum"] == pytest.approx(float(b.astype(np.float64).sum()), rel=1e-9, abs=1e-9)


def test_loader_shipped_model():
    from go2_onnx_controller_amd import engine
    v = engine.inspect_model(SHIPPED)
    assert v["inputs"] == [{"name": "observation", "shape": [1, 98]}]
    assert v["outputs"] == [{"name": "action", "shape": [1, 12]}]
    assert (v["in_dim"], v["out_dim"], v["ir_version"], v["opset"]) == (98, 12, 8, 17)
    _check_layers(v, _oracle_layers(SHIPPED))


@pytest.mark.parametrize("name", ["go2_mlp_512", "mlp_small_relu", "mlp_small_tanh"])
def test_loader_synthetic(synth_path, name):
    from go2_onnx_controller_amd import engine
    p = synth_path(name)
    _check_layers(engine.inspect_model(p), _oracle_layers(p))


@pytest.mark.parametrize("name", ["gru_small", "go2_gru_256", "gru_lbr0_small"])
def test_loader_gru(synth_path, name):
    from go2_onnx_controller_amd import engine
    from oracle import onnx_ref
    p = synth_path(name)
    v = engine.inspect_model(p)
    g = onnx_ref.load(p)
    gru = next(n for n in g.nodes if n.op_type == "GRU")
    W, R, B = (g.inits[gru.inputs[i]].astype(np.float64) for i in (1, 2, 3))
    assert v["gru"]["H"] == R.shape[2] and v["gru"]["I"] == W.shape[2]
    assert v["gru"]["lbr"] == (0 if "lbr0" in name else 1)
    assert v["gru"]["w_sum"] == pytest.approx(W.sum(), rel=1e-9)
    assert v["gru"]["r_sum"] == pytest.approx(R.sum(), rel=1e-9)
    assert v["gru"]["b_sum"] == pytest.approx(B.sum(), rel=1e-9)
    assert [io["name"] for io in v["inputs"]] == ["observation", "h_in"]
    assert [io["name"] for io in v["outputs"]] == ["action", "h_out"]
    assert v["layers"][0]["K"] == R.shape[2]


@pytest.mark.parametrize("kind", graphs.VARIANTS)
def test_loader_graph_variants(tmp_path, kind):
    from go2_onnx_controller_amd import engine
    p = graphs.write(tmp_path, kind)
    v = engine.inspect_model(p)
    _check_layers(v, _oracle_layers(p))
    if kind == "normalized_tanh_clip":
        assert v["pre_sub"] == 24 and v["pre_div"] == 24
        assert v["clip"] == pytest.approx([-0.5, 0.75])
    if kind == "relu6_mid_clip":  # the Clip is layer 0's activation, not an output clip
        assert v["clip"] == [-1e308, 1e308] and v["layers"][0]["act"] == 6
        assert (v["layers"][0]["alpha"], v["layers"][0]["beta"]) == (0.0, 6.0)
    if kind == "const_scales":
        assert v["pre_mul"] == 20 and v["pre_clip"] == pytest.approx([-2.5, 2.0])
        assert v["clip"] == pytest.approx([-0.4, 0.9]) and v["post_scale"] == 0.25
    if kind == "slice_concat_blocks":  # two blocks' (x - mean) / std: one per-column prologue
        assert (v["in_dim"], v["pre_sub"], v["pre_div"], v["pre_mul"]) == (98, 98, 98, 0)
    if kind == "slice_concat_mixed":  # a scalar Mul, an Identity, Sub + Mul; one shared Clip
        assert (v["pre_sub"], v["pre_div"], v["pre_mul"]) == (30, 0, 30)
        assert v["pre_clip"] == pytest.approx([-1.2, 1.1])


@pytest.mark.parametrize("kind,msg", [("conv", "unsupported operator 'Conv'"),
                                      ("dynamic_weight", "not an initializer"),
                                      ("clip_after_act_mid", "only supported at the end of the graph"),
                                      ("mul_then_clip_out", "Clip after a Mul"),
                                      ("vector_mul_out", "per-feature Mul after the final activation"),
                                      ("slice_reordered", "cover its columns in order"),
                                      ("slice_clip_differs", "Clip bounds differ"),
                                      ("slice_sub_reversed", "Sub in the observation front-end must take the "
                                                             "observation as its first input")])
def test_loader_rejects_unsupported(tmp_path, kind, msg):
    from go2_onnx_controller_amd import engine
    with pytest.raises(engine.Go2piError, match=msg):
        engine.inspect_model(graphs.write(tmp_path, kind))


def test_loader_rejects_missing_and_garbage(tmp_path):
    from go2_onnx_controller_amd import engine
    with pytest.raises(engine.Go2piError, match="cannot open"):
        engine.inspect_model(str(tmp_path / "nope.onnx"))
    bad = tmp_path / "bad.onnx"
    bad.write_bytes(b"\xff\xff\xff\xff\x0f" * 7)
    with pytest.raises(engine.Go2piError, match="GO2PI_E_MODEL"):
        engine.inspect_model(str(bad))


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from go2_onnx_controller_amd import Engine, Go2piError
    with pytest.raises(Go2piError, match="no CPU fallback"):
        Engine(SHIPPED)
    # model errors are reported before device errors
    with pytest.raises(Go2piError, match="GO2PI_E_MODEL"):
        Engine(os.path.join(ROOT, "README.md"))


def test_opts_struct_layout_matches_header():
    """ctypes mirror of go2pi_opts / go2pi_cost vs the C compiler's view."""
    from go2_onnx_controller_amd.engine import Cost, CtlParams, Opts
    src = r'''
#include <stddef.h>
#include <stdio.h>
#include "go2pi.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu ", sizeof(go2pi_opts), offsetof(go2pi_opts, obs_mean),
         offsetof(go2pi_opts, action_scale), sizeof(go2pi_cost), offsetof(go2pi_cost, n_layers),
         offsetof(go2pi_opts, small_batch));
  printf("%zu %zu %zu %zu ", sizeof(go2pi_ctl_params), offsetof(go2pi_ctl_params, gravity_w),
         offsetof(go2pi_ctl_params, action_scale), offsetof(go2pi_ctl_params, q0));
  go2pi_opts o;
  go2pi_default_opts(&o);
  printf("%zu %d\n", offsetof(go2pi_opts, resident_ms), o.resident_ms);
  return 0;
}'''
    exe = os.path.join(ROOT, "build", "abi_layout")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    lib = os.path.join(ROOT, "go2_onnx_controller_amd", "lib")
    subprocess.run(["gcc", "-x", "c", "-", "-I", os.path.join(ROOT, "include"), "-o", exe, "-L", lib, "-lgo2pi",
                    f"-Wl,-rpath,{lib}"], input=src, text=True, check=True)
    got = [int(x) for x in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    # the resident kernel is opt-in: go2pi_default_opts leaves resident_ms at 0
    assert got == [ctypes.sizeof(Opts), Opts.obs_mean.offset, Opts.action_scale.offset, ctypes.sizeof(Cost),
                   Cost.n_layers.offset, Opts.small_batch.offset, ctypes.sizeof(CtlParams),
                   CtlParams.gravity_w.offset, CtlParams.action_scale.offset, CtlParams.q0.offset,
                   Opts.resident_ms.offset, 0]


def build_controller_shape():
    exe = os.path.join(ROOT, "build", "controller_shape")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    lib = os.path.join(ROOT, "go2_onnx_controller_amd", "lib")
    subprocess.run(["g++", "-std=c++20", "-O2", "-Wall", "-Wextra", "-Wpedantic", "-Werror",
                    "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "controller_shape.cpp"),
                    "-L" + lib, "-lonnx_actor", "-Wl,-rpath," + lib, "-o", exe], check=True)
    return exe


def test_dropin_header_compiles_and_links():
    """The reference controller's use of the header compiles unchanged (-Wall -Wextra
    -Wpedantic as onnx_controller/CMakeLists.txt:33 adds) and links."""
    exe = build_controller_shape()
    import torch
    if not torch.cuda.is_available():
        r = subprocess.run([exe, SHIPPED], capture_output=True, text=True)
        assert r.returncode == 3 and "no CPU fallback" in r.stdout


def test_cmake_package_config(tmp_path):
    """find_package(onnx_inference) exports onnx_inference::onnx_actor and an
    `onnxruntime` target, as onnx_controller/CMakeLists.txt:45-51 links them."""
    cmake = shutil.which("cmake")
    if cmake is None:
        pytest.skip("cmake not available")
    proj = tmp_path / "consumer"
    proj.mkdir()
    (proj / "CMakeLists.txt").write_text(
        "cmake_minimum_required(VERSION 3.21)\nproject(consumer CXX)\nset(CMAKE_CXX_STANDARD 20)\n"
        "find_package(onnx_inference REQUIRED)\n"
        f"add_executable(controller_shape {os.path.join(ROOT, 'tests', 'cpp', 'controller_shape.cpp')})\n"
        "target_link_libraries(controller_shape onnx_inference::onnx_actor onnxruntime)\n")
    build = tmp_path / "b"
    r = subprocess.run([cmake, "-S", str(proj), "-B", str(build),
                        f"-Donnx_inference_DIR={os.path.join(ROOT, 'cmake')}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run([cmake, "--build", str(build)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("name", ["lstm_small", "go2_lstm_256"])
def test_loader_lstm(synth_path, name):
    """The C++ loader's view of an ONNX LSTM policy (gates i, o, f, c; h and c graph I/O)
    against the oracle's own protobuf decoder: dims, cell kind and weight checksums."""
    from go2_onnx_controller_amd.engine import inspect_model
    from oracle import onnx_ref
    p = synth_path(name)
    v = inspect_model(p)
    g = onnx_ref.load(p)
    lstm = next(n for n in g.nodes if n.op_type == "LSTM")
    W, R, B = (g.inits[lstm.inputs[i]].astype(np.float64) for i in (1, 2, 3))
    assert v["gru"]["cell"] == "LSTM"
    assert v["gru"]["H"] == R.shape[2] and v["gru"]["I"] == W.shape[2] and 4 * R.shape[2] == W.shape[1]
    assert v["gru"]["w_sum"] == pytest.approx(W.sum(), rel=1e-9)
    assert v["gru"]["r_sum"] == pytest.approx(R.sum(), rel=1e-9)
    assert v["gru"]["b_sum"] == pytest.approx(B.sum(), rel=1e-9)
    assert [i["name"] for i in v["inputs"]] == ["observation", "h_in", "c_in"]
    assert [o["name"] for o in v["outputs"]] == ["action", "h_out", "c_out"]
    assert v["layers"][0]["K"] == R.shape[2]


def test_loader_rejects_unsupported_lstm_forms(synth_path):
    """LSTM peepholes / input_forget / cell clip are refused at load with a clear message."""
    from go2_onnx_controller_amd import onnx_writer as ow
    from go2_onnx_controller_amd.engine import Go2piError, inspect_model
    import tempfile
    H, I = 16, 4
    rng = np.random.default_rng(0)
    W = rng.standard_normal((1, 4 * H, I)).astype(np.float32)
    R = rng.standard_normal((1, 4 * H, H)).astype(np.float32)
    Wh = rng.standard_normal((3, H)).astype(np.float32)
    for attrs, extra_in, msg in (([ow.attr_int("input_forget", 1)], [], "input_forget"),
                                 ([ow.attr_float("clip", 3.0)], [], "clip"),
                                 ([], ["lstm.P"], "peephole")):
        inits = [("lstm.W", W), ("lstm.R", R), ("axes0", np.array([0], np.int64)), ("w", Wh),
                 ("lstm.P", np.zeros((1, 3 * H), np.float32))]
        ins = ["x_seq", "lstm.W", "lstm.R", "", "", "", ""] + extra_in
        nodes = [ow.node("Unsqueeze", ["observation", "axes0"], ["x_seq"], "u"),
                 ow.node("LSTM", ins, ["Y", "h_out"], "lstm", [ow.attr_int("hidden_size", H)] + attrs),
                 ow.node("Squeeze", ["h_out", "axes0"], ["h"], "s"),
                 ow.node("Gemm", ["h", "w"], ["action"], "g", [ow.attr_int("transB", 1)])]
        data = ow.model(nodes, inits, [("observation", ["batch", I])], [("action", ["batch", 3])])
        with tempfile.NamedTemporaryFile(suffix=".onnx") as fh:
            fh.write(data)
            fh.flush()
            with pytest.raises(Go2piError, match=msg):
                inspect_model(fh.name)


def test_loader_state_io_traced_by_name(tmp_path):
    """An LSTM policy whose graph lists its state I/O as (c, h): the loader maps them
    to the cell's initial_h / initial_c and Y_h / Y_c by name and lists them (h, c),
    the engine's state-row order (they were taken by position)."""
    from go2_onnx_controller_amd import onnx_writer as ow
    from go2_onnx_controller_amd.engine import inspect_model
    H, I = 16, 6
    rng = np.random.default_rng(0)
    inits = [("lstm.W", rng.standard_normal((1, 4 * H, I)).astype(np.float32)),
             ("lstm.R", rng.standard_normal((1, 4 * H, H)).astype(np.float32)),
             ("axes0", np.array([0], np.int64)), ("w", rng.standard_normal((3, H)).astype(np.float32))]
    nodes = [ow.node("Unsqueeze", ["observation", "axes0"], ["x_seq"], "u"),
             ow.node("Identity", ["cc_in"], ["c0"], "ic"),
             ow.node("LSTM", ["x_seq", "lstm.W", "lstm.R", "", "", "hh_in", "c0"], ["Y", "h_o", "c_o"], "lstm",
                     [ow.attr_int("hidden_size", H)]),
             ow.node("Identity", ["c_o"], ["cc_out"], "oc"),
             ow.node("Squeeze", ["h_o", "axes0"], ["h"], "s"),
             ow.node("Identity", ["h_o"], ["hh_out"], "oh"),
             ow.node("Gemm", ["h", "w"], ["action"], "g", [ow.attr_int("transB", 1)])]
    data = ow.model(nodes, inits, [("observation", ["batch", I]), ("cc_in", [1, "batch", H]),
                                   ("hh_in", [1, "batch", H])],
                    [("action", ["batch", 3]), ("cc_out", [1, "batch", H]), ("hh_out", [1, "batch", H])])
    p = tmp_path / "lstm_ch.onnx"
    p.write_bytes(data)
    v = inspect_model(str(p))
    assert [i["name"] for i in v["inputs"]] == ["observation", "hh_in", "cc_in"]
    assert [o["name"] for o in v["outputs"]] == ["action", "hh_out", "cc_out"]
