"""CPU: the product's ONNX loader under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY §5 "Race detection / sanitizers").

go2_onnx_controller_amd/csrc/onnx_model.cpp parses caller-supplied files (the
reference hands its path to onnxruntime's session, onnx_actor.cpp:16). Here it is
built host-only with -fsanitize=address,undefined -fno-sanitize-recover=all beside
tests/cpp/fuzz_loader.cpp (parse_onnx + inspect_json, exactly what
go2pi_inspect_model runs), and fed hypothesis-generated mutations of the shipped
model and of the loader-breadth graphs: truncations, bit flips, oversized varints
(dims, lengths, field keys) and spliced byte runs. Every input must load or end in
a clean exception (GO2PI_E_MODEL at the ABI); no crash, no sanitizer report.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

import graphs
from conftest import ROOT, SHIPPED

EXE = os.path.join(ROOT, "build", "fuzz_loader_asan")
SRC = os.path.join(ROOT, "go2_onnx_controller_amd", "csrc")


@pytest.fixture(scope="module")
def harness():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    subprocess.run(["g++", "-std=c++20", "-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-I" + SRC, os.path.join(ROOT, "tests", "cpp", "fuzz_loader.cpp"),
                    os.path.join(SRC, "onnx_model.cpp"), "-o", EXE], check=True)
    return EXE


def _run(exe, paths):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe] + [str(p) for p in paths], capture_output=True, text=True, errors="replace", timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    lines = r.stdout.splitlines()
    assert len(lines) == len(paths)
    return lines


BASES = [open(SHIPPED, "rb").read()] + [graphs.variant_bytes(k, 3) for k in graphs.VARIANTS]


def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


@st.composite
def mutated(draw):
    data = bytearray(BASES[draw(st.integers(0, len(BASES) - 1))])
    kind = draw(st.sampled_from(["truncate", "flip", "varint", "splice", "mix"]))
    n = len(data)
    if kind in ("truncate", "mix"):
        data = data[: draw(st.integers(0, n))]
    if kind in ("flip", "mix") and data:
        for _ in range(draw(st.integers(1, 8))):
            i = draw(st.integers(0, len(data) - 1))
            data[i] ^= 1 << draw(st.integers(0, 7))
    if kind == "varint" and data:
        # an oversized varint (a huge dim, length or key) over a random position
        i = draw(st.integers(0, len(data) - 1))
        big = draw(st.sampled_from([(1 << 31) - 1, 1 << 31, (1 << 32) + 5, (1 << 62), (1 << 64) - 1, 1 << 40]))
        v = _varint(big)
        data[i:i + len(v)] = v
    if kind == "splice" and data:
        i = draw(st.integers(0, len(data)))
        data[i:i] = draw(st.binary(min_size=1, max_size=64))
    return bytes(data)


@settings(max_examples=400, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
@given(cases=st.lists(mutated(), min_size=25, max_size=25))
def _collect(cases, sink):
    sink.extend(cases)


def test_loader_sanitized_on_mutated_models(harness, tmp_path):
    cases = []
    _collect(sink=cases)
    assert len(cases) >= 2000
    paths = []
    for i, data in enumerate(cases):
        p = tmp_path / f"m{i}.onnx"
        p.write_bytes(data)
        paths.append(p)
    lines = []
    for k in range(0, len(paths), 500):  # (argument-list size)
        lines += _run(harness, paths[k:k + 500])
    assert all(l.startswith(("ok ", "error onnx: ", "error ")) for l in lines)
    assert sum(l.startswith("error") for l in lines) > len(lines) // 4  # most mutations are refused


def test_loader_sanitized_on_valid_graphs(harness, tmp_path, synth_path):
    """The unmutated inputs load cleanly under the sanitizers (every supported graph form)."""
    paths = [SHIPPED] + [graphs.write(tmp_path, k) for k in graphs.VARIANTS] + \
        [synth_path(n) for n in ("go2_mlp_512", "go2_gru_256", "go2_lstm_256", "gru_small", "lstm_small")]
    lines = _run(harness, paths)
    assert all(l.startswith("ok ") for l in lines), lines


def test_loader_sanitized_on_oversized_dims(harness, tmp_path):
    """Tensor dims whose product overflows, negative dims and a huge element count are
    refused with a message, not undefined behaviour or an allocation of the claimed size."""
    from go2_onnx_controller_amd import onnx_writer as ow
    W = np.zeros((4, 4), np.float32)
    good = ow.tensor("W", W)
    cases = []
    for dims in ([1 << 40, 1 << 40], [-1, 16], [1 << 62, 4], [4, (1 << 31)], [0, 4]):
        body = b"".join(ow.f_varint(1, d & ((1 << 64) - 1)) for d in dims) + good[good.index(ow.f_varint(2, 1)):]
        nodes = [ow.node("Gemm", ["obs", "W"], ["act"], "", [ow.attr_int("transB", 1)])]
        g = b"".join(ow.f_bytes(1, n) for n in nodes) + ow.f_bytes(5, body) + \
            ow.f_bytes(11, ow.value_info("obs", ["N", 4])) + ow.f_bytes(12, ow.value_info("act", ["N", 4]))
        cases.append(ow.f_varint(1, 8) + ow.f_bytes(7, g) + ow.f_bytes(8, ow.f_varint(2, 17)))
    paths = []
    for i, data in enumerate(cases):
        p = tmp_path / f"d{i}.onnx"
        p.write_bytes(data)
        paths.append(p)
    lines = _run(harness, paths)
    assert all(l.startswith("error onnx: ") for l in lines), lines
