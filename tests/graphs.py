"""Small ONNX policy graphs exercising the loader's supported patterns
(SURVEY §8f.3 "ONNX loader breadth"): Gemm with transB=0 / alpha / beta,
MatMul + Add, Sub/Div input normalisation, LeakyRelu / Sigmoid, trailing
Tanh + Clip. Built with the repo's own writer; evaluated by the oracle."""
import numpy as np

from go2_onnx_controller_amd import onnx_writer as ow


def _rng(seed):
    return np.random.default_rng(seed)


def variant_bytes(kind: str, seed: int = 0) -> bytes:
    r = _rng(seed)
    f32 = lambda *s: (r.standard_normal(s) * 0.3).astype(np.float32)  # noqa: E731
    if kind == "gemm_transB0_alpha_beta":
        W1, b1, W2, b2 = f32(20, 40), f32(40), f32(40, 7), f32(7)   # [K, N] layout (transB=0)
        nodes = [ow.node("Gemm", ["obs", "W1", "b1"], ["h1"], "g1",
                         [ow.attr_float("alpha", 0.5), ow.attr_float("beta", 2.0), ow.attr_int("transB", 0)]),
                 ow.node("LeakyRelu", ["h1"], ["a1"], "lr", [ow.attr_float("alpha", 0.1)]),
                 ow.node("Gemm", ["a1", "W2", "b2"], ["act"], "g2", [ow.attr_int("transB", 0)])]
        inits = [("W1", W1), ("b1", b1), ("W2", W2), ("b2", b2)]
        return ow.model(nodes, inits, [("obs", ["N", 20])], [("act", ["N", 7])])
    if kind == "matmul_add_sigmoid":
        W1, b1, W2, b2 = f32(17, 33), f32(33), f32(33, 5), f32(5)
        nodes = [ow.node("MatMul", ["obs", "W1"], ["m1"]), ow.node("Add", ["m1", "b1"], ["h1"]),
                 ow.node("Sigmoid", ["h1"], ["a1"]),
                 ow.node("MatMul", ["a1", "W2"], ["m2"]), ow.node("Add", ["b2", "m2"], ["act"])]
        inits = [("W1", W1), ("b1", b1), ("W2", W2), ("b2", b2)]
        return ow.model(nodes, inits, [("obs", ["N", 17])], [("act", ["N", 5])])
    if kind == "normalized_tanh_clip":
        mean, std = f32(24), (np.abs(f32(24)) + 0.5).astype(np.float32)
        W1, b1, W2, b2 = f32(64, 24), f32(64), f32(12, 64), f32(12)
        lo, hi = np.array(-0.5, np.float32), np.array(0.75, np.float32)
        nodes = [ow.node("Sub", ["obs", "mean"], ["c"]), ow.node("Div", ["c", "std"], ["n"]),
                 ow.node("Gemm", ["n", "W1", "b1"], ["h1"], "", [ow.attr_int("transB", 1)]),
                 ow.node("Elu", ["h1"], ["a1"], "", [ow.attr_float("alpha", 0.7)]),
                 ow.node("Gemm", ["a1", "W2", "b2"], ["h2"], "", [ow.attr_int("transB", 1)]),
                 ow.node("Tanh", ["h2"], ["t"]), ow.node("Clip", ["t", "lo", "hi"], ["act"])]
        inits = [("mean", mean), ("std", std), ("W1", W1), ("b1", b1), ("W2", W2), ("b2", b2), ("lo", lo),
                 ("hi", hi)]
        return ow.model(nodes, inits, [("obs", [1, 24])], [("act", [1, 12])])
    if kind == "relu_deep":
        dims = [30, 96, 160, 64, 200, 9]
        nodes, inits, cur = [], [], "obs"
        for i, (k, n) in enumerate(zip(dims[:-1], dims[1:])):
            inits += [(f"W{i}", f32(n, k)), (f"b{i}", f32(n))]
            out = "act" if i == len(dims) - 2 else f"h{i}"
            nodes.append(ow.node("Gemm", [cur, f"W{i}", f"b{i}"], [out], "", [ow.attr_int("transB", 1)]))
            cur = out
            if out != "act":
                nodes.append(ow.node("Relu", [cur], [f"a{i}"]))
                cur = f"a{i}"
        return ow.model(nodes, inits, [("obs", ["N", 30])], [("act", ["N", 9])])
    raise KeyError(kind)


VARIANTS = ["gemm_transB0_alpha_beta", "matmul_add_sigmoid", "normalized_tanh_clip", "relu_deep"]

UNSUPPORTED = {
    # op the loader must reject with a clear message (no silent fallback)
    "conv": lambda: ow.model([ow.node("Conv", ["obs", "W"], ["act"])],
                             [("W", np.zeros((1, 1, 1), np.float32))], [("obs", [1, 4])], [("act", [1, 4])]),
    "dynamic_weight": lambda: ow.model([ow.node("MatMul", ["obs", "w_in"], ["act"])], [],
                                       [("obs", [1, 4]), ("w_in", [4, 4])], [("act", [1, 4])]),
}


def write(tmp_path, kind, seed=0):
    p = tmp_path / f"{kind}.onnx"
    data = variant_bytes(kind, seed) if kind in VARIANTS else UNSUPPORTED[kind]()
    p.write_bytes(data)
    return str(p)
