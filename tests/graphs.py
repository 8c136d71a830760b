"""Small ONNX policy graphs exercising the loader's supported patterns
(SURVEY §8f.3 "ONNX loader breadth"): Gemm with transB=0 / alpha / beta,
MatMul + Add, Sub/Div input normalisation, LeakyRelu / Sigmoid, trailing
Tanh + Clip, Clip between dense layers (ReLU6), Constant nodes, Mul by a
constant at the input / after a Gemm / after an activation / at the output,
Selu / Softplus / HardSigmoid / HardSwish / Softsign, a Slice -> per-block
normalisation -> Concat observation front-end. Built with the repo's own
writer; evaluated by the oracle."""
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
    if kind == "relu6_mid_clip":
        # Gemm -> Clip(0, 6) -> Gemm -> Elu -> Gemm: a Clip between dense layers is the
        # first layer's activation (torch.onnx.export writes nn.ReLU6 so, opset >= 11)
        W1, b1, W2, b2, W3, b3 = f32(64, 30) * 4, f32(64) * 4, f32(48, 64), f32(48), f32(10, 48), f32(10)
        nodes = [ow.node("Gemm", ["obs", "W1", "b1"], ["h1"], "", [ow.attr_int("transB", 1)]),
                 ow.node("Clip", ["h1", "lo", "hi"], ["a1"]),
                 ow.node("Gemm", ["a1", "W2", "b2"], ["h2"], "", [ow.attr_int("transB", 1)]),
                 ow.node("Elu", ["h2"], ["a2"]),
                 ow.node("Gemm", ["a2", "W3", "b3"], ["act"], "", [ow.attr_int("transB", 1)])]
        inits = [("W1", W1), ("b1", b1), ("lo", np.array(0, np.float32)), ("hi", np.array(6, np.float32)),
                 ("W2", W2), ("b2", b2), ("W3", W3), ("b3", b3)]
        return ow.model(nodes, inits, [("obs", ["N", 30])], [("act", ["N", 10])])
    if kind == "relu6_pipeline":
        # uniform 256-wide hidden layers with Clip(-1, 1.5) activations: the 4-wave pipeline
        # (lean kernel, activation read at run time) with a two-parameter activation
        dims = [40, 256, 256, 256, 12]
        nodes, inits, cur = [], [("lo", np.array(-1.0, np.float32)), ("hi", np.array(1.5, np.float32))], "obs"
        for i, (k, n) in enumerate(zip(dims[:-1], dims[1:])):
            inits += [(f"W{i}", (f32(n, k) / np.sqrt(k / 12.0)).astype(np.float32)), (f"b{i}", f32(n))]
            out = "act" if i == len(dims) - 2 else f"h{i}"
            nodes.append(ow.node("Gemm", [cur, f"W{i}", f"b{i}"], [out], "", [ow.attr_int("transB", 1)]))
            cur = out
            if out != "act":
                nodes.append(ow.node("Clip", [cur, "lo", "hi"], [f"a{i}"]))
                cur = f"a{i}"
        return ow.model(nodes, inits, [("obs", ["N", 40])], [("act", ["N", 12])])
    if kind == "const_scales":
        # scales as Constant nodes (as torch.onnx.export writes Python scalars): the observation
        # scaled and clipped, a Mul right after a Gemm (folded into its rows), a per-feature Mul
        # after an activation (folded into the next layer's columns), and the output clipped,
        # then scaled (the action epilogue)
        W1, b1, W2, b2 = f32(32, 20), f32(32), f32(8, 32), f32(8)
        sc_in = (np.abs(f32(20)) + 0.5).astype(np.float32)
        nodes = [ow.node("Constant", [], ["k_in"], "", [ow.attr_tensor("value", sc_in)]),
                 ow.node("Constant", [], ["lo_in"], "", [ow.attr_tensor("value", np.array(-2.5, np.float32))]),
                 ow.node("Constant", [], ["hi_in"], "", [ow.attr_tensor("value", np.array(2.0, np.float32))]),
                 ow.node("Constant", [], ["k1"], "", [ow.attr_tensor("value", np.array(1.75, np.float32))]),
                 ow.node("Constant", [], ["k2"], "", [ow.attr_tensor("value", (np.abs(f32(32)) + 0.2).astype(np.float32))]),
                 ow.node("Constant", [], ["k_out"], "", [ow.attr_tensor("value", np.array(0.25, np.float32))]),
                 ow.node("Mul", ["obs", "k_in"], ["x1"]),
                 ow.node("Clip", ["x1", "lo_in", "hi_in"], ["x2"]),
                 ow.node("Gemm", ["x2", "W1", "b1"], ["h1"], "", [ow.attr_int("transB", 1)]),
                 ow.node("Mul", ["k1", "h1"], ["h1s"]),
                 ow.node("Tanh", ["h1s"], ["a1"]),
                 ow.node("Mul", ["a1", "k2"], ["a1s"]),
                 ow.node("Gemm", ["a1s", "W2", "b2"], ["h2"], "", [ow.attr_int("transB", 1)]),
                 ow.node("Elu", ["h2"], ["a2"]),
                 ow.node("Clip", ["a2"], ["c2"], "", [ow.attr_float("min", -0.4), ow.attr_float("max", 0.9)]),
                 ow.node("Mul", ["c2", "k_out"], ["act"])]
        inits = [("W1", W1), ("b1", b1), ("W2", W2), ("b2", b2)]
        return ow.model(nodes, inits, [("obs", ["N", 20])], [("act", ["N", 8])])
    if kind == "selu_softplus_hardswish":
        W1, b1, W2, b2, W3, b3, W4, b4 = (f32(40, 24), f32(40), f32(40, 40), f32(40), f32(24, 40), f32(24),
                                          f32(6, 24) * 0.25, f32(6))
        nodes = [ow.node("Gemm", ["obs", "W1", "b1"], ["h1"], "", [ow.attr_int("transB", 1)]),
                 ow.node("Selu", ["h1"], ["a1"]),
                 ow.node("Gemm", ["a1", "W2", "b2"], ["h2"], "", [ow.attr_int("transB", 1)]),
                 ow.node("Softplus", ["h2"], ["a2"]),
                 ow.node("Gemm", ["a2", "W3", "b3"], ["h3"], "", [ow.attr_int("transB", 1)]),
                 ow.node("HardSwish", ["h3"], ["a3"]),
                 ow.node("Gemm", ["a3", "W4", "b4"], ["h4"], "", [ow.attr_int("transB", 1)]),
                 ow.node("HardSigmoid", ["h4"], ["act"], "", [ow.attr_float("alpha", 0.3), ow.attr_float("beta", 0.4)])]
        inits = [("W1", W1), ("b1", b1), ("W2", W2), ("b2", b2), ("W3", W3), ("b3", b3), ("W4", W4), ("b4", b4)]
        return ow.model(nodes, inits, [("obs", ["N", 24])], [("act", ["N", 6])])
    if kind == "softsign_selu_attrs":
        W1, b1, W2, b2 = f32(48, 16), f32(48), f32(5, 48), f32(5)
        nodes = [ow.node("Gemm", ["obs", "W1", "b1"], ["h1"], "", [ow.attr_int("transB", 1)]),
                 ow.node("Softsign", ["h1"], ["a1"]),
                 ow.node("Gemm", ["a1", "W2", "b2"], ["h2"], "", [ow.attr_int("transB", 1)]),
                 ow.node("Selu", ["h2"], ["act"], "", [ow.attr_float("alpha", 1.2), ow.attr_float("gamma", 0.8)])]
        inits = [("W1", W1), ("b1", b1), ("W2", W2), ("b2", b2)]
        return ow.model(nodes, inits, [("obs", ["N", 16])], [("act", ["N", 5])])
    if kind == "slice_concat_blocks":
        # per-block normalisation of a 2-step history (49 + 49 columns, controller.hpp:45-68):
        # Slice each block, (x - mean) / std per block, Concat, then the shipped policy's shape
        # (98 -> 128 -> 128 -> 12, Elu): the 4-wave pipeline and the resident kernels with a prologue
        m0, m1 = f32(49), f32(49)
        s0, s1 = (np.abs(f32(49)) + 0.5).astype(np.float32), (np.abs(f32(49)) + 0.5).astype(np.float32)
        W1, b1 = (f32(128, 98) / 3).astype(np.float32), f32(128)
        W2, b2, W3, b3 = (f32(128, 128) / 3).astype(np.float32), f32(128), (f32(12, 128) / 3).astype(np.float32), f32(12)
        i64 = lambda *v: np.array(v, np.int64)  # noqa: E731
        nodes = [ow.node("Slice", ["obs", "st0", "en0", "ax"], ["blk0"]),
                 ow.node("Slice", ["obs", "st1", "en1", "ax"], ["blk1"]),
                 ow.node("Sub", ["blk0", "m0"], ["c0"]), ow.node("Div", ["c0", "s0"], ["n0"]),
                 ow.node("Sub", ["blk1", "m1"], ["c1"]), ow.node("Div", ["c1", "s1"], ["n1"]),
                 ow.node("Concat", ["n0", "n1"], ["x"], "", [ow.attr_int("axis", 1)]),
                 ow.node("Gemm", ["x", "W1", "b1"], ["h1"], "", [ow.attr_int("transB", 1)]), ow.node("Elu", ["h1"], ["a1"]),
                 ow.node("Gemm", ["a1", "W2", "b2"], ["h2"], "", [ow.attr_int("transB", 1)]), ow.node("Elu", ["h2"], ["a2"]),
                 ow.node("Gemm", ["a2", "W3", "b3"], ["act"], "", [ow.attr_int("transB", 1)])]
        inits = [("st0", i64(0)), ("en0", i64(49)), ("st1", i64(49)), ("en1", i64(2**63 - 1)), ("ax", i64(1)),
                 ("m0", m0), ("s0", s0), ("m1", m1), ("s1", s1), ("W1", W1), ("b1", b1), ("W2", W2), ("b2", b2),
                 ("W3", W3), ("b3", b3)]
        return ow.model(nodes, inits, [("obs", ["N", 98])], [("act", ["N", 12])])
    if kind == "slice_concat_mixed":
        # three blocks with different ops (a scalar Mul; nothing but an Identity; Sub and a
        # per-column Mul), every block clipped to the same interval, one Slice in the opset-1
        # attribute form and one with negative indices, then a small Tanh policy
        k0 = np.array(1.5, np.float32)
        sub2, mul2 = f32(10), (np.abs(f32(10)) + 0.3).astype(np.float32)
        W1, b1, W2, b2 = f32(40, 30), f32(40), f32(6, 40), f32(6)
        i64 = lambda *v: np.array(v, np.int64)  # noqa: E731
        lo, hi = np.array(-1.2, np.float32), np.array(1.1, np.float32)
        nodes = [ow.node("Slice", ["obs"], ["blk0"], "", [ow.attr_ints("starts", [0]), ow.attr_ints("ends", [7]),
                                                        ow.attr_ints("axes", [1])]),
                 ow.node("Slice", ["obs", "st1", "en1", "ax1"], ["blk1"]),
                 ow.node("Slice", ["obs", "st2", "en2", "ax2", "sp2"], ["blk2"]),
                 ow.node("Mul", ["k0", "blk0"], ["p0"]), ow.node("Clip", ["p0", "lo", "hi"], ["q0"]),
                 ow.node("Identity", ["blk1"], ["p1"]), ow.node("Clip", ["p1", "lo", "hi"], ["q1"]),
                 ow.node("Sub", ["blk2", "sub2"], ["c2"]), ow.node("Mul", ["c2", "mul2"], ["p2"]),
                 ow.node("Clip", ["p2", "lo", "hi"], ["q2"]),
                 ow.node("Concat", ["q0", "q1", "q2"], ["x"], "", [ow.attr_int("axis", -1)]),
                 ow.node("Gemm", ["x", "W1", "b1"], ["h1"], "", [ow.attr_int("transB", 1)]), ow.node("Tanh", ["h1"], ["a1"]),
                 ow.node("Gemm", ["a1", "W2", "b2"], ["act"], "", [ow.attr_int("transB", 1)])]
        inits = [("st1", i64(7)), ("en1", i64(-10)), ("ax1", i64(-1)), ("st2", i64(-10)), ("en2", i64(30)),
                 ("ax2", i64(1)), ("sp2", i64(1)), ("k0", k0), ("lo", lo), ("hi", hi), ("sub2", sub2), ("mul2", mul2),
                 ("W1", W1), ("b1", b1), ("W2", W2), ("b2", b2)]
        return ow.model(nodes, inits, [("obs", ["N", 30])], [("act", ["N", 6])])
    raise KeyError(kind)


VARIANTS = ["gemm_transB0_alpha_beta", "matmul_add_sigmoid", "normalized_tanh_clip", "relu_deep", "relu6_mid_clip",
            "relu6_pipeline", "const_scales", "selu_softplus_hardswish", "softsign_selu_attrs", "slice_concat_blocks",
            "slice_concat_mixed"]
# graphs whose every operator propagates a NaN (ONNX Clip included): a NaN observation
# row must come out as a NaN action row
NAN_VARIANTS = ["normalized_tanh_clip", "relu6_mid_clip", "relu6_pipeline", "const_scales"]

UNSUPPORTED = {
    # op the loader must reject with a clear message (no silent fallback)
    "conv": lambda: ow.model([ow.node("Conv", ["obs", "W"], ["act"])],
                             [("W", np.zeros((1, 1, 1), np.float32))], [("obs", [1, 4])], [("act", [1, 4])]),
    "dynamic_weight": lambda: ow.model([ow.node("MatMul", ["obs", "w_in"], ["act"])], [],
                                       [("obs", [1, 4]), ("w_in", [4, 4])], [("act", [1, 4])]),
    # a Clip after an activation between two dense layers (not an activation of its own:
    # the matcher fuses one activation per layer) must be refused, never moved to the output
    "clip_after_act_mid": lambda: _chain([("Relu",), ("Clip", 0.0, 6.0)]),
    # Mul after the last activation, then Clip: clip(s * y) is not post_fn's clip-then-scale
    "mul_then_clip_out": lambda: _chain([], tail=[("Tanh",), ("Mul", np.float32(2.0)), ("Clip", -1.0, 1.0)]),
    "vector_mul_out": lambda: _chain([], tail=[("Tanh",), ("Mul", np.arange(1, 5, dtype=np.float32))]),
    # observation front-ends the per-column prologue cannot express: blocks Concatenated out
    # of order (a column permutation), and blocks clipped to different intervals
    "slice_reordered": lambda: _front([(4, 8), (0, 4)], clips=None),
    "slice_clip_differs": lambda: _front([(0, 4), (4, 8)], clips=[(-1.0, 1.0), (-2.0, 2.0)]),
    # a block computing mean - x (the constant first): not the prologue's x - sub
    "slice_sub_reversed": lambda: _front([(0, 4), (4, 8)], clips=None, sub_first=True),
}


def _front(blocks, clips, sub_first=False):
    """obs[8] -> Slice blocks (-> Clip) -> Concat -> Gemm -> act[3] (refusal cases);
    sub_first: block 0 goes through Sub(constant, block) first."""
    r = _rng(6)
    inits = [("W", r.standard_normal((3, 8)).astype(np.float32)), ("ax", np.array([1], np.int64))]
    nodes, outs = [], []
    for i, (b, e) in enumerate(blocks):
        inits += [(f"s{i}", np.array([b], np.int64)), (f"e{i}", np.array([e], np.int64))]
        nodes.append(ow.node("Slice", ["obs", f"s{i}", f"e{i}", "ax"], [f"b{i}"]))
        out = f"b{i}"
        if sub_first and i == 0:
            inits.append(("m0", r.standard_normal(e - b).astype(np.float32)))
            nodes.append(ow.node("Sub", ["m0", out], ["d0"]))
            out = "d0"
        if clips:
            inits += [(f"lo{i}", np.array(clips[i][0], np.float32)), (f"hi{i}", np.array(clips[i][1], np.float32))]
            nodes.append(ow.node("Clip", [out, f"lo{i}", f"hi{i}"], [f"c{i}"]))
            out = f"c{i}"
        outs.append(out)
    nodes += [ow.node("Concat", outs, ["x"], "", [ow.attr_int("axis", 1)]),
              ow.node("Gemm", ["x", "W"], ["act"], "", [ow.attr_int("transB", 1)])]
    return ow.model(nodes, inits, [("obs", [1, 8])], [("act", [1, 3])])


def _chain(mid_ops, tail=()):
    """obs[4] -> Gemm -> mid_ops -> Gemm -> tail ops -> act[4] (for the refusal cases)."""
    r = _rng(5)
    inits = [("W0", r.standard_normal((4, 4)).astype(np.float32)), ("W1", r.standard_normal((4, 4)).astype(np.float32))]
    nodes, cur, k = [ow.node("Gemm", ["obs", "W0"], ["g0"], "", [ow.attr_int("transB", 1)])], "g0", 0

    def apply(op):
        nonlocal cur, k
        k += 1
        out = f"t{k}"
        if op[0] == "Clip":
            inits.extend([(f"lo{k}", np.array(op[1], np.float32)), (f"hi{k}", np.array(op[2], np.float32))])
            nodes.append(ow.node("Clip", [cur, f"lo{k}", f"hi{k}"], [out]))
        elif op[0] == "Mul":
            inits.append((f"m{k}", np.asarray(op[1], np.float32)))
            nodes.append(ow.node("Mul", [cur, f"m{k}"], [out]))
        else:
            nodes.append(ow.node(op[0], [cur], [out]))
        cur = out

    for op in mid_ops:
        apply(op)
    nodes.append(ow.node("Gemm", [cur, "W1"], ["g1"], "", [ow.attr_int("transB", 1)]))
    cur = "g1"
    for op in tail:
        apply(op)
    nodes.append(ow.node("Identity", [cur], ["act"]))
    return ow.model(nodes, inits, [("obs", ["N", 4])], [("act", ["N", 4])])


def write(tmp_path, kind, seed=0):
    p = tmp_path / f"{kind}.onnx"
    data = variant_bytes(kind, seed) if kind in VARIANTS else UNSUPPORTED[kind]()
    p.write_bytes(data)
    return str(p)
