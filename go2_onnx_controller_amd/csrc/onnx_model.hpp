// ONNX policy loader: a minimal protobuf reader plus a pattern matcher that
// lowers an exported policy graph to the engine's program (dense layers with a
// fused activation, optional leading GRU, optional affine prologue and clip
// epilogue). Replaces what the reference gets from onnxruntime's session
// creation (onnx_inference/src/cpp/onnx_actor.cpp:16, :23-28).
#pragma once

#include <cstddef>
#include <cstdint>
#include <limits>
#include <string>
#include <vector>

namespace go2pi {

// The activation fused into a dense layer's epilogue (device_fn.hpp act_t), with
// the ONNX node's attributes in alpha / beta: Elu / LeakyRelu alpha; Clip min / max
// (a Clip right after a Gemm, e.g. ReLU6); Selu alpha / gamma; HardSigmoid and
// HardSwish alpha / beta.
enum Act : int {
  ACT_NONE = 0, ACT_ELU = 1, ACT_RELU = 2, ACT_TANH = 3, ACT_SIGMOID = 4, ACT_LEAKY = 5,
  ACT_CLIP = 6, ACT_SELU = 7, ACT_SOFTPLUS = 8, ACT_HARDSIGMOID = 9, ACT_HARDSWISH = 10, ACT_SOFTSIGN = 11
};

struct Dense {
  int K = 0, N = 0;
  std::vector<float> W;  // [N][K] row-major (ONNX Gemm transB=1 layout)
  std::vector<float> b;  // [N]
  int act = ACT_NONE;
  float alpha = 0.f, beta = 0.f;
};

// ONNX GRU (opset 14), forward, layout 0, one layer; gates ordered z, r, h.
// The recurrent cell in front of the dense head: ONNX GRU (gates z, r, h) or
// LSTM (gates i, o, f, c; no peepholes). G = 3 or 4 gates.
struct Gru {
  int cell = 0;              // 0 GRU, 1 LSTM
  int G = 3;                 // gates
  int I = 0, H = 0;
  int lbr = 0;               // GRU linear_before_reset
  std::vector<float> W;      // [G*H][I]
  std::vector<float> R;      // [G*H][H]
  std::vector<float> Wb, Rb; // [G*H] each
};

struct IoInfo {
  std::string name;
  std::vector<int64_t> shape;  // -1 for symbolic dims
};

struct Model {
  std::vector<IoInfo> inputs, outputs;
  int64_t ir_version = 0, opset = 0;
  std::string producer;

  // program
  // optional prologue clip((x - sub) / div * mul, pre_lo, pre_hi), each [in_dim] or [1]
  std::vector<float> pre_sub, pre_div, pre_mul;
  float pre_lo = -std::numeric_limits<float>::infinity();
  float pre_hi = std::numeric_limits<float>::infinity();
  bool has_gru = false;
  Gru gru;
  std::vector<Dense> layers;
  // after the final layer's activation: y <- post_scale * clip(y, clip_lo, clip_hi)
  // (a trailing Clip and / or scalar Mul of the graph)
  float clip_lo = -std::numeric_limits<float>::infinity();
  float clip_hi = std::numeric_limits<float>::infinity();
  float post_scale = 1.f;
  int in_dim = 0, out_dim = 0;
};

// Throws std::runtime_error with a descriptive message on malformed or
// unsupported graphs.
Model parse_onnx(const uint8_t *data, size_t n);

// The loader's view of a model as JSON (go2pi_inspect_model): I/O, dims, each
// layer's activation and weight / bias checksums, the recurrent cell, the
// prologue / epilogue. Host-only (no device): tests/cpp/fuzz_loader.cpp drives
// parse_onnx + inspect_json under ASan / UBSan.
std::string inspect_json(const Model &m);

}  // namespace go2pi
