// ONNX policy loader (see onnx_model.hpp).
//
// Wire format: proto3 (varint=0, fixed64=1, length-delimited=2, fixed32=5).
// Field numbers from onnx.proto: ModelProto{ir_version=1, producer_name=2,
// graph=7, opset_import=8}; GraphProto{node=1, initializer=5, input=11,
// output=12}; NodeProto{input=1, output=2, name=3, op_type=4, attribute=5};
// AttributeProto{name=1, f=2, i=3, floats=7, ints=8}; TensorProto{dims=1,
// data_type=2, float_data=4, int64_data=7, name=8, raw_data=9};
// ValueInfoProto{name=1, type=2}; TypeProto{tensor_type=1};
// Tensor{elem_type=1, shape=2}; TensorShapeProto{dim=1};
// Dimension{dim_value=1, dim_param=2}.
//
// Initializer payloads sit at unaligned file offsets (e.g. 0.weight of the
// shipped model at byte 730), so every payload is memcpy'd, never aliased.
#include "onnx_model.hpp"

#include <cmath>
#include <cstring>
#include <map>
#include <stdexcept>
#include <unordered_map>

namespace go2pi {
namespace {

[[noreturn]] void fail(const std::string &m) { throw std::runtime_error("onnx: " + m); }

struct Span {
  const uint8_t *p = nullptr;
  size_t n = 0;
};

struct Field {
  uint32_t no = 0, wt = 0;
  uint64_t v = 0;  // varint / fixed payload
  Span s;          // length-delimited payload
};

class Reader {
 public:
  explicit Reader(Span s) : p_(s.p), end_(s.p + s.n) {}
  bool next(Field &f) {
    if (p_ >= end_) return false;
    uint64_t key = varint();
    f.no = uint32_t(key >> 3);
    f.wt = uint32_t(key & 7);
    f.v = 0;
    f.s = {};
    switch (f.wt) {
      case 0: f.v = varint(); break;
      case 1: need(8); std::memcpy(&f.v, p_, 8); p_ += 8; break;
      case 2: {
        uint64_t ln = varint();
        need(ln);
        f.s = {p_, size_t(ln)};
        p_ += ln;
        break;
      }
      case 5: { uint32_t w; need(4); std::memcpy(&w, p_, 4); f.v = w; p_ += 4; break; }
      default: fail("unsupported protobuf wire type " + std::to_string(f.wt));
    }
    return true;
  }

 private:
  void need(uint64_t k) {
    if (uint64_t(end_ - p_) < k) fail("truncated protobuf");
  }
  uint64_t varint() {
    uint64_t out = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      need(1);
      uint8_t b = *p_++;
      out |= uint64_t(b & 0x7F) << shift;
      if (!(b & 0x80)) return out;
    }
    fail("bad varint");
  }
  const uint8_t *p_, *end_;
};

std::string str(Span s) { return std::string(reinterpret_cast<const char *>(s.p), s.n); }

void packed_varints(const Field &f, std::vector<int64_t> &out) {
  if (f.wt == 0) {
    out.push_back(int64_t(f.v));
    return;
  }
  Reader r(f.s);
  // packed: a run of bare varints; reuse the reader by faking keys is awkward, decode directly
  const uint8_t *p = f.s.p, *e = f.s.p + f.s.n;
  while (p < e) {
    uint64_t v = 0;
    int shift = 0;
    while (true) {
      if (p >= e) fail("bad packed varint");
      uint8_t b = *p++;
      v |= uint64_t(b & 0x7F) << shift;
      if (!(b & 0x80)) break;
      shift += 7;
    }
    out.push_back(int64_t(v));
  }
  (void)r;
}

float as_f32(uint64_t v) {
  uint32_t w = uint32_t(v);
  float f;
  std::memcpy(&f, &w, 4);
  return f;
}

struct Tensor {
  std::string name;
  std::vector<int64_t> dims;
  std::vector<float> f;  // FLOAT data
  std::vector<int64_t> i; // INT64 data (Unsqueeze/Squeeze axes in opset 13+)
  int dtype = 0;
  int64_t numel() const {
    int64_t n = 1;
    for (auto d : dims) n *= d;
    return n;
  }
};

Tensor parse_tensor(Span s) {
  Tensor t;
  Span raw;
  bool has_raw = false;
  Reader r(s);
  Field f;
  while (r.next(f)) {
    switch (f.no) {
      case 1: packed_varints(f, t.dims); break;
      case 2: t.dtype = int(f.v); break;
      case 4:
        if (f.wt == 2) {
          size_t n = f.s.n / 4;
          size_t o = t.f.size();
          t.f.resize(o + n);
          std::memcpy(t.f.data() + o, f.s.p, n * 4);
        } else {
          t.f.push_back(as_f32(f.v));
        }
        break;
      case 7: packed_varints(f, t.i); break;
      case 8: t.name = str(f.s); break;
      case 9: raw = f.s; has_raw = true; break;
      default: break;
    }
  }
  if (has_raw) {
    if (t.dtype == 1) {
      if (raw.n % 4) fail("raw_data size of " + t.name);
      t.f.resize(raw.n / 4);
      std::memcpy(t.f.data(), raw.p, raw.n);  // unaligned source
    } else if (t.dtype == 7) {
      t.i.resize(raw.n / 8);
      std::memcpy(t.i.data(), raw.p, raw.n);
    }
  }
  if (t.dtype == 1 && int64_t(t.f.size()) != t.numel()) fail("element count mismatch in " + t.name);
  return t;
}

struct Attr {
  float f = 0.f;
  int64_t i = 0;
  bool has_f = false, has_i = false;
  std::vector<int64_t> ints;
  std::vector<float> floats;
};

struct Node {
  std::string op, name;
  std::vector<std::string> in, out;
  std::map<std::string, Attr> attrs;
  float fattr(const char *k, float d) const {
    auto it = attrs.find(k);
    return it == attrs.end() ? d : (it->second.has_f ? it->second.f : float(it->second.i));
  }
  int64_t iattr(const char *k, int64_t d) const {
    auto it = attrs.find(k);
    return it == attrs.end() ? d : (it->second.has_i ? it->second.i : int64_t(it->second.f));
  }
};

Node parse_node(Span s) {
  Node n;
  Reader r(s);
  Field f;
  while (r.next(f)) {
    switch (f.no) {
      case 1: n.in.push_back(str(f.s)); break;
      case 2: n.out.push_back(str(f.s)); break;
      case 3: n.name = str(f.s); break;
      case 4: n.op = str(f.s); break;
      case 5: {
        Attr a;
        std::string name;
        Reader ar(f.s);
        Field g;
        while (ar.next(g)) {
          if (g.no == 1) name = str(g.s);
          else if (g.no == 2) { a.f = as_f32(g.v); a.has_f = true; }
          else if (g.no == 3) { a.i = int64_t(g.v); a.has_i = true; }
          else if (g.no == 7) {
            if (g.wt == 2) {
              size_t k = g.s.n / 4, o = a.floats.size();
              a.floats.resize(o + k);
              std::memcpy(a.floats.data() + o, g.s.p, k * 4);
            } else a.floats.push_back(as_f32(g.v));
          } else if (g.no == 8) packed_varints(g, a.ints);
        }
        n.attrs[name] = a;
        break;
      }
      default: break;
    }
  }
  return n;
}

IoInfo parse_value_info(Span s) {
  IoInfo io;
  Reader r(s);
  Field f;
  while (r.next(f)) {
    if (f.no == 1) io.name = str(f.s);
    else if (f.no == 2) {
      Reader tr(f.s);
      Field t;
      while (tr.next(t)) {
        if (t.no != 1) continue;  // tensor_type
        Reader tt(t.s);
        Field u;
        while (tt.next(u)) {
          if (u.no != 2) continue;  // shape
          Reader sh(u.s);
          Field d;
          while (sh.next(d)) {
            if (d.no != 1) continue;
            int64_t val = -1;
            Reader dr(d.s);
            Field dv;
            while (dr.next(dv))
              if (dv.no == 1) val = int64_t(dv.v);
            io.shape.push_back(val);
          }
        }
      }
    }
  }
  return io;
}

int act_of(const std::string &op) {
  if (op == "Elu") return ACT_ELU;
  if (op == "Relu") return ACT_RELU;
  if (op == "Tanh") return ACT_TANH;
  if (op == "Sigmoid") return ACT_SIGMOID;
  if (op == "LeakyRelu") return ACT_LEAKY;
  return -1;
}

}  // namespace

Model parse_onnx(const uint8_t *data, size_t n) {
  if (!data || n == 0) fail("empty model");
  Model m;
  Span graph;
  bool has_graph = false;
  {
    Reader r({data, n});
    Field f;
    while (r.next(f)) {
      if (f.no == 1) m.ir_version = int64_t(f.v);
      else if (f.no == 2) m.producer = str(f.s);
      else if (f.no == 7) { graph = f.s; has_graph = true; }
      else if (f.no == 8) {
        Reader o(f.s);
        Field g;
        while (o.next(g))
          if (g.no == 2 && int64_t(g.v) > m.opset) m.opset = int64_t(g.v);
      }
    }
  }
  if (!has_graph) fail("model has no graph");

  std::vector<Node> nodes;
  std::unordered_map<std::string, Tensor> inits;
  std::vector<IoInfo> raw_inputs;
  {
    Reader r(graph);
    Field f;
    while (r.next(f)) {
      if (f.no == 1) nodes.push_back(parse_node(f.s));
      else if (f.no == 5) {
        Tensor t = parse_tensor(f.s);
        inits[t.name] = std::move(t);
      } else if (f.no == 11) raw_inputs.push_back(parse_value_info(f.s));
      else if (f.no == 12) m.outputs.push_back(parse_value_info(f.s));
    }
  }
  for (auto &io : raw_inputs)
    if (!inits.count(io.name)) m.inputs.push_back(io);
  if (m.inputs.empty() || m.outputs.empty()) fail("graph needs at least one input and one output");

  auto init = [&](const std::string &name) -> const Tensor & {
    auto it = inits.find(name);
    if (it == inits.end()) fail("'" + name + "' is not an initializer (dynamic weights unsupported)");
    if (it->second.dtype != 1) fail("'" + name + "' is not a FLOAT tensor");
    return it->second;
  };
  auto is_init = [&](const std::string &name) { return inits.count(name) > 0; };

  std::unordered_map<std::string, std::vector<size_t>> consumers;
  for (size_t i = 0; i < nodes.size(); ++i)
    for (auto &in : nodes[i].in)
      if (!in.empty()) consumers[in].push_back(i);

  // Walk the single-consumer chain from input 0 to output 0.
  std::string cur = m.inputs[0].name;
  std::vector<bool> used(nodes.size(), false);
  bool last_has_act = true;  // true => next Add cannot fold into a bias
  bool pending_bias_ok = false;
  const std::string &final_out = m.outputs[0].name;
  while (cur != final_out) {
    auto it = consumers.find(cur);
    size_t idx = SIZE_MAX;
    if (it != consumers.end())
      for (size_t k : it->second)
        if (!used[k]) { idx = k; break; }
    if (idx == SIZE_MAX) fail("dangling value '" + cur + "' does not reach output '" + final_out + "'");
    used[idx] = true;
    const Node &nd = nodes[idx];
    auto other_input = [&]() -> const std::string & {
      if (nd.in.size() < 2) fail(nd.op + " needs two inputs");
      return nd.in[0] == cur ? nd.in[1] : nd.in[0];
    };

    if (nd.op == "Gemm") {
      if (nd.in[0] != cur) fail("Gemm: activation must be input A");
      if (nd.iattr("transA", 0)) fail("Gemm transA=1 unsupported");
      const Tensor &B = init(nd.in[1]);
      if (B.dims.size() != 2) fail("Gemm: B must be 2-D");
      const bool tb = nd.iattr("transB", 0) != 0;
      const float alpha = nd.fattr("alpha", 1.f), beta = nd.fattr("beta", 1.f);
      Dense d;
      d.N = int(tb ? B.dims[0] : B.dims[1]);
      d.K = int(tb ? B.dims[1] : B.dims[0]);
      d.W.resize(size_t(d.N) * d.K);
      for (int i = 0; i < d.N; ++i)
        for (int k = 0; k < d.K; ++k) {
          float w = tb ? B.f[size_t(i) * d.K + k] : B.f[size_t(k) * d.N + i];
          d.W[size_t(i) * d.K + k] = alpha == 1.f ? w : alpha * w;
        }
      d.b.assign(d.N, 0.f);
      if (nd.in.size() > 2 && !nd.in[2].empty()) {
        const Tensor &C = init(nd.in[2]);
        if (C.numel() != d.N && C.numel() != 1) fail("Gemm: bias must broadcast over N");
        for (int i = 0; i < d.N; ++i) {
          float c = C.numel() == 1 ? C.f[0] : C.f[i];
          d.b[i] = beta == 1.f ? c : beta * c;
        }
      }
      m.layers.push_back(std::move(d));
      last_has_act = false;
      pending_bias_ok = true;
    } else if (nd.op == "MatMul") {
      if (nd.in[0] != cur) fail("MatMul: activation must be the left operand");
      const Tensor &B = init(nd.in[1]);
      if (B.dims.size() != 2) fail("MatMul: weight must be 2-D");
      Dense d;
      d.K = int(B.dims[0]);
      d.N = int(B.dims[1]);
      d.W.resize(size_t(d.N) * d.K);
      for (int i = 0; i < d.N; ++i)
        for (int k = 0; k < d.K; ++k) d.W[size_t(i) * d.K + k] = B.f[size_t(k) * d.N + i];
      d.b.assign(d.N, 0.f);
      m.layers.push_back(std::move(d));
      last_has_act = false;
      pending_bias_ok = true;
    } else if (nd.op == "Add" && is_init(other_input())) {
      const Tensor &C = init(other_input());
      if (m.layers.empty() || last_has_act || !pending_bias_ok) fail("Add: only a bias right after Gemm/MatMul is supported");
      Dense &d = m.layers.back();
      if (C.numel() != d.N && C.numel() != 1) fail("Add: bias must broadcast over N");
      for (int i = 0; i < d.N; ++i) d.b[i] += C.numel() == 1 ? C.f[0] : C.f[i];
    } else if ((nd.op == "Sub" || nd.op == "Div") && is_init(other_input()) && nd.in[0] == cur &&
               m.layers.empty() && !m.has_gru) {
      const Tensor &C = init(other_input());
      std::vector<float> &dst = nd.op == "Sub" ? m.pre_sub : m.pre_div;
      if (!dst.empty()) fail("only one " + nd.op + " in the prologue is supported");
      if (nd.op == "Sub" && !m.pre_div.empty()) fail("prologue must be Sub then Div");
      dst = C.f;
    } else if (act_of(nd.op) >= 0) {
      if (m.layers.empty()) fail(nd.op + " before any linear layer");
      if (last_has_act) fail("two activations in a row are unsupported");
      Dense &d = m.layers.back();
      d.act = act_of(nd.op);
      d.alpha = nd.op == "Elu" ? nd.fattr("alpha", 1.f) : (nd.op == "LeakyRelu" ? nd.fattr("alpha", 0.01f) : 0.f);
      last_has_act = true;
      pending_bias_ok = false;
    } else if (nd.op == "Clip") {
      // opset >= 11: min/max are optional inputs; opset 6: attributes
      float lo = nd.fattr("min", -INFINITY), hi = nd.fattr("max", INFINITY);
      if (nd.in.size() > 1 && !nd.in[1].empty()) lo = init(nd.in[1]).f.at(0);
      if (nd.in.size() > 2 && !nd.in[2].empty()) hi = init(nd.in[2]).f.at(0);
      m.clip_lo = std::max(m.clip_lo, lo);
      m.clip_hi = std::min(m.clip_hi, hi);
      last_has_act = true;
      pending_bias_ok = false;
    } else if (nd.op == "Identity" || nd.op == "Flatten") {
      // pass-through on [B, F]
    } else if (nd.op == "Unsqueeze") {
      // must feed the recurrent cell: X [1, B, I]
      const std::string u = nd.out[0];
      auto ci = consumers.find(u);
      if (ci == consumers.end() || ci->second.size() != 1 ||
          (nodes[ci->second[0]].op != "GRU" && nodes[ci->second[0]].op != "LSTM"))
        fail("Unsqueeze is only supported in front of a GRU or LSTM");
    } else if (nd.op == "GRU" || nd.op == "LSTM") {
      // ONNX GRU (opset 14: gates z, r, h) or LSTM (opset 14: gates i, o, f, c), one
      // forward direction, default activations, as torch.onnx.export writes nn.GRU / nn.LSTM
      const bool lstm = nd.op == "LSTM";
      const std::string op = nd.op;
      if (m.has_gru) fail("only one recurrent layer is supported");
      if (!m.layers.empty()) fail(op + " must be the first layer of the policy");
      if (nd.iattr("layout", 0) != 0) fail(op + " layout=1 unsupported");
      const Tensor &W = init(nd.in.at(1));
      const Tensor &R = init(nd.in.at(2));
      Gru g;
      g.cell = lstm ? 1 : 0;
      g.G = lstm ? 4 : 3;
      if (W.dims.size() != 3 || W.dims[0] != 1)
        fail(op + ": W must be [1, " + std::to_string(g.G) + "H, I] (one direction)");
      g.H = int(R.dims.at(2));
      g.I = int(W.dims[2]);
      if (W.dims[1] != g.G * g.H || R.dims[1] != g.G * g.H) fail(op + ": gate dims mismatch");
      g.lbr = lstm ? 0 : int(nd.iattr("linear_before_reset", 0));
      g.W = W.f;
      g.R = R.f;
      g.Wb.assign((size_t)g.G * g.H, 0.f);
      g.Rb.assign((size_t)g.G * g.H, 0.f);
      if (nd.in.size() > 3 && !nd.in[3].empty()) {
        const Tensor &B = init(nd.in[3]);
        if (B.numel() != (int64_t)2 * g.G * g.H) fail(op + ": B must be [1, " + std::to_string(2 * g.G) + "H]");
        std::copy(B.f.begin(), B.f.begin() + (long)g.G * g.H, g.Wb.begin());
        std::copy(B.f.begin() + (long)g.G * g.H, B.f.end(), g.Rb.begin());
      }
      if (nd.in.size() > 4 && !nd.in[4].empty()) fail(op + ": sequence_lens unsupported");
      if (nd.attrs.count("activations")) fail(op + ": custom activations unsupported");
      if (nd.attrs.count("clip")) fail(op + ": cell clip unsupported");
      if (lstm && nd.iattr("input_forget", 0) != 0) fail("LSTM: input_forget=1 unsupported");
      if (lstm && nd.in.size() > 7 && !nd.in[7].empty()) fail("LSTM: peepholes (input P) unsupported");
      m.gru = std::move(g);
      m.has_gru = true;
      // follow Y_h (output 1) if consumed, else Y (output 0)
      std::string next;
      if (nd.out.size() > 1 && !nd.out[1].empty() && consumers.count(nd.out[1])) next = nd.out[1];
      else next = nd.out.at(0);
      cur = next;
      last_has_act = true;
      pending_bias_ok = false;
      continue;
    } else if (nd.op == "Squeeze") {
      if (!m.has_gru) fail("Squeeze is only supported after a GRU or LSTM");
    } else {
      fail("unsupported operator '" + nd.op + "' (node '" + nd.name + "')");
    }
    if (nd.out.empty()) fail("node without output");
    cur = nd.out[0];
  }

  if (m.layers.empty()) fail("policy has no linear layer");
  const int first_in = m.has_gru ? m.gru.I : m.layers[0].K;
  m.in_dim = first_in;
  if (m.has_gru && m.layers[0].K != m.gru.H) fail("recurrent hidden size does not match the first dense layer");
  for (size_t l = 1; l < m.layers.size(); ++l)
    if (m.layers[l].K != m.layers[l - 1].N) fail("layer " + std::to_string(l) + " input dim mismatch");
  m.out_dim = m.layers.back().N;
  if (!m.pre_sub.empty() && int(m.pre_sub.size()) != m.in_dim && m.pre_sub.size() != 1) fail("prologue Sub size");
  if (!m.pre_div.empty() && int(m.pre_div.size()) != m.in_dim && m.pre_div.size() != 1) fail("prologue Div size");
  // check declared feature dims against the program (reference reads shape.at(1), onnx_actor.cpp:32,35)
  const auto &is = m.inputs[0].shape, &os = m.outputs[0].shape;
  if (is.size() >= 2 && is[1] > 0 && is[1] != m.in_dim) fail("input feature dim disagrees with weights");
  if (os.size() >= 2 && os[1] > 0 && os[1] != m.out_dim) fail("output feature dim disagrees with weights");
  return m;
}

}  // namespace go2pi
