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

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
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
  // -1 for a negative dim or a product past int64 (never equal to a real element count)
  int64_t numel() const {
    int64_t n = 1;
    for (auto d : dims)
      if (d < 0 || __builtin_mul_overflow(n, d, &n)) return -1;
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
          if (n) std::memcpy(t.f.data() + o, f.s.p, n * 4);
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
      if (raw.n) std::memcpy(t.f.data(), raw.p, raw.n);  // unaligned source
    } else if (t.dtype == 7) {
      if (raw.n % 8) fail("raw_data size of " + t.name);
      t.i.resize(raw.n / 8);
      if (raw.n) std::memcpy(t.i.data(), raw.p, raw.n);
    }
  }
  if (t.dtype == 1 && int64_t(t.f.size()) != t.numel()) fail("element count mismatch in " + t.name);
  return t;
}

struct Attr {
  float f = 0.f;
  int64_t i = 0;
  bool has_f = false, has_i = false, has_t = false;
  std::vector<int64_t> ints;
  std::vector<float> floats;
  Tensor t;  // AttributeProto.t (a Constant node's value)
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
          else if (g.no == 5 && g.wt == 2) { a.t = parse_tensor(g.s); a.has_t = true; }
          else if (g.no == 7) {
            if (g.wt == 2) {
              size_t k = g.s.n / 4, o = a.floats.size();
              a.floats.resize(o + k);
              if (k) std::memcpy(a.floats.data() + o, g.s.p, k * 4);
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
  if (op == "Selu") return ACT_SELU;
  if (op == "Softplus") return ACT_SOFTPLUS;
  if (op == "HardSigmoid") return ACT_HARDSIGMOID;
  if (op == "HardSwish") return ACT_HARDSWISH;
  if (op == "Softsign") return ACT_SOFTSIGN;
  return -1;
}

// The node's attributes with the ONNX defaults (opset 6+ for Elu / LeakyRelu /
// Selu / HardSigmoid, opset 14 HardSwish: alpha = 1/6, beta = 0.5 fixed).
void act_attrs(const Node &nd, int act, float &alpha, float &beta) {
  alpha = beta = 0.f;
  switch (act) {
    case ACT_ELU: alpha = nd.fattr("alpha", 1.f); break;
    case ACT_LEAKY: alpha = nd.fattr("alpha", 0.01f); break;
    case ACT_SELU:
      alpha = nd.fattr("alpha", 1.67326319217681884765625f);
      beta = nd.fattr("gamma", 1.05070102214813232421875f);
      break;
    case ACT_HARDSIGMOID:
      alpha = nd.fattr("alpha", 0.2f);
      beta = nd.fattr("beta", 0.5f);
      break;
    case ACT_HARDSWISH:
      alpha = 1.f / 6.f;
      beta = 0.5f;
      break;
    default: break;
  }
}

// An int64 vector input of a node (Slice starts / ends / axes / steps), or empty.
std::vector<int64_t> ints_of(const std::unordered_map<std::string, Tensor> &inits, const Node &nd, size_t k) {
  if (nd.in.size() <= k || nd.in[k].empty()) return {};
  auto it = inits.find(nd.in[k]);
  if (it == inits.end() || it->second.dtype != 7) fail(nd.op + ": input " + std::to_string(k) + " must be an INT64 constant");
  return it->second.i;
}

// The per-block observation front-end: the observation Sliced into column blocks,
// each block through its own Sub / Div / Mul / Clip, then Concatenated on the feature
// axis (e.g. per-block normalisation of a controller's history blocks, controller.hpp
// :45-68). When the blocks cover the observation's columns in order, the front-end is
// exactly a per-column prologue: (x - sub[k]) / div[k] * mul[k], clipped, with each
// block's constants at its columns and the identity where a block has no such op. The
// blocks' Clip bounds must agree (the prologue clip is one interval). The walk then
// starts at the Concat's output; a graph with no Slice on the observation is left as it
// is. (The reference hands any graph to onnxruntime, onnx_actor.cpp:16; a front-end
// this cannot lower exactly is refused, never approximated.)
void front_end(Model &m, const std::vector<Node> &nodes, const std::unordered_map<std::string, Tensor> &inits,
               const std::unordered_map<std::string, std::vector<size_t>> &consumers, std::vector<bool> &used,
               std::string &cur) {
  const std::string obs = m.inputs[0].name;
  auto ci = consumers.find(obs);
  if (ci == consumers.end()) return;
  bool any_slice = false;
  for (size_t k : ci->second) any_slice |= nodes[k].op == "Slice";
  if (!any_slice) return;
  const auto &shape = m.inputs[0].shape;
  if (shape.size() != 2 || shape[1] <= 0) fail("Slice on the observation needs a static [batch, features] input shape");
  const int64_t F = shape[1];
  auto only_consumer = [&](const std::string &v) -> size_t {
    auto it = consumers.find(v);
    if (it == consumers.end() || it->second.size() != 1) fail("front-end value '" + v + "' must have exactly one consumer");
    return it->second[0];
  };
  auto fconst = [&](const Node &nd, const std::string &x) -> const Tensor & {
    const std::string &o = nd.in.at(0) == x ? nd.in.at(1) : nd.in.at(0);
    auto it = inits.find(o);
    if (it == inits.end() || it->second.dtype != 1) fail(nd.op + " in the observation front-end needs a FLOAT constant");
    // (a constant first would be c / x or c - x: lowered as x / c or x - c, the wrong value)
    if ((nd.op == "Div" || nd.op == "Sub") && nd.in.at(0) != x)
      fail(nd.op + " in the observation front-end must take the observation as its first input");
    return it->second;
  };
  struct Block {
    int64_t b = 0, e = 0;
    std::vector<float> sub, div, mul;
    float lo = -INFINITY, hi = INFINITY;
    bool clip = false;
    std::string tail;
  };
  std::vector<Block> blocks;
  size_t concat = SIZE_MAX;
  for (size_t k : ci->second) {
    const Node &sl = nodes[k];
    if (sl.op != "Slice" || sl.in.at(0) != obs) fail("the observation feeds a Slice front-end and a '" + sl.op + "'");
    std::vector<int64_t> st, en, ax, sp;
    if (sl.in.size() > 1) {
      st = ints_of(inits, sl, 1);
      en = ints_of(inits, sl, 2);
      ax = ints_of(inits, sl, 3);
      sp = ints_of(inits, sl, 4);
    } else {  // opset 1-9: attributes
      auto a = sl.attrs.find("starts"), b = sl.attrs.find("ends"), c = sl.attrs.find("axes");
      if (a == sl.attrs.end() || b == sl.attrs.end()) fail("Slice without starts / ends");
      st = a->second.ints;
      en = b->second.ints;
      if (c != sl.attrs.end()) ax = c->second.ints;
    }
    if (ax.empty())
      for (size_t i = 0; i < st.size(); ++i) ax.push_back((int64_t)i);
    if (st.size() != en.size() || ax.size() != st.size() || (!sp.empty() && sp.size() != st.size()))
      fail("Slice: starts / ends / axes / steps lengths differ");
    Block bl;
    bl.b = 0;
    bl.e = F;
    for (size_t i = 0; i < st.size(); ++i) {
      const int64_t a = ax[i] < 0 ? ax[i] + 2 : ax[i];
      if (!sp.empty() && sp[i] != 1) fail("Slice with a step other than 1 is unsupported");
      auto clampi = [&](int64_t v, int64_t dim) { return std::max<int64_t>(0, std::min(v < 0 ? v + dim : v, dim)); };
      if (a == 0) {
        if (clampi(st[i], INT64_MAX) != 0 || en[i] < INT32_MAX) fail("Slice on the batch axis is unsupported");
      } else if (a == 1) {
        bl.b = clampi(st[i], F);
        bl.e = clampi(en[i], F);
      } else {
        fail("Slice axis out of range for a [batch, features] observation");
      }
    }
    if (bl.e <= bl.b) fail("empty Slice of the observation");
    used[k] = true;
    const int64_t w = bl.e - bl.b;
    auto per_col = [&](const Tensor &C, const std::string &what) {
      if (C.numel() != 1 && C.numel() != w) fail(what + " in the front-end must broadcast over its block's " +
                                                 std::to_string(w) + " columns");
      std::vector<float> v((size_t)w);
      for (int64_t j = 0; j < w; ++j) v[(size_t)j] = C.numel() == 1 ? C.f.at(0) : C.f.at((size_t)j);
      return v;
    };
    // the block's chain: Sub?, Div? / Mul?, Clip?, Identity anywhere, then the Concat
    std::string x = sl.out.at(0);
    for (int hop = 0; hop < 16; ++hop) {
      const size_t n = only_consumer(x);
      const Node &nd = nodes[n];
      if (nd.op == "Concat") {
        if (concat != SIZE_MAX && concat != n) fail("the observation's Slices feed different Concats");
        concat = n;
        break;
      }
      used[n] = true;
      if (nd.op == "Identity") {
      } else if (nd.op == "Sub") {
        if (!bl.sub.empty() || !bl.div.empty() || !bl.mul.empty() || bl.clip) fail("front-end block: Sub must come first");
        bl.sub = per_col(fconst(nd, x), "Sub");
      } else if (nd.op == "Div") {
        if (!bl.div.empty() || !bl.mul.empty() || bl.clip) fail("front-end block must be Sub, Div, Mul, then Clip");
        bl.div = per_col(fconst(nd, x), "Div");
      } else if (nd.op == "Mul") {
        if (!bl.mul.empty() || bl.clip) fail("front-end block must be Sub, Div, Mul, then Clip");
        bl.mul = per_col(fconst(nd, x), "Mul");
      } else if (nd.op == "Clip") {
        if (bl.clip) fail("front-end block: two Clips");
        bl.lo = nd.fattr("min", -INFINITY);
        bl.hi = nd.fattr("max", INFINITY);
        auto sc = [&](size_t k2, float &v) {
          if (nd.in.size() > k2 && !nd.in[k2].empty()) {
            auto it = inits.find(nd.in[k2]);
            if (it == inits.end() || it->second.dtype != 1 || it->second.numel() != 1 || it->second.f.empty())
              fail("front-end Clip bounds must be FLOAT scalars");
            v = it->second.f[0];
          }
        };
        sc(1, bl.lo);
        sc(2, bl.hi);
        bl.clip = true;
      } else {
        fail("unsupported operator '" + nd.op + "' in the observation front-end (node '" + nd.name + "')");
      }
      if (nd.out.empty()) fail("node without output");
      x = nd.out[0];
    }
    if (concat == SIZE_MAX) fail("the observation's Slice chain does not reach a Concat");
    bl.tail = x;
    blocks.push_back(std::move(bl));
  }
  const Node &cc = nodes[concat];
  const int64_t axis = cc.iattr("axis", 1);
  if (axis != 1 && axis != -1) fail("Concat of the observation blocks must be on the feature axis");
  if (cc.in.size() != blocks.size()) fail("the Concat after the observation Slices takes other inputs too");
  // the blocks in Concat order must cover [0, F) in order
  std::vector<Block *> order;
  for (const auto &name : cc.in) {
    Block *hit = nullptr;
    for (auto &bl : blocks)
      if (bl.tail == name && !hit) hit = &bl;
    if (!hit) fail("Concat input '" + name + "' is not an observation block");
    order.push_back(hit);
  }
  int64_t at = 0;
  for (Block *bl : order) {
    if (bl->b != at) fail("the observation blocks must cover its columns in order (a reordering front-end is unsupported)");
    at = bl->e;
  }
  if (at != F) fail("the observation blocks must cover all of its columns");
  bool any_sub = false, any_div = false, any_mul = false, any_clip = false;
  float lo = -INFINITY, hi = INFINITY;
  for (Block *bl : order) {
    any_sub |= !bl->sub.empty();
    any_div |= !bl->div.empty();
    any_mul |= !bl->mul.empty();
    if (bl->clip) {
      if (any_clip && (bl->lo != lo || bl->hi != hi)) fail("the observation blocks' Clip bounds differ");
      any_clip = true;
      lo = bl->lo;
      hi = bl->hi;
    }
  }
  if (any_clip)
    for (Block *bl : order)
      if (!bl->clip) fail("only some observation blocks are clipped");
  auto cat = [&](bool any, std::vector<float> Block::*f, float ident, std::vector<float> &dst) {
    if (!any) return;
    dst.clear();
    for (Block *bl : order) {
      const auto &v = bl->*f;
      if (v.empty()) dst.insert(dst.end(), (size_t)(bl->e - bl->b), ident);
      else dst.insert(dst.end(), v.begin(), v.end());
    }
  };
  cat(any_sub, &Block::sub, 0.f, m.pre_sub);
  cat(any_div, &Block::div, 1.f, m.pre_div);
  cat(any_mul, &Block::mul, 1.f, m.pre_mul);
  if (any_clip) {
    m.pre_lo = lo;
    m.pre_hi = hi;
  }
  used[concat] = true;
  cur = cc.out.at(0);
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
  // Constant nodes (torch.onnx.export writes scalars such as a Clip bound or a Mul
  // factor this way) become initializers of their output
  for (auto &nd : nodes) {
    if (nd.op != "Constant" || nd.out.empty()) continue;
    Tensor t;
    auto it = nd.attrs.find("value");
    if (it != nd.attrs.end() && it->second.has_t) t = it->second.t;
    else if ((it = nd.attrs.find("value_float")) != nd.attrs.end()) { t.dtype = 1; t.f = {it->second.f}; }
    else if ((it = nd.attrs.find("value_floats")) != nd.attrs.end()) {
      t.dtype = 1;
      t.f = it->second.floats;
      t.dims = {int64_t(t.f.size())};
    } else fail("Constant node '" + nd.name + "' without a value");
    t.name = nd.out[0];
    inits[t.name] = std::move(t);
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
  front_end(m, nodes, inits, consumers, used, cur);
  bool last_has_act = true;  // true => next Add cannot fold into a bias
  bool pending_bias_ok = false;
  // elementwise ops after the last layer's activation: a Mul by a constant is held
  // here (col_scale) and folded into the next Gemm's input columns; at the end of
  // the graph a scalar one becomes post_scale, and a Clip becomes the output clip
  std::vector<float> col_scale;
  bool post_clip = false;
  size_t rnn_node = SIZE_MAX;  // the recurrent cell's node
  const std::string &final_out = m.outputs[0].name;
  auto const_vec = [&](const Tensor &C, int n, const std::string &what) {
    if (C.numel() != n && C.numel() != 1) fail(what + " must broadcast over " + std::to_string(n) + " features");
    std::vector<float> v(n);
    for (int i = 0; i < n; ++i) v[i] = C.numel() == 1 ? C.f[0] : C.f[i];
    return v;
  };
  auto scalar_of = [&](const std::string &name) -> float {
    const Tensor &t = init(name);
    if (t.f.empty()) fail("'" + name + "' is empty");
    if (t.numel() != 1) fail("'" + name + "' must be a scalar");
    return t.f[0];
  };
  // a new linear layer: no trailing op may sit between it and the previous one,
  // except a held column scale, folded into its weights here
  auto begin_layer = [&](Dense &d, const std::string &op) {
    if (post_clip) fail(op + ": a Clip after an activation is only supported at the end of the graph");
    if (!col_scale.empty()) {
      if ((int)col_scale.size() != 1 && (int)col_scale.size() != d.K) fail(op + ": the Mul before it must broadcast over K");
      for (int i = 0; i < d.N; ++i)
        for (int k = 0; k < d.K; ++k) d.W[size_t(i) * d.K + k] *= col_scale[col_scale.size() == 1 ? 0 : k];
      col_scale.clear();
    }
  };
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
    const bool at_input = m.layers.empty() && !m.has_gru;  // still in front of the first layer

    if (nd.op == "Gemm") {
      if (nd.in[0] != cur) fail("Gemm: activation must be input A");
      if (nd.iattr("transA", 0)) fail("Gemm transA=1 unsupported");
      const Tensor &B = init(nd.in.at(1));
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
      begin_layer(d, "Gemm");
      m.layers.push_back(std::move(d));
      last_has_act = false;
      pending_bias_ok = true;
    } else if (nd.op == "MatMul") {
      if (nd.in[0] != cur) fail("MatMul: activation must be the left operand");
      const Tensor &B = init(nd.in.at(1));
      if (B.dims.size() != 2) fail("MatMul: weight must be 2-D");
      Dense d;
      d.K = int(B.dims[0]);
      d.N = int(B.dims[1]);
      d.W.resize(size_t(d.N) * d.K);
      for (int i = 0; i < d.N; ++i)
        for (int k = 0; k < d.K; ++k) d.W[size_t(i) * d.K + k] = B.f[size_t(k) * d.N + i];
      d.b.assign(d.N, 0.f);
      begin_layer(d, "MatMul");
      m.layers.push_back(std::move(d));
      last_has_act = false;
      pending_bias_ok = true;
    } else if (nd.op == "Add" && is_init(other_input())) {
      const Tensor &C = init(other_input());
      if (m.layers.empty() || last_has_act || !pending_bias_ok) fail("Add: only a bias right after Gemm/MatMul is supported");
      Dense &d = m.layers.back();
      if (C.numel() != d.N && C.numel() != 1) fail("Add: bias must broadcast over N");
      for (int i = 0; i < d.N; ++i) d.b[i] += C.numel() == 1 ? C.f[0] : C.f[i];
    } else if ((nd.op == "Sub" || nd.op == "Div") && at_input && nd.in[0] == cur && is_init(other_input())) {
      // observation normalisation, evaluated as written: (x - sub) / div
      const Tensor &C = init(other_input());
      std::vector<float> &dst = nd.op == "Sub" ? m.pre_sub : m.pre_div;
      if (!dst.empty()) fail("only one " + nd.op + " in the prologue is supported");
      if (nd.op == "Sub" && (!m.pre_div.empty() || !m.pre_mul.empty())) fail("prologue must be Sub, then Div / Mul");
      if (!m.pre_mul.empty() || std::isfinite(m.pre_lo) || std::isfinite(m.pre_hi))
        fail("prologue must be Sub, Div, Mul, then Clip");
      dst = C.f;
    } else if (nd.op == "Mul" && at_input && is_init(other_input())) {
      if (!m.pre_mul.empty()) fail("only one Mul in the prologue is supported");
      if (std::isfinite(m.pre_lo) || std::isfinite(m.pre_hi)) fail("prologue must be Sub, Div, Mul, then Clip");
      m.pre_mul = init(other_input()).f;
    } else if ((nd.op == "Mul" || (nd.op == "Div" && nd.in[0] == cur)) && is_init(other_input())) {
      // a constant scale between or after the layers (its reciprocal for a Div)
      const Tensor &C = init(other_input());
      if (m.has_gru && m.layers.empty()) fail(nd.op + " right after the recurrent cell is unsupported");
      if (post_clip && C.numel() != 1) fail("a per-feature " + nd.op + " after the output Clip is unsupported");
      const bool div = nd.op == "Div";
      if (!last_has_act) {
        // straight after Gemm (+ bias): scale the layer's rows and bias
        Dense &d = m.layers.back();
        const std::vector<float> sc = const_vec(C, d.N, nd.op);
        for (int i = 0; i < d.N; ++i) {
          const float f = div ? 1.f / sc[i] : sc[i];
          for (int k = 0; k < d.K; ++k) d.W[size_t(i) * d.K + k] *= f;
          d.b[i] *= f;
        }
      } else {
        // after an activation: held for the next layer's input columns (or the output)
        const int n = m.layers.back().N;
        std::vector<float> sc = const_vec(C, n, nd.op);
        if (C.numel() == 1) sc.resize(1);
        for (auto &v : sc) v = div ? 1.f / v : v;
        if (col_scale.empty()) col_scale = sc;
        else if (col_scale.size() == 1 && sc.size() == 1) col_scale[0] *= sc[0];
        else fail("two vector Mul / Div in a row are unsupported");
      }
    } else if (nd.op == "Clip") {
      // opset >= 11: min/max are optional inputs; opset 6: attributes
      float lo = nd.fattr("min", -INFINITY), hi = nd.fattr("max", INFINITY);
      if (nd.in.size() > 1 && !nd.in[1].empty()) lo = scalar_of(nd.in[1]);
      if (nd.in.size() > 2 && !nd.in[2].empty()) hi = scalar_of(nd.in[2]);
      if (at_input) {
        // clip of the observation (after any normalisation)
        m.pre_lo = std::max(m.pre_lo, lo);
        m.pre_hi = std::min(m.pre_hi, hi);
      } else if (m.has_gru && m.layers.empty()) {
        fail("Clip right after the recurrent cell is unsupported");
      } else if (!last_has_act) {
        // the layer's activation (ReLU6 = Clip(0, 6)), applied in its epilogue
        Dense &d = m.layers.back();
        d.act = ACT_CLIP;
        d.alpha = lo;
        d.beta = hi;
        last_has_act = true;
        pending_bias_ok = false;
      } else {
        // after an activation: only as the output clip (the action epilogue)
        if (!col_scale.empty()) fail("Clip after a Mul that follows an activation is unsupported");
        m.clip_lo = std::max(m.clip_lo, lo);
        m.clip_hi = std::min(m.clip_hi, hi);
        post_clip = true;
      }
    } else if (act_of(nd.op) >= 0) {
      if (m.layers.empty()) fail(nd.op + " before any linear layer");
      if (last_has_act) fail("two activations in a row are unsupported");
      Dense &d = m.layers.back();
      d.act = act_of(nd.op);
      act_attrs(nd, d.act, d.alpha, d.beta);
      last_has_act = true;
      pending_bias_ok = false;
    } else if (nd.op == "Identity" || nd.op == "Flatten") {
      // pass-through on [B, F]
    } else if (nd.op == "Unsqueeze") {
      // must feed the recurrent cell: X [1, B, I]
      const std::string u = nd.out.at(0);
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
      if (R.dims.size() != 3 || R.dims[0] != 1 || g.H <= 0 || g.I <= 0) fail(op + ": R must be [1, G*H, H], H > 0");
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
      rnn_node = idx;
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
  if (rnn_node != SIZE_MAX) {
    // The recurrent state I/O listed as (h, c) after the observation / action, whatever
    // the graph's order: traced by name to the cell's initial_h / initial_c (inputs 5,
    // 6) through Unsqueeze / Identity / Reshape, and Y_h / Y_c (outputs 1, 2) through
    // Squeeze / Identity / Reshape. Other extra graph inputs / outputs keep their order.
    const Node &cell = nodes[rnn_node];
    auto producer = [&](const std::string &v) -> const Node * {
      for (auto &nd : nodes)
        for (auto &o : nd.out)
          if (o == v) return &nd;
      return nullptr;
    };
    auto is_pass = [](const std::string &op, bool in) {
      return op == "Identity" || op == "Reshape" || op == (in ? "Unsqueeze" : "Squeeze");
    };
    auto find_io = [](std::vector<IoInfo> &v, const std::string &name) -> long {
      for (size_t i = 1; i < v.size(); ++i)
        if (v[i].name == name) return (long)i;
      return -1;
    };
    auto trace_in = [&](size_t k) -> long {
      if (cell.in.size() <= k || cell.in[k].empty()) return -1;
      std::string v = cell.in[k];
      for (int hop = 0; hop < 8; ++hop) {
        const long i = find_io(m.inputs, v);
        if (i >= 0) return i;
        const Node *pr = producer(v);
        if (!pr || !is_pass(pr->op, true) || pr->in.empty()) return -1;
        v = pr->in[0];
      }
      return -1;
    };
    auto trace_out = [&](size_t k) -> long {
      if (cell.out.size() <= k || cell.out[k].empty()) return -1;
      std::string v = cell.out[k];
      for (int hop = 0; hop < 8; ++hop) {
        const long i = find_io(m.outputs, v);
        if (i >= 0) return i;
        auto ci = consumers.find(v);
        if (ci == consumers.end()) return -1;
        const Node *nx = nullptr;
        for (size_t c : ci->second)
          if (is_pass(nodes[c].op, false)) nx = &nodes[c];
        if (!nx || nx->out.empty()) return -1;
        v = nx->out[0];
      }
      return -1;
    };
    auto reorder = [](std::vector<IoInfo> &v, long h, long c) {
      std::vector<IoInfo> r{v[0]};
      if (h > 0) r.push_back(v[h]);
      if (c > 0) r.push_back(v[c]);
      for (long i = 1; i < (long)v.size(); ++i)
        if (i != h && i != c) r.push_back(v[i]);
      v = std::move(r);
    };
    const bool lstm = m.gru.cell == 1;
    const long hi = trace_in(5), ci = lstm ? trace_in(6) : -1, ho = trace_out(1), co = lstm ? trace_out(2) : -1;
    //  the state I/O is (h) or (h, c) positionally after the observation /
    // action (actor.py maps them so): an LSTM exposes both or neither, and h and c are
    // distinct graph values
    if (lstm && ((hi >= 0) != (ci >= 0) || (ho >= 0) != (co >= 0)))
      fail("LSTM: initial_h / initial_c (and Y_h / Y_c) must both be graph I/O, or neither");
    if ((hi >= 0 && hi == ci) || (ho >= 0 && ho == co)) fail(std::string(lstm ? "LSTM" : "GRU") + ": h and c trace to the same graph I/O");
    reorder(m.inputs, hi, ci);
    reorder(m.outputs, ho, co);
  }
  if (!col_scale.empty()) {
    if (col_scale.size() != 1) fail("a per-feature Mul after the final activation is unsupported");
    m.post_scale = col_scale[0];
  }
  const int first_in = m.has_gru ? m.gru.I : m.layers[0].K;
  m.in_dim = first_in;
  if (m.has_gru && m.layers[0].K != m.gru.H) fail("recurrent hidden size does not match the first dense layer");
  for (size_t l = 1; l < m.layers.size(); ++l)
    if (m.layers[l].K != m.layers[l - 1].N) fail("layer " + std::to_string(l) + " input dim mismatch");
  m.out_dim = m.layers.back().N;
  if (!m.pre_sub.empty() && int(m.pre_sub.size()) != m.in_dim && m.pre_sub.size() != 1) fail("prologue Sub size");
  if (!m.pre_div.empty() && int(m.pre_div.size()) != m.in_dim && m.pre_div.size() != 1) fail("prologue Div size");
  if (!m.pre_mul.empty() && int(m.pre_mul.size()) != m.in_dim && m.pre_mul.size() != 1) fail("prologue Mul size");
  // check declared feature dims against the program (reference reads shape.at(1), onnx_actor.cpp:32,35)
  const auto &is = m.inputs[0].shape, &os = m.outputs[0].shape;
  if (is.size() >= 2 && is[1] > 0 && is[1] != m.in_dim) fail("input feature dim disagrees with weights");
  if (os.size() >= 2 && os[1] > 0 && os[1] != m.out_dim) fail("output feature dim disagrees with weights");
  return m;
}

namespace {

std::string json_num(double v) {
  if (std::isnan(v)) return "null";
  if (std::isinf(v)) return v > 0 ? "1e308" : "-1e308";
  char t[64];
  std::snprintf(t, sizeof t, "%.17g", v);
  return t;
}

// a JSON string literal (names come from the file: quotes, backslashes and control bytes escaped)
std::string json_str(const std::string &s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += (char)c;
    } else if (c < 0x20 || c >= 0x7F) {
      char t[8];
      std::snprintf(t, sizeof t, "\\u%04x", c);
      o += t;
    } else {
      o += (char)c;
    }
  }
  return o + "\"";
}

double sum_of(const std::vector<float> &v) {
  double s = 0;
  for (float x : v) s += x;
  return s;
}

std::string io_json(const std::vector<IoInfo> &v) {
  std::string s = "[";
  for (size_t i = 0; i < v.size(); ++i) {
    s += (i ? "," : "") + std::string("{\"name\":") + json_str(v[i].name) + ",\"shape\":[";
    for (size_t d = 0; d < v[i].shape.size(); ++d) s += (d ? "," : "") + std::to_string(v[i].shape[d]);
    s += "]}";
  }
  return s + "]";
}

}  // namespace

std::string inspect_json(const Model &m) {
  std::string j = "{\"ir_version\":" + std::to_string(m.ir_version) + ",\"opset\":" + std::to_string(m.opset) +
                  ",\"producer\":" + json_str(m.producer) + ",\"inputs\":" + io_json(m.inputs) +
                  ",\"outputs\":" + io_json(m.outputs) + ",\"in_dim\":" + std::to_string(m.in_dim) +
                  ",\"out_dim\":" + std::to_string(m.out_dim) + ",\"layers\":[";
  for (size_t l = 0; l < m.layers.size(); ++l) {
    const auto &d = m.layers[l];
    j += (l ? "," : "") + std::string("{\"K\":") + std::to_string(d.K) + ",\"N\":" + std::to_string(d.N) +
         ",\"act\":" + std::to_string(d.act) + ",\"alpha\":" + json_num(d.alpha) + ",\"beta\":" + json_num(d.beta) +
         ",\"w_sum\":" + json_num(sum_of(d.W)) + ",\"b_sum\":" + json_num(sum_of(d.b)) + "}";
  }
  j += "],\"gru\":";
  if (m.has_gru)
    j += "{\"cell\":\"" + std::string(m.gru.cell ? "LSTM" : "GRU") + "\",\"I\":" + std::to_string(m.gru.I) +
         ",\"H\":" + std::to_string(m.gru.H) + ",\"lbr\":" + std::to_string(m.gru.lbr) +
         ",\"w_sum\":" + json_num(sum_of(m.gru.W)) + ",\"r_sum\":" + json_num(sum_of(m.gru.R)) +
         ",\"b_sum\":" + json_num(sum_of(m.gru.Wb) + sum_of(m.gru.Rb)) + "}";
  else
    j += "null";
  j += ",\"pre_sub\":" + std::to_string(m.pre_sub.size()) + ",\"pre_div\":" + std::to_string(m.pre_div.size()) +
       ",\"pre_mul\":" + std::to_string(m.pre_mul.size()) + ",\"pre_clip\":[" + json_num(m.pre_lo) + "," +
       json_num(m.pre_hi) + "],\"clip\":[" + json_num(m.clip_lo) + "," + json_num(m.clip_hi) +
       "],\"post_scale\":" + json_num(m.post_scale) + "}";
  return j;
}

}  // namespace go2pi
