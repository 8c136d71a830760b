// Drop-in ONNXActor over the go2pi C ABI.
// Mirrors onnx_inference/src/cpp/onnx_actor.cpp:
//   ctor (:6-36)        -> go2pi_create + input/output name & shape discovery
//   act() (:38-48)      -> go2pi_run on the aliased spans, batch 1
//   check_dims (:50-58) -> obs.size()==in_shape[1] && act.size()==out_shape[1]
//   print_model_info (:60-66) -> the same four lines
// Errors throw std::runtime_error (the reference lets Ort::Exception escape).
#include "../../include/onnx_actor.hpp"

#include <cstdlib>
#include <iostream>
#include <stdexcept>

#include "../../include/go2pi.h"

struct ONNXActor::Impl {
  go2pi_engine *engine = nullptr;
  std::span<float> observation, action;
  std::string model_path;
  std::string input_name, output_name;
  std::vector<int64_t> input_shape, output_shape;
  OrtLoggingLevel log_level;
  int64_t in_dim = 0, out_dim = 0;
  ~Impl() { go2pi_destroy(engine); }
};

namespace {
void check(int rc, const char *what) {
  if (rc != GO2PI_OK) throw std::runtime_error(std::string("ONNXActor: ") + what + ": " + go2pi_last_error());
}

std::vector<int64_t> shape_of(go2pi_engine *e, int is_out) {
  int64_t dims[8];
  int32_t rank = 0;
  check(go2pi_io_shape(e, is_out, 0, dims, 8, &rank), "io shape");
  return std::vector<int64_t>(dims, dims + std::min<int32_t>(rank, 8));
}

std::string name_of(go2pi_engine *e, int is_out) {
  char buf[512];
  check(go2pi_io_name(e, is_out, 0, buf, sizeof buf), "io name");
  return buf;
}
}  // namespace

ONNXActor::ONNXActor(const std::string &model_path, const std::span<float> observation,
                     const std::span<float> action, OrtLoggingLevel log_level)
    : impl_(std::make_unique<Impl>()) {
  impl_->observation = observation;
  impl_->action = action;
  impl_->model_path = model_path;
  impl_->log_level = log_level;
  go2pi_opts opts;
  go2pi_default_opts(&opts);
  opts.log_level = static_cast<int32_t>(log_level);
  opts.max_batch = 64;  // one robot per act(); keep device buffers small
  // act() is one robot's tick at the controller's 50 Hz (controller.cpp:61): a
  // resident kernel serves it without a launch per call and leaves after 100 ms
  // without one (GO2PI_RESIDENT_MS overrides; 0 = one launch per call).
  opts.resident_ms = 100;
  if (const char *v = std::getenv("GO2PI_RESIDENT_MS")) opts.resident_ms = std::atoi(v);
  check(go2pi_create(model_path.c_str(), &opts, &impl_->engine), "cannot load model");
  impl_->input_name = name_of(impl_->engine, 0);
  impl_->output_name = name_of(impl_->engine, 1);
  impl_->input_shape = shape_of(impl_->engine, 0);
  impl_->output_shape = shape_of(impl_->engine, 1);
  check(go2pi_io_dims(impl_->engine, &impl_->in_dim, &impl_->out_dim), "io dims");
  // The reference wraps the spans with element count shape.at(1) (onnx_actor.cpp:31-35):
  // it requires a 2-D I/O and reads exactly in_dim floats / writes out_dim floats.
  if (impl_->input_shape.size() < 2 || impl_->output_shape.size() < 2)
    throw std::runtime_error("ONNXActor: model input/output must be 2-D [batch, features]");
  if (observation.size() < static_cast<size_t>(impl_->in_dim) || action.size() < static_cast<size_t>(impl_->out_dim))
    throw std::runtime_error("ONNXActor: observation/action buffer smaller than the model's feature dims");
}

ONNXActor::~ONNXActor() = default;

void ONNXActor::act() {
  check(go2pi_run(impl_->engine, impl_->observation.data(), impl_->action.data(), 1), "act");
}

bool ONNXActor::check_dims() {
  bool result = true;
  result &= impl_->observation.size() == static_cast<size_t>(impl_->input_shape.at(1));
  result &= impl_->action.size() == static_cast<size_t>(impl_->output_shape.at(1));
  return result;
}

void ONNXActor::print_model_info() {
  std::cout << "Input dimension: " << impl_->input_shape.at(1) << std::endl;
  std::cout << "Output dimension: " << impl_->output_shape.at(1) << std::endl;
  std::cout << "Input name: " << impl_->input_name << std::endl;
  std::cout << "Output name: " << impl_->output_name << std::endl;
}
