#pragma once
/*
 * Drop-in replacement for the reference's `onnx_actor.hpp`
 * (onnx_inference/include/onnx_actor.hpp:1-76): same global class name,
 * constructor signature, default argument, act(), print_model_info() and
 * check_dims(), so `onnx_controller` (controller.cpp:25,49,215) compiles
 * unchanged, and so does the demo driver's use of the actor and of the Ort
 * namespace (src/cpp/main.cpp:26-45; tests/cpp/controller_shape.cpp). The rest of
 * main.cpp is not ours to provide: its model path comes from ROS's
 * ament_index_cpp (:29), and its `std::cout << duration` (:42) needs a C++20
 * standard library with P0355's chrono output (libstdc++ >= 14).
 *
 * Differences that are deliberate:
 *  - no onnxruntime header: OrtLoggingLevel is defined here with ORT's values
 *    (VERBOSE=0 … FATAL=4) so `ORT_LOGGING_LEVEL_WARNING` still names 2, and
 *    `Ort::Env` is an empty environment object (the reference's callers create
 *    one before the actor, main.cpp:26; ORT keeps its thread pools and logging
 *    there, go2pi needs neither). The header's includes cover what callers got
 *    through onnxruntime_cxx_api.h (<array>: main.cpp:32);
 *  - private state lives behind a pimpl over the go2pi C ABI (include/go2pi.h);
 *  - errors throw std::runtime_error (a std::exception, like Ort::Exception).
 *
 * Contract kept from the reference: the observation and action spans are
 * aliased, not copied — they must outlive the actor; act() reads the
 * observation at call time and overwrites the action in place; one call at a
 * time per instance.
 */
#include <array>
#include <cstdint>
#include <memory>
#include <span>
#include <string>
#include <vector>

#ifndef ORT_API_VERSION  // real onnxruntime headers not included: provide the enum
typedef enum OrtLoggingLevel {
  ORT_LOGGING_LEVEL_VERBOSE = 0,
  ORT_LOGGING_LEVEL_INFO = 1,
  ORT_LOGGING_LEVEL_WARNING = 2,
  ORT_LOGGING_LEVEL_ERROR = 3,
  ORT_LOGGING_LEVEL_FATAL = 4,
} OrtLoggingLevel;

namespace Ort {
/** onnxruntime's process environment (main.cpp:26): nothing to hold here. */
struct Env {
  Env() = default;
  Env(OrtLoggingLevel /*log_level*/, const char * /*logid*/) {}
  Env(const Env &) = delete;
  Env & operator=(const Env &) = delete;
};
}  // namespace Ort
#endif

/**
 * @class ONNXActor
 * @brief Runs an ONNX reinforcement-learning policy on an AMD Instinct GPU.
 */
class ONNXActor
{
public:
  /**
   * @param model_path  Path to the ONNX model file.
   * @param observation Span over the caller's observation buffer (read by act()).
   * @param action      Span over the caller's action buffer (written by act()).
   * @param log_level   Logging level (default: ORT_LOGGING_LEVEL_WARNING).
   */
  ONNXActor(
    const std::string & model_path,
    const std::span<float> observation,
    const std::span<float> action,
    OrtLoggingLevel log_level = ORT_LOGGING_LEVEL_WARNING);

  ~ONNXActor();
  ONNXActor(const ONNXActor &) = delete;
  ONNXActor & operator=(const ONNXActor &) = delete;

  /** @brief Compute the action for the current observation (one policy step). */
  void act();

  /** @brief Print input/output dimension and name (same four lines as the reference). */
  void print_model_info();

  /** @brief True iff observation.size() == input dim and action.size() == output dim. */
  bool check_dims();

private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};
