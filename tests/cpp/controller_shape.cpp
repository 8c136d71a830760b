// "Controller-shaped" use of the drop-in header, exactly as the reference's
// callers use it (onnx_controller/src/controller.cpp:25,49,215 with the
// std::array members of controller.hpp:148-149; onnx_inference/src/cpp/main.cpp:32-45).
// Usage: controller_shape <model.onnx> [zeros|twos|ticks N]
#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>

#include "onnx_actor.hpp"

constexpr size_t kDimDOF = 12;
constexpr size_t kDimObs = 49;
constexpr size_t kHistory = 2;

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  std::array<float, kDimObs * kHistory> observation{};
  std::array<float, kDimDOF> action{};
  std::string mode = argc > 2 ? argv[2] : "zeros";
  try {
    auto actor = std::make_unique<ONNXActor>(argv[1], observation, action);
    actor->print_model_info();
    std::printf("check_dims: %d\n", actor->check_dims() ? 1 : 0);
    if (mode == "twos") observation.fill(2.0f);
    int ticks = mode == "ticks" && argc > 3 ? std::atoi(argv[3]) : 1;
    double best = 1e30;
    for (int t = 0; t < ticks; ++t) {
      if (mode == "ticks") observation[t % observation.size()] += 0.001f;  // obs changes every tick
      auto t0 = std::chrono::steady_clock::now();
      actor->act();
      auto t1 = std::chrono::steady_clock::now();
      best = std::min(best, std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::printf("Action:");
    for (float a : action) std::printf(" %.9g", a);
    std::printf("\nbest_us: %.3f\n", best);
  } catch (const std::exception &ex) {
    std::printf("exception: %s\n", ex.what());
    return 3;
  }
  return 0;
}
