// "Controller-shaped" use of the drop-in header, exactly as the reference's
// callers use it (onnx_controller/src/controller.cpp:25,49,215 with the
// std::array members of controller.hpp:148-149; onnx_inference/src/cpp/main.cpp:26-45,
// including the Ort::Env that main.cpp:26 creates before the actor).
// Usage: controller_shape <model.onnx> [zeros|twos|ticks N [actions.bin]]
//   ticks: N act() calls on an observation the caller changes in place before each
//   (observation[t % 98] += 0.001f, as populate_buffer rewrites it every tick); with
//   actions.bin, every tick's 12 actions are written there as float32 [N][12].
//        controller_shape <model.onnx> lat <iters> <warmup> <in_dim> <out_dim>
//   lat: act() latency as the reference's main.cpp:38-42 measures it (steady_clock
//   around one act()), over <warmup> untimed then <iters> timed calls on spans of
//   the given sizes; prints p50 / p99 in microseconds.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "onnx_actor.hpp"

constexpr size_t kDimDOF = 12;
constexpr size_t kDimObs = 49;
constexpr size_t kHistory = 2;

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  Ort::Env env(ORT_LOGGING_LEVEL_WARNING, "test");  // main.cpp:26
  std::array<float, kDimObs * kHistory> observation{};
  std::array<float, kDimDOF> action{};
  std::string mode = argc > 2 ? argv[2] : "zeros";
  if (mode == "lat") {
    if (argc < 7) return 2;
    const int iters = std::atoi(argv[3]), warm = std::atoi(argv[4]);
    std::vector<float> obs((size_t)std::atoi(argv[5]), 0.f), act((size_t)std::atoi(argv[6]), 0.f);
    try {
      ONNXActor actor(argv[1], obs, act);
      std::vector<double> ts;
      ts.reserve((size_t)iters);
      for (int t = 0; t < warm + iters; ++t) {
        obs[(size_t)t % obs.size()] += 0.001f;  // the observation changes every call
        const auto t0 = std::chrono::steady_clock::now();
        actor.act();
        const auto t1 = std::chrono::steady_clock::now();
        if (t >= warm) ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      }
      std::sort(ts.begin(), ts.end());
      std::printf("p50_us: %.3f\np99_us: %.3f\n", ts[ts.size() / 2], ts[ts.size() * 99 / 100]);
    } catch (const std::exception &ex) {
      std::printf("exception: %s\n", ex.what());
      return 3;
    }
    return 0;
  }
  try {
    auto actor = std::make_unique<ONNXActor>(argv[1], observation, action);
    actor->print_model_info();
    std::printf("check_dims: %d\n", actor->check_dims() ? 1 : 0);
    if (mode == "twos") observation.fill(2.0f);
    int ticks = mode == "ticks" && argc > 3 ? std::atoi(argv[3]) : 1;
    std::FILE *dump = mode == "ticks" && argc > 4 ? std::fopen(argv[4], "wb") : nullptr;
    double best = 1e30;
    for (int t = 0; t < ticks; ++t) {
      if (mode == "ticks") observation[t % observation.size()] += 0.001f;  // obs changes every tick
      auto t0 = std::chrono::steady_clock::now();
      actor->act();
      auto t1 = std::chrono::steady_clock::now();
      best = std::min(best, std::chrono::duration<double, std::micro>(t1 - t0).count());
      if (dump && std::fwrite(action.data(), sizeof(float), action.size(), dump) != action.size()) return 4;
    }
    if (dump) std::fclose(dump);
    std::printf("Action:");
    for (float a : action) std::printf(" %.9g", a);
    std::printf("\nbest_us: %.3f\n", best);
  } catch (const std::exception &ex) {
    std::printf("exception: %s\n", ex.what());
    return 3;
  }
  return 0;
}
