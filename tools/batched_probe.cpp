// Diagnostics (r06): the batched kernel's time per launch from C++,
// measured the way tools/launch_probe.hip measures its spin kernels (back-to-back
// go2pi_run_device launches on one non-blocking HIP stream, HIP events around n of
// them), so that the two can be compared without the Python / torch path in between.
// Build (repo root): g++ -O2 -std=c++20 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
//   tools/batched_probe.cpp -Lgo2_onnx_controller_amd/lib -lgo2pi -L/opt/rocm/lib -lamdhip64
//   -Wl,-rpath,$PWD/go2_onnx_controller_amd/lib -o tools/batched_probe.bin
// Run: tools/batched_probe.bin MODEL.onnx [batch] [launches]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "go2pi.h"

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s MODEL.onnx [batch] [launches]\n", argv[0]);
    return 2;
  }
  const int B = argc > 2 ? std::atoi(argv[2]) : 4096, n = argc > 3 ? std::atoi(argv[3]) : 1000;
  go2pi_opts o{};
  o.struct_size = sizeof(o);
  go2pi_default_opts(&o);
  o.max_batch = B;
  go2pi_engine *e = nullptr;
  if (go2pi_create(argv[1], &o, &e) != GO2PI_OK) {
    std::fprintf(stderr, "create: %s\n", go2pi_last_error());
    return 1;
  }
  int64_t in_dim = 0, out_dim = 0;
  go2pi_io_dims(e, &in_dim, &out_dim);
  float *obs = nullptr, *act = nullptr;
  if (hipMalloc(&obs, sizeof(float) * B * in_dim) != hipSuccess || hipMalloc(&act, sizeof(float) * B * out_dim) != hipSuccess)
    return 1;
  std::vector<float> h((size_t)B * in_dim);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 2000) / 1000.f - 1.f;
  if (hipMemcpy(obs, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return 1;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  char name[128];
  go2pi_batched_kernel(e, name, sizeof(name));
  std::vector<double> per;
  for (int rep = 0; rep < 5; ++rep) {
    for (int i = 0; i < 200; ++i) go2pi_run_device(e, obs, act, B, s);
    (void)hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, s);
    for (int i = 0; i < n; ++i)
      if (go2pi_run_device(e, obs, act, B, s) != GO2PI_OK) {
        std::fprintf(stderr, "run: %s\n", go2pi_last_error());
        return 1;
      }
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    per.push_back(ms * 1000.0 / n);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  std::sort(per.begin(), per.end());
  std::printf("%s batch %d: %.3f us per launch (median of 5 x %d; min %.3f max %.3f)\n", name, B, per[2], n, per[0],
              per[4]);
  go2pi_destroy(e);
  return 0;
}
