/* Batch-1 controller tick latency through the C ABI, as a C controller would call it
 * in place of the work publish() does around act() (onnx_controller/src/controller.cpp
 * :156-251): go2pi_controller_step on one robot's raw state and
 * joystick rows, the observation history and previous action updated in place, q_des /
 * kp / kd and the NaN status out. The resident kernel serves it (resident_ms = 100;
 * argv[4] = 0: one launch per tick). Timed per call with CLOCK_MONOTONIC over <warm>
 * untimed then <iters> timed ticks; prints p50 / p99 in microseconds.
 * Usage: ctl_lat <model.onnx> <iters> <warm> [resident_ms] [min]
 * ("min": q_des / kp / kd / status not asked for, only the observation and the action) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "go2pi.h"

static int cmp_d(const void *a, const void *b) {
  const double x = *(const double *)a, y = *(const double *)b;
  return (x > y) - (x < y);
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  const int iters = atoi(argv[2]), warm = atoi(argv[3]);
  const int lean = argc > 5 && strcmp(argv[5], "min") == 0;
  go2pi_opts o;
  go2pi_default_opts(&o);
  o.max_batch = 8;
  o.resident_ms = argc > 4 ? atoi(argv[4]) : 100;
  go2pi_engine *e = NULL;
  if (go2pi_create(argv[1], &o, &e)) {
    printf("create: %s\n", go2pi_last_error());
    return 3;
  }
  int64_t in_dim = 0, out_dim = 0;
  go2pi_io_dims(e, &in_dim, &out_dim);
  float state[GO2PI_CTL_STATE_DIM] = {1.f, 0.f, 0.f, 0.f}; /* upright: quaternion (1, 0, 0, 0) */
  float joy[GO2PI_CTL_JOY_DIM] = {1.f, 0.2f, 0.3f, 0.f, 0.f};
  float *obs = calloc((size_t)in_dim, sizeof(float)), action[GO2PI_CTL_DOF] = {0};
  double q_des[GO2PI_CTL_DOF], kp[GO2PI_CTL_DOF], kd[GO2PI_CTL_DOF];
  uint32_t status = 0;
  double *ts = malloc(sizeof(double) * (size_t)iters);
  for (int t = 0; t < warm + iters; ++t) {
    state[7 + t % 12] += 0.001f; /* the joints move every tick */
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    const int rc = lean ? go2pi_controller_step(e, state, joy, obs, action, NULL, NULL, NULL, NULL, 1)
                        : go2pi_controller_step(e, state, joy, obs, action, q_des, kp, kd, &status, 1);
    clock_gettime(CLOCK_MONOTONIC, &b);
    if (rc) {
      printf("controller_step: %s\n", go2pi_last_error());
      return 4;
    }
    if (t >= warm) ts[t - warm] = (double)(b.tv_sec - a.tv_sec) * 1e6 + (double)(b.tv_nsec - a.tv_nsec) * 1e-3;
  }
  qsort(ts, (size_t)iters, sizeof(double), cmp_d);
  printf("p50_us: %.3f\np99_us: %.3f\nstatus: %u\n", ts[iters / 2], ts[(size_t)iters * 99 / 100], status);
  go2pi_destroy(e);
  free(ts);
  free(obs);
  return 0;
}
