/*
 * go2pi — MI355X-native batched policy-inference engine, C ABI.
 *
 * This is the boundary the drop-in `ONNXActor` (include/onnx_actor.hpp) and any
 * FFI (ctypes, cgo, JNI …) bind to. Plain pointers and sizes only; no HIP or
 * torch types in any signature (a HIP stream travels as `void*`).
 *
 * Each entry point replaces one piece of the reference's onnxruntime-backed
 * operator (inria-paris-robotics-lab/go2_onnx_controller):
 *
 *   go2pi_create        <- ONNXActor::ONNXActor  onnx_inference/src/cpp/onnx_actor.cpp:6-36
 *                          (Ort::Session(env, path, SessionOptions{nullptr}) :16,
 *                           input/output name+shape discovery :23-28)
 *   go2pi_io_name /
 *   go2pi_io_shape      <- GetInputNameAllocated / GetInputTypeInfo … GetShape  onnx_actor.cpp:23-28
 *                          (consumed by print_model_info :60-66 and check_dims :50-58)
 *   go2pi_run           <- ONNXActor::act()  onnx_actor.cpp:38-48 (Session::Run :47),
 *                          generalised to a batch of robots (rows)
 *   go2pi_run_device    <- same, device-resident obs/action (many-robot path)
 *   go2pi_reset_hidden  <- (build-defined, recurrent policies)
 *   go2pi_last_error    <- Ort::Exception::what()  (the reference throws; the C ABI returns a
 *                          status and the C++ shim rethrows std::runtime_error)
 *   go2pi_destroy       <- ~ONNXActor  onnx_actor.hpp:38
 *
 * Return codes: 0 = OK, negative = error (message via go2pi_last_error(), per
 * thread). An engine instance is NOT re-entrant: one call at a time, exactly as
 * the reference binds fixed tensors per ONNXActor (onnx_actor.cpp:31-35).
 */
#ifndef GO2PI_H_
#define GO2PI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GO2PI_OK 0
#define GO2PI_E_INVALID (-1)   /* bad argument */
#define GO2PI_E_MODEL (-2)     /* unreadable / unsupported ONNX model */
#define GO2PI_E_DEVICE (-3)    /* no HIP device / HIP runtime error */
#define GO2PI_E_CAPACITY (-4)  /* batch above the engine's capacity */

typedef struct go2pi_engine go2pi_engine;

/* Engine options. Zero-initialise, then call go2pi_default_opts(). */
typedef struct go2pi_opts {
  int32_t struct_size;   /* = sizeof(go2pi_opts) */
  int32_t device;        /* HIP device ordinal, default 0 */
  int64_t max_batch;     /* robots per call capacity (device buffers), default 4096 */
  int32_t use_graph;     /* 1 (default): the small-batch host path replays a captured hipGraph */
  int32_t log_level;     /* OrtLoggingLevel-compatible: 0 VERBOSE … 4 FATAL, default 2 */
  int32_t waves;         /* waves per workgroup of the batched kernel: 4, 8 or 16 (0 = auto: 4 for a uniform MLP, else 8) */
  int32_t small_batch;   /* host batches <= this use the GEMV chain (0 = auto: 8; -1 = never) */
  /* Optional fused prologue / epilogue (north_star: obs normalisation, action tanh/clip).
     All OFF by default so act() stays comparable to the shipped graph. */
  const float *obs_mean; /* [in_dim] or NULL */
  const float *obs_std;  /* [in_dim] or NULL: x <- (x - mean) / std */
  float obs_clip;        /* > 0: clamp normalised obs to [-obs_clip, obs_clip] */
  int32_t action_tanh;   /* 1: action <- tanh(action) */
  float action_clip;     /* > 0: clamp action to [-action_clip, action_clip]
                            (the caller's kActionLimit clamp, controller.cpp:217-223) */
  float action_scale;    /* != 0 and != 1: action <- action * action_scale (after clip) */
  /* > 0: go2pi_run and go2pi_controller_step at batch <= 8 are served by a RESIDENT
     kernel (no launch per call: the request and its input rows travel as tagged
     granules in host-mapped memory); the kernel leaves after this many ms without a
     request and is relaunched by the next call. Dense (non-recurrent) policies whose
     final layer is <= 16 wide; others keep the launch path. 0 (default): one launch
     per call. Any other call on the engine first stops the resident kernel. */
  int32_t resident_ms;
} go2pi_opts;

void go2pi_default_opts(go2pi_opts *opts);

/* Load an ONNX policy (Gemm/MatMul+Add with Elu/Relu/Tanh/Sigmoid/LeakyRelu, optional GRU)
   and upload it to the device. `opts` may be NULL (defaults). */
int go2pi_create(const char *onnx_path, const go2pi_opts *opts, go2pi_engine **out);
int go2pi_create_from_memory(const void *onnx_bytes, size_t nbytes, const go2pi_opts *opts,
                             go2pi_engine **out);
void go2pi_destroy(go2pi_engine *e);

/* I/O metadata of graph input/output `index` (0 = the bound observation / action). */
int go2pi_num_io(const go2pi_engine *e, int32_t *n_inputs, int32_t *n_outputs);
int go2pi_io_name(const go2pi_engine *e, int32_t is_output, int32_t index, char *buf, size_t cap);
/* Writes up to `cap` dims; *rank receives the true rank. Symbolic dims read as -1. */
int go2pi_io_shape(const go2pi_engine *e, int32_t is_output, int32_t index, int64_t *dims, int32_t cap,
                   int32_t *rank);
/* Per-robot feature counts of the bound observation / action (shape[1]). */
int go2pi_io_dims(const go2pi_engine *e, int64_t *in_dim, int64_t *out_dim);

/* Synchronous host path: obs [batch][in_dim] -> act [batch][out_dim], host memory
   (the act() contract: reads obs at call time, overwrites act in place). */
int go2pi_run(go2pi_engine *e, const float *obs, float *act, int64_t batch);

/* Asynchronous device path: obs/act are device pointers on e's device; enqueued on
   `hip_stream` (a hipStream_t; NULL = the HIP null stream, as in HIP). No host sync.
   The caller must use the same HIP runtime instance as this library (e.g. load
   PyTorch's libamdhip64 first when sharing torch streams/tensors). */
int go2pi_run_device(go2pi_engine *e, const float *obs_dev, float *act_dev, int64_t batch, void *hip_stream);

/* Recurrent policies carry one hidden row per robot (engine-resident, HBM).
   Run `steps` ticks back to back with the hidden rows kept on-chip between ticks:
   obs_dev [steps][batch][in_dim] -> act_dev [steps][batch][out_dim]. For a
   feed-forward policy this is `steps` independent batched calls. */
int go2pi_run_sequence_device(go2pi_engine *e, const float *obs_dev, float *act_dev, int64_t steps,
                              int64_t batch, void *hip_stream);

/* Zero the hidden state of robots whose mask byte is non-zero (mask NULL = all). */
int go2pi_reset_hidden(go2pi_engine *e, const uint8_t *mask, int64_t batch);
/* Copy hidden state rows [0,batch) to/from host (hidden_dim floats per robot). */
int go2pi_get_hidden(go2pi_engine *e, float *h, int64_t batch);
int go2pi_set_hidden(go2pi_engine *e, const float *h, int64_t batch);
int go2pi_hidden_dim(const go2pi_engine *e, int64_t *hidden_dim);

/* Wait for all work queued on the engine's own stream. */
int go2pi_sync(go2pi_engine *e);

/* Algorithmic cost per robot-step (for roofline accounting in bench.py). */
typedef struct go2pi_cost {
  double flops_per_row;    /* 2*MAC of every contraction (+ nothing for activations) */
  double weight_bytes;     /* fp32 parameter bytes (unpadded) */
  double io_bytes_per_row; /* obs + action (+ 2x hidden for recurrent) bytes */
  int32_t n_layers;
  int32_t has_gru;         /* recurrent cell in front of the dense layers: 0 none, 1 GRU, 2 LSTM */
} go2pi_cost;
int go2pi_get_cost(const go2pi_engine *e, go2pi_cost *cost);

/* Name of the batched kernel instantiation this engine launches for batches
   above the small-batch paths, e.g. "policy_fused_kernel<4, 8, 1>" (waves per
   workgroup, tiles per wave of the 4-wave pipeline, head tiles), as rocprofv3
   reports it. Writes a NUL-terminated string into buf (truncated to cap-1). For
   profiling tools; no compute. */
int go2pi_batched_kernel(const go2pi_engine *e, char *buf, size_t cap);

/* Name of the resident kernel that serves go2pi_run at batch <= 8 on this engine
   (opts.resident_ms > 0), then " ring=vram" when the request ring is in device
   memory the host writes through the large-BAR mapping, " ring=host" when it is in
   pinned host memory; "none" when no resident kernel serves act(). E.g.
   "policy_wide_kernel<4, 8, 12, 0> ring=vram". For tests and profiling tools; no
   compute. */
int go2pi_resident_kernel(const go2pi_engine *e, char *buf, size_t cap);

/* Resident kernel launches this engine has made so far (one serves every request
   until it idles out or another call stops it; a kernel that aborts on a request
   shows up as a launch per call). For tests and profiling tools; no compute. */
int go2pi_resident_launches(const go2pi_engine *e, int64_t *n);

/* Parse and lower an ONNX policy WITHOUT touching a device (no compute): writes a
   JSON description (I/O names and shapes, the lowered layer program with
   per-layer weight/bias checksums) into buf. Returns the JSON length (>= 0) or an
   error code; truncates to cap-1 bytes. For loader tests and tooling. */
int go2pi_inspect_model(const char *onnx_path, char *buf, size_t cap);

/* ---------------------------------------------------------------------------
   Controller tick: the Go2 ONNXController's per-tick work around act(), fused
   into the policy launch (many robots or one):
     prologue  <- observation assembly, controller.cpp:173-212 + lowstate_cb_
                  controller.hpp:93-110 (gravity projection of the IMU quaternion,
                  q - q0, joystick velocity command, foot contacts, and the
                  kHistory-step history shift of populate_buffer, controller.hpp:45-68)
     epilogue  <- action post-processing, controller.cpp:217-223 (clamp to
                  +-kActionLimit, joystick stop button zeroes the action) and
                  240-248 (q_des = q0 + 0.25 a, kp/kd arrays for send_command)
   Needs a policy whose observation is kHistory x 49 features (kDimObs,
   controller.hpp:14; the shipped model: 98) and whose action has 12.
   Per-robot raw state row, GO2PI_CTL_STATE_DIM floats:
     [0:4]  imu_state.quaternion (w, x, y, z)     [4:7]   imu_state.gyroscope
     [7:19] joint q (Isaac order)                 [19:31] joint dq
     [31:35] foot_force (Unitree order, as in LowState)   [35] reserved
   Per-robot joystick row, GO2PI_CTL_JOY_DIM floats:
     {has_axes, axes[0], axes[1], axes[3], buttons[0]}; has_axes = 0 keeps the
     previous velocity command (the reference only updates it when axes are
     present). A NULL joystick pointer means no message for any robot (velocity
     command kept, stop button released).
   State carried between ticks (caller-owned, in place, as the reference's
   observation_ / action_ members): obs [batch][in_dim] holds the previous
   observation on entry and this tick's on return (the ObservationAction log
   row, controller.cpp:226); action [batch][12] holds the previous action on
   entry and this tick's post-processed action on return. Zero both to start.
   Outputs q_des / kp / kd [batch][12] (double, as send_command takes them) may
   be NULL. status [batch] (may be NULL): bit 0 set when a NaN entered the
   observation (the reference exit(1)s in populate_buffer's check,
   controller.hpp:57-64); the tick still completes. */
#define GO2PI_CTL_STATE_DIM 36
#define GO2PI_CTL_JOY_DIM 5
#define GO2PI_CTL_DOF 12

typedef struct go2pi_ctl_params {
  int32_t struct_size;     /* = sizeof(go2pi_ctl_params) */
  float kp;                /* kp_ (controller.hpp:119), default 28 */
  float kd;                /* kd_ (:120), default 0.5 */
  float kp_stop;           /* kp while the stop button is held (controller.cpp:246), default 5 */
  float action_limit;      /* kActionLimit (controller.hpp:17), default 1000 */
  float contact_threshold; /* foot_force >= this is a contact (controller.hpp:100-103), default 22 */
  float gravity_w[3];      /* gravity_w_ (controller.hpp:131), default (0, 0, -1) */
  double action_scale;     /* q_des = q0 + action_scale * a (controller.cpp:244), default 0.25 */
  double q0[12];           /* q0_ (controller.hpp:165), Isaac order */
} go2pi_ctl_params;

void go2pi_ctl_default_params(go2pi_ctl_params *params);
/* Set the engine's controller parameters (synchronous; defaults at create). */
int go2pi_ctl_set_params(go2pi_engine *e, const go2pi_ctl_params *params);
/* kHistory of the bound policy (in_dim / 49), or GO2PI_E_MODEL if its I/O is not
   a Go2 controller's (in_dim a multiple of 49, out_dim 12). */
int go2pi_ctl_history(const go2pi_engine *e, int32_t *history);

/* One tick for `batch` robots, host buffers (synchronous; batch <= 8 runs as
   one launch on host-mapped staging, larger batches stage through HBM). */
int go2pi_controller_step(go2pi_engine *e, const float *state, const float *joy, float *obs, float *action,
                          double *q_des, double *kp, double *kd, uint32_t *status, int64_t batch);
/* Same on device pointers, enqueued on `hip_stream`, no host sync. */
int go2pi_controller_step_device(go2pi_engine *e, const float *state_dev, const float *joy_dev, float *obs_dev,
                                 float *action_dev, double *q_des_dev, double *kp_dev, double *kd_dev,
                                 uint32_t *status_dev, int64_t batch, void *hip_stream);

/* Diagnostics: copy up to n per-workgroup clock stamps of the last batched launch
   ({s_memtime, s_memrealtime} at start and end, 4 per workgroup). Needs a
   GO2PI_DIAG_CLOCK build and GO2PI_DIAG_STAMPS set at create; returns the count. */
int go2pi_diag_stamps(go2pi_engine *e, uint64_t *out, int64_t n);

/* Thread-local message of the last failing call on this thread ("" if none). */
const char *go2pi_last_error(void);

/* Library version string. */
const char *go2pi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GO2PI_H_ */
