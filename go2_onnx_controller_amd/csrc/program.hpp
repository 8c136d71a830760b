// Device-side description of a loaded policy ("program"), passed to the HIP
// kernels by value. Shared by engine.cpp (builds it) and kernels.hip (runs it).
//
// Weight layout in HBM ("fragment order", built once at load time):
// a dense layer W[N][K] (ONNX Gemm transB=1 layout) is zero-padded to
// N_pad (64 for hidden layers, 16 for the final one), K_pad = ceil64(K) and
// stored chunk-major:
//     packed[c][t][lane] : float4,  c < K_pad/16, t < N_pad/16, lane < 64
//     packed[c][t][lane].j = W[16t + (lane & 15)][16c + 4(lane >> 4) + j]
// so one wave-instruction (64 lanes x 16 B) reads 1 KiB of contiguous memory
// and the float4 feeds four v_mfma_f32_16x16x4_f32 as the B operand (B[k][n] =
// W[n][k]) — see kernels.hip. Chunk-major order keeps the slab that every CU
// of an XCD reads at the same moment (chunk c of all tiles) contiguous, so it
// spreads over all L2 channels instead of striding one (tile-major measured
// slower). The GRU gates use the same idea with three gate fragments per
// (chunk, tile): packed[c][t][gate][lane].
#pragma once

#include <cstdint>

#define GO2PI_MAX_LAYERS 8
#define GO2PI_TILE_ROWS 16      // robots per workgroup tile in the batched kernel
#define GO2PI_SMALL_MAXB 8      // max rows of the GEMV chain
#define GO2PI_STAMPS_PER_WG 64  // diagnostics: {start,end} x {memtime,realtime}, phase marks, per-wave layer-1 marks
// A batched launch of more than this many workgroups (one per CU: ~100 KiB of LDS
// each) bumps the device's yield counter, so idle resident kernels (<= 32 CUs for the
// 48->512^3->12 policy, 8 for the shipped one) give their CUs back; smaller launches
// (a per-tick recurrent or controller launch at a few robots) fit beside them and
// must not evict them on every call.
#define GO2PI_YIELD_MIN_GRID 64

// Clock stamps (GO2PI_DIAG_CLOCK builds, tools/clock_probe.py): s_memtime (or the
// 100 MHz s_memrealtime) of a workgroup's phases into P.stamps[block][slot]. In the
// shipped build the macros are empty: no load, no store, no condition evaluated.
#ifdef GO2PI_DIAG_CLOCK
#define GO2PI_STAMP_AT(row, cond, slot)                                  \
  do {                                                                   \
    if ((row) && (cond)) ((__attribute__((address_space(1))) unsigned long long *)(row))[slot] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define GO2PI_STAMP(P, cond, slot) \
  GO2PI_STAMP_AT((P).stamps ? (P).stamps + blockIdx.x * GO2PI_STAMPS_PER_WG : nullptr, cond, slot)
#define GO2PI_STAMP_RT(P, cond, slot)                                                                       \
  do {                                                                                                      \
    if ((P).stamps && (cond))                                                                              \
      ((__attribute__((address_space(1))) unsigned long long *)(P).stamps)[blockIdx.x * GO2PI_STAMPS_PER_WG + (slot)] = \
          __builtin_amdgcn_s_memrealtime();                                                                  \
  } while (0)
// (r06) the workgroup's start, taken at kernel entry and stored as slots 0 / 1 once the
// stamp row is known: a start stamp taken where the row pointer is first read waits for
// that program load (~1K cycles into a cold launch), which moved that time out of the
// measured workgroup life and into "event - span"
#define GO2PI_ENTRY_CLOCK()                                                   \
  const unsigned long long go2pi_t_entry = __builtin_amdgcn_s_memtime(),     \
                           go2pi_rt_entry = __builtin_amdgcn_s_memrealtime()
#define GO2PI_STAMP_ENTRY(P, cond)                                                                       \
  do {                                                                                                   \
    if ((P).stamps && (cond)) {                                                                          \
      auto *r_ = (__attribute__((address_space(1))) unsigned long long *)(P).stamps + blockIdx.x * GO2PI_STAMPS_PER_WG; \
      r_[0] = go2pi_t_entry;                                                                             \
      r_[1] = go2pi_rt_entry;                                                                            \
    }                                                                                                    \
  } while (0)
#else
#define GO2PI_ENTRY_CLOCK() \
  do {                      \
  } while (0)
#define GO2PI_STAMP_ENTRY(P, cond) \
  do {                             \
  } while (0)
#define GO2PI_STAMP_AT(row, cond, slot) \
  do {                                  \
    (void)sizeof(row);                  \
  } while (0)
#define GO2PI_STAMP(P, cond, slot) \
  do {                             \
  } while (0)
#define GO2PI_STAMP_RT(P, cond, slot) \
  do {                                \
  } while (0)
#endif

namespace go2pi {

struct DevLayer {
  const float *w;     // packed fragments (float4 granules), see above
  const float *bias;  // [N_pad], zero padded
  int K_pad, N_pad, N;
  int act;
  float alpha, beta;  // the activation's attributes (onnx_model.hpp Dense)
  int pad1, pad2;
};

// The recurrent cell in front of the dense head (ONNX GRU or LSTM; the field
// names are the GRU's). State per robot in HBM: h [H] (GRU), h [H] | c [H] (LSTM).
struct DevGru {
  const float *w;    // packed [Cx + Ch][Ht][G gates][64] float4 (chunk-major)
  const float *bzr;  // GRU: [2H] Wb_z + Rb_z | Wb_r + Rb_r; LSTM: [4H] Wb + Rb, gates i, o, f, c
  const float *bh;   // GRU: [2H] Wb_h | Rb_h; LSTM: unused
  int I, I_pad, H, lbr;
  int cell;          // 0 GRU, 1 LSTM
  int sw;            // state floats per robot: H (GRU), 2H (LSTM)
};

struct DevProgram {
  // ---- hot block (the first 80 bytes): every field the 4-wave pipeline reads,
  // so that one scalar burst at kernel start fetches all of it (the fields'
  // scattered lazy loads were a chain of ~7 dependent scalar round trips before
  // the first observation load; fused_impl.hpp W4Hot). Set for pipeline programs.
  const float *l0_w;       // = L[0].w, the base of the packed dense layers (back to back)
  const float *head_w;     // = L[nl - 1].w
  const float *head_bias;  // = L[nl - 1].bias
  const float *bpack;      // = w4_bpack
  const float *zero_hot;   // = zero
  unsigned *err_hot;       // = err
  int nbias;               // = w4_bias
  int head_n;              // = L[nl - 1].N
  int c0;                  // = L[0].K_pad / 16 (layer 0's k-chunks)
  int in_dim_hot;          // = in_dim
  int hid_act, head_act;   // activation of every hidden layer (uniform), of the head
  float hid_alpha, head_alpha;
  int post_plain;          // 1: no action post-processing (tanh / clip / scale): the head's plain store
  // ---- the rest
  int nl;
  int in_dim, in_pad, out_dim;
  int lds_stride;  // floats per row of an LDS activation buffer
  int has_gru;
  int head_fuse;   // >0: the final layer (this many 16-col tiles) is fused into the one before it
  int zero_fill;   // 1: clear LDS activation buffers at kernel start (padded columns never written)
  int w4_tpw;      // >0: 4-wave uniform-MLP pipeline (kernels.hip, w4_step), tiles per wave of every hidden layer
  int w4_bias;     // pipeline: LDS floats holding every hidden layer's bias (sum of their N_pad), else 0
  const float *w4_bpack;  // pipeline: those biases packed back to back in device memory (one LDS-DMA stream)
  int w4_plain;           // pipeline, 1: no prologue / epilogue arithmetic, no recurrent cell (the lean kernel)
  int w4_gru_lean;        // 1: a GRU policy served by the lean GRU tick (policy_gru_kernel, r05)
  int ctl_general;        // 1: the controller tick runs the general body, not the lean tick kernel (A/B)
  int w4_c0m;             // pipeline: layer 0's k-chunks mod 4 (0 or 3; K padded to 16, not 64, when 3)
  int w4_actc;            // lean kernel: the hidden activation as a compile-time constant (1 = Elu), or -1
  int w4_nhc;             // lean kernel: the hidden-layer count as a compile-time constant (3), or 0 (runtime)
  float hid_beta, head_beta;  // second activation attribute of the hidden layers / the head (Clip max, ...)
  // prologue: x <- clamp((x - sub) / div * mul, -obs_clip, obs_clip); sub/div/mul may be null
  const float *pre_sub;
  const float *pre_div;
  const float *pre_mul;
  int pre_sub_bcast, pre_div_bcast, pre_mul_bcast;  // 1: single scalar broadcast over features
  int pre_clip;         // 1: x <- clip(x, obs_lo, obs_hi) (a graph's input Clip and / or go2pi_opts.obs_clip)
  float obs_lo, obs_hi;
  // epilogue on the final layer: y <- scale * clamp(tanh?(act(y)), lo, hi)
  int post_tanh;
  float clip_lo, clip_hi, scale;
  DevGru gru;
  unsigned long long *stamps;  // diagnostics only (GO2PI_DIAG_CLOCK builds): 4 per workgroup
  const float *zero;           // >= 64 zero floats in device memory (source of the padding lanes' loads)
  unsigned *err;               // host-mapped word: set to 1 when a wave-to-wave layer hand-off times out
  unsigned *yield;             // the device's batched-launch counter (one per device and process): every
                               // batched kernel adds 1 at its start, an idle resident kernel that sees it
                               // move leaves (it holds CUs the batched kernel needs; resident.hip)
  DevLayer L[GO2PI_MAX_LAYERS];
};

// ---------------------------------------------------------------------------
// Controller tick: the Go2 controller's observation
// assembly (onnx_controller/src/controller.cpp:173-212, controller.hpp:45-68,
// 93-110) fused as the policy's prologue and its action post-processing
// (controller.cpp:217-223, 240-248) fused into the final layer's store.
// Raw per-robot state row (floats), see include/go2pi.h GO2PI_CTL_*:
//   [0:4] imu quaternion (w,x,y,z)  [4:7] gyroscope  [7:19] q  [19:31] dq
//   [31:35] foot_force (Unitree order)  [35] reserved
// Joystick row: {has_axes, axes[0], axes[1], axes[3], buttons[0]}.
#define GO2PI_CTL_STATE_DIM 36
#define GO2PI_CTL_JOY_DIM 5
#define GO2PI_CTL_DOF 12
#define GO2PI_CTL_STEP_DIM 49  // kDimObs, controller.hpp:14

struct DevCtlParams {  // device memory, set by go2pi_ctl_set_params
  double q0[GO2PI_CTL_DOF];
  double action_scale;
  double kp_run, kd_run, kp_stop;  // already widened as the reference widens them (float -> double)
  float action_limit, contact_threshold;
  float gravity_w[3];
  int hist;  // kHistory (in_dim / 49)
};

struct DevCtl {  // per call (kernel argument)
  const DevCtlParams *prm;
  const float *state;  // [B][GO2PI_CTL_STATE_DIM]
  const float *joy;    // [B][GO2PI_CTL_JOY_DIM] or null (no joystick message: vel_cmd kept, buttons[0] = 0)
  float *obs;          // [B][in_dim]  observation_ with history: read (t-1), written (t)
  float *action;       // [B][12]      action_: read (t-1, history), written (t)
  double *q_des, *kp, *kd;  // [B][12] each, or null
  unsigned *status;         // [B] or null: bit 0 = NaN entered the observation
};

// Host-side launchers (kernels.hip). All launches are asynchronous on `stream`.
// Return a hipError_t as int.
// p: host copy (grid, LDS size, kernel choice); p_dev: its device-memory copy (the kernel reads that)
int launch_policy_fused(const DevProgram &p, const DevProgram *p_dev, int waves, const float *obs, float *act,
                        float *hidden, int batch, int steps, void *stream);
size_t fused_lds_bytes(const DevProgram &p, int waves);
int launch_gemv_layer(const DevProgram &p, int layer, const float *x, int x_stride, float *y, int y_stride,
                      int batch, void *stream);
size_t gemv_lds_bytes(const DevProgram &p, int layer);
int configure_kernels(const DevProgram &p, int waves);
// batch <= GO2PI_SMALL_MAXB act() in one launch; gran: [nl-1][gstride] u64 granules
// (tag = epoch0 + layer), err: host-visible word set to 1 on a hand-off timeout,
// done: host-visible word set to epoch0 once the action is written (final layer
// must be a single 16-output tile; may be null).
// p_dev: a device-memory copy of p (the kernel reads the program from it).
int launch_latency(const DevProgram &p, const DevProgram *p_dev, const float *obs, float *act, int batch,
                   unsigned epoch0,
                   unsigned long long *gran, int gstride, unsigned *err, unsigned *done, void *stream);
int latency_grid(const DevProgram &p);
// Controller tick variants of the two launchers above (steps = 1; ctl.obs / ctl.action
// replace obs / act). The latency variant needs the final layer to be one tile.
int launch_policy_fused_ctl(const DevProgram &p, const DevProgram *p_dev, int waves, const DevCtl &ctl,
                            float *hidden, int batch, void *stream);
int launch_latency_ctl(const DevProgram &p, const DevProgram *p_dev, const DevCtl &ctl, int batch, unsigned epoch0,
                       unsigned long long *gran, int gstride, unsigned *err, unsigned *done, void *stream);

// Resident batch <= GO2PI_SMALL_MAXB path (resident.hip): ONE launch serves act()
// requests until it is told to leave or sits idle for idle_ticks of the 100 MHz
// wall clock. req: host-mapped [1 + SMALL_MAXB * in_dim] {tag, value} granules,
// req[0] = {epoch, batch} (tag GO2PI_RES_LEAVE: leave), req[1 + i] = {epoch, obs[i]};
// act: host-mapped [SMALL_MAXB][out_dim]; done: set to the epoch once the action is
// written, to GO2PI_RES_LEAVE when the kernel leaves. Layer-l granules carry tag
// epoch + 1 + l. gran must be zeroed before every launch (a leaving workgroup tags
// its slots GO2PI_RES_LEAVE so waiting consumers leave too). mirror: device
// [1 + SMALL_MAXB * in_dim] granules, workgroup 0's copy of each request for the
// other workgroups (zeroed before every launch, like gran). ctl non-null: the
// controller-tick form (go2pi_controller_step at batch <= 8): ctl's rows are the
// pinned host staging of the outputs; req[0] = {epoch, batch | GO2PI_RES_* flags},
// req[1 ..] = the tick's rows as {epoch, value} granules: state [B][36], joystick
// [B][5], previous obs [B][in_dim], previous action [B][12].
#define GO2PI_RES_LEAVE 0xFFFFFFFFu
// Controller-tick request flags (header low word, bits 8..): the optional rows the call passed.
#define GO2PI_CTL_RAW (GO2PI_CTL_STATE_DIM + GO2PI_CTL_JOY_DIM + GO2PI_CTL_DOF)  // request floats per robot + in_dim
#define GO2PI_RES_JOY (1u << 8)
#define GO2PI_RES_QDES (1u << 9)
#define GO2PI_RES_KP (1u << 10)
#define GO2PI_RES_KD (1u << 11)
#define GO2PI_RES_STATUS (1u << 12)
// yield: the device's batched-launch counter (DevProgram::yield): an idle resident
// kernel leaves when a batched kernel starts.
// A GRU policy (p.has_gru, GRU lbr = 1, H % 64 == 0, ctl null) runs the cell as a
// tiled layer: hgran = device [2][SMALL_MAXB][H] granules (zeroed before every
// launch) carry h' between requests, hidden = the engine's state rows (read for
// rows not yet written in this launch, written back when the kernel leaves).
// act() form: the action rows travel to the host as {epoch, value} granules in actg
// (host-mapped [SMALL_MAXB][out_dim]): the host checks the data itself, so no drain
// and no done word sit between the last store and the answer.
int launch_resident(const DevProgram &p, const DevProgram *p_dev, const unsigned long long *req,
                    unsigned long long *actg,
                    unsigned long long *gran, int gstride, unsigned long long *mirror, unsigned *err,
                    unsigned *done, unsigned long long idle_ticks, const DevCtl *ctl, unsigned long long *hgran,
                    float *hidden, const unsigned *yield, void *stream);

// The single-workgroup resident form (resident.hip policy_resident1_kernel, r04):
// dense policies of <= 4 layers whose weights fit one CU's registers, at most 16
// outputs. Same request / answer / leave protocol as launch_resident.
bool resident1_fits(const DevProgram &p, bool ctl);  // ctl: the controller form (512 threads)
// The controller form answers in granules too when policy_act1_kernel serves it (r05;
// true here): actg holds ctl_gran(in_dim).total granules, each output value tagged with
// the request's epoch, and there is no done word per request (the r04 forms and
// launch_resident's drain the plain outputs into ctl's staging, then set done).
bool resident1_ctl_granules(const DevProgram &p);
// Offsets (in granules) of the controller form's answer, fixed for GO2PI_SMALL_MAXB rows:
// action [8][12], q_des / kp / kd [8][12][2] (each double's low then high 32 bits),
// the new observation rows [8][in_dim], status [8]. Only the requested outputs are written.
struct CtlGran {
  int act, qdes, kp, kd, obs, status, total;
};
constexpr CtlGran ctl_gran(int in_dim) {  // (constexpr: callable from device code too)
  constexpr int R = GO2PI_SMALL_MAXB, D = GO2PI_CTL_DOF;
  return CtlGran{0, R * D, 3 * R * D, 5 * R * D, 7 * R * D, 7 * R * D + R * in_dim, 7 * R * D + R * in_dim + R};
}
// ctl non-null: the controller-tick form (launch_resident's ctl semantics).
int launch_resident1(const DevProgram &p, const DevProgram *p_dev, const unsigned long long *req,
                     unsigned long long *actg, unsigned *err, unsigned *done, unsigned long long idle_ticks,
                     const unsigned *yield, const DevCtl *ctl, void *stream);

// The resident act() for wide dense policies (resident_wide.hip policy_wide_kernel, r06):
// 3..5 dense layers, every hidden layer H = 256 or 512 wide, a head of <= 16 outputs,
// layer 0 of K_pad <= 64. H / 16 workgroups, each polling the request ring itself (the
// ring must be in device memory: the host writes it through the large-BAR mapping).
// Same request / answer / leave protocol as launch_resident1 (act() form only); gran:
// [nl - 1][gstride >= 8 H] granules, zeroed before every launch.
struct WideShape {
  int nl, cw, f0;
};
WideShape wide_shape(const DevProgram &p);  // nl = 0: does not apply
int launch_resident_wide(const DevProgram &p, const DevProgram *p_dev, const unsigned long long *req,
                         unsigned long long *actg, unsigned long long *gran, int gstride, unsigned *err, unsigned *done,
                         unsigned long long idle_ticks, const unsigned *yield, void *stream);

}  // namespace go2pi
