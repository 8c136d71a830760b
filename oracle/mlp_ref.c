/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), and the
 * cpu_baseline leg of bench.py). Never linked into the product.
 *
 * Parity status: parity unpinned (see oracle/onnx_ref.py header): onnxruntime,
 * where the reference's arithmetic lives (onnx_inference/cmake/dependencies.cmake:14-31),
 * is absent, and the reference ships no expected outputs.
 *
 * Plain-C restatement of the reference's hot path, ONNXActor::act()
 * (onnx_inference/src/cpp/onnx_actor.cpp:38-48) -> Session::Run over the graph
 * Gemm(transB=1) -> Elu -> Gemm -> Elu -> Gemm -> Elu -> Gemm
 * (onnx_inference/data/model.onnx), i.e. per layer
 *     y[n] = act( b[n] + sum_k x[k] * W[n][k] )
 * with ONNX Elu: x > 0 ? x : alpha * (exp(x) - 1).
 *
 * Two precisions:
 *   mlpref_run_f32 — fp32 storage and arithmetic, k-sequential accumulation per
 *                    output (the "reference CPU path" timed by bench.py: it
 *                    stands in for onnxruntime's CPU EP, which cannot run here).
 *   mlpref_run_f64 — fp64 accumulation: the parity oracle.
 * And the build-defined GRU cell (ONNX GRU semantics, gate order z,r,h;
 * linear_before_reset selectable), SURVEY §8a row a8, in fp64.
 *
 * Rows are independent; OpenMP splits row blocks over `nthreads` threads.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { ACT_NONE = 0, ACT_ELU = 1, ACT_RELU = 2, ACT_TANH = 3, ACT_SIGMOID = 4, ACT_LEAKY = 5 };

#define MAXL 16
#define RB 8 /* rows per register block */

typedef struct {
  int nl;
  int K[MAXL], N[MAXL], act[MAXL];
  float alpha[MAXL];
  float *wt32[MAXL]; /* [K][N] transposed copy */
  float *b32[MAXL];
  double *wt64[MAXL];
  double *b64[MAXL];
  int maxw;
} mlpref_t;

static float actf(int a, float al, float x) {
  switch (a) {
    case ACT_ELU: return x > 0.f ? x : al * expm1f(x);
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_TANH: return tanhf(x);
    case ACT_SIGMOID: return 1.f / (1.f + expf(-x));
    case ACT_LEAKY: return x >= 0.f ? x : al * x;
    default: return x;
  }
}
static double actd(int a, double al, double x) {
  switch (a) {
    case ACT_ELU: return x > 0. ? x : al * expm1(x);
    case ACT_RELU: return x > 0. ? x : 0.;
    case ACT_TANH: return tanh(x);
    case ACT_SIGMOID: return 1. / (1. + exp(-x));
    case ACT_LEAKY: return x >= 0. ? x : al * x;
    default: return x;
  }
}

void *mlpref_create(int nl, const int *K, const int *N, const float *const *W, const float *const *b,
                    const int *act, const float *alpha) {
  if (nl < 1 || nl > MAXL) return NULL;
  mlpref_t *h = (mlpref_t *)calloc(1, sizeof(mlpref_t));
  h->nl = nl;
  h->maxw = 0;
  for (int l = 0; l < nl; ++l) {
    int k = K[l], n = N[l];
    h->K[l] = k; h->N[l] = n; h->act[l] = act[l]; h->alpha[l] = alpha[l];
    if (k > h->maxw) h->maxw = k;
    if (n > h->maxw) h->maxw = n;
    h->wt32[l] = (float *)malloc(sizeof(float) * (size_t)k * n);
    h->wt64[l] = (double *)malloc(sizeof(double) * (size_t)k * n);
    h->b32[l] = (float *)malloc(sizeof(float) * n);
    h->b64[l] = (double *)malloc(sizeof(double) * n);
    for (int i = 0; i < n; ++i) {
      h->b32[l][i] = b ? b[l][i] : 0.f;
      h->b64[l][i] = h->b32[l][i];
      for (int j = 0; j < k; ++j) {
        h->wt32[l][(size_t)j * n + i] = W[l][(size_t)i * k + j];
        h->wt64[l][(size_t)j * n + i] = W[l][(size_t)i * k + j];
      }
    }
  }
  return h;
}

void mlpref_destroy(void *p) {
  mlpref_t *h = (mlpref_t *)p;
  if (!h) return;
  for (int l = 0; l < h->nl; ++l) {
    free(h->wt32[l]); free(h->wt64[l]); free(h->b32[l]); free(h->b64[l]);
  }
  free(h);
}

/* one block of up to RB rows through every layer, fp32 */
static void block_f32(const mlpref_t *h, const float *x, float *y, int rows, int in_stride, int out_stride,
                      float *bufa, float *bufb) {
  const int W = h->maxw;
  for (int r = 0; r < rows; ++r) memcpy(bufa + (size_t)r * W, x + (size_t)r * in_stride, sizeof(float) * h->K[0]);
  float *cur = bufa, *nxt = bufb;
  for (int l = 0; l < h->nl; ++l) {
    const int K = h->K[l], N = h->N[l];
    const float *wt = h->wt32[l], *bb = h->b32[l];
    for (int r = 0; r < rows; ++r) memcpy(nxt + (size_t)r * W, bb, sizeof(float) * N);
    for (int k = 0; k < K; ++k) {
      const float *wr = wt + (size_t)k * N;
      for (int r = 0; r < rows; ++r) {
        const float xv = cur[(size_t)r * W + k];
        float *yr = nxt + (size_t)r * W;
        for (int n = 0; n < N; ++n) yr[n] = fmaf(xv, wr[n], yr[n]);
      }
    }
    for (int r = 0; r < rows; ++r)
      for (int n = 0; n < N; ++n) nxt[(size_t)r * W + n] = actf(h->act[l], h->alpha[l], nxt[(size_t)r * W + n]);
    float *t = cur; cur = nxt; nxt = t;
  }
  for (int r = 0; r < rows; ++r) memcpy(y + (size_t)r * out_stride, cur + (size_t)r * W, sizeof(float) * h->N[h->nl - 1]);
}

static void block_f64(const mlpref_t *h, const float *x, double *y, int rows, int in_stride, int out_stride,
                      double *bufa, double *bufb) {
  const int W = h->maxw;
  for (int r = 0; r < rows; ++r)
    for (int k = 0; k < h->K[0]; ++k) bufa[(size_t)r * W + k] = x[(size_t)r * in_stride + k];
  double *cur = bufa, *nxt = bufb;
  for (int l = 0; l < h->nl; ++l) {
    const int K = h->K[l], N = h->N[l];
    const double *wt = h->wt64[l], *bb = h->b64[l];
    for (int r = 0; r < rows; ++r) memcpy(nxt + (size_t)r * W, bb, sizeof(double) * N);
    for (int k = 0; k < K; ++k) {
      const double *wr = wt + (size_t)k * N;
      for (int r = 0; r < rows; ++r) {
        const double xv = cur[(size_t)r * W + k];
        double *yr = nxt + (size_t)r * W;
        for (int n = 0; n < N; ++n) yr[n] += xv * wr[n];
      }
    }
    for (int r = 0; r < rows; ++r)
      for (int n = 0; n < N; ++n) nxt[(size_t)r * W + n] = actd(h->act[l], h->alpha[l], nxt[(size_t)r * W + n]);
    double *t = cur; cur = nxt; nxt = t;
  }
  for (int r = 0; r < rows; ++r)
    for (int n = 0; n < h->N[h->nl - 1]; ++n) y[(size_t)r * out_stride + n] = cur[(size_t)r * W + n];
}

int mlpref_run_f32(void *p, const float *x, float *y, long B, int nthreads) {
  const mlpref_t *h = (const mlpref_t *)p;
  if (!h || B < 0) return -1;
  const long nblk = (B + RB - 1) / RB;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
  {
    float *a = (float *)malloc(sizeof(float) * RB * h->maxw);
    float *bb = (float *)malloc(sizeof(float) * RB * h->maxw);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (long i = 0; i < nblk; ++i) {
      long r0 = i * RB;
      int rows = (int)((B - r0) < RB ? (B - r0) : RB);
      block_f32(h, x + r0 * h->K[0], y + r0 * h->N[h->nl - 1], rows, h->K[0], h->N[h->nl - 1], a, bb);
    }
    free(a); free(bb);
  }
  return 0;
}

int mlpref_run_f64(void *p, const float *x, double *y, long B, int nthreads) {
  const mlpref_t *h = (const mlpref_t *)p;
  if (!h || B < 0) return -1;
  const long nblk = (B + RB - 1) / RB;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
  {
    double *a = (double *)malloc(sizeof(double) * RB * h->maxw);
    double *bb = (double *)malloc(sizeof(double) * RB * h->maxw);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (long i = 0; i < nblk; ++i) {
      long r0 = i * RB;
      int rows = (int)((B - r0) < RB ? (B - r0) : RB);
      block_f64(h, x + r0 * h->K[0], y + r0 * h->N[h->nl - 1], rows, h->K[0], h->N[h->nl - 1], a, bb);
    }
    free(a); free(bb);
  }
  return 0;
}

/*
 * ONNX GRU, one time step, fp64 (onnx GRU opset 14).
 * W [3H][I] gates (z,r,h); R [3H][H]; Wb, Rb [3H]; x [B][I]; h [B][H] in/out.
 */
int gruref_step_f64(int I, int H, const float *W, const float *R, const float *Wb, const float *Rb, int lbr,
                    const float *x, double *h, long B, int nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
  for (long r = 0; r < B; ++r) {
    double *hr = h + r * H;
    const float *xr = x + r * I;
    double *hn = (double *)malloc(sizeof(double) * H);
    double *rg = (double *)malloc(sizeof(double) * H);
    double *zg = (double *)malloc(sizeof(double) * H);
    for (int j = 0; j < H; ++j) {
      double az = (double)Wb[j] + (double)Rb[j], ar = (double)Wb[H + j] + (double)Rb[H + j];
      for (int k = 0; k < I; ++k) {
        az += (double)W[(size_t)j * I + k] * xr[k];
        ar += (double)W[(size_t)(H + j) * I + k] * xr[k];
      }
      for (int k = 0; k < H; ++k) {
        az += (double)R[(size_t)j * H + k] * hr[k];
        ar += (double)R[(size_t)(H + j) * H + k] * hr[k];
      }
      zg[j] = 1. / (1. + exp(-az));
      rg[j] = 1. / (1. + exp(-ar));
    }
    for (int j = 0; j < H; ++j) {
      double ax = Wb[2 * H + j], ah = 0.;
      for (int k = 0; k < I; ++k) ax += (double)W[(size_t)(2 * H + j) * I + k] * xr[k];
      if (lbr) {
        ah = Rb[2 * H + j];
        for (int k = 0; k < H; ++k) ah += (double)R[(size_t)(2 * H + j) * H + k] * hr[k];
        hn[j] = tanh(ax + rg[j] * ah);
      } else {
        for (int k = 0; k < H; ++k) ah += (double)R[(size_t)(2 * H + j) * H + k] * (rg[k] * hr[k]);
        hn[j] = tanh(ax + ah + (double)Rb[2 * H + j]);
      }
    }
    for (int j = 0; j < H; ++j) hr[j] = (1. - zg[j]) * hn[j] + zg[j] * hr[j];
    free(hn); free(rg); free(zg);
  }
  return 0;
}

/*
 * cpu_baseline leg of bench.py (BASELINE configs[0]): the reference's own
 * measurement is one timed act() at batch 1 (onnx_inference/src/cpp/main.cpp:38-42,
 * steady_clock around Session::Run). This times `warm + iters` single-robot fp32
 * forwards on the calling thread (no OpenMP), each bracketed by CLOCK_MONOTONIC,
 * and writes the `iters` per-call durations in microseconds to out_us. Each call
 * reads the observation row and writes the action row, as act() does.
 */
#include <time.h>
int mlpref_time_b1(void *p, const float *x, float *y, int warm, int iters, double *out_us) {
  const mlpref_t *h = (const mlpref_t *)p;
  if (!h || iters < 0 || warm < 0) return -1;
  float *a = (float *)malloc(sizeof(float) * RB * h->maxw);
  float *bb = (float *)malloc(sizeof(float) * RB * h->maxw);
  for (int i = 0; i < warm + iters; ++i) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    block_f32(h, x, y, 1, h->K[0], h->N[h->nl - 1], a, bb);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (i >= warm) out_us[i - warm] = (double)(t1.tv_sec - t0.tv_sec) * 1e6 + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-3;
  }
  free(a); free(bb);
  return 0;
}
