// Optimizer step of the training loop: torch.optim.RAdam (L2 weight decay added to the
// gradient, decoupled_weight_decay=False) followed by the Lookahead slow-weight sync,
// over every parameter tensor in ONE elementwise launch.
//
// Reference: code/MyOptimizer/optim_factory.py:77-79 (optim.RAdam), :118-121 and
// code/MyOptimizer/lookahead.py (Lookahead(alpha=0.5, k=6)).  The per-element update
// restates torch/optim/radam.py (_multi_tensor_radam, capturable branch):
//   g  = grad + wd * p
//   m  = lerp(m, g, 1 - b1);   v = b2 * v + (1 - b2) * g^2
//   rho_t = rho_inf - 2 t b2^t / (1 - b2^t)
//   rect  = rho_t > 5 ? sqrt((rho_t-4)(rho_t-2) rho_inf / ((rho_inf-4)(rho_inf-2) rho_t)) : 0
//   p += m * (rect > 0 ? -lr rect sqrt(1-b2^t) / ((1-b1^t)(sqrt(v)+eps)) : -lr / (1-b1^t))
// and Lookahead every k-th step: slow = first_sync ? p : slow + alpha (p - slow); p = slow.
//
// The step counters live in device memory (counters[0] = RAdam step, counters[1] = Lookahead
// step; counters[2] unused), advanced by a 1-thread launch before the update, so the pair is
// hipGraph-replayable.  (Advancing them from the last-finishing workgroup instead -- one
// agent-scope fence + one same-address atomic per workgroup -- made the step 3.4x slower:
// 108 vs 32 us.)  Flat-state offsets are multiples of 4 (each tensor padded), so a thread
// updates 4 consecutive elements with 16-B loads / stores; tensors whose param / grad pointers
// are not 16-B aligned fall back to element-wise access.
// HBM traffic per element: p, m, v read+write, g read = 28 B (+8 B slow on sync steps).
#include "../../include/transmil_hip.h"
#include "common.h"

namespace {

constexpr int OPT_THREADS = 256, OPT_PER_BLOCK = OPT_THREADS * 4;

__global__ void optim_tick_kernel(int* counters) {
  counters[0] += 1;
  counters[1] += 1;
}

struct RAdamScal {
  float bc1, bc2, rect;
  bool sync, first_sync;
};

TM_DEV float radam_elem(float p, float g, float& m, float& v, const RAdamScal& r, float lr, float wd, float beta1,
                        float beta2, float eps) {
  g += wd * p;
  m = m + (1.0f - beta1) * (g - m);
  v = v * beta2 + (1.0f - beta2) * g * g;
  float coef;
  if (r.rect > 0.0f) {
    const float bc2f = -(sqrtf(r.bc2) * lr * r.rect) / r.bc1;
    coef = 1.0f / ((sqrtf(v) + eps) / bc2f);
  } else {
    coef = -lr / r.bc1;
  }
  return fmaf(m, coef, p);
}

__global__ __launch_bounds__(OPT_THREADS) void radam_lookahead_kernel(tm_optim_table tab, float* __restrict__ exp_avg,
                                                                      float* __restrict__ exp_avg_sq,
                                                                      float* __restrict__ slow,
                                                                      int* __restrict__ counters, float beta1,
                                                                      float beta2, float eps, int la_k,
                                                                      float la_alpha) {
  // the element loads go out first: nothing they address depends on the step counters, so the
  // counter load and the bias-correction math overlap them (no LDS hand-off or barrier)
  const long long total = tab.offset[tab.count];
  const long long blk0 = (long long)blockIdx.x * OPT_PER_BLOCK;
  const long long i0 = blk0 + 4LL * threadIdx.x;
  if (i0 >= total) return;
  int ti = 0;
  while (ti < tab.count - 1 && blk0 >= tab.offset[ti + 1]) ++ti;  // block-uniform
  while (i0 >= tab.offset[ti + 1]) ++ti;
  const tm_optim_tensor& T = tab.t[ti];
  const long long j0 = i0 - tab.offset[ti];
  const int n = (int)min(4LL, T.numel - j0);   // the tensor's padding tail: n < 4 (or <= 0)
  if (n <= 0) return;
  const bool vec = n == 4 && ((uintptr_t)(T.param + j0) % 16) == 0 && ((uintptr_t)(T.grad + j0) % 16) == 0;
  f32x4 m4 = *(const f32x4*)(exp_avg + i0), v4 = *(const f32x4*)(exp_avg_sq + i0);
  f32x4 p4, g4, s4 = {0.f, 0.f, 0.f, 0.f};
  if (vec) {
    p4 = *(const f32x4*)(T.param + j0);
    g4 = *(const f32x4*)(T.grad + j0);
  } else {
    for (int e = 0; e < 4; ++e) {
      p4[e] = e < n ? T.param[j0 + e] : 0.f;
      g4[e] = e < n ? T.grad[j0 + e] : 0.f;
    }
  }
  const float step = (float)counters[0];
  const int la_step = counters[1];
  RAdamScal r;
  r.bc1 = 1.0f - powf(beta1, step);
  const float b2t = powf(beta2, step);
  r.bc2 = 1.0f - b2t;
  const float rho_inf = 2.0f / (1.0f - beta2) - 1.0f;
  const float rho_t = rho_inf - 2.0f * step * b2t / r.bc2;
  r.rect = rho_t > 5.0f ? sqrtf((rho_t - 4.0f) * (rho_t - 2.0f) * rho_inf /
                                ((rho_inf - 4.0f) * (rho_inf - 2.0f) * rho_t))
                        : 0.0f;
  r.sync = la_k > 0 && la_step % la_k == 0;
  r.first_sync = la_step <= la_k;
  if (r.sync && !r.first_sync) s4 = *(const f32x4*)(slow + i0);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float m = m4[e], v = v4[e];
    float p = radam_elem(p4[e], g4[e], m, v, r, T.lr, T.weight_decay, beta1, beta2, eps);
    if (r.sync) {
      p = r.first_sync ? p : s4[e] + la_alpha * (p - s4[e]);
      s4[e] = p;
    }
    m4[e] = m;
    v4[e] = v;
    p4[e] = p;
  }
  *(f32x4*)(exp_avg + i0) = m4;
  *(f32x4*)(exp_avg_sq + i0) = v4;
  if (r.sync) *(f32x4*)(slow + i0) = s4;
  if (vec) {
    *(f32x4*)(T.param + j0) = p4;
  } else {
    for (int e = 0; e < n; ++e) T.param[j0 + e] = p4[e];
  }
}

}  // namespace

extern "C" int tm_radam_lookahead_step(const tm_optim_table* table, float* exp_avg, float* exp_avg_sq, float* slow,
                                       int* counters, float beta1, float beta2, float eps, int lookahead_k,
                                       float lookahead_alpha, void* stream) {
  TM_REQUIRE(table && table->count > 0 && table->count <= TM_OPTIM_MAX_TENSORS, "optim: 1..40 tensors per call");
  TM_REQUIRE(table->offset[0] == 0, "optim: offsets must start at 0");
  for (int i = 0; i < table->count; ++i) {
    TM_REQUIRE(table->t[i].param && table->t[i].grad, "optim: every tensor needs a param and a grad");
    const long long span = table->offset[i + 1] - table->offset[i];
    TM_REQUIRE(table->offset[i] % 4 == 0 && span >= table->t[i].numel && span < table->t[i].numel + 4,
               "optim: offsets must be the prefix sums of numel rounded up to multiples of 4");
  }
  TM_REQUIRE(((uintptr_t)exp_avg % 16) == 0 && ((uintptr_t)exp_avg_sq % 16) == 0 && (!slow || ((uintptr_t)slow % 16) == 0),
             "optim: state buffers must be 16-B aligned");
  TM_REQUIRE(lookahead_k == 0 || slow, "optim: lookahead needs the slow buffer");
  const long long total = table->offset[table->count];
  if (total == 0) return 0;
  const long long blocks = (total + OPT_PER_BLOCK - 1) / OPT_PER_BLOCK;
  optim_tick_kernel<<<1, 1, 0, (hipStream_t)stream>>>(counters);
  radam_lookahead_kernel<<<(unsigned)blocks, OPT_THREADS, 0, (hipStream_t)stream>>>(
      *table, exp_avg, exp_avg_sq, slow, counters, beta1, beta2, eps, lookahead_k, lookahead_alpha);
  TM_CHECK_LAUNCH();
  return 0;
}
