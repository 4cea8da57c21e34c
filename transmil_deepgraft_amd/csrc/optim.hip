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
// The step counters live in device memory (counters[0] = RAdam step, counters[1] =
// Lookahead step), advanced by a 1-thread launch, so the pair is hipGraph-replayable.
// HBM traffic per element: p, m, v read+write, g read = 28 B (+8 B slow on sync steps).
#include "../../include/transmil_hip.h"
#include "common.h"

namespace {

__global__ void optim_tick_kernel(int* counters) {
  counters[0] += 1;
  counters[1] += 1;
}

__global__ __launch_bounds__(256) void radam_lookahead_kernel(tm_optim_table tab, float* __restrict__ exp_avg,
                                                              float* __restrict__ exp_avg_sq,
                                                              float* __restrict__ slow,
                                                              const int* __restrict__ counters, float beta1,
                                                              float beta2, float eps, int la_k, float la_alpha) {
  const long long total = tab.offset[tab.count];
  const float step = (float)counters[0];
  const int la_step = counters[1];
  const float bc1 = 1.0f - powf(beta1, step);
  const float b2t = powf(beta2, step);
  const float bc2 = 1.0f - b2t;
  const float rho_inf = 2.0f / (1.0f - beta2) - 1.0f;
  const float rho_t = rho_inf - 2.0f * step * b2t / bc2;
  const float rect = rho_t > 5.0f
                         ? sqrtf((rho_t - 4.0f) * (rho_t - 2.0f) * rho_inf /
                                 ((rho_inf - 4.0f) * (rho_inf - 2.0f) * rho_t))
                         : 0.0f;
  const bool sync = la_k > 0 && la_step % la_k == 0;
  const bool first_sync = la_step <= la_k;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int ti = 0;
    while (i >= tab.offset[ti + 1]) ++ti;
    const tm_optim_tensor& T = tab.t[ti];
    const long long j = i - tab.offset[ti];
    float p = T.param[j];
    const float g = T.grad[j] + T.weight_decay * p;
    float m = exp_avg[i];
    m = m + (1.0f - beta1) * (g - m);
    const float v = exp_avg_sq[i] * beta2 + (1.0f - beta2) * g * g;
    exp_avg[i] = m;
    exp_avg_sq[i] = v;
    float coef;
    if (rect > 0.0f) {
      const float bc2f = -(sqrtf(bc2) * T.lr * rect) / bc1;
      coef = 1.0f / ((sqrtf(v) + eps) / bc2f);
    } else {
      coef = -T.lr / bc1;
    }
    p = fmaf(m, coef, p);
    if (sync) {
      const float s = first_sync ? p : slow[i] + la_alpha * (p - slow[i]);
      slow[i] = s;
      p = s;
    }
    T.param[j] = p;
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
    TM_REQUIRE(table->offset[i + 1] - table->offset[i] == table->t[i].numel, "optim: offsets != prefix sum of numel");
  }
  TM_REQUIRE(lookahead_k == 0 || slow, "optim: lookahead needs the slow buffer");
  hipStream_t st = (hipStream_t)stream;
  optim_tick_kernel<<<1, 1, 0, st>>>(counters);
  TM_CHECK_LAUNCH();
  const long long total = table->offset[table->count];
  if (total == 0) return 0;
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  radam_lookahead_kernel<<<(unsigned)blocks, 256, 0, st>>>(*table, exp_avg, exp_avg_sq, slow, counters, beta1, beta2,
                                                            eps, lookahead_k, lookahead_alpha);
  TM_CHECK_LAUNCH();
  return 0;
}
