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
// The step counters live in device memory, one (RAdam step, Lookahead step) pair per workgroup
// (tm_radam_counters_len ints; pair 0 is the canonical one a checkpoint stores): a workgroup reads
// its own pair, updates with pair + 1 and writes pair + 1 back after its threads have read it, so
// no launch or cross-workgroup ordering advances them and the step stays hipGraph-replayable.
// Every workgroup runs every step (the tensor set is fixed once the optimizer is active), so the
// pairs stay equal.  (A one-thread tick launch before the update cost 4.6 us per step; advancing
// one shared pair from the last-finishing workgroup -- an agent-scope fence + a same-address
// atomic per workgroup -- made the step 3.4x slower.)  Flat-state offsets are multiples of 4 (each tensor padded), so a thread
// updates 4 consecutive elements with 16-B loads / stores; tensors whose param / grad pointers
// are not 16-B aligned fall back to element-wise access.
// HBM traffic per element: p, m, v read+write, g read = 28 B (+8 B slow on sync steps).
// lr / weight decay per tensor come from the table, or from the device array tab.hyper when set (an
// LR scheduler then acts on a captured, replayed step).
#include "../../include/transmil_hip.h"
#include "common.h"

namespace {

constexpr int OPT_THREADS = 256, OPT_PIECES = 2, OPT_PER_BLOCK = OPT_THREADS * 4 * OPT_PIECES;

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
  // each thread updates OPT_PIECES 4-element pieces (a block's pieces OPT_THREADS*4 apart, so
  // every load is coalesced).  The tensor of a piece is found wave-uniformly (scalar loads of the
  // table; a per-lane search indexes the kernarg table with vector loads, a dependent round trip
  // per level ahead of the element loads); a wave that straddles a tensor boundary walks the few
  // tensors it touches.  Every element load goes out before the counters are read and before any store (a
  // param store of one piece could alias another piece's loads).
  const long long total = tab.offset[tab.count];
  const long long blk0 = (long long)blockIdx.x * OPT_PER_BLOCK;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int ti = 0;
  struct Piece { float* param; long long j0; float lr, wd; int n; bool vec; };
  long long i0[OPT_PIECES];
  Piece pc[OPT_PIECES];
  f32x4 m4[OPT_PIECES], v4[OPT_PIECES], p4[OPT_PIECES], g4[OPT_PIECES], s4[OPT_PIECES];
#pragma unroll
  for (int u = 0; u < OPT_PIECES; ++u) {
    const long long wbase = blk0 + (long long)u * OPT_THREADS * 4 + wave * 256;  // wave-uniform
    i0[u] = wbase + 4 * (threadIdx.x & 63);
    pc[u].n = 0;
    s4[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (wbase >= total) continue;
    {   // the last tensor starting at or before wbase: a binary search (a linear walk from tensor 0
        // was up to tab.count dependent scalar loads per wave ahead of its element loads)
      int lo = ti, hi = tab.count - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tab.offset[mid] <= wbase) lo = mid; else hi = mid - 1;
      }
      ti = lo;
    }
    const float* grad = nullptr;
    for (int t = ti; t < tab.count && tab.offset[t] < wbase + 256; ++t) {  // wave-uniform t
      if (i0[u] >= tab.offset[t] && i0[u] < tab.offset[t + 1]) {
        const tm_optim_tensor& T = tab.t[t];
        pc[u].param = T.param; grad = T.grad;
        pc[u].lr = tab.hyper ? tab.hyper[2 * t] : T.lr;
        pc[u].wd = tab.hyper ? tab.hyper[2 * t + 1] : T.weight_decay;
        pc[u].j0 = i0[u] - tab.offset[t];
        pc[u].n = (int)min(4LL, T.numel - pc[u].j0);   // the tensor's padding tail: n < 4 (or <= 0)
      }
    }
    const int n = pc[u].n;
    if (n <= 0) continue;
    const long long j0 = pc[u].j0;
    pc[u].vec = n == 4 && ((uintptr_t)(pc[u].param + j0) % 16) == 0 && ((uintptr_t)(grad + j0) % 16) == 0;
    m4[u] = *(const f32x4*)(exp_avg + i0[u]);
    v4[u] = *(const f32x4*)(exp_avg_sq + i0[u]);
    if (pc[u].vec) {
      p4[u] = *(const f32x4*)(pc[u].param + j0);
      g4[u] = *(const f32x4*)(grad + j0);
    } else {
      for (int e = 0; e < 4; ++e) {
        p4[u][e] = e < n ? pc[u].param[j0 + e] : 0.f;
        g4[u][e] = e < n ? grad[j0 + e] : 0.f;
      }
    }
  }
  const int step_i = counters[2 * blockIdx.x] + 1, la_step = counters[2 * blockIdx.x + 1] + 1;
  const float step = (float)step_i;
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
  if (r.sync && !r.first_sync) {
#pragma unroll
    for (int u = 0; u < OPT_PIECES; ++u)
      if (pc[u].n > 0) s4[u] = *(const f32x4*)(slow + i0[u]);
  }
#pragma unroll
  for (int u = 0; u < OPT_PIECES; ++u) {
    const int n = pc[u].n;
    if (n <= 0) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float m = m4[u][e], v = v4[u][e];
      float p = radam_elem(p4[u][e], g4[u][e], m, v, r, pc[u].lr, pc[u].wd, beta1, beta2, eps);
      if (r.sync) {
        p = r.first_sync ? p : s4[u][e] + la_alpha * (p - s4[u][e]);
        s4[u][e] = p;
      }
      m4[u][e] = m;
      v4[u][e] = v;
      p4[u][e] = p;
    }
    *(f32x4*)(exp_avg + i0[u]) = m4[u];
    *(f32x4*)(exp_avg_sq + i0[u]) = v4[u];
    if (r.sync) *(f32x4*)(slow + i0[u]) = s4[u];
    if (pc[u].vec) {
      *(f32x4*)(pc[u].param + pc[u].j0) = p4[u];
    } else {
      for (int e = 0; e < n; ++e) pc[u].param[pc[u].j0 + e] = p4[u][e];
    }
  }
  __syncthreads();   // every thread of the workgroup has read its counter pair
  if (threadIdx.x == 0) {
    counters[2 * blockIdx.x] = step_i;
    counters[2 * blockIdx.x + 1] = la_step;
  }
}

}  // namespace

extern "C" long long tm_radam_counters_len(long long total_elements) {
  return 2 * ((total_elements + OPT_PER_BLOCK - 1) / OPT_PER_BLOCK);
}

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
  radam_lookahead_kernel<<<(unsigned)blocks, OPT_THREADS, 0, (hipStream_t)stream>>>(
      *table, exp_avg, exp_avg_sq, slow, counters, beta1, beta2, eps, lookahead_k, lookahead_alpha);
  TM_CHECK_LAUNCH();
  return 0;
}
