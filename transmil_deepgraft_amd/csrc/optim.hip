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

// a grid of at most OPT_MAX_BLOCKS workgroups walks the flat state in 4-element pieces, grid-strided
// (a wave's piece = 256 consecutive elements), with the next piece's loads issued before the
// current piece's update and stores: one 16-B piece per thread per pass, reads and writes of the
// step overlapped.  (One piece pair per thread over ceil(total / 2048) workgroups put every
// workgroup in the same phase -- the whole state read, then computed, then written: 18.8 us for
// 67 MB.)
#ifndef OPT_MAX_BLOCKS_SET
#define OPT_MAX_BLOCKS_SET 1024
#endif
constexpr int OPT_THREADS = 256, OPT_MAX_BLOCKS = OPT_MAX_BLOCKS_SET;

inline long long opt_blocks(long long total) {
  const long long need = (total + OPT_THREADS * 4 - 1) / (OPT_THREADS * 4);
  return std::max(1LL, std::min((long long)OPT_MAX_BLOCKS, need));
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

struct OptPiece {
  float* param;
  const float* grad;
  long long i0, j0;   // flat-state index of the thread's 4 elements; their index in the tensor
  float lr, wd;
  int n;              // valid elements (<= 0: none)
  bool vec;
};

// the tensor of the piece at flat index i0 (wave base wbase, wave-uniform): found with scalar loads
// of the table (a per-lane search indexes the kernarg table with vector loads, a dependent round
// trip per level ahead of the element loads); a wave that straddles a tensor boundary walks the
// few tensors it touches.  ti: the search's lower bound, advanced (pieces only move forward).
TM_DEV OptPiece opt_find(const tm_optim_table& tab, long long total, long long wbase, long long i0, int& ti) {
  OptPiece pc;
  pc.n = 0;
  pc.i0 = i0;
  pc.param = nullptr;
  pc.grad = nullptr;
  pc.j0 = 0;
  pc.lr = pc.wd = 0.f;
  pc.vec = false;
  if (wbase >= total) return pc;
  {
    int lo = ti, hi = tab.count - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tab.offset[mid] <= wbase) lo = mid; else hi = mid - 1;
    }
    ti = lo;
  }
  for (int t = ti; t < tab.count && tab.offset[t] < wbase + 256; ++t) {  // wave-uniform t
    if (i0 >= tab.offset[t] && i0 < tab.offset[t + 1]) {
      const tm_optim_tensor& T = tab.t[t];
      pc.param = T.param;
      pc.grad = T.grad;
      pc.lr = tab.hyper ? tab.hyper[2 * t] : T.lr;
      pc.wd = tab.hyper ? tab.hyper[2 * t + 1] : T.weight_decay;
      pc.j0 = i0 - tab.offset[t];
      pc.n = (int)min(4LL, T.numel - pc.j0);   // the tensor's padding tail: n < 4 (or <= 0)
    }
  }
  if (pc.n > 0)
    pc.vec = pc.n == 4 && ((uintptr_t)(pc.param + pc.j0) % 16) == 0 && ((uintptr_t)(pc.grad + pc.j0) % 16) == 0;
  return pc;
}

struct OptRegs { f32x4 m, v, p, g, s; };

TM_DEV void opt_load(const OptPiece& pc, const float* exp_avg, const float* exp_avg_sq, const float* slow,
                     bool read_slow, OptRegs& x) {
  if (pc.n <= 0) return;
  x.m = *(const f32x4*)(exp_avg + pc.i0);
  x.v = *(const f32x4*)(exp_avg_sq + pc.i0);
  if (pc.vec) {
    x.p = *(const f32x4*)(pc.param + pc.j0);
    x.g = *(const f32x4*)(pc.grad + pc.j0);
  } else {
    for (int e = 0; e < 4; ++e) {
      x.p[e] = e < pc.n ? pc.param[pc.j0 + e] : 0.f;
      x.g[e] = e < pc.n ? pc.grad[pc.j0 + e] : 0.f;
    }
  }
  if (read_slow) x.s = *(const f32x4*)(slow + pc.i0);
}

TM_DEV void opt_update_store(const OptPiece& pc, OptRegs& x, const RAdamScal& r, float* exp_avg, float* exp_avg_sq,
                             float* slow, float beta1, float beta2, float eps, float la_alpha) {
  if (pc.n <= 0) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float m = x.m[e], v = x.v[e];
    float p = radam_elem(x.p[e], x.g[e], m, v, r, pc.lr, pc.wd, beta1, beta2, eps);
    if (r.sync) {
      p = r.first_sync ? p : x.s[e] + la_alpha * (p - x.s[e]);
      x.s[e] = p;
    }
    x.m[e] = m;
    x.v[e] = v;
    x.p[e] = p;
  }
  *(f32x4*)(exp_avg + pc.i0) = x.m;
  *(f32x4*)(exp_avg_sq + pc.i0) = x.v;
  if (r.sync) *(f32x4*)(slow + pc.i0) = x.s;
  if (pc.vec) {
    *(f32x4*)(pc.param + pc.j0) = x.p;
  } else {
    for (int e = 0; e < pc.n; ++e) pc.param[pc.j0 + e] = x.p[e];
  }
}

__global__ __launch_bounds__(OPT_THREADS) void radam_lookahead_kernel(tm_optim_table tab, float* __restrict__ exp_avg,
                                                                      float* __restrict__ exp_avg_sq,
                                                                      float* __restrict__ slow,
                                                                      int* __restrict__ counters, float beta1,
                                                                      float beta2, float eps, int la_k,
                                                                      float la_alpha) {
  const long long total = tab.offset[tab.count];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  // this workgroup's step pair first: the sync decision says which loads a piece needs
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
  const bool read_slow = r.sync && !r.first_sync;

  const long long stride = (long long)gridDim.x * OPT_THREADS * 4;
  long long wb = (long long)blockIdx.x * OPT_THREADS * 4 + wave * 256;   // wave-uniform
  int ti = 0;
  OptPiece cur = opt_find(tab, total, wb, wb + 4 * lane, ti);
  OptRegs xc;
  opt_load(cur, exp_avg, exp_avg_sq, slow, read_slow, xc);
  for (; wb < total; wb += stride) {
    // the next piece's loads go out before this piece's stores (a load issued behind a store waits
    // for it on vmcnt; pieces are disjoint, so the order is free)
    const long long wn = wb + stride;
    const OptPiece nxt = opt_find(tab, total, wn, wn + 4 * lane, ti);
    OptRegs xn;
    opt_load(nxt, exp_avg, exp_avg_sq, slow, read_slow, xn);
    opt_update_store(cur, xc, r, exp_avg, exp_avg_sq, slow, beta1, beta2, eps, la_alpha);
    cur = nxt;
    xc = xn;
  }
  __syncthreads();   // every thread of the workgroup has read its counter pair
  if (threadIdx.x == 0) {
    counters[2 * blockIdx.x] = step_i;
    counters[2 * blockIdx.x + 1] = la_step;
  }
}

}  // namespace

extern "C" long long tm_radam_counters_len(long long total_elements) { return 2 * opt_blocks(total_elements); }

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
  const long long blocks = opt_blocks(total);
  radam_lookahead_kernel<<<(unsigned)blocks, OPT_THREADS, 0, (hipStream_t)stream>>>(
      *table, exp_avg, exp_avg_sq, slow, counters, beta1, beta2, eps, lookahead_k, lookahead_alpha);
  TM_CHECK_LAUNCH();
  return 0;
}
