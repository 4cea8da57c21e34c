// C5 tile encoder in train mode: BatchNorm with batch statistics, as the reference's frozen
// encoder runs under Lightning's model.train() (code/models/ResNet.py:95-117 Bottleneck with
// nn.BatchNorm2d; code/models/model_interface.py:243-245 freezes the parameters, not the mode).
//
// Per BatchNorm two passes over the channels-last [rows, C] activation, instead of MIOpen's
// statistics + normalise passes followed by separate ReLU / residual-add passes:
//   1. tm_bn_train_stats: per-channel shifted sums (shift = row 0, so E[x^2] - E[x]^2 does not
//      cancel) per row block in fp32, combined in fp64 in a fixed order (deterministic); yields
//      scale = gamma / sqrt(var + eps), shift = beta - mean * scale (biased variance, as
//      F.batch_norm normalises) and updates running_mean / running_var with the unbiased
//      variance and the module's momentum (nn.BatchNorm2d semantics);
//   2. tm_bn_apply: y = act(y * scale + shift [+ residual | + residual * rscale + rshift]) in place
//      -- bn1 / bn2 + ReLU, and bn3 + (downsample BN'd) identity + ReLU as one pass.
// HBM-bound elementwise / column-reduction work: 16-B vector accesses, no LDS tiling needed
// beyond the stats kernel's cross-row combine.
#include "common.h"

namespace {

constexpr int kStatParts = 2048;     // row blocks of the statistics pass (fixed: partial slab size)
constexpr int kMaxPieces = 64;       // row pieces one statistics call combines

// the row pieces of one statistics call: piece p owns partial slots [pbeg[p], pbeg[p + 1])
struct BnPieces {
  const void* x[kMaxPieces];
  long long rows[kMaxPieces];
  int pbeg[kMaxPieces + 1];
  int n;
};

// ONE launch over every piece (workgroup b = partial slot b): all ~2 K workgroups of the call are
// in flight together, where one launch per piece put one 256-thread workgroup on each CU
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(BnPieces pcs, int C, long long rows_per_part,
                                                               float* __restrict__ part) {
  __shared__ float red[2][256 * 8];
  int p = 0;
  while (p < pcs.n - 1 && (int)blockIdx.x >= pcs.pbeg[p + 1]) ++p;   // workgroup-uniform
  const T* __restrict__ x = (const T*)pcs.x[p];
  const long long rows = pcs.rows[p];
  const int tpr = C >> 3;                      // threads per row (8 channels each), divides 256
  const int rpi = 256 / tpr;                   // rows per iteration
  const int c8 = (threadIdx.x % tpr) * 8, r0 = threadIdx.x / tpr;
  const vec8<T> shv = load8((const T*)pcs.x[0] + c8);   // shift: row 0 of the first piece
  float sh[8], s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sh[e] = to_f(shv[e]); s[e] = 0.f; q[e] = 0.f; }
  const long long beg = (long long)(blockIdx.x - pcs.pbeg[p]) * rows_per_part;
  const long long end = beg + rows_per_part < rows ? beg + rows_per_part : rows;
  long long r = beg + r0;
  for (; r + 3LL * rpi < end; r += 4LL * rpi) {          // four rows in flight per thread
    vec8<T> v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = load8(x + (r + (long long)u * rpi) * C + c8);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = to_f(v[u][e]) - sh[e];
        s[e] += d;
        q[e] = fmaf(d, d, q[e]);
      }
  }
  for (; r < end; r += rpi) {
    const vec8<T> v = load8(x + r * C + c8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = to_f(v[e]) - sh[e];
      s[e] += d;
      q[e] = fmaf(d, d, q[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][r0 * C + c8 + e] = s[e];
    red[1][r0 * C + c8 + e] = q[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float ss = 0.f, qq = 0.f;
    for (int r = 0; r < rpi; ++r) {
      ss += red[0][r * C + c];
      qq += red[1][r * C + c];
    }
    part[((size_t)blockIdx.x * 2 + 0) * C + c] = ss;
    part[((size_t)blockIdx.x * 2 + 1) * C + c] = qq;
  }
}

// The fp64 combine of the partial sums: a workgroup owns CB = min(C, 64) channels, its 1024 / CB
// thread groups each sum every G-th part (G = number of groups) in fp64 with 8 parts' loads in
// flight, then group 0 adds the groups' sums in group order -- a fixed order, so deterministic.
// (One thread per channel walking all ~2 K parts serially was ~0.75 ms per call: one dependent
// load round trip per part on 1-8 workgroups.)
constexpr int kFinalThreads = 1024;
template <typename T>
__global__ __launch_bounds__(kFinalThreads) void bn_stats_final_kernel(const T* __restrict__ x, long long rows, int C,
                                                                       int nparts, const float* __restrict__ part,
                                                                       const float* __restrict__ gamma,
                                                                       const float* __restrict__ beta,
                                                                       float* running_mean, float* running_var,
                                                                       float momentum, float eps,
                                                                       float* __restrict__ scale,
                                                                       float* __restrict__ shift) {
  __shared__ double red[2][kFinalThreads];
  const int CB = C < 64 ? C : 64, G = kFinalThreads / CB;
  const int cl = threadIdx.x % CB, grp = threadIdx.x / CB, c = blockIdx.x * CB + cl;
  double S = 0.0, Q = 0.0;
  constexpr int U = 8;
  for (int g0 = grp; g0 < nparts; g0 += U * G) {
    float sv[U], qv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int g = min(g0 + u * G, nparts - 1);
      sv[u] = part[((size_t)g * 2 + 0) * C + c];
      qv[u] = part[((size_t)g * 2 + 1) * C + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (g0 + u * G < nparts) { S += (double)sv[u]; Q += (double)qv[u]; }
  }
  red[0][threadIdx.x] = S;
  red[1][threadIdx.x] = Q;
  __syncthreads();
  if (grp != 0) return;
  S = 0.0;
  Q = 0.0;
  for (int g = 0; g < G; ++g) { S += red[0][g * CB + cl]; Q += red[1][g * CB + cl]; }
  const double n = (double)rows, md = S / n;
  double var = Q / n - md * md;
  var = var > 0.0 ? var : 0.0;
  const double mean = (double)to_f(x[c]) + md;
  const double sc = (double)gamma[c] / sqrt(var + (double)eps);
  scale[c] = (float)sc;
  shift[c] = (float)((double)beta[c] - mean * sc);
  if (running_mean) running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
  if (running_var)
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * (rows > 1 ? var * n / (n - 1.0) : var));
}

template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(T* y, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const T* __restrict__ res,
                                                       const float* __restrict__ rscale,
                                                       const float* __restrict__ rshift, long long count, int C,
                                                       int relu) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= count) return;
  const int c = (int)(i % C);
  const vec8<T> v = load8(y + i);
  float o[8], sc[8], sf[8];
  *(float4*)sc = *(const float4*)(scale + c);
  *(float4*)(sc + 4) = *(const float4*)(scale + c + 4);
  *(float4*)sf = *(const float4*)(shift + c);
  *(float4*)(sf + 4) = *(const float4*)(shift + c + 4);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = fmaf(to_f(v[e]), sc[e], sf[e]);
  if (res) {
    const vec8<T> r = load8(res + i);
    if (rscale) {
      *(float4*)sc = *(const float4*)(rscale + c);
      *(float4*)(sc + 4) = *(const float4*)(rscale + c + 4);
      *(float4*)sf = *(const float4*)(rshift + c);
      *(float4*)(sf + 4) = *(const float4*)(rshift + c + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += fmaf(to_f(r[e]), sc[e], sf[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += to_f(r[e]);
    }
  }
  vec8<T> out;
  const float lo = relu ? 0.f : -INFINITY;
#pragma unroll
  for (int e = 0; e < 8; ++e) out[e] = from_f<T>(fmaxf(o[e], lo));
  store8<T>(y + i, out);
}

}  // namespace

extern "C" long long tm_bn_train_workspace(int C) {
  return 2LL * (kStatParts + kMaxPieces) * (C > 0 ? C : 0);
}

// The activation may come as up to kMaxPieces row pieces (the bag in tile pieces, each its own
// channels-last tensor): statistics span all of them; piece p's rows get partial slots in
// proportion to its row count, so the combine order is fixed by the piece list.
extern "C" int tm_bn_train_stats(int dtype, const void* const* xs, const long long* rows, int npieces, int C,
                                 const float* gamma, const float* beta, float* running_mean, float* running_var,
                                 float momentum, float eps, float* scale, float* shift, float* workspace,
                                 long long ws_floats, void* stream) {
  TM_REQUIRE(xs && rows && npieces > 0 && npieces <= kMaxPieces, "bn_train_stats: 1..64 pieces");
  TM_REQUIRE(gamma && beta && scale && shift && workspace, "bn_train_stats: bad args");
  TM_REQUIRE(C >= 8 && C <= 2048 && (C & (C - 1)) == 0, "bn_train_stats: C must be a power of two in [8, 2048]");
  TM_REQUIRE(ws_floats >= tm_bn_train_workspace(C), "bn_train_stats: workspace too small");
  long long total = 0;
  for (int p = 0; p < npieces; ++p) {
    TM_REQUIRE(xs[p] && rows[p] > 0 && ((uintptr_t)xs[p] % 16) == 0, "bn_train_stats: piece (16-B aligned, rows > 0)");
    total += rows[p];
  }
  TM_REQUIRE(dtype == TM_BF16 || dtype == TM_F32, "bn_train_stats: dtype");
  const long long per = (total + kStatParts - 1) / kStatParts;
  hipStream_t st = (hipStream_t)stream;
  BnPieces pcs{};
  int nparts = 0;
  for (int p = 0; p < npieces; ++p) {
    pcs.x[p] = xs[p];
    pcs.rows[p] = rows[p];
    pcs.pbeg[p] = nparts;
    nparts += (int)((rows[p] + per - 1) / per);
  }
  pcs.pbeg[npieces] = nparts;
  pcs.n = npieces;
  if (dtype == TM_BF16)
    bn_stats_partial_kernel<bf16><<<nparts, 256, 0, st>>>(pcs, C, per, workspace);
  else
    bn_stats_partial_kernel<float><<<nparts, 256, 0, st>>>(pcs, C, per, workspace);
  TM_CHECK_LAUNCH();
  if (dtype == TM_BF16)
    bn_stats_final_kernel<bf16><<<(C + 63) / 64, kFinalThreads, 0, st>>>((const bf16*)xs[0], total, C, nparts,
                                                                          workspace, gamma, beta, running_mean,
                                                                          running_var, momentum, eps, scale, shift);
  else
    bn_stats_final_kernel<float><<<(C + 63) / 64, kFinalThreads, 0, st>>>((const float*)xs[0], total, C, nparts,
                                                                           workspace, gamma, beta, running_mean,
                                                                           running_var, momentum, eps, scale, shift);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_bn_apply(int dtype, void* y, const float* scale, const float* shift, const void* residual,
                           const float* rscale, const float* rshift, long long rows, int C, int relu, void* stream) {
  TM_REQUIRE(y && scale && shift && rows >= 0 && C > 0 && C % 8 == 0, "bn_apply: bad args (C % 8 == 0)");
  TM_REQUIRE(!rscale == !rshift && (!rscale || residual), "bn_apply: rscale / rshift come with a residual");
  TM_REQUIRE(((uintptr_t)y % 16) == 0 && ((uintptr_t)residual % 16) == 0, "bn_apply: 16-B aligned buffers");
  TM_REQUIRE(((uintptr_t)scale % 16) == 0 && ((uintptr_t)shift % 16) == 0 && ((uintptr_t)rscale % 16) == 0 &&
                 ((uintptr_t)rshift % 16) == 0, "bn_apply: 16-B aligned scale / shift vectors");
  const long long count = rows * (long long)C;
  if (count == 0) return 0;
  const unsigned blocks = (unsigned)((count + 2047) / 2048);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TM_BF16)
    bn_apply_kernel<bf16><<<blocks, 256, 0, st>>>((bf16*)y, scale, shift, (const bf16*)residual, rscale, rshift,
                                                  count, C, relu);
  else if (dtype == TM_F32)
    bn_apply_kernel<float><<<blocks, 256, 0, st>>>((float*)y, scale, shift, (const float*)residual, rscale, rshift,
                                                   count, C, relu);
  else {
    tm_set_error("bn_apply: dtype");
    return 1;
  }
  TM_CHECK_LAUNCH();
  return 0;
}
