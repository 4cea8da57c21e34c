// Glue around the TransMIL forward (code/models/TransMIL.py:167-211) that is not
// a GEMM, attention or stencil: class-token rows, the dropout backward of
// NystromAttention.to_out, the _fc1 GELU backward with the grid-padding fold
// (:177-180), and the class-token gradient.  All HBM-bound, one pass each.
#include "common.h"
#include "../../include/transmil_hip.h"

namespace {

// fp32 -> T copies of up to 8 tensors in one launch (the per-step GEMM weight operands)
template <typename T>
__global__ void cast_many_kernel(tm_cast_table tab) {
  const long long i4 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= tab.offset[tab.count]) return;
  int t = 0;
  while (i4 >= tab.offset[t + 1]) ++t;
  const long long j = i4 - tab.offset[t], n = tab.offset[t + 1] - tab.offset[t];
  const float* src = tab.src[t];
  T* dst = (T*)tab.dst[t];
  for (int e = 0; e < 4 && j + e < n; ++e) dst[j + e] = from_f<T>(src[j + e]);
}

constexpr int CAST_PIECES = 4;

// The per-step preparation of the fused forward as ONE launch: blocks [0, cast_blocks) convert
// the cast table (GEMM weights + the bag to T), the next ceil(49 D/256) blocks fold PPEG's
// 7x7 + 5x5 + 3x3 + identity into one 7x7 kernel (code/models/TransMIL.py:72), and the last
// block advances the dropout counter and writes this forward's seed snapshot.
template <typename T>
__global__ void __launch_bounds__(256) step_prepare_kernel(tm_cast_table tab, long long cast_blocks,
                                                           const float* __restrict__ w7, const float* __restrict__ b7,
                                                           const float* __restrict__ w5, const float* __restrict__ b5,
                                                           const float* __restrict__ w3, const float* __restrict__ b3,
                                                           int D, float* __restrict__ wf, float* __restrict__ bf,
                                                           long long* __restrict__ counter,
                                                           long long* __restrict__ seed_out,
                                                           const float* __restrict__ cls, float* __restrict__ H,
                                                           int B, int S) {
  if (blockIdx.x < cast_blocks) {
    // CAST_PIECES 4-element pieces per lane (block b, piece k: elements from (b CAST_PIECES + k)
    // 1024, a wave 256 of them), all loads issued before any store: 16 KB in flight per block.  The
    // tensor is found wave-uniformly (scalar loads of the table); a wave span inside one aligned
    // tensor moves as one 16-B load / one 4-T store per lane, the rare span across a tensor
    // boundary or the table's end goes piece by piece
    const long long total = tab.offset[tab.count];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    f32x4 v[CAST_PIECES];
    T* dp[CAST_PIECES];
#pragma unroll
    for (int k = 0; k < CAST_PIECES; ++k) {
      dp[k] = nullptr;
      const long long wbase = ((long long)blockIdx.x * CAST_PIECES + k) * 1024 + wave * 256;
      if (wbase >= total) continue;
      const long long i4 = wbase + 4 * lane;
      int t0 = 0;
      while (t0 < tab.count - 1 && wbase >= tab.offset[t0 + 1]) ++t0;
      const bool aligned = ((uintptr_t)tab.src[t0] % 16) == 0 && ((uintptr_t)tab.dst[t0] % (4 * sizeof(T))) == 0;
      if (aligned && tab.offset[t0 + 1] >= wbase + 256) {
        const long long j = i4 - tab.offset[t0];
        v[k] = *(const f32x4*)(tab.src[t0] + j);
        dp[k] = (T*)tab.dst[t0] + j;
        continue;
      }
      for (int t = t0; t < tab.count && tab.offset[t] < wbase + 256; ++t) {  // wave-uniform t
        if (i4 < tab.offset[t] || i4 >= tab.offset[t + 1]) continue;
        const long long j = i4 - tab.offset[t];
        const float* src = tab.src[t] + j;
        T* dst = (T*)tab.dst[t] + j;
        for (int e = 0; e < 4; ++e) dst[e] = from_f<T>(src[e]);
      }
    }
#pragma unroll
    for (int k = 0; k < CAST_PIECES; ++k) {
      if (!dp[k]) continue;
      vec4<T> o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = from_f<T>(v[k][e]);
      *(vec4<T>*)dp[k] = o;
    }
    return;
  }
  const long long fb = blockIdx.x - cast_blocks;
  const int nfold = w7 ? (49 * D + 255) / 256 : 0;
  if (fb < nfold) {  // one thread per (tap, channel), channels fastest
    const int i = (int)fb * 256 + threadIdx.x;
    if (i >= 49 * D) return;
    const int tap = i / D, ch = i - tap * D, dy = tap / 7, dx = tap - dy * 7;
    float v = w7[(size_t)ch * 49 + tap];
    if (dy >= 1 && dy <= 5 && dx >= 1 && dx <= 5) v += w5[(size_t)ch * 25 + (dy - 1) * 5 + (dx - 1)];
    if (dy >= 2 && dy <= 4 && dx >= 2 && dx <= 4) v += w3[(size_t)ch * 9 + (dy - 2) * 3 + (dx - 2)];
    if (dy == 3 && dx == 3) v += 1.0f;
    wf[(size_t)tap * D + ch] = v;  // tap-major [49][D] (coalesced stencil reads)
    if (tap == 0) bf[ch] = b7[ch] + b5[ch] + b3[ch];
    return;
  }
  if (threadIdx.x == 0 && counter) {
    const long long c = counter[0] + 1;
    counter[0] = c;
    seed_out[0] = c;
  }
  if (cls)   // the class-token rows H[b*S + 0][:] (code/models/TransMIL.py:184-186)
    for (int i = threadIdx.x; i < B * D; i += blockDim.x) H[(size_t)(i / D) * S * D + i % D] = cls[i % D];
}

// H[b*S + 0][:] = cls[:]; grid (B), block 256
__global__ void put_cls_kernel(const float* __restrict__ cls, int S, int D, float* __restrict__ H) {
  for (int c = threadIdx.x; c < D; c += blockDim.x) H[(size_t)blockIdx.x * S * D + c] = cls[c];
}

// out[b][pad + i][c] = dH[b*S + i][c] * keep(b*S+i, c) * scale ; out[b][0..pad)[c] = 0
// grid (n_pad, B), block 256
template <typename T>
__global__ void dropout_bwd_pad_kernel(const float* __restrict__ dH, int S, int n_pad, int pad, int D, float p,
                                       float scale, uint64_t seed0, const uint64_t* __restrict__ seed_ptr,
                                       T* __restrict__ out) {
  const int t = blockIdx.x, b = blockIdx.y;
  const uint64_t seed = p > 0.f ? effective_seed(seed0, seed_ptr) : 0;
  T* dst = out + ((size_t)b * n_pad + t) * D;
  const int i = t - pad;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float v = 0.f;
    if (i >= 0) {
      const int row = b * S + i;
      v = dH[(size_t)row * D + c];
      if (p > 0.f) v = dropout_u01(seed, (uint32_t)row, (uint32_t)c) >= p ? v * scale : 0.f;
    }
    dst[c] = from_f<T>(v);
  }
}

// dpre = (dH[token] + dH[duplicated pad row]) * GELU'(pre) for the N token rows of every bag, 8
// columns per thread (16-B loads, one 16-B T store), 4 rows per 256-thread block; block (0, 0) also
// writes the class-token gradient dcls = sum_b dH[b, 0, :] (one launch for both).
template <typename T>
__global__ __launch_bounds__(256) void fc1_gelu_bwd_kernel(const float* __restrict__ dH, const T* __restrict__ pre,
                                                           int B, int N, int S, int add, int D, T* __restrict__ dpre,
                                                           float* __restrict__ dcls) {
  const int b = blockIdx.y, i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && b == 0 && dcls) {
    for (int c = threadIdx.x; c < D; c += 256) {
      float sacc = 0.f;
      for (int bb = 0; bb < B; ++bb) sacc += dH[(size_t)bb * S * D + c];
      dcls[c] = sacc;
    }
  }
  if (i >= N) return;
  const float* g0 = dH + ((size_t)b * S + 1 + i) * D;
  const float* g1 = dH + ((size_t)b * S + 1 + N + i) * D;
  const size_t o = ((size_t)b * N + i) * D;
  for (int c = lane * 8; c < D; c += 64 * 8) {
    const f32x4 a0 = *(const f32x4*)(g0 + c), a1 = *(const f32x4*)(g0 + c + 4);
    const vec8<T> pv = load8<T>(pre + o + c);   // the pre-activation in T (bf16 step: bf16)
    const f32x4 p0 = {to_f(pv[0]), to_f(pv[1]), to_f(pv[2]), to_f(pv[3])};
    const f32x4 p1 = {to_f(pv[4]), to_f(pv[5]), to_f(pv[6]), to_f(pv[7])};
    f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
    if (i < add) { d0 = *(const f32x4*)(g1 + c); d1 = *(const f32x4*)(g1 + c + 4); }
    vec8<T> out;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      out[e] = from_f<T>((a0[e] + d0[e]) * gelu_erf_grad(p0[e]));
      out[4 + e] = from_f<T>((a1[e] + d1[e]) * gelu_erf_grad(p1[e]));
    }
    store8<T>(dpre + o + c, out);
  }
}

// dpre[i] = dy[i] * gelu'(pre[i]) over a flat [rows, D] block (the Linear+GELU stages of the
// _fc1 branches other than the last, code/models/TransMIL.py:100-111); 4 elements per lane
template <typename T>
__global__ void gelu_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ pre, size_t count,
                                T* __restrict__ dpre) {
  const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 4 <= count) {
    const float4 g = *(const float4*)(dy + i);
    const float4 x = *(const float4*)(pre + i);
    dpre[i] = from_f<T>(g.x * gelu_erf_grad(x.x));
    dpre[i + 1] = from_f<T>(g.y * gelu_erf_grad(x.y));
    dpre[i + 2] = from_f<T>(g.z * gelu_erf_grad(x.z));
    dpre[i + 3] = from_f<T>(g.w * gelu_erf_grad(x.w));
  } else {
    for (size_t j = i; j < count; ++j) dpre[j] = from_f<T>(dy[j] * gelu_erf_grad(pre[j]));
  }
}

// y[b][pad + i][c] = x[b*S + i][c] (cast to T), y[b][0..pad)[c] = 0; grid (n_pad, B)
template <typename T>
__global__ void pad_rows_kernel(const float* __restrict__ x, int S, int n_pad, int pad, int D, T* __restrict__ y) {
  const int t = blockIdx.x, b = blockIdx.y, i = t - pad;
  T* dst = y + ((size_t)b * n_pad + t) * D;
  for (int c = threadIdx.x; c < D; c += blockDim.x)
    dst[c] = from_f<T>(i >= 0 ? x[((size_t)b * S + i) * D + c] : 0.f);
}


// y = max(a + b, 0), elementwise over 8-element pieces (the C5 encoder's residual add + ReLU in
// one pass instead of two; a and y may alias).  grid-stride, block 256.
template <typename T>
__global__ __launch_bounds__(256) void add_relu_kernel(const T* __restrict__ a, const T* __restrict__ b, T* y,
                                                       long long count) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i + 8 <= count) {
    const vec8<T> x = load8(a + i), z = load8(b + i);
    vec8<T> o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = from_f<T>(fmaxf(to_f(x[e]) + to_f(z[e]), 0.f));
    store8<T>(y + i, o);
  } else {
    for (long long j = i; j < count; ++j) y[j] = from_f<T>(fmaxf(to_f(a[j]) + to_f(b[j]), 0.f));
  }
}

// y[r, c] = act(y[r, c] + bias[c]) in place over channels-last rows of C channels (C % 8 == 0):
// the C5 encoder's 3x3 convolutions' folded conv+BN bias and ReLU in one pass (MIOpen's
// convolution + a bias add + a ReLU clamp were two extra read+write passes).
template <typename T>
__global__ __launch_bounds__(256) void bias_act_kernel(T* y, const T* __restrict__ bias, long long count, int C,
                                                       int relu) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= count) return;
  const int c = (int)(i % C);
  const vec8<T> x = load8(y + i), b = load8(bias + c);
  vec8<T> o;
  const float lo = relu ? 0.f : -INFINITY;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = from_f<T>(fmaxf(to_f(x[e]) + to_f(b[e]), lo));
  store8<T>(y + i, o);
}

}  // namespace

// CrossEntropyLoss(logits, one_hot(label).float()) averaged over the B rows
// (code/models/model_interface.py:346-347; the soft-target form equals -log_softmax at the label),
// with Y_prob = softmax(logits) and Y_hat = argmax(logits) (:339-341, first index on ties) in the
// same pass; one block.  Backward: dlogits = g (prob - one_hot) / B, g = the upstream scalar.
__global__ void __launch_bounds__(256) ce_fwd_kernel(const float* __restrict__ logits,
                                                     const long long* __restrict__ label, int B, int C,
                                                     float* __restrict__ loss, float* __restrict__ prob,
                                                     long long* __restrict__ yhat, int* __restrict__ stats) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const float* l = logits + (size_t)b * C;
    float m = l[0];
    int am = 0;
    for (int c = 1; c < C; ++c)
      if (l[c] > m) { m = l[c]; am = c; }
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += expf(l[c] - m);
    const float inv = 1.f / s, lse = m + logf(s);
    for (int c = 0; c < C; ++c) prob[(size_t)b * C + c] = expf(l[c] - m) * inv;
    const long long y = label[b];      // out of range: NaN loss, no out-of-bounds read
    acc += (y >= 0 && y < C) ? lse - l[y] : __builtin_nanf("");
    yhat[b] = am;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    loss[0] = (red[0] + red[1] + red[2] + red[3]) / (float)B;
    // the reference's per-class bookkeeping (self.data[y]["count"/"correct"], :350-356), kept on
    // the device instead of one host sync per step
    if (stats)
      for (int b = 0; b < B; ++b) {
        const long long yl = label[b];
        if (yl < 0 || yl >= C) continue;
        const int y = (int)yl;
        stats[2 * y] += 1;
        stats[2 * y + 1] += yhat[b] == y;
      }
  }
}

__global__ void __launch_bounds__(256) ce_bwd_kernel(const float* __restrict__ prob,
                                                     const long long* __restrict__ label, int B, int C,
                                                     const float* __restrict__ g, float* __restrict__ dlogits) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i % C;
  dlogits[i] = g[0] * (prob[i] - (c == (int)label[b] ? 1.f : 0.f)) / (float)B;
}

#define TM_DTYPE_DISPATCH(dt, CALL)                               \
  if ((dt) == TM_BF16) { using T = bf16; CALL; }                  \
  else if ((dt) == TM_F32) { using T = float; CALL; }             \
  else { tm_set_error("glue: dtype must be TM_F32 or TM_BF16"); return 1; }

extern "C" int tm_ce_fwd(const float* logits, const long long* label, int B, int C, float* loss, float* prob,
                         long long* yhat, int* class_stats, void* stream) {
  TM_REQUIRE(B >= 1 && C >= 1, "ce_fwd: empty logits");
  ce_fwd_kernel<<<1, 256, 0, (hipStream_t)stream>>>(logits, label, B, C, loss, prob, yhat, class_stats);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_ce_bwd(const float* prob, const long long* label, int B, int C, const float* g, float* dlogits,
                         void* stream) {
  ce_bwd_kernel<<<(B * C + 255) / 256, 256, 0, (hipStream_t)stream>>>(prob, label, B, C, g, dlogits);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_put_cls(const float* cls, int B, int S, int D, float* H, void* stream) {
  put_cls_kernel<<<B, 256, 0, (hipStream_t)stream>>>(cls, S, D, H);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_dropout_bwd_pad(int dtype, const float* dH, int B, int S, int n_pad, int pad, int D, float p,
                                  uint64_t seed, const uint64_t* seed_ptr, void* out, void* stream) {
  TM_REQUIRE(n_pad >= S + pad, "dropout_bwd_pad: n_pad < S + pad");
  const float scale = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  TM_DTYPE_DISPATCH(dtype, (dropout_bwd_pad_kernel<T><<<dim3(n_pad, B), 256, 0, (hipStream_t)stream>>>(
                               dH, S, n_pad, pad, D, p, scale, seed, seed_ptr, (T*)out)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_pad_rows(int dtype, const float* x, int B, int S, int n_pad, int pad, int D, void* y,
                           void* stream) {
  TM_REQUIRE(n_pad >= S + pad, "pad_rows: n_pad < S + pad");
  TM_DTYPE_DISPATCH(dtype, (pad_rows_kernel<T><<<dim3(n_pad, B), 256, 0, (hipStream_t)stream>>>(
                               x, S, n_pad, pad, D, (T*)y)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_fc1_gelu_bwd(int dtype, const float* dH, const void* pre, int B, int N, int S, int add, int D,
                               void* dpre, float* dcls, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  TM_REQUIRE(D % 8 == 0 && ((uintptr_t)dH % 16) == 0 && ((uintptr_t)pre % 16) == 0 && ((uintptr_t)dpre % 16) == 0,
             "fc1_gelu_bwd: D % 8 == 0 and 16-B aligned rows");
  TM_DTYPE_DISPATCH(dtype, (fc1_gelu_bwd_kernel<T><<<dim3((N + 3) / 4, B), 256, 0, st>>>(dH, (const T*)pre, B, N, S,
                                                                                         add, D, (T*)dpre, dcls)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_gelu_bwd(int dtype, const float* dy, const float* pre, long long count, void* dpre,
                           void* stream) {
  TM_REQUIRE(dy && pre && dpre && count >= 0, "gelu_bwd: bad args");
  TM_REQUIRE(((uintptr_t)dy % 16) == 0 && ((uintptr_t)pre % 16) == 0, "gelu_bwd: dy / pre must be 16-B aligned");
  if (count == 0) return 0;
  const unsigned blocks = (unsigned)(((count + 3) / 4 + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
  TM_DTYPE_DISPATCH(dtype, (gelu_bwd_kernel<T><<<blocks, 256, 0, st>>>(dy, pre, (size_t)count, (T*)dpre)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_step_prepare(int dtype, const tm_cast_table* table, const float* w7, const float* b7,
                               const float* w5, const float* b5, const float* w3, const float* b3, int D,
                               float* wfold, float* bfold, long long* counter, long long* seed_out,
                               const float* cls, float* H, int B, int S, void* stream) {
  TM_REQUIRE(table && table->count >= 0 && table->count <= TM_CAST_MAX, "step_prepare: 0..8 tensors");
  TM_REQUIRE(!cls || (H && B >= 1 && S >= 1), "step_prepare: class-token rows need H, B, S");
  TM_REQUIRE(!counter || seed_out, "step_prepare: the counter needs a seed output");
  long long off = 0;
  for (int i = 0; i < table->count; ++i) {
    TM_REQUIRE(table->src[i] && table->dst[i], "step_prepare: null tensor");
    TM_REQUIRE(table->offset[i] == off && table->offset[i + 1] >= off && table->offset[i + 1] % 4 == 0,
               "step_prepare: offsets must be a prefix sum of multiples of 4");
    off = table->offset[i + 1];
  }
  const long long cast_blocks = (off + 1024 * CAST_PIECES - 1) / (1024 * CAST_PIECES);
  const long long blocks = cast_blocks + (w7 ? (49LL * D + 255) / 256 : 0) + 1;
  TM_DTYPE_DISPATCH(dtype, (step_prepare_kernel<T><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(
                               *table, cast_blocks, w7, b7, w5, b5, w3, b3, D, wfold, bfold, counter, seed_out,
                               cls, H, B, S)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_cast_f32_many(int dtype, const tm_cast_table* table, void* stream) {
  TM_REQUIRE(table && table->count >= 1 && table->count <= TM_CAST_MAX, "cast_many: 1..8 tensors");
  long long off = 0;
  for (int i = 0; i < table->count; ++i) {
    TM_REQUIRE(table->src[i] && table->dst[i], "cast_many: null tensor");
    TM_REQUIRE(table->offset[i] == off && table->offset[i + 1] >= off, "cast_many: offsets must be a prefix sum");
    // a thread converts 4 consecutive elements of the concatenated index space: a tensor that
    // ended mid-quad would leave the next one's first elements unconverted
    TM_REQUIRE(table->offset[i + 1] % 4 == 0, "cast_many: every tensor's element count must be a multiple of 4");
    off = table->offset[i + 1];
  }
  if (off == 0) return 0;
  const long long threads = (off + 3) / 4;
  TM_DTYPE_DISPATCH(dtype, (cast_many_kernel<T><<<(unsigned)((threads + 255) / 256), 256, 0, (hipStream_t)stream>>>(
                               *table)));
  TM_CHECK_LAUNCH();
  return 0;
}

// ResNet stem tail (code/models/ResNet.py:240-245: conv1 -> bn1 -> relu -> maxpool 3x3/2 pad 1) on
// the raw stem convolution output, channels-last bf16: out = relu(max over the window of y + b)
// (= max of relu(y + b): + b and ReLU are monotone), one thread per 8 channels of one output
// pixel; the 9 window rows' 16-B pieces are loaded before the max (out-of-range taps skipped, as
// the -inf padding of max_pool2d).
// AFFINE: train-mode BatchNorm instead of the folded bias: each tap is bf16(relu(y * scale + shift))
// (tm_bn_apply's per-element arithmetic; the scale may be negative, so the affine map is applied
// before the max), then the max of the window.
template <bool AFFINE = false>
__global__ __launch_bounds__(256) void bias_relu_maxpool_kernel(const bf16* __restrict__ y, const bf16* __restrict__ bias,
                                                                bf16* __restrict__ out, long long npix, int H, int W,
                                                                int OH, int OW, int C,
                                                                const float* __restrict__ scale = nullptr,
                                                                const float* __restrict__ shift = nullptr) {
  const int cg = C / 8;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= npix * cg) return;
  const int c8 = (int)(i % cg) * 8;
  const long long pix = i / cg;
  const int ow = (int)(pix % OW), oh = (int)((pix / OW) % OH);
  const long long nimg = pix / ((long long)OW * OH);
  const bf16* base = y + nimg * H * W * (long long)C + c8;
  bf16x8 v[9];
  bool ok[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ih = 2 * oh - 1 + t / 3, iw = 2 * ow - 1 + t % 3;
    ok[t] = ih >= 0 && ih < H && iw >= 0 && iw < W;
    v[t] = ok[t] ? *(const bf16x8*)(base + ((long long)ih * W + iw) * C) : (bf16x8){};
  }
  float m[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
  if constexpr (AFFINE) {
    float sc[8], sf[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = scale[c8 + e]; sf[e] = shift[c8 + e]; }
#pragma unroll
    for (int t = 0; t < 9; ++t)
      if (ok[t])
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], (float)(bf16)fmaxf(fmaf((float)v[t][e], sc[e], sf[e]), 0.f));
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)m[e];
    *(bf16x8*)(out + pix * C + c8) = o;
    return;
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
    if (ok[t])
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], (float)v[t][e]);
  const bf16x8 b8 = *(const bf16x8*)(bias + c8);
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    // the reference rounds y + b to bf16 before the ReLU / pool: same here (the max of the
    // rounded sums equals the rounded sum of the max: rounding is monotone)
    const float sb = (float)(bf16)(m[e] + (float)b8[e]);
    o[e] = (bf16)fmaxf(sb, 0.f);
  }
  *(bf16x8*)(out + pix * C + c8) = o;
}

extern "C" int tm_bias_relu_maxpool(const void* y, const void* bias, void* out, int N, int H, int W, int C,
                                    void* stream) {
  TM_REQUIRE(y && bias && out && N > 0 && H > 0 && W > 0 && C > 0 && C % 8 == 0, "bias_relu_maxpool: bad args");
  TM_REQUIRE(((uintptr_t)y % 16) == 0 && ((uintptr_t)bias % 16) == 0 && ((uintptr_t)out % 16) == 0,
             "bias_relu_maxpool: 16-B aligned buffers");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const long long npix = (long long)N * OH * OW;
  const long long threads = npix * (C / 8);
  bias_relu_maxpool_kernel<false><<<(unsigned)((threads + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const bf16*)y, (const bf16*)bias, (bf16*)out, npix, H, W, OH, OW, C);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_bn_relu_maxpool(const void* y, const float* scale, const float* shift, void* out, int N, int H, int W,
                                  int C, void* stream) {
  TM_REQUIRE(y && scale && shift && out && N > 0 && H > 0 && W > 0 && C > 0 && C % 8 == 0,
             "bn_relu_maxpool: bad args");
  TM_REQUIRE(((uintptr_t)y % 16) == 0 && ((uintptr_t)out % 16) == 0, "bn_relu_maxpool: 16-B aligned buffers");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const long long npix = (long long)N * OH * OW;
  const long long threads = npix * (C / 8);
  bias_relu_maxpool_kernel<true><<<(unsigned)((threads + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const bf16*)y, nullptr, (bf16*)out, npix, H, W, OH, OW, C, scale, shift);
  TM_CHECK_LAUNCH();
  return 0;
}

// Strided spatial subsample of a channels-last activation (the input of a stride-s 1x1 downsample
// convolution, code/models/ResNet.py:130-135): out[n, i, j, :] = x[n, s*i, s*j, :], one thread per
// 16-B piece of a pixel's channels (the channel rows stay contiguous on both sides).
__global__ __launch_bounds__(256) void subsample_kernel(const uint4* __restrict__ x, uint4* __restrict__ out,
                                                        long long npix_out, int H, int W, int OH, int OW, int s,
                                                        int pieces) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= npix_out * pieces) return;
  const int q = (int)(i % pieces);
  const long long pix = i / pieces;
  const int ow = (int)(pix % OW), oh = (int)((pix / OW) % OH);
  const long long n = pix / ((long long)OW * OH);
  out[i] = x[((n * H + (long long)oh * s) * W + (long long)ow * s) * pieces + q];
}

extern "C" int tm_subsample2d(int dtype, const void* x, void* out, int N, int H, int W, int C, int stride,
                              void* stream) {
  TM_REQUIRE(x && out && N > 0 && H > 0 && W > 0 && C > 0 && stride > 0, "subsample2d: bad args");
  const int esz = dtype == TM_BF16 ? 2 : 4;
  TM_REQUIRE((C * esz) % 16 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)out % 16) == 0,
             "subsample2d: 16-B channel rows and buffers");
  const int OH = (H - 1) / stride + 1, OW = (W - 1) / stride + 1, pieces = C * esz / 16;
  const long long npix = (long long)N * OH * OW;
  const long long threads = npix * pieces;
  subsample_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const uint4*)x, (uint4*)out, npix, H, W, OH, OW, stride, pieces);
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_bias_act(int dtype, void* y, const void* bias, long long rows, int C, int relu, void* stream) {
  TM_REQUIRE(y && bias && rows >= 0 && C > 0 && C % 8 == 0, "bias_act: bad args (C % 8 == 0)");
  TM_REQUIRE(((uintptr_t)y % 16) == 0 && ((uintptr_t)bias % 16) == 0, "bias_act: 16-B aligned buffers");
  const long long count = rows * (long long)C;
  if (count == 0) return 0;
  const unsigned blocks = (unsigned)((count + 2047) / 2048);
  if (dtype == TM_BF16)
    bias_act_kernel<bf16><<<blocks, 256, 0, (hipStream_t)stream>>>((bf16*)y, (const bf16*)bias, count, C, relu);
  else if (dtype == TM_F32)
    bias_act_kernel<float><<<blocks, 256, 0, (hipStream_t)stream>>>((float*)y, (const float*)bias, count, C, relu);
  else {
    tm_set_error("bias_act: dtype");
    return 1;
  }
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_add_relu(int dtype, const void* a, const void* b, void* y, long long count, void* stream) {
  TM_REQUIRE(a && b && y && count >= 0, "add_relu: bad args");
  TM_REQUIRE(((uintptr_t)a % 16) == 0 && ((uintptr_t)b % 16) == 0 && ((uintptr_t)y % 16) == 0,
             "add_relu: 16-B aligned buffers");
  if (count == 0) return 0;
  const unsigned blocks = (unsigned)((count + 2047) / 2048);
  if (dtype == TM_BF16)
    add_relu_kernel<bf16><<<blocks, 256, 0, (hipStream_t)stream>>>((const bf16*)a, (const bf16*)b, (bf16*)y, count);
  else if (dtype == TM_F32)
    add_relu_kernel<float><<<blocks, 256, 0, (hipStream_t)stream>>>((const float*)a, (const float*)b, (float*)y, count);
  else {
    tm_set_error("add_relu: dtype");
    return 1;
  }
  TM_CHECK_LAUNCH();
  return 0;
}
