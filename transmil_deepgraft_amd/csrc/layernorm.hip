// LayerNorm forward/backward and the class-token head.
//
// Replaces: TransLayer.norm (code/models/TransMIL.py:23, applied at :47) and the
// final `self.norm` + `_fc` head (code/models/TransMIL.py:154-155, 202-204).
// One wave per token row (HBM-bound; D/64 fp32 values per lane in registers).
// The forward writes the normalised rows straight into the FRONT-padded
// [B, n', D] layout NystromAttention consumes (SURVEY.md App. A eq. 1), with
// the pad rows zeroed, so no separate pad copy exists.
#include "common.h"
#include "head_bwd.h"
#include "../../include/transmil_hip.h"

namespace {

template <int VPL>
TM_DEV void load_row(float (&v)[VPL], const float* p, int lane) {
  if constexpr (VPL % 4 == 0) {
#pragma unroll
    for (int i = 0; i < VPL; i += 4) {
      f32x4 t = *(const f32x4*)(p + lane * VPL + i);
      v[i] = t[0]; v[i + 1] = t[1]; v[i + 2] = t[2]; v[i + 3] = t[3];
    }
  } else {
#pragma unroll
    for (int i = 0; i < VPL; ++i) v[i] = p[lane * VPL + i];
  }
}

template <typename T, int VPL>
TM_DEV void load_row_t(float (&v)[VPL], const T* p, int lane) {
  if constexpr (VPL == 8) {
    const vec8<T> t = load8(p + lane * VPL);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = to_f(t[i]);
  } else {
#pragma unroll
    for (int i = 0; i < VPL; ++i) v[i] = to_f(p[lane * VPL + i]);
  }
}

// rows: B*S input rows (fp32 residual stream); out row = (r / S) * n_pad + pad + r % S
template <typename T, int VPL>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps, int rows, int S,
                                                     int n_pad, int pad, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int D = VPL * 64;
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nbags = rows / S;
  // extra rows beyond `rows` zero the pad rows of every bag
  if (r >= rows) {
    const int z = r - rows;  // pad row index over all bags
    if (z < nbags * pad) {
      const int b = z / pad, t = z % pad;
      T* dst = y + ((size_t)b * n_pad + t) * D;
#pragma unroll
      for (int i = 0; i < VPL; ++i) dst[lane * VPL + i] = from_f<T>(0.f);
    }
    return;
  }
  float v[VPL];
  load_row<VPL>(v, x + (size_t)r * D, lane);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += v[i];
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) { const float d = v[i] - mean; q += d * d; }
  const float var = wave_sum(q) * (1.0f / D);
  const float rstd = 1.0f / sqrtf(var + eps);
  const int b = r / S, t = r % S;
  T* dst = y + ((size_t)b * n_pad + pad + t) * D;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane * VPL + i;
    dst[c] = from_f<T>((v[i] - mean) * rstd * gamma[c] + beta[c]);
  }
  if (lane == 0) { mean_out[r] = mean; rstd_out[r] = rstd; }
}

// dx accumulated into dx_accum (fp32, [rows, D]); dy read from the padded layout.
// Each block handles `rows_per_block` rows (4 waves interleaved) and writes one
// partial row of dgamma / dbeta: part[2][nblocks][D].
// SEG: dy of row t (bag b) + seg[b][(pad + t) / len] (+ seg[b][nseg] at t = 0): the class-row
// layer's q-part gradient rows (tm_layernorm_bwd_seg)
struct SegAdd { const float* p; int len, nseg, rows; };
template <typename T, int VPL, bool SEG = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const float* __restrict__ x,
                                                     const float* __restrict__ gamma, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, int rows, int S, int n_pad, int pad,
                                                     int rows_per_block, int resid_cls_only, float* __restrict__ dx_accum,
                                                     float* __restrict__ part, SegAdd sg = SegAdd{nullptr, 1, 0, 0}) {
  constexpr int D = VPL * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dg[VPL], db[VPL], gm[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) { dg[i] = 0.f; db[i] = 0.f; gm[i] = gamma[lane * VPL + i]; }
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  // software pipeline: the next row's dy, x, mean/rstd and dx_accum are requested before
  // this row is processed (one HBM round trip in flight instead of one per row)
  auto fetch = [&](int r, float (&g)[VPL], float (&xv)[VPL], float (&acc)[VPL], float& mu, float& rs,
                   float (&sa)[VPL]) {
    const int rr = min(r, rows - 1);
    const int b = rr / S, t = rr % S;
    load_row_t<T, VPL>(g, dy + ((size_t)b * n_pad + pad + t) * D, lane);
    if constexpr (SEG) {
      load_row<VPL>(sa, sg.p + ((size_t)b * sg.rows + (pad + t) / sg.len) * D, lane);
      if (t == 0) {   // the class row also carries its own q term (one row per bag: a waited load)
        float sc[VPL];
        load_row<VPL>(sc, sg.p + ((size_t)b * sg.rows + sg.nseg) * D, lane);
#pragma unroll
        for (int i = 0; i < VPL; ++i) sa[i] += sc[i];
      }
    }
    load_row<VPL>(xv, x + (size_t)rr * D, lane);
    if (!resid_cls_only || t == 0) {
      load_row<VPL>(acc, dx_accum + (size_t)rr * D, lane);
    } else {
#pragma unroll
      for (int i = 0; i < VPL; ++i) acc[i] = 0.f;
    }
    mu = mean[rr];
    rs = rstd[rr];
  };
  float g[VPL], xv[VPL], dacc[VPL], sa[VPL], mu, rs;
  int r = r0 + wave;
  if (r < r1) fetch(r, g, xv, dacc, mu, rs, sa);
  for (; r < r1; r += 4) {
    float g2[VPL], xv2[VPL], dacc2[VPL], sa2[VPL], mu2 = 0.f, rs2 = 0.f;
    const bool more = r + 4 < r1;
    if (more) fetch(r + 4, g2, xv2, dacc2, mu2, rs2, sa2);
    if constexpr (SEG) {
#pragma unroll
      for (int i = 0; i < VPL; ++i) g[i] += sa[i];
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const float xh = (xv[i] - mu) * rs;
      dg[i] += g[i] * xh;
      db[i] += g[i];
      const float gg = g[i] * gm[i];
      xv[i] = xh;
      g[i] = gg;
      s1 += gg;
      s2 += gg * xh;
    }
    s1 = wave_sum(s1) * (1.0f / D);
    s2 = wave_sum(s2) * (1.0f / D);
    float* dst = dx_accum + (size_t)r * D;
    if constexpr (VPL % 4 == 0) {
#pragma unroll
      for (int i = 0; i < VPL; i += 4)
        *(f32x4*)(dst + lane * VPL + i) =
            (f32x4){dacc[i] + rs * (g[i] - s1 - xv[i] * s2), dacc[i + 1] + rs * (g[i + 1] - s1 - xv[i + 1] * s2),
                    dacc[i + 2] + rs * (g[i + 2] - s1 - xv[i + 2] * s2), dacc[i + 3] + rs * (g[i + 3] - s1 - xv[i + 3] * s2)};
    } else {
#pragma unroll
      for (int i = 0; i < VPL; ++i) dst[lane * VPL + i] = dacc[i] + rs * (g[i] - s1 - xv[i] * s2);
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < VPL; ++i) { g[i] = g2[i]; xv[i] = xv2[i]; dacc[i] = dacc2[i]; sa[i] = sa2[i]; }
      mu = mu2;
      rs = rs2;
    }
  }
  __shared__ float red[2][4][D];
#pragma unroll
  for (int i = 0; i < VPL; ++i) { red[0][wave][lane * VPL + i] = dg[i]; red[1][wave][lane * VPL + i] = db[i]; }
  __syncthreads();
  const size_t nb = gridDim.x;
  for (int c = threadIdx.x; c < D; c += 256) {
    part[(size_t)blockIdx.x * D + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    part[(nb + blockIdx.x) * D + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

// Head forward: per bag, LN(h[b, 0]) -> logits = y W^T + bias.  One wave per bag.
template <int VPL>
__global__ void head_fwd_kernel(const float* __restrict__ h, int S, const float* __restrict__ gamma,
                                const float* __restrict__ beta, float eps, const float* __restrict__ W,
                                const float* __restrict__ bias, int C, float* __restrict__ logits,
                                float* __restrict__ xhat, float* __restrict__ rstd_out) {
  constexpr int D = VPL * 64;
  const int b = blockIdx.x, lane = threadIdx.x;
  float v[VPL];
  load_row<VPL>(v, h + (size_t)b * S * D, lane);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += v[i];
  const float mu = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) { const float d = v[i] - mu; q += d * d; }
  const float rs = 1.0f / sqrtf(wave_sum(q) * (1.0f / D) + eps);
  float y[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane * VPL + i;
    const float xh = (v[i] - mu) * rs;
    xhat[(size_t)b * D + c] = xh;
    y[i] = xh * gamma[c] + beta[c];
  }
  if (lane == 0) rstd_out[b] = rs;
  for (int k = 0; k < C; ++k) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) acc += y[i] * W[(size_t)k * D + lane * VPL + i];
    acc = wave_sum(acc);
    if (lane == 0) logits[b * C + k] = acc + bias[k];
  }
}

// Head backward: one block of 64 threads loops over bags (B is small).
// Writes dW [C,D], db [C], dgamma/dbeta [D] and dh[b*S*D + :] (row 0 of each bag).
template <int VPL>
__global__ void head_bwd_kernel(const float* __restrict__ dlogits, int B, int C, int S,
                                const float* __restrict__ xhat, const float* __restrict__ rstd,
                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                const float* __restrict__ W, float* __restrict__ dW, float* __restrict__ dbias,
                                float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dh) {
  constexpr int D = VPL * 64;
  const int lane = threadIdx.x;
  if (B == 1 && C <= 4) {
    // one bag (the reference's batch size), few classes: every load first, one memory round trip
    float dl[4], gm[VPL], bt[VPL], xh[VPL], w[4][VPL];
#pragma unroll
    for (int k = 0; k < 4; ++k) dl[k] = k < C ? dlogits[k] : 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane * VPL + i;
      gm[i] = gamma[c]; bt[i] = beta[c]; xh[i] = xhat[c];
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k][i] = k < C ? W[(size_t)k * D + c] : 0.f;
    }
    float g[VPL], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane * VPL + i;
      float dy = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < C) {
          dW[(size_t)k * D + c] = 0.f + dl[k] * (xh[i] * gm[i] + bt[i]);
          dy += dl[k] * w[k][i];
        }
      dgamma[c] = 0.f + dy * xh[i];
      dbeta[c] = 0.f + dy;
      g[i] = dy * gm[i];
      s1 += g[i];
      s2 += g[i] * xh[i];
    }
    if (lane == 0)
      for (int k = 0; k < C; ++k) dbias[k] = 0.f + dl[k];
    s1 = wave_sum(s1) * (1.0f / D);
    s2 = wave_sum(s2) * (1.0f / D);
    const float rs = rstd[0];
#pragma unroll
    for (int i = 0; i < VPL; ++i) dh[lane * VPL + i] = rs * (g[i] - s1 - xh[i] * s2);
    return;
  }
  float dgm[VPL], dbt[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) { dgm[i] = 0.f; dbt[i] = 0.f; }
  for (int k = 0; k < C; ++k) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dlogits[b * C + k];
    if (lane == 0) dbias[k] = s;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane * VPL + i;
      float acc = 0.f;
      for (int b = 0; b < B; ++b) acc += dlogits[b * C + k] * (xhat[(size_t)b * D + c] * gamma[c] + beta[c]);
      dW[(size_t)k * D + c] = acc;
    }
  }
  for (int b = 0; b < B; ++b) {
    float g[VPL], xh[VPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane * VPL + i;
      float dy = 0.f;
      for (int k = 0; k < C; ++k) dy += dlogits[b * C + k] * W[(size_t)k * D + c];
      xh[i] = xhat[(size_t)b * D + c];
      dgm[i] += dy * xh[i];
      dbt[i] += dy;
      g[i] = dy * gamma[c];
      s1 += g[i];
      s2 += g[i] * xh[i];
    }
    s1 = wave_sum(s1) * (1.0f / D);
    s2 = wave_sum(s2) * (1.0f / D);
    const float rs = rstd[b];
#pragma unroll
    for (int i = 0; i < VPL; ++i) dh[(size_t)b * S * D + lane * VPL + i] = rs * (g[i] - s1 - xh[i] * s2);
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) { dgamma[lane * VPL + i] = dgm[i]; dbeta[lane * VPL + i] = dbt[i]; }
}

// Head + loss of the training step in ONE launch (the step's tail was four latency-bound launches:
// head, CE, CE backward, head backward -- two of them now):
// forward: the head above for every bag (wave w takes bags w, w + NW, ...), then
// CrossEntropyLoss(logits, one_hot(label).float()) averaged over the bags with Y_prob, Y_hat and
// the per-class count / correct (as ce_fwd_kernel, glue.hip), from the logits through LDS.
constexpr int HEAD_CE_WAVES = 4;
template <int VPL>
__global__ __launch_bounds__(64 * HEAD_CE_WAVES) void head_ce_fwd_kernel(
    const float* __restrict__ h, int B, int S, const float* __restrict__ gamma, const float* __restrict__ beta,
    float eps, const float* __restrict__ W, const float* __restrict__ bias, int C, const long long* __restrict__ label,
    float* __restrict__ logits, float* __restrict__ xhat, float* __restrict__ rstd_out, float* __restrict__ loss,
    float* __restrict__ prob, long long* __restrict__ yhat, int* __restrict__ stats) {
  constexpr int D = VPL * 64;
  __shared__ float red[HEAD_CE_WAVES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int b = wave; b < B; b += HEAD_CE_WAVES) {
    float v[VPL];
    load_row<VPL>(v, h + (size_t)b * S * D, lane);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) s += v[i];
    const float mu = wave_sum(s) * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) { const float d = v[i] - mu; q += d * d; }
    const float rs = 1.0f / sqrtf(wave_sum(q) * (1.0f / D) + eps);
    float y[VPL];
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane * VPL + i;
      const float xh = (v[i] - mu) * rs;
      xhat[(size_t)b * D + c] = xh;
      y[i] = xh * gamma[c] + beta[c];
    }
    if (lane == 0) rstd_out[b] = rs;
    for (int k = 0; k < C; ++k) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < VPL; ++i) acc += y[i] * W[(size_t)k * D + lane * VPL + i];
      acc = wave_sum(acc);
      if (lane == 0) logits[b * C + k] = acc + bias[k];
    }
  }
  __syncthreads();   // the block's logits stores are visible to the block (same workgroup)
  float acc = 0.f;
  for (int b = threadIdx.x; b < B; b += 64 * HEAD_CE_WAVES) {
    const float* l = logits + (size_t)b * C;
    float m = l[0];
    int am = 0;
    for (int c = 1; c < C; ++c)
      if (l[c] > m) { m = l[c]; am = c; }
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += expf(l[c] - m);
    const float inv = 1.f / s, lse = m + logf(s);
    for (int c = 0; c < C; ++c) prob[(size_t)b * C + c] = expf(l[c] - m) * inv;
    // an out-of-range label (F.one_hot raises in the reference) poisons the loss with NaN instead
    // of reading past the logits row
    const long long y = label[b];
    acc += (y >= 0 && y < C) ? lse - l[y] : __builtin_nanf("");
    yhat[b] = am;
  }
  acc = wave_sum(acc);
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < HEAD_CE_WAVES; ++w) t += red[w];
    loss[0] = t / (float)B;
    if (stats)
      for (int b = 0; b < B; ++b) {
        const long long y = label[b];
        if (y < 0 || y >= C) continue;     // never index class_stats out of bounds
        const int yv = (int)y;
        stats[2 * yv] += 1;
        stats[2 * yv + 1] += yhat[b] == yv;
      }
  }
}

// backward of the above: dlogits = g (prob - one_hot(label)) / B (+ dlogits_in, the gradient
// reaching the logits from other uses; null: none), then the head backward of head_bwd_kernel.
template <int VPL>
__global__ void head_ce_bwd_kernel(const float* __restrict__ prob, const long long* __restrict__ label,
                                   const float* __restrict__ g, const float* __restrict__ dlogits_in, int B, int C,
                                   int S, const float* __restrict__ xhat, const float* __restrict__ rstd,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   const float* __restrict__ W, float* __restrict__ dW, float* __restrict__ dbias,
                                   float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dh,
                                   float* __restrict__ dl_scratch) {
  constexpr int D = VPL * 64;
  const int lane = threadIdx.x;
  const float gs = g[0] / (float)B;
  if (B == 1 && C <= 4) {
    head_bwd_b1<VPL>(prob, label, g, dlogits_in, C, xhat, rstd, gamma, beta, W, dW, dbias, dgamma, dbeta, dh, nullptr,
                     lane);
    return;
  }
  // general B / C: dlogits into the scratch, then the general head backward
  for (int i = lane; i < B * C; i += 64) {
    const int b = i / C, c = i % C;
    dl_scratch[i] = gs * (prob[i] - (c == (int)label[b] ? 1.f : 0.f)) + (dlogits_in ? dlogits_in[i] : 0.f);
  }
  __syncthreads();
  const float* dlogits = dl_scratch;
  float dgm[VPL], dbt[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) { dgm[i] = 0.f; dbt[i] = 0.f; }
  for (int k = 0; k < C; ++k) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dlogits[b * C + k];
    if (lane == 0) dbias[k] = s;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane * VPL + i;
      float acc = 0.f;
      for (int b = 0; b < B; ++b) acc += dlogits[b * C + k] * (xhat[(size_t)b * D + c] * gamma[c] + beta[c]);
      dW[(size_t)k * D + c] = acc;
    }
  }
  for (int b = 0; b < B; ++b) {
    float gg[VPL], xh[VPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane * VPL + i;
      float dy = 0.f;
      for (int k = 0; k < C; ++k) dy += dlogits[b * C + k] * W[(size_t)k * D + c];
      xh[i] = xhat[(size_t)b * D + c];
      dgm[i] += dy * xh[i];
      dbt[i] += dy;
      gg[i] = dy * gamma[c];
      s1 += gg[i];
      s2 += gg[i] * xh[i];
    }
    s1 = wave_sum(s1) * (1.0f / D);
    s2 = wave_sum(s2) * (1.0f / D);
    const float rs = rstd[b];
#pragma unroll
    for (int i = 0; i < VPL; ++i) dh[(size_t)b * S * D + lane * VPL + i] = rs * (gg[i] - s1 - xh[i] * s2);
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) { dgamma[lane * VPL + i] = dgm[i]; dbeta[lane * VPL + i] = dbt[i]; }
}

}  // namespace

#define TM_VPL_DISPATCH(D, CALL)                        \
  switch (D) {                                          \
    case 64: { constexpr int VPL = 1; CALL; break; }    \
    case 128: { constexpr int VPL = 2; CALL; break; }   \
    case 256: { constexpr int VPL = 4; CALL; break; }   \
    case 384: { constexpr int VPL = 6; CALL; break; }   \
    case 512: { constexpr int VPL = 8; CALL; break; }   \
    case 768: { constexpr int VPL = 12; CALL; break; }  \
    case 1024: { constexpr int VPL = 16; CALL; break; } \
    default: tm_set_error("layernorm: D must be 64/128/256/384/512/768/1024"); return 1; \
  }

extern "C" int tm_layernorm_fwd(const float* x, const float* gamma, const float* beta, float eps, int rows, int D,
                                int S, int n_pad, int pad, int dtype, void* y, float* mean, float* rstd,
                                void* stream) {
  TM_REQUIRE(x && gamma && beta && y && mean && rstd && S > 0 && rows % S == 0, "layernorm_fwd: bad args");
  TM_REQUIRE(n_pad >= S + pad, "layernorm_fwd: n_pad < S + pad");
  const int total = rows + (rows / S) * pad;
  const dim3 grid((total + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TM_BF16) {
    TM_VPL_DISPATCH(D, (ln_fwd_kernel<bf16, VPL><<<grid, 256, 0, st>>>(x, gamma, beta, eps, rows, S, n_pad, pad,
                                                                       (bf16*)y, mean, rstd)));
  } else {
    TM_VPL_DISPATCH(D, (ln_fwd_kernel<float, VPL><<<grid, 256, 0, st>>>(x, gamma, beta, eps, rows, S, n_pad, pad,
                                                                        (float*)y, mean, rstd)));
  }
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" long long tm_layernorm_bwd_workspace(int rows, int D, int rows_per_block) {
  return 2LL * ((rows + rows_per_block - 1) / rows_per_block) * D * (long long)sizeof(float);
}

extern "C" int tm_layernorm_bwd(const void* dy, int dtype, const float* x, const float* gamma, const float* mean,
                                const float* rstd, int rows, int D, int S, int n_pad, int pad, int rows_per_block,
                                int resid_cls_only, float* dx_accum, float* work, float* dgamma, float* dbeta,
                                tm_reduce_queue* rq, void* stream) {
  TM_REQUIRE(dy && x && gamma && mean && rstd && dx_accum && work && dgamma && dbeta, "layernorm_bwd: null arg");
  TM_REQUIRE(rows_per_block > 0 && S > 0, "layernorm_bwd: bad args");
  const int nb = (rows + rows_per_block - 1) / rows_per_block;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TM_BF16) {
    TM_VPL_DISPATCH(D, (ln_bwd_kernel<bf16, VPL><<<nb, 256, 0, st>>>((const bf16*)dy, x, gamma, mean, rstd, rows, S,
                                                                     n_pad, pad, rows_per_block, resid_cls_only, dx_accum, work)));
  } else {
    TM_VPL_DISPATCH(D, (ln_bwd_kernel<float, VPL><<<nb, 256, 0, st>>>((const float*)dy, x, gamma, mean, rstd, rows,
                                                                      S, n_pad, pad, rows_per_block, resid_cls_only, dx_accum, work)));
  }
  TM_CHECK_LAUNCH();
  int rc = tm_splitk_reduce(work, dgamma, nb, D, 1.0f, 0, rq, stream);
  if (rc) return rc;
  return tm_splitk_reduce(work + (size_t)nb * D, dbeta, nb, D, 1.0f, 0, rq, stream);
}

extern "C" int tm_layernorm_bwd_seg(const void* dy, int dtype, const float* x, const float* gamma, const float* mean,
                                    const float* rstd, int rows, int D, int S, int n_pad, int pad, int rows_per_block,
                                    int resid_cls_only, const float* seg_add, int seg_len, int nseg, int seg_rows,
                                    float* dx_accum, float* work, float* dgamma, float* dbeta, tm_reduce_queue* rq,
                                    void* stream) {
  TM_REQUIRE(dy && x && gamma && mean && rstd && dx_accum && work && dgamma && dbeta && seg_add,
             "layernorm_bwd_seg: null arg");
  TM_REQUIRE(rows_per_block > 0 && S > 0 && seg_len > 0 && nseg >= 0 && seg_rows > nseg, "layernorm_bwd_seg: bad args");
  TM_REQUIRE((long long)(pad + S - 1) / seg_len < nseg && pad + S <= n_pad, "layernorm_bwd_seg: rows past the segments");
  TM_REQUIRE(dtype == TM_BF16, "layernorm_bwd_seg: bf16 dy only");
  const int nb = (rows + rows_per_block - 1) / rows_per_block;
  hipStream_t st = (hipStream_t)stream;
  const SegAdd sg{seg_add, seg_len, nseg, seg_rows};
  TM_VPL_DISPATCH(D, (ln_bwd_kernel<bf16, VPL, true><<<nb, 256, 0, st>>>((const bf16*)dy, x, gamma, mean, rstd, rows, S,
                                                                         n_pad, pad, rows_per_block, resid_cls_only,
                                                                         dx_accum, work, sg)));
  TM_CHECK_LAUNCH();
  int rc = tm_splitk_reduce(work, dgamma, nb, D, 1.0f, 0, rq, stream);
  if (rc) return rc;
  return tm_splitk_reduce(work + (size_t)nb * D, dbeta, nb, D, 1.0f, 0, rq, stream);
}

extern "C" int tm_head_fwd(const float* h, int B, int S, int D, const float* gamma, const float* beta, float eps,
                           const float* W, const float* bias, int C, float* logits, float* xhat, float* rstd,
                           void* stream) {
  TM_REQUIRE(h && gamma && beta && W && bias && logits && xhat && rstd && B > 0 && C > 0, "head_fwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  TM_VPL_DISPATCH(D, (head_fwd_kernel<VPL><<<B, 64, 0, st>>>(h, S, gamma, beta, eps, W, bias, C, logits, xhat, rstd)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_head_ce_fwd(const float* h, int B, int S, int D, const float* gamma, const float* beta, float eps,
                              const float* W, const float* bias, int C, const long long* label, float* logits,
                              float* xhat, float* rstd, float* loss, float* prob, long long* yhat, int* class_stats,
                              void* stream) {
  TM_REQUIRE(h && gamma && beta && W && bias && label && logits && xhat && rstd && loss && prob && yhat && B > 0 &&
                 C > 0, "head_ce_fwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  TM_VPL_DISPATCH(D, (head_ce_fwd_kernel<VPL><<<1, 64 * HEAD_CE_WAVES, 0, st>>>(
                         h, B, S, gamma, beta, eps, W, bias, C, label, logits, xhat, rstd, loss, prob, yhat,
                         class_stats)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_head_ce_bwd(const float* prob, const long long* label, const float* gloss, const float* dlogits_in,
                              int B, int C, int S, int D, const float* xhat, const float* rstd, const float* gamma,
                              const float* beta, const float* W, float* dW, float* dbias, float* dgamma, float* dbeta,
                              float* dh, float* scratch, void* stream) {
  TM_REQUIRE(prob && label && gloss && xhat && rstd && gamma && beta && W && dW && dbias && dgamma && dbeta && dh,
             "head_ce_bwd: null arg");
  TM_REQUIRE((B == 1 && C <= 4) || scratch, "head_ce_bwd: scratch [B*C] needed unless B == 1 and C <= 4");
  hipStream_t st = (hipStream_t)stream;
  TM_VPL_DISPATCH(D, (head_ce_bwd_kernel<VPL><<<1, 64, 0, st>>>(prob, label, gloss, dlogits_in, B, C, S, xhat, rstd,
                                                                gamma, beta, W, dW, dbias, dgamma, dbeta, dh,
                                                                scratch)));
  TM_CHECK_LAUNCH();
  return 0;
}

extern "C" int tm_head_bwd(const float* dlogits, int B, int C, int S, int D, const float* xhat, const float* rstd,
                           const float* gamma, const float* beta, const float* W, float* dW, float* dbias,
                           float* dgamma, float* dbeta, float* dh, void* stream) {
  TM_REQUIRE(dlogits && xhat && rstd && gamma && beta && W && dW && dbias && dgamma && dbeta && dh,
             "head_bwd: null arg");
  hipStream_t st = (hipStream_t)stream;
  TM_VPL_DISPATCH(D, (head_bwd_kernel<VPL><<<1, 64, 0, st>>>(dlogits, B, C, S, xhat, rstd, gamma, beta, W, dW, dbias,
                                                             dgamma, dbeta, dh)));
  TM_CHECK_LAUNCH();
  return 0;
}
