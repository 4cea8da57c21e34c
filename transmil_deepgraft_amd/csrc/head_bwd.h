// Head + CrossEntropy backward of one bag (B = 1, <= 4 classes) on one wave, VPL channels per lane
// (code/models/TransMIL.py:202-204 LayerNorm + _fc; model_interface.py:346-347 the soft-target CE):
//   dl[k] = g (prob[k] - onehot(label)[k]) (+ dlogits_in[k])
//   dW[k][c] = dl[k] y[c] (y = x^ gamma + beta),  dbias[k] = dl[k]
//   dy[c] = sum_k dl[k] W[k][c],  dgamma = dy x^,  dbeta = dy
//   dh = rstd (dy gamma - mean(dy gamma) - x^ mean(dy gamma x^))
// Shared by layernorm.hip's head_ce_bwd_kernel and clsrow.hip's fused class-row backward, so the
// two launch shapes produce the same bits.  dW == NULL: no parameter-gradient writes; dh_out /
// dh_lds: where dh goes (either may be NULL).
#pragma once
#include "common.h"

template <int VPL>
TM_DEV void head_bwd_b1(const float* __restrict__ prob, const long long* __restrict__ label, const float* __restrict__ g,
                        const float* __restrict__ dlogits_in, int C, const float* __restrict__ xhat,
                        const float* __restrict__ rstd, const float* __restrict__ gamma, const float* __restrict__ beta,
                        const float* __restrict__ W, float* dW, float* dbias, float* dgamma, float* dbeta,
                        float* dh_out, float* dh_lds, int lane) {
  constexpr int D = VPL * 64;
  const float gs = g[0];
  const int lab = (int)label[0];
  float dl[4], gm[VPL], bt[VPL], xh[VPL], w[4][VPL];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    dl[k] = k < C ? gs * (prob[k] - (k == lab ? 1.f : 0.f)) + (dlogits_in ? dlogits_in[k] : 0.f) : 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane * VPL + i;
    gm[i] = gamma[c]; bt[i] = beta[c]; xh[i] = xhat[c];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k][i] = k < C ? W[(size_t)k * D + c] : 0.f;
  }
  float gg[VPL], s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane * VPL + i;
    float dy = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < C) {
        if (dW) dW[(size_t)k * D + c] = 0.f + dl[k] * (xh[i] * gm[i] + bt[i]);
        dy += dl[k] * w[k][i];
      }
    if (dW) { dgamma[c] = 0.f + dy * xh[i]; dbeta[c] = 0.f + dy; }
    gg[i] = dy * gm[i];
    s1 += gg[i];
    s2 += gg[i] * xh[i];
  }
  if (dW && lane == 0)
    for (int k = 0; k < C; ++k) dbias[k] = 0.f + dl[k];
  s1 = wave_sum(s1) * (1.0f / D);
  s2 = wave_sum(s2) * (1.0f / D);
  const float rs = rstd[0];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const float v = rs * (gg[i] - s1 - xh[i] * s2);
    if (dh_out) dh_out[lane * VPL + i] = v;
    if (dh_lds) dh_lds[lane * VPL + i] = v;
  }
}
