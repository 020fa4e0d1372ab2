// The Adam element update of every table / flat-parameter kernel (adam.hip) and of the fused
// embedding-backward + apply (embedding_bwd.hip): one definition, so every schedule takes the
// same bits.  torch.optim.Adam semantics (src/model/trainer.py:71-75, :285); see adam.hip.
#pragma once
#include <cmath>
#include "ncf_common.h"

namespace ncf_adam {
namespace {

struct AdamScalars {
  float neg_step, w1, b2, c2, inv_bc2_sqrt, eps, wd;
  float b1, k1, k2;   // zero-gradient step: beta1, (1-beta1) wd, (1-beta2) wd^2
  float ra, rb;       // zero-gradient step s: inv_bc2_sqrt / neg_step, eps / neg_step
};

// One Adam element update, written as explicit fmas with the hardware square root and
// reciprocal (v_sqrt_f32 / v_rcp_f32, ~1 ulp) and 1/sqrt(1-b2^t) folded on the host:
//   g' = g + wd*p;  m += (1-b1)(g' - m);  v = b2 v + (1-b2) g'^2
//   p += (-lr/(1-b1^t)) * m * 1/(sqrt(v) * 1/sqrt(1-b2^t) + eps)
// 11 VALU ops (2 transcendental) per element-step.  Every kernel that applies a step (dense
// sweep, deferred catch-up, touched-row apply) calls this one function with the same fp32
// scalars, so the deferred schedule reproduces the dense schedule bit for bit; against torch's
// correctly rounded CPU Adam the difference is ~1 ulp of the step (parity tests: abs 1e-6).
__device__ __forceinline__ void adam1(float& p, float& m, float& v, float g, float neg_step,
                                      float inv_bc, const AdamScalars& s) {
  g = __builtin_fmaf(s.wd, p, g);
  m = __builtin_fmaf(s.w1, g - m, m);
  v = __builtin_fmaf(s.c2 * g, g, v * s.b2);
  const float denom = __builtin_fmaf(__builtin_amdgcn_sqrtf(v), inv_bc, s.eps);
  p = __builtin_fmaf(neg_step * m, __builtin_amdgcn_rcpf(denom), p);
}

// The step of an element whose gradient is zero (an untouched table row: weight decay only),
// the same update with the constants folded (9 VALU ops, 2 transcendental, instead of 11):
//   m = b1 m + ((1-b1) wd) p;   v = b2 v + ((1-b2) wd^2) p p
//   p += m / (sqrt(v) ra + rb),   ra = inv_bc2_sqrt / neg_step, rb = eps / neg_step
// Used by every schedule for exactly the untouched elements (the dense sweep for rows without a
// gradient slot, the deferred replay for the zero-gradient steps it owes), so the schedules stay
// bit-identical to each other; against torch's Adam it differs by rounding (~1 ulp of m, v).
__device__ __forceinline__ void adam0(float& p, float& m, float& v, float ra, float rb,
                                      const AdamScalars& s) {
  m = __builtin_fmaf(s.b1, m, s.k1 * p);
  v = __builtin_fmaf(s.k2 * p, p, v * s.b2);
  const float den = __builtin_fmaf(__builtin_amdgcn_sqrtf(v), ra, rb);
  p = __builtin_fmaf(m, __builtin_amdgcn_rcpf(den), p);
}

__device__ __forceinline__ void adam1(float& p, float& m, float& v, float g, const AdamScalars& s) {
  adam1(p, m, v, g, s.neg_step, s.inv_bc2_sqrt, s);
}

__device__ __forceinline__ void adam4(float4& p, float4& m, float4& v, float4 g, float ns,
                                      float bc, const AdamScalars& s) {
  adam1(p.x, m.x, v.x, g.x, ns, bc, s);
  adam1(p.y, m.y, v.y, g.y, ns, bc, s);
  adam1(p.z, m.z, v.z, g.z, ns, bc, s);
  adam1(p.w, m.w, v.w, g.w, ns, bc, s);
}

__device__ __forceinline__ void adam4(float4& p, float4& m, float4& v, float4 g, const AdamScalars& s) {
  adam4(p, m, v, g, s.neg_step, s.inv_bc2_sqrt, s);
}

inline AdamScalars make_scalars(double lr, double beta1, double beta2, double eps, double wd, double step) {
  AdamScalars s;
  const double bc1 = 1.0 - pow(beta1, step);
  const double bc2 = 1.0 - pow(beta2, step);
  s.neg_step = (float)(-(lr / bc1));
  s.w1 = (float)(1.0 - beta1);
  s.b2 = (float)beta2;
  s.c2 = (float)(1.0 - beta2);
  s.inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
  s.eps = (float)eps;
  s.wd = (float)wd;
  s.b1 = (float)beta1;
  s.k1 = (float)((1.0 - beta1) * wd);
  s.k2 = (float)((1.0 - beta2) * wd * wd);
  // zero-gradient form: ns folded into the denominator (lr == 0: a finite huge denominator, the
  // step vanishes instead of 0 * inf)
  const double ns = -(lr / bc1);
  s.ra = ns != 0.0 ? (float)((1.0 / sqrt(bc2)) / ns) : -3.0e38f;
  s.rb = ns != 0.0 ? (float)(eps / ns) : -3.0e38f;
  return s;
}

inline AdamScalars consts_of(double beta1, double beta2, double eps, double wd) {
  AdamScalars s = make_scalars(1.0, beta1, beta2, eps, wd, 1.0);
  s.neg_step = 0.f;
  s.inv_bc2_sqrt = 1.f;
  return s;
}

}  // namespace
}  // namespace ncf_adam
