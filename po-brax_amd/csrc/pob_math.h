// pob_math.h -- device math for the rollout kernels (gfx950).
//
// Every expression here has a FIXED evaluation order and the library is compiled with
// -ffp-contract=off, so results are reproducible IEEE-754 binary32 (add/sub/mul/div/sqrt
// and the explicit fused multiply-adds FMA() are correctly rounded on gfx950, and the
// oracle spells the same fmaf() calls).  The vector / quaternion helpers are written as
// chains of fused multiply-adds (one v_fma_f32 per product-sum term).  Transcendentals use explicit polynomial forms instead of
// ocml so that the float results are a deterministic function of the inputs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define POB_D __device__ __forceinline__

struct v3 { float x, y, z; };
struct q4 { float w, x, y, z; };

#define FMA(a, b, c) __builtin_fmaf((a), (b), (c))

POB_D v3 V(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
POB_D v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
POB_D v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
POB_D v3 vscl(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
// Correctly rounded 1/x and sqrt(x) for |x| in [2^-96, 2^96] without the full IEEE
// expansions: hardware estimate + FMA correction (checked against IEEE 1/x and sqrtf on
// every float32 in that range by scripts/check_fast_ieee.hip); other inputs take the IEEE
// operation.  Same results as the oracle's 1.0f / x and sqrtf(x).
POB_D bool pob_fast_range(float x) {
  const float a = fabsf(x);
  return a >= 0x1p-96f && a <= 0x1p+96f;
}
POB_D float pob_rcp_fast(float x) {
  const float y = __builtin_amdgcn_rcpf(x);
  const float e = FMA(-x, y, 1.0f);
  return FMA(e, y, y);
}
POB_D float pob_sqrt_fast(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
  const float rdn = FMA(-sdn, s, x), rup = FMA(-sup, s, x);
  float r = rdn <= 0.0f ? sdn : s;
  r = rup > 0.0f ? sup : r;
  return r;
}
// the IEEE slow paths are out-of-line so that the compiler does not speculate them
__device__ __attribute__((noinline)) float pob_rcp_ieee(float x) { return 1.0f / x; }
__device__ __attribute__((noinline)) float pob_sqrt_ieee(float x) { return sqrtf(x); }
// wave-uniform guard: the common case (every lane in range) is one compare and a
// not-taken scalar branch, without exec-mask save/restore
POB_D float pob_rcp(float x) {
  float r = pob_rcp_fast(x);
  const bool slow = !pob_fast_range(x);
  if (__builtin_expect(__any(slow), 0)) {
    if (slow) r = pob_rcp_ieee(x);
  }
  return r;
}
POB_D float pob_sqrt(float x) {
  float r = pob_sqrt_fast(x);
  const bool slow = !pob_fast_range(x);
  if (__builtin_expect(__any(slow), 0)) {
    if (slow) r = pob_sqrt_ieee(x);
  }
  return r;
}

// s = sqrt(x) and inv = 1 / s (for use where s > 0) under ONE range guard: x in
// [2^-96, 2^96] puts s in [2^-48, 2^48], inside the reciprocal's fast range, so the
// separate guard of pob_rcp(pob_sqrt(x)) never fires there.  Same values as the pair.
POB_D void pob_sqrt_rcp(float x, float &s, float &inv) {
  s = pob_sqrt_fast(x);
  inv = pob_rcp_fast(s);
  const bool slow = !pob_fast_range(x);
  if (__builtin_expect(__any(slow), 0)) {
    if (slow) s = pob_sqrt_ieee(x);
    const float r = pob_rcp_fast(s);
    inv = pob_fast_range(s) ? r : pob_rcp_ieee(s);
  }
}

// a / b of the physics step as a * (1 / b) with the correctly rounded reciprocal (spec:
// the oracle spells a * (1.0f / b)); <= 1.5 ulp, and a quarter of an IEEE division's cost
#define POB_DIV(a, b) ((a) * pob_rcp(b))
POB_D v3 vdivs(v3 a, float s) { float inv = pob_rcp(s); return V(a.x * inv, a.y * inv, a.z * inv); }
POB_D float vdot(v3 a, v3 b) { return FMA(a.z, b.z, FMA(a.y, b.y, a.x * b.x)); }
POB_D v3 vcross(v3 a, v3 b) {
  return V(FMA(a.y, b.z, -(a.z * b.y)), FMA(a.z, b.x, -(a.x * b.z)), FMA(a.x, b.y, -(a.y * b.x)));
}
POB_D v3 vload(const float *p) { return V(p[0], p[1], p[2]); }
// min(max(x, -h), h) for h >= 0 as one v_med3_f32 (equal to the oracle's fminf(fmaxf(..))
// for every non-NaN x; no canonicalising moves)
POB_D float clamp_sym(float x, float h) { return __builtin_amdgcn_fmed3f(x, -h, h); }
// component-wise selects of vectors / quaternions: a ternary on the structs may be lowered
// to a select of their addresses, i.e. a private array in scratch memory
POB_D v3 vsel3(bool c, v3 a, v3 b) { return V(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }
POB_D q4 qsel(bool c, q4 a, q4 b) {
  q4 r; r.w = c ? a.w : b.w; r.x = c ? a.x : b.x; r.y = c ? a.y : b.y; r.z = c ? a.z : b.z; return r;
}

// brax.math.rotate(v, q) = 2 (u.v) u + (s^2 - u.u) v + 2 s (u x v)
POB_D v3 qrot(v3 v, q4 q) {
  v3 u = V(q.x, q.y, q.z);
  float t2 = 2.0f * vdot(u, v);
  float c = FMA(q.w, q.w, -vdot(u, u));
  float s2 = 2.0f * q.w;
  v3 cr = vcross(u, v);
  return V(FMA(t2, u.x, FMA(c, v.x, s2 * cr.x)), FMA(t2, u.y, FMA(c, v.y, s2 * cr.y)),
           FMA(t2, u.z, FMA(c, v.z, s2 * cr.z)));
}
// rotation matrix of q from brax.math.rotate's formula, R v = (s^2 - u.u) v + 2 (u.v) u
// + 2 s (u x v): several vectors rotated by one quaternion cost 9 operations each
struct m3 { float m00, m01, m02, m10, m11, m12, m20, m21, m22; };
POB_D m3 qmat(q4 q) {
  const float c = FMA(q.w, q.w, -FMA(q.z, q.z, FMA(q.y, q.y, q.x * q.x)));
  const float x2 = 2.0f * q.x, y2 = 2.0f * q.y, z2 = 2.0f * q.z, s2 = 2.0f * q.w;
  const float sx = s2 * q.x, sy = s2 * q.y, sz = s2 * q.z;
  m3 r;
  r.m00 = FMA(x2, q.x, c); r.m11 = FMA(y2, q.y, c); r.m22 = FMA(z2, q.z, c);
  r.m01 = FMA(x2, q.y, -sz); r.m10 = FMA(x2, q.y, sz);
  r.m02 = FMA(x2, q.z, sy); r.m20 = FMA(x2, q.z, -sy);
  r.m12 = FMA(y2, q.z, -sx); r.m21 = FMA(y2, q.z, sx);
  return r;
}
POB_D v3 mrot(const m3 &R, v3 v) {
  return V(FMA(R.m02, v.z, FMA(R.m01, v.y, R.m00 * v.x)), FMA(R.m12, v.z, FMA(R.m11, v.y, R.m10 * v.x)),
           FMA(R.m22, v.z, FMA(R.m21, v.y, R.m20 * v.x)));
}
// mrot / qrot for the Ant's joint frames (pob_system.cpp checks the pattern): the products
// with exactly-zero components dropped, which leaves every result unchanged (up to the sign
// of a zero).  v in the xy-plane (v.z == 0):
POB_D v3 mrot_xy(const m3 &R, v3 v) {
  return V(FMA(R.m01, v.y, R.m00 * v.x), FMA(R.m11, v.y, R.m10 * v.x), FMA(R.m21, v.y, R.m20 * v.x));
}
POB_D v3 mcol0(const m3 &R) { return V(R.m00, R.m10, R.m20); }  // R (1, 0, 0)
POB_D v3 mcol2(const m3 &R) { return V(R.m02, R.m12, R.m22); }  // R (0, 0, 1)
// qrot((0, 0, 1), q)
POB_D v3 qrot_ez(q4 q) {
  const float t2 = 2.0f * q.z, c = FMA(q.w, q.w, -FMA(q.z, q.z, FMA(q.y, q.y, q.x * q.x)));
  const float s2 = 2.0f * q.w;
  return V(FMA(t2, q.x, s2 * q.y), FMA(t2, q.y, -(s2 * q.x)), FMA(t2, q.z, c));
}
// qrot(v, q) with v.z == 0
POB_D v3 qrot_xy(v3 v, q4 q) {
  const float t2 = 2.0f * FMA(q.y, v.y, q.x * v.x);
  const float c = FMA(q.w, q.w, -FMA(q.z, q.z, FMA(q.y, q.y, q.x * q.x)));
  const float s2 = 2.0f * q.w;
  const v3 cr = V(-(q.z * v.y), q.z * v.x, FMA(q.x, v.y, -(q.y * v.x)));
  return V(FMA(t2, q.x, FMA(c, v.x, s2 * cr.x)), FMA(t2, q.y, FMA(c, v.y, s2 * cr.y)), FMA(t2, q.z, s2 * cr.z));
}
// brax.math.quat_mul
POB_D q4 qmul(q4 u, q4 v) {
  q4 r;
  r.w = FMA(-u.z, v.z, FMA(-u.y, v.y, FMA(-u.x, v.x, u.w * v.w)));
  r.x = FMA(-u.z, v.y, FMA(u.y, v.z, FMA(u.x, v.w, u.w * v.x)));
  r.y = FMA(u.z, v.x, FMA(u.y, v.w, FMA(-u.x, v.z, u.w * v.y)));
  r.z = FMA(u.z, v.w, FMA(-u.y, v.x, FMA(u.x, v.y, u.w * v.z)));
  return r;
}
// quat_mul([0, a], q)
POB_D q4 qmul_vq(v3 a, q4 q) {
  q4 r;
  r.w = FMA(-a.z, q.z, FMA(-a.y, q.y, -(a.x * q.x)));
  r.x = FMA(-a.z, q.y, FMA(a.y, q.z, a.x * q.w));
  r.y = FMA(a.z, q.x, FMA(a.y, q.w, -(a.x * q.z)));
  r.z = FMA(a.z, q.w, FMA(-a.y, q.x, a.x * q.y));
  return r;
}
POB_D q4 qinv(q4 q) { q4 r; r.w = q.w; r.x = -q.x; r.y = -q.y; r.z = -q.z; return r; }
// Torque actuator gate (oracle actuator_inside): no actuator torque while the joint angle is
// outside its limits.  The angle's direction from the relative rotation M = R(q_p^-1 q_c) (the
// qmat formula): hip (reference -x, axis +z) gx = M00, gy = M10; knee (reference +z, axis in
// the xy-plane) gx = M22, gy = M02 ay - M12 ax -- the oracle's generic (ref . M ref,
// (ref x M ref) . axis) with the products of the frames' exact zeros and ones folded.  Inside
// [lo, hi] (both in (-pi/2, pi/2)) iff gx > 0 and tan(lo) gx <= gy <= tan(hi) gx.
POB_D bool actuator_inside(q4 qp, q4 qc, bool hip, v3 axis, float tlo, float thi) {
  const q4 r = qmul(qinv(qp), qc);
  const float c = FMA(r.w, r.w, -FMA(r.z, r.z, FMA(r.y, r.y, r.x * r.x)));
  const float s2 = 2.0f * r.w, x2 = 2.0f * r.x;
  float gx, gy;
  if (hip) {
    gx = FMA(x2, r.x, c);
    gy = FMA(x2, r.y, s2 * r.z);
  } else {
    const float y2 = 2.0f * r.y, z2 = 2.0f * r.z;
    const float m02 = FMA(x2, r.z, s2 * r.y), m12 = FMA(y2, r.z, -(s2 * r.x));
    gx = FMA(z2, r.z, c);
    gy = FMA(m02, axis.y, -m12 * axis.x);
  }
  return gx > 0.0f && gy >= tlo * gx && gy <= thi * gx;
}
// a * s + b, fused per component
POB_D v3 vfma(v3 a, float s, v3 b) { return V(FMA(a.x, s, b.x), FMA(a.y, s, b.y), FMA(a.z, s, b.z)); }
// x + rotate(v, q) with the translation folded into the rotation's fused chain
POB_D v3 qrot_add(v3 v, q4 q, v3 x) {
  v3 u = V(q.x, q.y, q.z);
  float t2 = 2.0f * vdot(u, v);
  float c = FMA(q.w, q.w, -vdot(u, u));
  float s2 = 2.0f * q.w;
  v3 cr = vcross(u, v);
  return V(FMA(t2, u.x, FMA(c, v.x, FMA(s2, cr.x, x.x))), FMA(t2, u.y, FMA(c, v.y, FMA(s2, cr.y, x.y))),
           FMA(t2, u.z, FMA(c, v.z, FMA(s2, cr.z, x.z))));
}
// Substep quaternion normalisation (spec, oracle qnormalize): with e = |q|^2 - 1 (exact by
// Sterbenz), 1/|q| = 1 - e/2 + 3e^2/8 - 5e^3/16 + O(e^4), truncation error <= 35/128 e^4
// < 2^-27 for |e| <= 2^-6; |e| stays below 2.4e-3 in rollouts (the integration and
// correction steps move a unit q by far less), so the three-FMA polynomial replaces the
// correctly rounded sqrt + reciprocal; outside that range (never in practice) the element
// takes 1 / sqrt(|q|^2) as before, behind a wave-uniform guard.
POB_D q4 qnormalize(q4 q) {
  const float n2 = FMA(q.z, q.z, FMA(q.y, q.y, FMA(q.x, q.x, q.w * q.w)));
  const float e = n2 - 1.0f;
  float inv = FMA(FMA(FMA(-0.3125f, e, 0.375f), e, -0.5f), e, 1.0f);
  const bool far = !(fabsf(e) <= 0x1p-6f);
  if (__builtin_expect(__any(far), 0)) {
    if (far) inv = pob_rcp(pob_sqrt(n2));
  }
  q4 r; r.w = q.w * inv; r.x = q.x * inv; r.y = q.y * inv; r.z = q.z * inv;
  return r;
}
// acc += sign * 0.5 * d, one fused multiply-add per component (sign * 0.5 is exact)
POB_D void qadd_half(q4 &acc, q4 d, float sign) {
  const float h = 0.5f * sign;
  acc.w = FMA(h, d.w, acc.w); acc.x = FMA(h, d.x, acc.x);
  acc.y = FMA(h, d.y, acc.y); acc.z = FMA(h, d.z, acc.z);
}

// atan2f (spec, oracle orc_atan2f): branch-free octant reduction t = min(|x|,|y|) / max(|x|,|y|)
// (correctly rounded reciprocal, then one multiply), atan t = t P(t^2) with a degree-7 minimax
// polynomial on [0, 1] (7.2e-8 relative), then pi/2 - r, pi - r and the sign of y by selects:
// <= 4 ulp against atan2 over the whole plane (no divergent branches, no division).  NaN
// inputs give NaN.
template <class G>
POB_D float pob_atan2f_g(G &g, float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  float t = mn * g.rcp(mx);
  t = mx > 0.0f ? t : 0.0f;
  const float s = t * t;
  float p = FMA(s, -0.0047533135f, 0.024452504f);
  p = FMA(p, s, -0.059750218f);
  p = FMA(p, s, 0.09932368f);
  p = FMA(p, s, -0.14026737f);
  p = FMA(p, s, 0.19971494f);
  p = FMA(p, s, -0.33332205f);
  p = FMA(p, s, 0.99999994f);
  float r = t * p;
  r = ay > ax ? 1.5707964f - r : r;
  r = x < 0.0f ? 3.1415927f - r : r;
  r = __builtin_copysignf(r, y);
  return r + (x * 0.0f + y * 0.0f);  // + 0, or NaN for NaN / infinite inputs
}

// Range-guard policies of the exact fast forms (pob_rcp / pob_sqrt_rcp / qnormalize).
// GuardBranch: each operation checks its operand and takes the exact slow form behind its
// own wave-uniform branch.  GuardAcc: no branches -- every operand's magnitude bits are
// folded into one per-lane register (distance above the range's low end, shifted so the
// sign drops out: out of range <=> above 0xC0000000), and the caller reruns the whole
// computation under GuardBranch when any lane of the wave saw an operand out of range.
// In range both give the same bits (the fast forms are exact there), so a rerun changes
// nothing for the lanes that were in range.  The branches split the latency-bound
// kernels' basic blocks; the accumulator is one or two VALU operations off the chain.
struct GuardBranch {
  POB_D float rcp(float x) { return pob_rcp(x); }
  POB_D float sqrt(float x) { return pob_sqrt(x); }
  POB_D void sqrt_rcp(float x, float &s, float &i) { pob_sqrt_rcp(x, s, i); }
  POB_D q4 qnorm(q4 q) { return qnormalize(q); }
};
struct GuardAcc {
  uint32_t m = 0u;
  POB_D void note(float x) {  // |x| in [2^-96, 2^96] <=> (bits << 1) - bits(2^-96) << 1 <= 0xC0000000
    const uint32_t t = (__float_as_uint(x) << 1) - 0x1F000000u;
    m = m > t ? m : t;
  }
  POB_D bool bad() const { return m > 0xC0000000u; }
  POB_D float rcp(float x) { note(x); return pob_rcp_fast(x); }
  POB_D float sqrt(float x) { note(x); return pob_sqrt_fast(x); }
  POB_D void sqrt_rcp(float x, float &s, float &i) {
    note(x);
    s = pob_sqrt_fast(x);
    i = pob_rcp_fast(s);
  }
  POB_D q4 qnorm(q4 q) {  // qnormalize's polynomial; |e| > 2^-6 (or NaN) maps above 2^96
    const float n2 = FMA(q.z, q.z, FMA(q.y, q.y, FMA(q.x, q.x, q.w * q.w)));
    const float e = n2 - 1.0f;
    const float inv = FMA(FMA(FMA(-0.3125f, e, 0.375f), e, -0.5f), e, 1.0f);
    note(FMA(fabsf(e), 0x1p102f, 1.0f));
    q4 r; r.w = q.w * inv; r.x = q.x * inv; r.y = q.y * inv; r.z = q.z * inv;
    return r;
  }
};
POB_D float pob_atan2f(float y, float x) {
  GuardBranch g;
  return pob_atan2f_g(g, y, x);
}
// Cephes-form sinf/cosf (Cody-Waite reduction by pi/4)
POB_D void pob_sincosf(float x, float *s, float *c) {
  float sgn_s = 1.0f, sgn_c = 1.0f;
  if (x < 0.0f) { x = -x; sgn_s = -1.0f; }
  int j = (int)(1.27323954473516f * x);
  float y = (float)j;
  if (j & 1) { j += 1; y += 1.0f; }
  j &= 7;
  if (j > 3) { sgn_s = -sgn_s; sgn_c = -sgn_c; j -= 4; }
  if (j > 1) sgn_c = -sgn_c;
  float xr = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
  float z = xr * xr;
  float ps = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * xr + xr;
  float pc = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) *
                 z * z - 0.5f * z + 1.0f;
  if (j == 1 || j == 2) { *s = sgn_s * pc; *c = sgn_c * ps; }
  else { *s = sgn_s * ps; *c = sgn_c * pc; }
}

// ------------------------------------------------------------------------- threefry
// jax.random threefry2x32 (20 rounds), pre-partitionable scheme.
POB_D uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

POB_D void threefry2x32(uint32_t k0, uint32_t k1, uint32_t x0, uint32_t x1, uint32_t &y0,
                        uint32_t &y1) {
  const uint32_t k2 = k0 ^ k1 ^ 0x1BD11BDAu;
  uint32_t a = x0 + k0, b = x1 + k1;
#define POB_TF_R(r) a += b; b = rotl32(b, r); b ^= a;
  POB_TF_R(13) POB_TF_R(15) POB_TF_R(26) POB_TF_R(6)
  a += k1; b += k2 + 1u;
  POB_TF_R(17) POB_TF_R(29) POB_TF_R(16) POB_TF_R(24)
  a += k2; b += k0 + 2u;
  POB_TF_R(13) POB_TF_R(15) POB_TF_R(26) POB_TF_R(6)
  a += k0; b += k1 + 3u;
  POB_TF_R(17) POB_TF_R(29) POB_TF_R(16) POB_TF_R(24)
  a += k1; b += k2 + 4u;
  POB_TF_R(13) POB_TF_R(15) POB_TF_R(26) POB_TF_R(6)
  a += k2; b += k0 + 5u;
#undef POB_TF_R
  y0 = a; y1 = b;
}

// element j of threefry_2x32(key, iota(n)) (odd n padded with a zero count)
POB_D uint32_t tf_elem(uint32_t k0, uint32_t k1, uint32_t n, uint32_t j) {
  const uint32_t h = (n + 1u) >> 1;
  uint32_t y0, y1;
  if (j < h) {
    uint32_t x1 = j + h;
    if (x1 >= n) x1 = 0u;
    threefry2x32(k0, k1, j, x1, y0, y1);
    return y0;
  }
  threefry2x32(k0, k1, j - h, j, y0, y1);
  return y1;
}
// row i of split(key, num)
POB_D void tf_split(uint32_t k0, uint32_t k1, uint32_t num, uint32_t i, uint32_t &o0, uint32_t &o1) {
  o0 = tf_elem(k0, k1, 2u * num, 2u * i);
  o1 = tf_elem(k0, k1, 2u * num, 2u * i + 1u);
}
POB_D float bits_to_unit(uint32_t b) { return __uint_as_float((b >> 9) | 0x3F800000u) - 1.0f; }
// jax.random.uniform element: max(lo, f*(hi-lo)+lo)
POB_D float tf_uniform(uint32_t k0, uint32_t k1, uint32_t n, uint32_t i, float lo, float hi) {
  float f = bits_to_unit(tf_elem(k0, k1, n, i));
  float v = f * (hi - lo) + lo;
  return v > lo ? v : lo;
}
