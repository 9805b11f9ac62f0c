// pob_physics.h -- shared physics pieces of the rollout kernels (gfx950): the system-table
// access helpers, the per-lane LDS view and one contact's position / velocity / legacy
// impulse response (the contacts themselves: ground in each kernel, walls pob_mesh.h).
//
// Algorithm = brax v1 System.step with dynamics_mode "pbd" as restated in DESIGN.md §3
// (brax is not vendored: reference call sites ant_heavenhell.py:108, ant_gather.py:127,
// ant_tag.py:109).  Op order matches oracle/pob_oracle.c expression for expression.
#pragma once
#include "pob_math.h"
#include "pob_sys.h"
#include "pob_mesh.h"

struct Body {
  v3 x[POB_NDYN];
  q4 q[POB_NDYN];
  v3 v[POB_NDYN];
  v3 w[POB_NDYN];
};

// launder(): with POB_LAUNDER the table pointer is hidden from loop-invariant code motion
// (each table value's scalar load stays next to its use).  Round 1 needed it against SGPR
// spills; with the scheduling fences and the current kernels the compiler's own placement
// measured 0.7-0.9 % faster at B = 65 536 (HH, TAG, ant; no new scratch), so it is off.
typedef __attribute__((address_space(4))) const pob_sys csys_t;  // constant address space
POB_D csys_t *launder(csys_t *p) {
#ifdef POB_LAUNDER
  asm volatile("" : "+s"(p));
#endif
  return p;
}
// the walls' face constants (pob_sys::face_c, pob_mesh.h MFace)
POB_D fcptr_t pob_face_table(csys_t &S) { return (fcptr_t)&S.face_c[0][0][0]; }
// Scheduling fence between the independent joint / contact blocks: without it the machine
// scheduler interleaves all of them for ILP and the live set blows past 512 registers.
#ifdef POB_NO_FENCE
#define POB_FENCE() ((void)0)
#else
#define POB_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif

// Per-lane LDS scratch, lane-minor (element e of lane t at base[e * BS + t]): conflict-free
// ds_read/ds_write_b32.  Holds what the substep keeps live but rarely touches (the
// substep-start pose and the Info.contact accumulators, pob_quad.h).
struct Lds {
  float *base;
  int stride, t;
  POB_D float get(int e) const { return base[e * stride + t]; }
  POB_D void set(int e, float v) const { base[e * stride + t] = v; }
  POB_D v3 get3(int e) const { return V(get(e), get(e + 1), get(e + 2)); }
  POB_D v3 get3_lane(int e, int lane) const {  // another lane's slot (same wave)
    return V(base[e * stride + lane], base[(e + 1) * stride + lane], base[(e + 2) * stride + lane]);
  }
  POB_D void set3(int e, v3 v) const { set(e, v.x); set(e + 1, v.y); set(e + 2, v.z); }
  POB_D q4 get4(int e) const { q4 q; q.w = get(e); q.x = get(e + 1); q.y = get(e + 2); q.z = get(e + 3); return q; }
  POB_D void set4(int e, q4 q) const { set(e, q.w); set(e + 1, q.x); set(e + 2, q.y); set(e + 3, q.z); }
};

POB_D constexpr int jparent(int j) { return (j & 1) ? j : 0; }
POB_D constexpr int jchild(int j) { return j + 1; }
POB_D constexpr int ground_body(int g) { return 2 * g; }
POB_D constexpr int contact_body(int k) { return k < POB_NGROUND ? 2 * k : k - POB_NGROUND; }

#define SV(a) V((a)[0], (a)[1], (a)[2])

// ------------------------------------------------------------------ contact responses
// One contact's position-level projection (normal + static friction) and velocity-level solve
// (dynamic friction + inelastic normal) on its body (oracle contact_position /
// contact_velocity, shared by every kernel).  pe = the contact's sphere centre (the capsule
// point x + rotate(end, q), or x + tau rotate(e0, q) for a wall contact), n the world normal.
// (the contact functions' view of the table: S.friction and S.inv_h)
struct HCon {
  float friction, inv_h;
};
// position-level ground contact (n = +z: the general form with the products by the normal's
// exact zeros dropped, same values up to the sign of a zero)
template <class G = GuardBranch, class SS = HCon>
POB_D void oground_position(G &g, const SS &S, const float pen, const v3 pe, const float rad, const float im, const v3 x,
                            const q4 q, const q4 pq, const v3 px, v3 &DX, v3 &DA) {
  const v3 cp = V(pe.x, pe.y, pe.z - rad);
  const v3 rr = vsub(cp, x);
  const float w = im + FMA(rr.x, rr.x, rr.y * rr.y);  // |rr x n|^2
  const float lam = (pen * g.rcp(w));
  DX.z = FMA(lam, im, DX.z);  // P = (0, 0, lam)
  DA = V(DA.x + rr.y * lam, DA.y + -(rr.x * lam), DA.z);  // rr x P
  const v3 cprev = qrot_add(qrot(rr, qinv(q)), pq, px);
  const float dpx = cp.x - cprev.x, dpy = cp.y - cprev.y;  // tangential part of cp - cprev
  float lt, inv;
  g.sqrt_rcp(FMA(dpy, dpy, dpx * dpx), lt, inv);
  if (lt > 0.0f) {
    const float tx = dpx * inv, ty = dpy * inv;
    const v3 ctn = V(-(rr.z * ty), rr.z * tx, FMA(rr.x, ty, -(rr.y * tx)));  // rr x t
    const float wt = im + vdot(ctn, ctn);
    const float lamt = (lt * g.rcp(wt));
    if (lamt < S.friction * lam) {
      const float px_ = tx * -lamt, py_ = ty * -lamt;
      DX.x = FMA(px_, im, DX.x);
      DX.y = FMA(py_, im, DX.y);
      DA = vadd(DA, V(-(rr.z * py_), rr.z * px_, FMA(rr.x, py_, -(rr.y * px_))));  // rr x Pt
    }
  }
}

// position-level wall contact (the general form)
template <class G = GuardBranch, class SS = HCon>
POB_D void owall_position(G &g, const SS &S, const float pen, const v3 pe, const v3 n, const float rad, const float im,
                          const v3 x, const q4 q, const q4 pq, const v3 px, v3 &DX, v3 &DA) {
  v3 cp = vfma(n, -rad, pe);
  v3 rr = vsub(cp, x);
  v3 cn = vcross(rr, n);
  float w = im + vdot(cn, cn);
  float lam = (pen * g.rcp(w));
  v3 P = vscl(n, lam);
  DX = vfma(P, im, DX);
  DA = vadd(DA, vcross(rr, P));
  v3 cprev = qrot_add(qrot(rr, qinv(q)), pq, px);
  v3 dp = vsub(cp, cprev);
  v3 dpt = vfma(n, -vdot(dp, n), dp);
  float lt, ilt;
  g.sqrt_rcp(vdot(dpt, dpt), lt, ilt);
  if (lt > 0.0f) {
    v3 t = vscl(dpt, ilt);
    v3 ctn = vcross(rr, t);
    float wt = im + vdot(ctn, ctn);
    float lamt = (lt * g.rcp(wt));
    if (lamt < S.friction * lam) {
      v3 Pt = vscl(t, -lamt);
      DX = vfma(Pt, im, DX);
      DA = vadd(DA, vcross(rr, Pt));
    }
  }
}

// velocity-level contact at the contact point pe (ground: n = +z with the zero products dropped)
template <class G = GuardBranch, class SS = HCon>
POB_D void ocontact_vel_pe(G &g, const SS &S, const bool ground, const float pen, const v3 pe, const v3 n,
                           const float rad, const float im, const v3 x, const v3 v, const v3 w, v3 &dV, v3 &dW) {
  v3 cp = vfma(n, -rad, pe);
  v3 rr = vsub(cp, x);
  v3 vr = vadd(v, vcross(w, rr));
  v3 dv = V(0.0f, 0.0f, 0.0f);
  if (ground) {
    const float vn = vr.z;
    float lt, ilt;
    g.sqrt_rcp(FMA(vr.y, vr.y, vr.x * vr.x), lt, ilt);
    if (lt > 0.0f) {
      const float fr = fminf(S.friction * pen * S.inv_h, lt);
      const float k = -(fr * ilt);
      dv = V(vr.x * k, vr.y * k, 0.0f);
    }
    if (vn < 0.0f) dv.z = -vn;
  } else {
    float vn = vdot(vr, n);
    v3 vt = vfma(n, -vn, vr);
    float lt, ilt;
    g.sqrt_rcp(vdot(vt, vt), lt, ilt);
    if (lt > 0.0f) {
      float fr = fminf(S.friction * pen * S.inv_h, lt);
      dv = vscl(vt, -(fr * ilt));
    }
    if (vn < 0.0f) dv = vfma(n, -vn, dv);
  }
  float D, iD;
  g.sqrt_rcp(vdot(dv, dv), D, iD);
  if (D > 0.0f) {
    v3 dh = vscl(dv, iD);
    v3 cd = vcross(rr, dh);
    float wgt = im + vdot(cd, cd);
    v3 P = vscl(dv, g.rcp(wgt));
    dV = vfma(P, im, dV);
    dW = vadd(dW, vcross(rr, P));
  }
}
// the same with the body-frame end point e (pe = x + rotate(e, q), e in the body xy-plane)
template <class G = GuardBranch, class SS = HCon>
POB_D void ocontact_vel_one(G &g, const SS &S, const bool ground, const float pen, const v3 e, const v3 n, const float rad,
                            const float im, const v3 x, const q4 q, const v3 v, const v3 w, v3 &dV, v3 &dW) {
  ocontact_vel_pe(g, S, ground, pen, vadd(x, qrot_xy(e, q)), n, rad, im, x, v, w, dV, dW);
}

// One-way contact impulse of brax <= 0.0.12 (oracle legacy_contacts: Baumgarte-stabilised
// inelastic normal impulse, Coulomb drag capped by friction * impulse; applied when
// penetrating, approaching and positive) at the contact point pe
template <class SS>
POB_D void olegacy_contact(const SS &S, const float pen, const v3 pe, const v3 n, const float rad, const float im,
                           const v3 x, const v3 v, const v3 w, v3 &dV, v3 &dW) {
  const v3 rel = vsub(vfma(n, -rad, pe), x);
  const v3 cv = vadd(v, vcross(w, rel));
  const float nv = vdot(n, cv);
  const float ang = vdot(n, vcross(vcross(rel, n), rel));
  const float rden = pob_rcp(im + ang);
  const float imp = (S.erp * pen - nv) * rden;
  if (nv < 0.0f && imp > 0.0f) {
    const v3 vd = vfma(n, -nv, cv);
    const float nd = pob_sqrt(vdot(vd, vd));
    v3 P = vscl(n, imp);
    if (nd > 0.01f) {
      const float impd = fminf(nd * rden, S.friction * imp);
      P = vfma(vd, -(impd * pob_rcp(1e-6f + nd)), P);
    }
    dV = vfma(P, im, dV);
    dW = vadd(dW, vcross(rel, P));
  }
}
