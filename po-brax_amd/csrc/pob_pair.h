// pob_pair.h -- the PBD Ant step with TWO lanes per environment (gfx950).
//
// Why: with one lane per env the physics needs ~450 VGPR+AGPR and 117 LDS floats per lane,
// which pins the kernel to one wave per SIMD, where a wave can issue a VALU op at most
// every 4 cycles (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost').  Splitting each
// env over a lane pair halves the per-lane state, so two waves share each SIMD.
//
// Split: lane half h (0/1) of the pair owns the torso (replicated in both lanes) and the
// two legs of joints 4h..4h+3 (global bodies 4h+1..4h+4).  Local body l in 0..4 maps to
// global body (l == 0 ? 0 : l + 4h); local joint jl in 0..3 to global joint jl + 4h, and the
// local topology (parent(jl) = jl odd ? jl : 0, child = jl + 1) is the same in both lanes.
// Everything a body accumulates is computed by its owner in the oracle's order; the only
// cross-lane sums are the torso's (joint torques and joint corrections from joints
// 0,2 | 4,6), handed over with DPP as a running partial sum: lane 0 sums its joints from
// zero, lane 1 continues from lane 0's partial, and sends the total back -- the exact
// left-to-right float order of oracle/pob_oracle.c, so results stay bit-identical.
// Torso contacts are evaluated redundantly (identically) in both lanes.
#pragma once
#include "pob_physics.h"

// The pair kernel's live set leaves room for the compiler to keep table values in
// registers (measured +5 % over per-use scalar reloads), so its table accesses are NOT
// laundered (cf. launder() in pob_physics.h, which the one-lane kernel needs).
POB_D csys_t *plain_tbl(csys_t *p) { return p; }

#define PNB 5  // local bodies per lane
#define PNJ 4  // local joints per lane

struct HBody {
  v3 x[PNB];
  q4 q[PNB];
  v3 v[PNB];
  v3 w[PNB];
};

// partner lane's value (lane ^ 1) via DPP quad_perm [1,0,3,2].  Inline asm on purpose: the
// update_dpp builtin may be sunk into a lane-masked branch (e.g. `h ? swap(x) : x`), and a
// DPP read from a disabled lane returns 0.  A volatile asm statement is never moved into
// control flow, so it always runs with the pair's full exec mask.  The s_nop covers the
// VALU-write -> DPP-read hazard (hipcc does not insert hazards for asm statements).
POB_D float pair_swap(float x) {
  float r;
  asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
               : "=&v"(r) : "v"(x));
  return r;
}
POB_D v3 pair_swap3(v3 a) { return V(pair_swap(a.x), pair_swap(a.y), pair_swap(a.z)); }
POB_D q4 pair_swap4(q4 a) {
  q4 r; r.w = pair_swap(a.w); r.x = pair_swap(a.x); r.y = pair_swap(a.y); r.z = pair_swap(a.z);
  return r;
}
// lane-half select of two (scalar) table values
POB_D float hsel(bool h, float a, float b) { return h ? b : a; }
#define HSV(h, a, b) V(hsel(h, (a)[0], (b)[0]), hsel(h, (a)[1], (b)[1]), hsel(h, (a)[2], (b)[2]))

POB_D constexpr int lbody_global(int l, int h) { return l == 0 ? 0 : l + 4 * h; }

// Per-lane LDS scratch for the pair kernel (lane-minor): substep-start pose of the 5 local
// bodies (35 floats) and their Info.contact accumulators (30 floats).
#define PL_PX(l) (7 * (l))
#define PL_PQ(l) (7 * (l) + 3)
#define PL_CV(l) (35 + 6 * (l))
#define PL_CA(l) (35 + 6 * (l) + 3)
#define PL_FLOATS 65

struct HContacts {
  // local contacts: [0] torso ground, [1] ground of local body 2, [2] ground of local body 4,
  // [3 + l] deepest wall contact of local capsule l (l = 0..4)
  float pen[3 + PNB];
  v3 n[PNB];
  bool sel[PNB];
};
POB_D constexpr int hcontact_body(int k) { return k == 0 ? 0 : (k == 1 ? 2 : (k == 2 ? 4 : k - 3)); }
// global ground-contact index of local ground contact k: torso 0, body 2/6 -> 1/3, body 4/8 -> 2/4
POB_D int hground_index(int k, bool h) { return k == 0 ? 0 : (k + (h ? 2 : 0)); }

POB_D void hdetect(csys_t *Sp, const HBody &b, HContacts &ct, const bool h) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    csys_t &S = *plain_tbl(Sp);
    const int l = hcontact_body(k);
    const int g0 = k == 0 ? 0 : k, g1 = k == 0 ? 0 : k + 2;
    v3 pe = vadd(b.x[l], qrot(HSV(h, S.ground_end[g0], S.ground_end[g1]), b.q[l]));
    ct.pen[k] = hsel(h, S.ground_r[g0], S.ground_r[g1]) - pe.z;
  }
  uint32_t near_mask = 0u;
  {
    v3 mn = b.x[0], mx = b.x[0];
#pragma unroll
    for (int l = 1; l < PNB; ++l) {
      mn = V(fminf(mn.x, b.x[l].x), fminf(mn.y, b.x[l].y), fminf(mn.z, b.x[l].z));
      mx = V(fmaxf(mx.x, b.x[l].x), fmaxf(mx.y, b.x[l].y), fmaxf(mx.z, b.x[l].z));
    }
    csys_t &S = *plain_tbl(Sp);
    const int nw = S.n_walls;
    for (int w = 0; w < nw; ++w) {
      const bool near = mn.x <= S.wall_hi[w][0] && mx.x >= S.wall_lo[w][0] && mn.y <= S.wall_hi[w][1] &&
                        mx.y >= S.wall_lo[w][1] && mn.z <= S.wall_hi[w][2] && mx.z >= S.wall_lo[w][2];
      if (__any(near)) near_mask |= 1u << w;
    }
  }
#pragma unroll
  for (int l = 0; l < PNB; ++l) {
    POB_FENCE();
    csys_t &S = *plain_tbl(Sp);
    const int nend = (l == 0) ? 1 : 2;
    v3 pe[2];
#pragma unroll
    for (int q = 0; q < nend; ++q)
      pe[q] = vadd(b.x[l], qrot(l == 0 ? SV(S.cap_end[0][0]) : HSV(h, S.cap_end[l][q], S.cap_end[l + 4][q]), b.q[l]));
    float best = 0.0f;
    v3 bn = V(0.0f, 0.0f, 0.0f);
    bool bsel = false;
    const float r = l == 0 ? S.cap_r[0] : hsel(h, S.cap_r[l], S.cap_r[l + 4]);
    const int nw = S.n_walls;
    for (int w = 0; w < nw; ++w) {
      if (!(near_mask & (1u << w))) continue;
#pragma unroll
      for (int q = 0; q < nend; ++q) {
        v3 n;
        float pen = sphere_box(*plain_tbl(Sp), w, pe[q], r, n);
        if (pen > best) { best = pen; bn = n; bsel = q == 1; }
      }
    }
    ct.pen[3 + l] = best;
    ct.n[l] = bn;
    ct.sel[l] = bsel;
  }
}

POB_D void hcontact_geom(csys_t &S, const HContacts &ct, int k, const bool h, v3 &e, v3 &n, float &r) {
  if (k < 3) {
    const int g0 = k == 0 ? 0 : k, g1 = k == 0 ? 0 : k + 2;
    e = HSV(h, S.ground_end[g0], S.ground_end[g1]);
    n = V(0.0f, 0.0f, 1.0f);
    r = hsel(h, S.ground_r[g0], S.ground_r[g1]);
  } else {
    const int l = k - 3;
    v3 e0, e1;
    if (l == 0) { e0 = SV(S.cap_end[0][0]); e1 = SV(S.cap_end[0][1]); r = S.cap_r[0]; }
    else {
      e0 = HSV(h, S.cap_end[l][0], S.cap_end[l + 4][0]);
      e1 = HSV(h, S.cap_end[l][1], S.cap_end[l + 4][1]);
      r = hsel(h, S.cap_r[l], S.cap_r[l + 4]);
    }
    e = ct.sel[l] ? e1 : e0;
    n = ct.n[l];
  }
}

// contact processing order of one body = oracle order (ground contact first, then wall);
// hcontact order [torso ground, b2 ground, b4 ground, walls 0..4] visits each body's
// contacts in that relative order.
POB_D void hcontact_position(csys_t *Sp, const HBody &b, const Lds &L, const HContacts &ct, const bool h,
                             v3 (&DX)[PNB], q4 (&DQ)[PNB]) {
#pragma unroll
  for (int k = 0; k < 3 + PNB; ++k) {
    POB_FENCE();
    const int l = hcontact_body(k);
    const float pen = ct.pen[k];
    if (pen > 0.0f) {
      csys_t &S = *plain_tbl(Sp);
      v3 e, n;
      float rad;
      hcontact_geom(S, ct, k, h, e, n, rad);
      const float im = l == 0 ? S.inv_mass[0] : hsel(h, S.inv_mass[l], S.inv_mass[l + 4]);
      v3 pe = vadd(b.x[l], qrot(e, b.q[l]));
      v3 cp = vsub(pe, vscl(n, rad));
      v3 rr = vsub(cp, b.x[l]);
      v3 cn = vcross(rr, n);
      float w = im + vdot(cn, cn);
      float lam = pen / w;
      v3 P = vscl(n, lam);
      q4 dq = qmul_vq(vcross(rr, P), b.q[l]);
      DX[l] = vadd(DX[l], vscl(P, im));
      DQ[l].w += 0.5f * dq.w; DQ[l].x += 0.5f * dq.x; DQ[l].y += 0.5f * dq.y; DQ[l].z += 0.5f * dq.z;
      v3 cprev = vadd(L.get3(PL_PX(l)), qrot(qrot(rr, qinv(b.q[l])), L.get4(PL_PQ(l))));
      v3 dp = vsub(cp, cprev);
      v3 dpt = vsub(dp, vscl(n, vdot(dp, n)));
      float lt = sqrtf(vdot(dpt, dpt));
      if (lt > 0.0f) {
        v3 t = vdivs(dpt, lt);
        v3 ctn = vcross(rr, t);
        float wt = im + vdot(ctn, ctn);
        float lamt = lt / wt;
        if (lamt < S.friction * lam) {
          v3 Pt = vscl(t, -lamt);
          q4 dqt = qmul_vq(vcross(rr, Pt), b.q[l]);
          DX[l] = vadd(DX[l], vscl(Pt, im));
          DQ[l].w += 0.5f * dqt.w; DQ[l].x += 0.5f * dqt.x; DQ[l].y += 0.5f * dqt.y; DQ[l].z += 0.5f * dqt.z;
        }
      }
    }
  }
}

POB_D void hcontact_velocity(csys_t *Sp, const HBody &b, const HContacts &ct, const bool h, v3 (&dV)[PNB],
                             v3 (&dW)[PNB]) {
#pragma unroll
  for (int k = 0; k < 3 + PNB; ++k) {
    POB_FENCE();
    const int l = hcontact_body(k);
    const float pen = ct.pen[k];
    if (pen > 0.0f) {
      csys_t &S = *plain_tbl(Sp);
      v3 e, n;
      float rad;
      hcontact_geom(S, ct, k, h, e, n, rad);
      const float im = l == 0 ? S.inv_mass[0] : hsel(h, S.inv_mass[l], S.inv_mass[l + 4]);
      v3 pe = vadd(b.x[l], qrot(e, b.q[l]));
      v3 cp = vsub(pe, vscl(n, rad));
      v3 rr = vsub(cp, b.x[l]);
      v3 vr = vadd(b.v[l], vcross(b.w[l], rr));
      float vn = vdot(vr, n);
      v3 vt = vsub(vr, vscl(n, vn));
      float lt = sqrtf(vdot(vt, vt));
      v3 dv = V(0.0f, 0.0f, 0.0f);
      if (lt > 0.0f) {
        float fr = fminf(S.friction * pen * S.inv_h, lt);
        dv = vscl(vt, -(fr / lt));
      }
      if (vn < 0.0f) dv = vadd(dv, vscl(n, -vn));
      float D = sqrtf(vdot(dv, dv));
      if (D > 0.0f) {
        v3 dh = vdivs(dv, D);
        v3 cd = vcross(rr, dh);
        float w = im + vdot(cd, cd);
        v3 P = vdivs(dv, w);
        dV[l] = vadd(dV[l], vscl(P, im));
        dW[l] = vadd(dW[l], vcross(rr, P));
      }
    }
  }
}

// Torso terms of one even local joint (the torso is their parent): the values the oracle
// adds to DX[0] / DQ[0], kept separate so the pair can chain them in global joint order.
struct TorsoTerms {
  v3 dx;        // point constraint: P * imp (zero if the anchors coincide)
  q4 dqp, dqh, dql;  // point, hinge and limit rotation terms (sign * 0.5 * dq)
};
POB_D q4 half_term(q4 d, float sign) {
  q4 r; r.w = sign * (0.5f * d.w); r.x = sign * (0.5f * d.x); r.y = sign * (0.5f * d.y); r.z = sign * (0.5f * d.z);
  return r;
}
POB_D void qacc(q4 &a, q4 t) { a.w += t.w; a.x += t.x; a.y += t.y; a.z += t.z; }

// joint jl's point / hinge / limit corrections, accumulated into DX/DQ (local indices);
// for even jl the parent (torso) terms go to *tt instead
POB_D void hjoint_position(csys_t *Sp, const HBody &b, const int jl, const bool h, v3 (&DX)[PNB], q4 (&DQ)[PNB],
                           TorsoTerms *tt) {
  csys_t &S = *plain_tbl(Sp);
  const int p = jparent(jl), c = jchild(jl);
  const float imp = p == 0 ? S.inv_mass[0] : hsel(h, S.inv_mass[p], S.inv_mass[p + 4]);
  const float imc = hsel(h, S.inv_mass[c], S.inv_mass[c + 4]);
  const bool torso_parent = p == 0;
  v3 rp = qrot(HSV(h, S.off_p[jl], S.off_p[jl + 4]), b.q[p]);
  v3 rc = qrot(HSV(h, S.off_c[jl], S.off_c[jl + 4]), b.q[c]);
  v3 d = vsub(vadd(b.x[c], rc), vadd(b.x[p], rp));
  float L = sqrtf(vdot(d, d));
  if (torso_parent) {
    tt->dx = V(0.0f, 0.0f, 0.0f);
    tt->dqp.w = tt->dqp.x = tt->dqp.y = tt->dqp.z = 0.0f;
  }
  if (L > 0.0f) {
    v3 n = vdivs(d, L);
    v3 cp = vcross(rp, n), cc = vcross(rc, n);
    float wsum = (imp + vdot(cp, cp)) + (imc + vdot(cc, cc));
    float lam = (L / wsum) * S.s_pos;
    v3 P = vscl(n, lam);
    if (torso_parent) {
      tt->dx = vscl(P, imp);
      tt->dqp = half_term(qmul_vq(vcross(rp, P), b.q[p]), 1.0f);
    } else {
      DX[p] = vadd(DX[p], vscl(P, imp));
      qadd_half(DQ[p], qmul_vq(vcross(rp, P), b.q[p]), 1.0f);
    }
    DX[c] = vsub(DX[c], vscl(P, imc));
    qadd_half(DQ[c], qmul_vq(vcross(rc, P), b.q[c]), -1.0f);
  }
  const v3 axis = HSV(h, S.axis[jl], S.axis[jl + 4]);
  v3 ap = qrot(axis, b.q[p]), ac = qrot(axis, b.q[c]);
  v3 Pa = vscl(vcross(ap, ac), S.half_s_ang);
  if (torso_parent) tt->dqh = half_term(qmul_vq(Pa, b.q[p]), 1.0f);
  else qadd_half(DQ[p], qmul_vq(Pa, b.q[p]), 1.0f);
  qadd_half(DQ[c], qmul_vq(Pa, b.q[c]), -1.0f);
  const v3 ref = HSV(h, S.ref[jl], S.ref[jl + 4]);
  v3 fp = qrot(ref, b.q[p]), fc = qrot(ref, b.q[c]);
  float psi = pob_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
  const float lo = hsel(h, S.lim_lo[jl], S.lim_lo[jl + 4]), hi = hsel(h, S.lim_hi[jl], S.lim_hi[jl + 4]);
  float dl = 0.0f;
  if (psi < lo) dl = psi - lo;
  else if (psi > hi) dl = psi - hi;
  v3 Pl = vscl(ap, dl * S.half_s_ang);
  if (torso_parent) tt->dql = half_term(qmul_vq(Pl, b.q[p]), 1.0f);
  else qadd_half(DQ[p], qmul_vq(Pl, b.q[p]), 1.0f);
  qadd_half(DQ[c], qmul_vq(Pl, b.q[c]), -1.0f);
}

// add the two even joints' torso terms onto (dx, dq) in the oracle's order
POB_D void torso_chain(v3 &dx, q4 &dq, const TorsoTerms (&tt)[2]) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    dx = vadd(dx, tt[k].dx);
    qacc(dq, tt[k].dqp);
    qacc(dq, tt[k].dqh);
    qacc(dq, tt[k].dql);
  }
}

// One XPBD substep on a lane pair (see the header comment for the split).
POB_D void hpbd_substep(csys_t *Sp, HBody &b, const float (&act)[PNJ], const Lds &L, const bool h,
                        const bool COLLIDE) {
#pragma unroll
  for (int l = 0; l < PNB; ++l) { L.set3(PL_PX(l), b.x[l]); L.set4(PL_PQ(l), b.q[l]); }
  // 1. acceleration level.  Torso: dw0 = (((0 - t0) - t2) - t4) - t6 across the pair.
  {
    v3 tt[PNJ];
#pragma unroll
    for (int jl = 0; jl < PNJ; ++jl) {
      csys_t &S = *plain_tbl(Sp);
      const int p = jparent(jl), c = jchild(jl);
      v3 a = qrot(HSV(h, S.axis[jl], S.axis[jl + 4]), b.q[p]);
      v3 t = vscl(a, act[jl] * hsel(h, S.strength[jl], S.strength[jl + 4]));
      v3 d = vscl(vsub(b.w[p], b.w[c]), hsel(h, S.jdamp[jl], S.jdamp[jl + 4]));
      tt[jl] = vadd(t, d);
    }
    v3 dw[PNB];
    {
      v3 zero = V(0.0f, 0.0f, 0.0f);
      v3 part = vsub(vsub(zero, tt[0]), tt[2]);      // lane 0: first half of the sum
      v3 from0 = pair_swap3(part);                   // lane 1 receives lane 0's partial
      v3 full = vsub(vsub(from0, tt[0]), tt[2]);     // lane 1: continue with joints 4, 6
      v3 from1 = pair_swap3(full);                   // lane 0 receives the total
      dw[0] = h ? full : from1;
    }
    dw[1] = vsub(vadd(V(0.0f, 0.0f, 0.0f), tt[0]), tt[1]);
    dw[2] = vadd(V(0.0f, 0.0f, 0.0f), tt[1]);
    dw[3] = vsub(vadd(V(0.0f, 0.0f, 0.0f), tt[2]), tt[3]);
    dw[4] = vadd(V(0.0f, 0.0f, 0.0f), tt[3]);
    csys_t &S = *plain_tbl(Sp);
#pragma unroll
    for (int l = 0; l < PNB; ++l) {
      const v3 v = b.v[l], w = b.w[l];
      b.v[l] = V(S.lin_damp * v.x + 0.0f * S.h, S.lin_damp * v.y + 0.0f * S.h, S.lin_damp * v.z + S.gz * S.h);
      b.w[l] = V(S.ang_damp * w.x + dw[l].x * S.h, S.ang_damp * w.y + dw[l].y * S.h,
                 S.ang_damp * w.z + dw[l].z * S.h);
    }
    // 2. kinetic
#pragma unroll
    for (int l = 0; l < PNB; ++l) {
      b.x[l] = vadd(b.x[l], vscl(b.v[l], S.h));
      q4 dq = qmul_vq(b.w[l], b.q[l]);
      q4 q = b.q[l];
      q.w = q.w + S.half_h * dq.w; q.x = q.x + S.half_h * dq.x;
      q.y = q.y + S.half_h * dq.y; q.z = q.z + S.half_h * dq.z;
      b.q[l] = qnormalize(q);
    }
  }
  // 3. position projection
  HContacts ct;
  {
    v3 DX[PNB];
    q4 DQ[PNB];
#pragma unroll
    for (int l = 0; l < PNB; ++l) { DX[l] = V(0.0f, 0.0f, 0.0f); DQ[l].w = DQ[l].x = DQ[l].y = DQ[l].z = 0.0f; }
    // local joints in order; the torso terms of the even joints are chained across the
    // pair: lane 0 sums global joints 0, 2 from zero, lane 1 continues with 4, 6
    TorsoTerms tt[2];
    POB_FENCE();
    hjoint_position(Sp, b, 0, h, DX, DQ, &tt[0]);
    POB_FENCE();
    hjoint_position(Sp, b, 1, h, DX, DQ, nullptr);
    POB_FENCE();
    hjoint_position(Sp, b, 2, h, DX, DQ, &tt[1]);
    POB_FENCE();
    hjoint_position(Sp, b, 3, h, DX, DQ, nullptr);
    POB_FENCE();
    {
      v3 dx = V(0.0f, 0.0f, 0.0f);
      q4 dq; dq.w = dq.x = dq.y = dq.z = 0.0f;
      torso_chain(dx, dq, tt);                 // lane 0: partial over joints 0, 2
      v3 dx1 = pair_swap3(dx);                 // lane 1 receives lane 0's partial
      q4 dq1 = pair_swap4(dq);
      torso_chain(dx1, dq1, tt);               // lane 1: continue with joints 4, 6
      v3 dxf = pair_swap3(dx1);                // lane 0 receives the total
      q4 dqf = pair_swap4(dq1);
      DX[0] = h ? dx1 : dxf;
      DQ[0] = h ? dq1 : dqf;
    }
    if (COLLIDE) {
      hdetect(Sp, b, ct, h);
      hcontact_position(Sp, b, L, ct, h, DX, DQ);
    }
#pragma unroll
    for (int l = 0; l < PNB; ++l) {
      b.x[l] = vadd(b.x[l], DX[l]);
      b.q[l].w += DQ[l].w; b.q[l].x += DQ[l].x; b.q[l].y += DQ[l].y; b.q[l].z += DQ[l].z;
    }
  }
  // 4. velocity projection
  {
    csys_t &S = *plain_tbl(Sp);
#pragma unroll
    for (int l = 0; l < PNB; ++l) {
      b.q[l] = qnormalize(b.q[l]);
      b.v[l] = vscl(vsub(b.x[l], L.get3(PL_PX(l))), S.inv_h);
      q4 dq = qmul(b.q[l], qinv(L.get4(PL_PQ(l))));
      float sg = dq.w >= 0.0f ? 1.0f : -1.0f;
      b.w[l] = V(sg * ((2.0f * dq.x) * S.inv_h), sg * ((2.0f * dq.y) * S.inv_h), sg * ((2.0f * dq.z) * S.inv_h));
    }
  }
  // 5. velocity-level contacts
  if (COLLIDE) {
    v3 dV[PNB], dW[PNB];
#pragma unroll
    for (int l = 0; l < PNB; ++l) { dV[l] = V(0.0f, 0.0f, 0.0f); dW[l] = V(0.0f, 0.0f, 0.0f); }
    hcontact_velocity(Sp, b, ct, h, dV, dW);
#pragma unroll
    for (int l = 0; l < PNB; ++l) {
      b.v[l] = vadd(b.v[l], dV[l]); b.w[l] = vadd(b.w[l], dW[l]);
      L.set3(PL_CV(l), vadd(L.get3(PL_CV(l)), dV[l]));
      L.set3(PL_CA(l), vadd(L.get3(PL_CA(l)), dW[l]));
    }
  }
}
