// pob_quad.h -- the PBD Ant step with FOUR lanes per environment (gfx950).
//
// Why: the two-lane kernel (pob_pair.h) runs 2 waves per SIMD and its VALU pipe is busy
// about a third of the time -- the rest is dependency and memory latency that two waves
// cannot cover (profiles/r1g_summary.md).  One leg per lane cuts the per-lane state to
// three bodies (VGPRs and 39 LDS floats per lane), so four waves share each SIMD, and it
// shortens every wave's instruction stream, which is what bounds small batches.
//
// Split: lane k (0..3) of an env's lane quad owns the torso (replicated in all four
// lanes) and leg k: local body 0 = torso, 1 = Aux k+1 (global 2k+1), 2 = lower leg
// (global 2k+2); local joint 0 = global 2k (torso -> aux), 1 = global 2k+1 (aux -> leg).
// Leg tables come from an LDS copy of pob_sys::leg (one row per leg); the scalar table
// (torso and global constants) is laundered per stage (pob_physics.h).
// Every body's accumulations run in its owner lane in the oracle's order.  The torso's
// cross-leg sums (actuator + damping torques of joints 0,2,4,6; the position corrections
// those joints apply to the torso) are gathered with DPP quad broadcasts, and every lane
// adds the four legs' terms in global joint order -- the exact left-to-right float order of
// oracle/pob_oracle.c, so the four torso replicas stay bit-identical to the oracle's.
#pragma once
#include "pob_physics.h"

#define QNB 3  // local bodies per lane
#define QNJ 2  // local joints per lane

struct QBody {
  v3 x[QNB];
  q4 q[QNB];
  v3 v[QNB];
  v3 w[QNB];
};

// value of quad lane J broadcast to the lane's quad (DPP quad_perm [J,J,J,J]).  Inline asm
// so that it is never sunk into lane-masked control flow (a DPP read of a disabled lane
// returns 0); the s_nop covers the VALU-write -> DPP-read hazard.
template <int J>
POB_D float quad_bcast(float x) {
  float r;
  if (J == 0)
    asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf" : "=&v"(r) : "v"(x));
  else if (J == 1)
    asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf" : "=&v"(r) : "v"(x));
  else if (J == 2)
    asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf" : "=&v"(r) : "v"(x));
  else
    asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf" : "=&v"(r) : "v"(x));
  return r;
}
// The same broadcast through the DPP builtin, for values consumed unconditionally in
// straight-line code (the torso sums): the compiler then places the hazard wait states
// and schedules the moves, instead of one s_nop per asm statement.
template <int J>
POB_D float quad_bcast_b(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), J * 0x55, 0xf, 0xf, true));
}
template <int J> POB_D v3 quad_bcast3(v3 a) { return V(quad_bcast_b<J>(a.x), quad_bcast_b<J>(a.y), quad_bcast_b<J>(a.z)); }

// Leg tables: each block stages pob_sys::leg (4 legs x POB_LEG_FLOATS) in LDS, and a lane
// reads its own leg's row through LT = leg table + k * POB_LEG_FLOATS (ds_read_b32; the
// four rows sit in distinct banks).  Selecting among four scalar table values per lane
// instead costs either four vector loads or a divergent branch per value (measured).
#define QJV(LT, jl, f) V((LT)[POB_LEG_JOINT(jl) + (f)], (LT)[POB_LEG_JOINT(jl) + (f) + 1], (LT)[POB_LEG_JOINT(jl) + (f) + 2])
#define QJ_OFFP 0
#define QJ_OFFC 3
#define QJ_AXIS 6
#define QJ_TLO 9   // tan(lim_lo), tan(lim_hi): the actuator gate
#define QJ_THI 10
#define QJ_LO 12
#define QJ_HI 13
#define QJ_DAMP 14
#define QJ_STRENGTH 15
#define QJS(LT, jl, f) ((LT)[POB_LEG_JOINT(jl) + (f)])
POB_D float q_inv_mass(csys_t &S, const float *LT, int l) { return l == 0 ? S.inv_mass[0] : LT[POB_LEG_BODY(l)]; }
POB_D float q_cap_r(csys_t &S, const float *LT, int l) { return l == 0 ? S.cap_r[0] : LT[POB_LEG_BODY(l) + 1]; }

POB_D constexpr int qbody_global(int l, int k) { return l == 0 ? 0 : l + 2 * k; }

// Per-lane LDS scratch (lane-minor): substep-start pose of the 3 local bodies (21 floats)
// and their Info.contact accumulators (18 floats).
#define QL_PX(l) (7 * (l))
#define QL_PQ(l) (7 * (l) + 3)
#define QL_CV(l) (21 + 6 * (l))
#define QL_CA(l) (21 + 6 * (l) + 3)
#define QL_FLOATS 39

struct QContacts {
  // [0] torso ground, [1] lower-leg ground, [2 + l] deepest wall contact of local capsule l
  float pen[2 + QNB];
  v3 n[QNB];
  bool sel[QNB];
  v3 pe[2 + QNB];  // the contact's sphere centre in world (x + rotate(e, q)), reused by the position pass
};
POB_D constexpr int qcontact_body(int c) { return c == 0 ? 0 : (c == 1 ? 2 : c - 2); }

// capsule end point q of local body l (torso: the sphere centre)
POB_D v3 qcap_end(csys_t &S, const float *LT, int l, int q) {
  if (l == 0) return SV(S.cap_end[0][q]);
  const float *e = LT + POB_LEG_BODY(l) + 2 + 3 * q;
  return V(e[0], e[1], e[2]);
}
// ground contact c (0 torso, 1 lower leg k = ground collider k + 1)
POB_D v3 qground_end(csys_t &S, const float *LT, int c) {
  if (c == 0) return SV(S.ground_end[0]);
  return V(LT[POB_LEG_GROUND], LT[POB_LEG_GROUND + 1], LT[POB_LEG_GROUND + 2]);
}
POB_D float qground_r(csys_t &S, const float *LT, int c) {
  return c == 0 ? S.ground_r[0] : LT[POB_LEG_GROUND + 3];
}

// sphere_box (pob_physics.h) of end point p against the wall row R staged in LDS
// (centre x, y, cos, sin, half-extent x, y; z from the system), folded into the deepest-
// contact search: same operations in the same order, but the square root, normal and
// compare run only when d2 < T = r^2 (1 + 2^-20) (or d2 is NaN).  Exact: d2 >= T gives
// sqrt_rn(d2) >= r, so pen = r - dist <= 0 never beats best (>= 0, strict ">").
// (the row's six floats given as values: LDS rows for a per-lane wall walk, the system
// table's scalars for a wave-uniform one)
// (wall_hz / wall_cz given as values: the eight- and sixteen-lane kernels keep them in registers)
template <class G = GuardBranch>
POB_D void qwall_end_vz(G &g, const float wall_hz, const float wall_cz, const float cx, const float cy, const float c,
                        const float s, const float hx, const float hy, v3 p, float r, float T, bool on, bool q1,
                        float &best, v3 &bn, bool &bsel, v3 &bpe) {
  const v3 h = V(hx, hy, wall_hz);
  v3 d = vsub(p, V(cx, cy, wall_cz));
  float lx = FMA(d.y, s, d.x * c), ly = FMA(d.y, c, -(d.x * s)), lz = d.z;
  float qx = clamp_sym(lx, h.x), qy = clamp_sym(ly, h.y), qz = clamp_sym(lz, h.z);
  float ex = lx - qx, ey = ly - qy, ez = lz - qz;
  float d2 = FMA(ez, ez, FMA(ey, ey, ex * ex));
  if (!(d2 >= T)) {
    float pen, nx, ny, nz;
    if (d2 > 0.0f) {
      float dist, inv;
      g.sqrt_rcp(d2, dist, inv);
      pen = r - dist; nx = ex * inv; ny = ey * inv; nz = ez * inv;
    } else {
      float fx = h.x - fabsf(lx), fy = h.y - fabsf(ly), fz = h.z - fabsf(lz);
      nx = 0.0f; ny = 0.0f; nz = 0.0f;
      if (fx <= fy && fx <= fz) { pen = r + fx; nx = lx < 0.0f ? -1.0f : 1.0f; }
      else if (fy <= fz) { pen = r + fy; ny = ly < 0.0f ? -1.0f : 1.0f; }
      else { pen = r + fz; nz = lz < 0.0f ? -1.0f : 1.0f; }
    }
    if (on && pen > best) {
      best = pen;
      bn = V(FMA(-ny, s, nx * c), FMA(ny, c, nx * s), nz);
      bsel = q1;
      bpe = p;
    }
  }
}
template <class G = GuardBranch>
POB_D void qwall_end_v(G &g, csys_t &S, const float cx, const float cy, const float c, const float s, const float hx,
                       const float hy, v3 p, float r, float T, bool on, bool q1, float &best, v3 &bn, bool &bsel,
                       v3 &bpe) {
  qwall_end_vz(g, S.wall_hz, S.wall_cz, cx, cy, c, s, hx, hy, p, r, T, on, q1, best, bn, bsel, bpe);
}
POB_D void qwall_end(csys_t &S, const float *R, v3 p, float r, float T, bool on, bool q1, float &best, v3 &bn,
                     bool &bsel, v3 &bpe) {
  const float2 r01 = *reinterpret_cast<const float2 *>(R);
  const float2 r23 = *reinterpret_cast<const float2 *>(R + 2);
  const float2 r45 = *reinterpret_cast<const float2 *>(R + 4);
  GuardBranch g;
  qwall_end_v(g, S, r01.x, r01.y, r23.x, r23.y, r45.x, r45.y, p, r, T, on, q1, best, bn, bsel, bpe);
}

// Contact detection of a collide substep on a lane quad.  Walls: every lane keeps a mask
// of the walls whose grown box (pob_sys::wall_lo/hi) meets the AABB of its three body
// centres, and walks ITS OWN mask in increasing wall order, so one pass over a wall row
// serves lanes near different walls (a wave-uniform wall loop would run every wall any of
// the 16 envs is near).  Culled pairs have penetration < 0 and the walk keeps the oracle's
// (wall, end) order with the strict ">" -- the deepest contact is unchanged.
// WALLS = false compiles the wall search out (the stock ant has no walls).
// Contact points are x + rotate(e, q) (oracle cpoint).  The Ant's capsules (checked by
// pob_system.cpp) have opposite end points +-e0 in the body xy-plane, so one rotation
// rv = rotate(e0, q) serves both (rotate(-e0) = -rv exactly), and a lower leg's ground point
// is its end 1 (x - rv).  The torso sphere's points are its centre x (rotate(0) = 0).
template <bool WALLS>
POB_D void qdetect(csys_t *Sp, const float *LT, const float *WT, const QBody &b, QContacts &ct) {
  v3 rv_leg;
  {
    csys_t &S = *launder(Sp);
    rv_leg = qrot_xy(qcap_end(S, LT, 2, 0), b.q[2]);
    const v3 pe0 = S.torso_point ? b.x[0] : vadd(b.x[0], qrot(qground_end(S, LT, 0), b.q[0]));
    const v3 pe1 = vsub(b.x[2], rv_leg);
    ct.pen[0] = qground_r(S, LT, 0) - pe0.z;
    ct.pen[1] = qground_r(S, LT, 1) - pe1.z;
    ct.pe[0] = pe0;
    ct.pe[1] = pe1;
  }
  uint32_t lane_mask = 0u;
  if (WALLS) {
    float mnx = b.x[0].x, mxx = b.x[0].x, mny = b.x[0].y, mxy = b.x[0].y;
#pragma unroll
    for (int l = 1; l < QNB; ++l) {
      mnx = fminf(mnx, b.x[l].x); mxx = fmaxf(mxx, b.x[l].x);
      mny = fminf(mny, b.x[l].y); mxy = fmaxf(mxy, b.x[l].y);
    }
    csys_t &S = *launder(Sp);
#ifdef POB_EXP_NO_WALLS
    const int nw = 0;  // timing experiment only
#else
    const int nw = S.n_walls;
#endif
#pragma unroll
    for (int w = 0; w < POB_MAXW; ++w) {
      // xy only: dropping the z test can only keep more walls (the cull stays exact)
      // all POB_MAXW boxes loaded at once, w < nw as a predicate (a runtime loop waited
      // one scalar-load round trip per wall)
      const float lx = S.wall_lo[w][0], ly = S.wall_lo[w][1], hx = S.wall_hi[w][0], hy = S.wall_hi[w][1];
      const bool near = (mnx <= hx) & (mxx >= lx) & (mny <= hy) & (mxy >= ly);
      lane_mask |= (near & (w < nw)) ? 1u << w : 0u;
    }
  }
  const bool any_near = WALLS && __any(lane_mask != 0u);
#pragma unroll
  for (int l = 0; l < QNB; ++l) {
    POB_FENCE();
    csys_t &S = *launder(Sp);
    const int nend = (l == 0) ? 1 : 2;
    float best = 0.0f;
    v3 bn = V(0.0f, 0.0f, 0.0f);
    bool bsel = false;
    v3 bpe = bn;
    if (any_near) {
      v3 pe[2];
      if (l == 0) {
        pe[0] = S.torso_point ? b.x[0] : vadd(b.x[0], qrot(qcap_end(S, LT, 0, 0), b.q[0]));
      } else {
        const v3 rv = l == 2 ? rv_leg : qrot_xy(qcap_end(S, LT, 1, 0), b.q[1]);
        pe[0] = vadd(b.x[l], rv);
        pe[1] = vsub(b.x[l], rv);
      }
      const float r = q_cap_r(S, LT, l);
      const float T = (r * r) * 1.00000095367431640625f;  // r^2 (1 + 2^-20), rounded products
      uint32_t m = lane_mask;
      while (__any(m != 0u)) {
        const bool on = m != 0u;
        const int w = on ? __builtin_ctz(m) : 0;
        m &= m - 1u;
#pragma unroll
        for (int q = 0; q < nend; ++q) qwall_end(S, WT + POB_WALL_FLOATS * w, pe[q], r, T, on, q == 1, best, bn, bsel, bpe);
      }
    }
    ct.pen[2 + l] = best;
    ct.n[l] = bn;
    ct.sel[l] = bsel;
    ct.pe[2 + l] = bpe;
  }
}

POB_D void qcontact_geom(csys_t &S, const float *LT, const QContacts &ct, int c, v3 &e, v3 &n, float &r) {
  if (c < 2) {
    e = qground_end(S, LT, c);
    n = V(0.0f, 0.0f, 1.0f);
    r = qground_r(S, LT, c);
  } else {
    const int l = c - 2;
    e = ct.sel[l] ? qcap_end(S, LT, l, 1) : qcap_end(S, LT, l, 0);
    r = q_cap_r(S, LT, l);
    n = ct.n[l];
  }
}

// contact processing order of one body = oracle order (ground contact first, then wall)
POB_D void qcontact_position(csys_t *Sp, const float *LT, const QBody &b, const Lds &L, const QContacts &ct,
                             v3 (&DX)[QNB], v3 (&DA)[QNB], const float fric) {
#pragma unroll
  for (int c = 0; c < 2 + QNB; ++c) {
    POB_FENCE();
    const int l = qcontact_body(c);
    const float pen = ct.pen[c];
    if (pen > 0.0f) {
      csys_t &S = *launder(Sp);
      v3 e, n;
      float rad;
      qcontact_geom(S, LT, ct, c, e, n, rad);
      const float im = q_inv_mass(S, LT, l);
      const v3 pe = ct.pe[c];  // = x + rotate(e, q) of the detection (same q, x)
      if (c < 2) {
        // ground contact, n = (0, 0, 1): the expressions below with the products by the
        // normal's exact zeros dropped (same values up to the sign of a zero)
        const v3 cp = V(pe.x, pe.y, pe.z - rad);
        const v3 rr = vsub(cp, b.x[l]);
        const float w = im + FMA(rr.x, rr.x, rr.y * rr.y);  // |rr x n|^2
        const float lam = POB_DIV(pen, w);
        DX[l].z = FMA(lam, im, DX[l].z);  // P = (0, 0, lam)
        DA[l] = V(DA[l].x + rr.y * lam, DA[l].y + -(rr.x * lam), DA[l].z);  // rr x P
        const v3 cprev = qrot_add(qrot(rr, qinv(b.q[l])), L.get4(QL_PQ(l)), L.get3(QL_PX(l)));
        const float dpx = cp.x - cprev.x, dpy = cp.y - cprev.y;  // tangential part of cp - cprev
        float lt, inv;
        pob_sqrt_rcp(FMA(dpy, dpy, dpx * dpx), lt, inv);
        if (lt > 0.0f) {
          const float tx = dpx * inv, ty = dpy * inv;
          const v3 ctn = V(-(rr.z * ty), rr.z * tx, FMA(rr.x, ty, -(rr.y * tx)));  // rr x t
          const float wt = im + vdot(ctn, ctn);
          const float lamt = POB_DIV(lt, wt);
          if (lamt < fric * lam) {
            const float px = tx * -lamt, py = ty * -lamt;
            DX[l].x = FMA(px, im, DX[l].x);
            DX[l].y = FMA(py, im, DX[l].y);
            DA[l] = vadd(DA[l], V(-(rr.z * py), rr.z * px, FMA(rr.x, py, -(rr.y * px))));  // rr x Pt
          }
        }
        continue;
      }
      v3 cp = vfma(n, -rad, pe);
      v3 rr = vsub(cp, b.x[l]);
      v3 cn = vcross(rr, n);
      float w = im + vdot(cn, cn);
      float lam = POB_DIV(pen, w);
      v3 P = vscl(n, lam);
      DX[l] = vfma(P, im, DX[l]);
      DA[l] = vadd(DA[l], vcross(rr, P));
      v3 cprev = qrot_add(qrot(rr, qinv(b.q[l])), L.get4(QL_PQ(l)), L.get3(QL_PX(l)));
      v3 dp = vsub(cp, cprev);
      v3 dpt = vfma(n, -vdot(dp, n), dp);
      float lt, ilt;
      pob_sqrt_rcp(vdot(dpt, dpt), lt, ilt);
      if (lt > 0.0f) {
        v3 t = vscl(dpt, ilt);
        v3 ctn = vcross(rr, t);
        float wt = im + vdot(ctn, ctn);
        float lamt = POB_DIV(lt, wt);
        if (lamt < fric * lam) {
          v3 Pt = vscl(t, -lamt);
          DX[l] = vfma(Pt, im, DX[l]);
          DA[l] = vadd(DA[l], vcross(rr, Pt));
        }
      }
    }
  }
}

POB_D void qcontact_velocity(csys_t *Sp, const float *LT, const QBody &b, const QContacts &ct, v3 (&dV)[QNB],
                             v3 (&dW)[QNB], const float fric) {
#pragma unroll
  for (int c = 0; c < 2 + QNB; ++c) {
    POB_FENCE();
    const int l = qcontact_body(c);
    const float pen = ct.pen[c];
    if (pen > 0.0f) {
      csys_t &S = *launder(Sp);
      v3 e, n;
      float rad;
      qcontact_geom(S, LT, ct, c, e, n, rad);
      const float im = q_inv_mass(S, LT, l);
      v3 pe = l == 0 ? vadd(b.x[0], qrot(e, b.q[0])) : vadd(b.x[l], qrot_xy(e, b.q[l]));
      v3 cp = vfma(n, -rad, pe);
      v3 rr = vsub(cp, b.x[l]);
      v3 vr = vadd(b.v[l], vcross(b.w[l], rr));
      v3 dv = V(0.0f, 0.0f, 0.0f);
      if (c < 2) {
        // ground, n = (0, 0, 1) (zero products dropped, as in the position pass)
        const float vn = vr.z;
        float lt, ilt;
        pob_sqrt_rcp(FMA(vr.y, vr.y, vr.x * vr.x), lt, ilt);
        if (lt > 0.0f) {
          const float fr = fminf(fric * pen * S.inv_h, lt);
          const float k = -(fr * ilt);
          dv = V(vr.x * k, vr.y * k, 0.0f);
        }
        if (vn < 0.0f) dv.z = -vn;
      } else {
        float vn = vdot(vr, n);
        v3 vt = vfma(n, -vn, vr);
        float lt, ilt;
        pob_sqrt_rcp(vdot(vt, vt), lt, ilt);
        if (lt > 0.0f) {
          float fr = fminf(fric * pen * S.inv_h, lt);
          dv = vscl(vt, -(fr * ilt));
        }
        if (vn < 0.0f) dv = vfma(n, -vn, dv);
      }
      float D, iD;
      pob_sqrt_rcp(vdot(dv, dv), D, iD);
      if (D > 0.0f) {
        v3 dh = vscl(dv, iD);
        v3 cd = vcross(rr, dh);
        float w = im + vdot(cd, cd);
        v3 P = vdivs(dv, w);
        dV[l] = vfma(P, im, dV[l]);
        dW[l] = vadd(dW[l], vcross(rr, P));
      }
    }
  }
}

// torso terms of the lane's hip joint (global 2k): the oracle adds P * imp to DX[0] and
// t = (rp x P) + (Pa + Pl) to DA[0], in joint order
struct QTorso {
  v3 P;  // point-constraint impulse (zero if the anchors coincide)
  v3 t;  // angular correction of the torso
};

// local joint jl's point / hinge / limit corrections into DX / DA (local bodies; DA = the
// angular correction vectors, applied as one rotation update per body -- oracle
// joints_position); for the hip (jl = 0) the torso terms go to *tt
POB_D void qjoint_position(csys_t *Sp, const float *LT, const QBody &b, const int jl, v3 (&DX)[QNB], v3 (&DA)[QNB],
                           QTorso *tt) {
  csys_t &S = *launder(Sp);
  const int p = jparent(jl), c = jchild(jl);
  const float imp = q_inv_mass(S, LT, p);
  const float imc = q_inv_mass(S, LT, c);
  const bool torso_parent = p == 0;
  // the six joint vectors through the two bodies' rotation matrices (oracle joints_position)
  v3 ap, ac, rp, rc;
  float psi;
  {
    // Ant joint frames (checked by pob_system.cpp): offsets in the body xy-plane; the hip's
    // axis is +z and reference -x, the knee's axis lies in the xy-plane and reference is +z
    const m3 Rp = qmat(b.q[p]), Rc = qmat(b.q[c]);
    v3 fp, fc;
    if (jl == 0) {
      ap = mcol2(Rp); ac = mcol2(Rc);
      fp = vscl(mcol0(Rp), -1.0f); fc = vscl(mcol0(Rc), -1.0f);
    } else {
      const v3 axis = QJV(LT, jl, QJ_AXIS);
      ap = mrot_xy(Rp, axis); ac = mrot_xy(Rc, axis);
      fp = mcol2(Rp); fc = mcol2(Rc);
    }
    psi = pob_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
    rp = mrot_xy(Rp, QJV(LT, jl, QJ_OFFP));
    rc = mrot_xy(Rc, QJV(LT, jl, QJ_OFFC));
  }
  // hinge axis alignment and angle limits
  const float lo = QJS(LT, jl, QJ_LO), hi = QJS(LT, jl, QJ_HI);
  float dl = 0.0f;
  if (psi < lo) dl = psi - lo;
  else if (psi > hi) dl = psi - hi;
  const v3 Pa = vscl(vcross(ap, ac), S.half_s_ang);
  const v3 Pl = vscl(ap, dl * S.half_s_ang);
  const v3 s = vadd(Pa, Pl);
#ifndef POB_EXP_JOINT_ILP
  POB_FENCE();
#endif
  // point-to-point
  csys_t &S2 = *launder(Sp);
  // (oracle joints_position: P = d k, r x P = (r x d) k with k = s_pos L^2 / (L^2 (imp + imc)
  // + |rp x d|^2 + |rc x d|^2); all zero when the anchors coincide)
  v3 d = vsub(vadd(b.x[c], rc), vadd(b.x[p], rp));
  const float L2 = vdot(d, d);
  v3 P = V(0.0f, 0.0f, 0.0f), xp = P, xc = P;
  if (L2 > 0.0f) {
    const v3 ep = vcross(rp, d), ec = vcross(rc, d);
    const float den = FMA(L2, imp + imc, vdot(ep, ep) + vdot(ec, ec));
    const float k = POB_DIV(L2 * S2.s_pos, den);
    P = vscl(d, k); xp = vscl(ep, k); xc = vscl(ec, k);
  }
  if (torso_parent) tt->P = P;
  else DX[p] = vfma(P, imp, DX[p]);
  DX[c] = vfma(P, -imc, DX[c]);
  const v3 tp = vadd(xp, s);
  if (torso_parent) tt->t = tp;
  else DA[p] = vadd(DA[p], tp);
  DA[c] = vsub(DA[c], vadd(xc, s));
}

// add quad lane J's hip terms onto the torso accumulators (global joint 2J)
template <int J>
POB_D void qtorso_add(v3 &dx, v3 &da, const QTorso &t, const float imp0) {
  dx = vfma(quad_bcast3<J>(t.P), imp0, dx);
  da = vadd(da, quad_bcast3<J>(t.t));
}

// The friction coefficient for the substep loop (POB_QFRIC_REG, default on): read once and
// passed through an empty asm, so the compiler holds it in a register instead of
// re-issuing a scalar load of pob_sys::friction at each of the ten contact sites of every
// collide substep (and waiting for it).
#ifndef POB_QFRIC_REG
#define POB_QFRIC_REG 1
#endif
POB_D float quad_friction(const csys_t &S) {
  float f = S.friction;
#if POB_QFRIC_REG
  asm volatile("" : "+s"(f));
#endif
  return f;
}

// One XPBD substep on a lane quad (see the header comment for the split).
template <bool WALLS>
POB_D void qpbd_substep(csys_t *Sp, const float *LT, const float *WT, QBody &b, const float (&act)[QNJ], const Lds &L,
                        const bool COLLIDE, const float fric) {
#pragma unroll
  for (int l = 0; l < QNB; ++l) { L.set3(QL_PX(l), b.x[l]); L.set4(QL_PQ(l), b.q[l]); }
  // 1. acceleration level.  Torso: dw0 = (((0 - t0) - t2) - t4) - t6 over the quad.
  {
    v3 tt[QNJ];
#pragma unroll
    for (int jl = 0; jl < QNJ; ++jl) {
      const int p = jparent(jl), c = jchild(jl);
      const v3 axis = QJV(LT, jl, QJ_AXIS);
      const v3 a = jl == 0 ? qrot_ez(b.q[p]) : qrot_xy(axis, b.q[p]);
      const bool in = actuator_inside(b.q[p], b.q[c], jl == 0, axis, QJS(LT, jl, QJ_TLO), QJS(LT, jl, QJ_THI));
      v3 t = vscl(a, (in ? act[jl] : 0.0f) * QJS(LT, jl, QJ_STRENGTH));
      v3 d = vscl(vsub(b.w[p], b.w[c]), QJS(LT, jl, QJ_DAMP));
      tt[jl] = vadd(t, d);
    }
    v3 dw[QNB];
    {
      const v3 t0 = quad_bcast3<0>(tt[0]), t2 = quad_bcast3<1>(tt[0]);
      const v3 t4 = quad_bcast3<2>(tt[0]), t6 = quad_bcast3<3>(tt[0]);
      dw[0] = vsub(vsub(vsub(vsub(V(0.0f, 0.0f, 0.0f), t0), t2), t4), t6);
    }
    dw[1] = vsub(vadd(V(0.0f, 0.0f, 0.0f), tt[0]), tt[1]);
    dw[2] = vadd(V(0.0f, 0.0f, 0.0f), tt[1]);
    csys_t &S = *launder(Sp);
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      const v3 v = b.v[l], w = b.w[l];
      b.v[l] = V(FMA(S.lin_damp, v.x, 0.0f * S.h), FMA(S.lin_damp, v.y, 0.0f * S.h), FMA(S.lin_damp, v.z, S.gz * S.h));
      b.w[l] = V(FMA(S.ang_damp, w.x, dw[l].x * S.h), FMA(S.ang_damp, w.y, dw[l].y * S.h),
                 FMA(S.ang_damp, w.z, dw[l].z * S.h));
    }
    // 2. kinetic
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      b.x[l] = vfma(b.v[l], S.h, b.x[l]);
      q4 dq = qmul_vq(b.w[l], b.q[l]);
      q4 q = b.q[l];
      q.w = FMA(S.half_h, dq.w, q.w); q.x = FMA(S.half_h, dq.x, q.x);
      q.y = FMA(S.half_h, dq.y, q.y); q.z = FMA(S.half_h, dq.z, q.z);
      b.q[l] = qnormalize(q);
    }
  }
  // 3. position projection
  QContacts ct;
  {
    v3 DX[QNB];
    v3 DA[QNB];
#pragma unroll
    for (int l = 0; l < QNB; ++l) { DX[l] = V(0.0f, 0.0f, 0.0f); DA[l] = V(0.0f, 0.0f, 0.0f); }
    QTorso tq;
    POB_FENCE();
#ifdef POB_EXP_NO_JOINTS
    tq.P = V(0.0f, 0.0f, 0.0f);  // timing experiment only
    tq.t = tq.P;
#else
    qjoint_position(Sp, LT, b, 0, DX, DA, &tq);
#ifndef POB_EXP_JOINT_ILP
    POB_FENCE();
#endif
    qjoint_position(Sp, LT, b, 1, DX, DA, nullptr);
#endif
    POB_FENCE();
    // torso: global joints 0, 2, 4, 6 (quad lanes 0..3) in order
    {
      const float imp0 = launder(Sp)->inv_mass[0];
      qtorso_add<0>(DX[0], DA[0], tq, imp0);
      qtorso_add<1>(DX[0], DA[0], tq, imp0);
      qtorso_add<2>(DX[0], DA[0], tq, imp0);
      qtorso_add<3>(DX[0], DA[0], tq, imp0);
    }
    if (COLLIDE) {
      qdetect<WALLS>(Sp, LT, WT, b, ct);
      qcontact_position(Sp, LT, b, L, ct, DX, DA, fric);
    }
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      b.x[l] = vadd(b.x[l], DX[l]);
      qadd_half(b.q[l], qmul_vq(DA[l], b.q[l]), 1.0f);
    }
  }
  // 4. velocity projection
#pragma unroll
  for (int l = 0; l < QNB; ++l) {
    csys_t &S = *launder(Sp);
    b.q[l] = qnormalize(b.q[l]);
    b.v[l] = vscl(vsub(b.x[l], L.get3(QL_PX(l))), S.inv_h);
    q4 dq = qmul(b.q[l], qinv(L.get4(QL_PQ(l))));
    // sg ((2 dq) inv_h) == dq (sg 2 inv_h) bit for bit (scaling by 2 and by +-1 is exact)
    const float k2 = 2.0f * S.inv_h;
    const float kw = dq.w >= 0.0f ? k2 : -k2;
    b.w[l] = V(dq.x * kw, dq.y * kw, dq.z * kw);
  }
  // 5. velocity-level contacts
  if (COLLIDE) {
    v3 dV[QNB], dW[QNB];
#pragma unroll
    for (int l = 0; l < QNB; ++l) { dV[l] = V(0.0f, 0.0f, 0.0f); dW[l] = V(0.0f, 0.0f, 0.0f); }
    qcontact_velocity(Sp, LT, b, ct, dV, dW, fric);
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      b.v[l] = vadd(b.v[l], dV[l]); b.w[l] = vadd(b.w[l], dW[l]);
      L.set3(QL_CV(l), vadd(L.get3(QL_CV(l)), dV[l]));
      L.set3(QL_CA(l), vadd(L.get3(QL_CA(l)), dW[l]));
    }
  }
}

// ------------------------------------------------------------- legacy spring dynamics
// brax <= 0.0.12 spring/impulse step (oracle legacy_substep; pinned by the 20 frames of
// notebooks/ant_tag.ipynb:449) on the same lane quads: kinetic, then spring joints + torque
// actuators as accelerations, then one-way contact impulses.  Every expression follows the
// oracle's generic form (no frame specialisation: this mode is the parity reference for the
// notebook, not the throughput path).

// one-way contact impulses of the detected contacts into dV / dW (oracle legacy_contacts;
// per body: ground contact first, then wall)
POB_D void qlegacy_contacts(csys_t *Sp, const float *LT, const QBody &b, const QContacts &ct, v3 (&dV)[QNB],
                            v3 (&dW)[QNB]) {
#pragma unroll
  for (int c = 0; c < 2 + QNB; ++c) {
    const int l = qcontact_body(c);
    const float pen = ct.pen[c];
    if (pen > 0.0f) {
      csys_t &S = *launder(Sp);
      v3 e, n;
      float rad;
      qcontact_geom(S, LT, ct, c, e, n, rad);
      const float im = q_inv_mass(S, LT, l);
      const v3 rel = vsub(vfma(n, -rad, ct.pe[c]), b.x[l]);  // pe = x + rotate(e, q) of the detection
      const v3 cv = vadd(b.v[l], vcross(b.w[l], rel));
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
        dV[l] = vfma(P, im, dV[l]);
        dW[l] = vadd(dW[l], vcross(rel, P));
      }
    }
  }
}

// spring joint jl of the lane (oracle legacy_joints): the anchor impulse imp and the angular
// term tw (parent: + tw + rp x -imp, child: - tw + rc x imp)
struct QSpring {
  v3 imp, tp, tc;  // impulse; parent and child angular terms
};
POB_D QSpring qlegacy_joint(csys_t &S, const float *LT, const QBody &b, const int jl, const float act) {
  const int p = jparent(jl), c = jchild(jl);
  const v3 axis = QJV(LT, jl, QJ_AXIS);
  const v3 ref = jl == 0 ? V(-1.0f, 0.0f, 0.0f) : V(0.0f, 0.0f, 1.0f);  // the Ant's (pob_system.cpp)
  const v3 rp = qrot(QJV(LT, jl, QJ_OFFP), b.q[p]), rc = qrot(QJV(LT, jl, QJ_OFFC), b.q[c]);
  const v3 dpos = vsub(vadd(b.x[p], rp), vadd(b.x[c], rc));
  const v3 dvel = vsub(vadd(b.v[p], vcross(b.w[p], rp)), vadd(b.v[c], vcross(b.w[c], rc)));
  QSpring J;
  J.imp = vfma(dpos, S.k_spring, vscl(dvel, S.c_spring));
  const v3 ap = qrot(axis, b.q[p]), ac = qrot(axis, b.q[c]);
  const v3 fp = qrot(ref, b.q[p]), fc = qrot(ref, b.q[c]);
  const float psi = pob_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
  const float lo = QJS(LT, jl, QJ_LO), hi = QJS(LT, jl, QJ_HI);
  float dang = 0.0f;
  if (psi < lo) dang = lo - psi;
  else if (psi > hi) dang = hi - psi;
  v3 tq = vscl(vcross(ap, ac), S.k_spring);
  tq = vfma(ap, -(S.k_limit * dang), tq);
  tq = vfma(vsub(b.w[p], b.w[c]), -QJS(LT, jl, QJ_DAMP), tq);
  const v3 ta = vscl(ap, (dang != 0.0f ? 0.0f : act) * QJS(LT, jl, QJ_STRENGTH));
  const v3 tw = vsub(tq, ta);
  J.tp = vadd(vcross(rp, vscl(J.imp, -1.0f)), tw);
  J.tc = vsub(vcross(rc, J.imp), tw);
  return J;
}

template <bool WALLS>
POB_D void qlegacy_substep(csys_t *Sp, const float *LT, const float *WT, QBody &b, const float (&act)[QNJ],
                           const Lds &L) {
  // kinetic
  {
    csys_t &S = *launder(Sp);
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      b.x[l] = vfma(b.v[l], S.h, b.x[l]);
      q4 dq = qmul_vq(b.w[l], b.q[l]);
      q4 q = b.q[l];
      q.w = FMA(S.half_h, dq.w, q.w); q.x = FMA(S.half_h, dq.x, q.x);
      q.y = FMA(S.half_h, dq.y, q.y); q.z = FMA(S.half_h, dq.z, q.z);
      b.q[l] = qnormalize(q);
    }
  }
  // joints + actuators (accelerations), summed per body in joint order
  v3 dv[QNB], dw[QNB];
  {
    csys_t &S = *launder(Sp);
    const QSpring hip = qlegacy_joint(S, LT, b, 0, act[0]);
    const QSpring knee = qlegacy_joint(S, LT, b, 1, act[1]);
    const float im0 = S.inv_mass[0], im1 = q_inv_mass(S, LT, 1), im2 = q_inv_mass(S, LT, 2);
    // torso: parent of the hips (global joints 0, 2, 4, 6 = quad lanes 0..3)
    v3 v0 = V(0.0f, 0.0f, 0.0f), w0 = v0;
    v0 = vfma(quad_bcast3<0>(hip.imp), -im0, v0); w0 = vadd(w0, quad_bcast3<0>(hip.tp));
    v0 = vfma(quad_bcast3<1>(hip.imp), -im0, v0); w0 = vadd(w0, quad_bcast3<1>(hip.tp));
    v0 = vfma(quad_bcast3<2>(hip.imp), -im0, v0); w0 = vadd(w0, quad_bcast3<2>(hip.tp));
    v0 = vfma(quad_bcast3<3>(hip.imp), -im0, v0); w0 = vadd(w0, quad_bcast3<3>(hip.tp));
    dv[0] = v0; dw[0] = w0;
    // aux: child of the hip, then parent of the knee; lower leg: child of the knee
    dv[1] = vfma(knee.imp, -im1, vfma(hip.imp, im1, V(0.0f, 0.0f, 0.0f)));
    dw[1] = vadd(vadd(V(0.0f, 0.0f, 0.0f), hip.tc), knee.tp);
    dv[2] = vfma(knee.imp, im2, V(0.0f, 0.0f, 0.0f));
    dw[2] = vadd(V(0.0f, 0.0f, 0.0f), knee.tc);
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      const v3 v = b.v[l], w = b.w[l];
      b.v[l] = V(FMA(S.lin_damp, v.x, (dv[l].x + 0.0f) * S.h), FMA(S.lin_damp, v.y, (dv[l].y + 0.0f) * S.h),
                 FMA(S.lin_damp, v.z, (dv[l].z + S.gz) * S.h));
      b.w[l] = V(FMA(S.ang_damp, w.x, dw[l].x * S.h), FMA(S.ang_damp, w.y, dw[l].y * S.h),
                 FMA(S.ang_damp, w.z, dw[l].z * S.h));
    }
  }
  // collisions: velocity impulses at the post-kinetic pose
  QContacts ct;
  qdetect<WALLS>(Sp, LT, WT, b, ct);
  v3 dV[QNB], dW[QNB];
#pragma unroll
  for (int l = 0; l < QNB; ++l) { dV[l] = V(0.0f, 0.0f, 0.0f); dW[l] = V(0.0f, 0.0f, 0.0f); }
  qlegacy_contacts(Sp, LT, b, ct, dV, dW);
#pragma unroll
  for (int l = 0; l < QNB; ++l) {
    b.v[l] = vadd(b.v[l], dV[l]); b.w[l] = vadd(b.w[l], dW[l]);
    L.set3(QL_CV(l), vadd(L.get3(QL_CV(l)), dV[l]));
    L.set3(QL_CA(l), vadd(L.get3(QL_CA(l)), dW[l]));
  }
}
