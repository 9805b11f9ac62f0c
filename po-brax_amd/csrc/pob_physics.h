// pob_physics.h -- shared physics pieces of the rollout kernels (gfx950): the system-table
// access helpers, the per-lane LDS view, sphere-box and the whole-ant (one lane) contact
// detection + velocity-level contact solve used by the reset kernel's sys.info(qp)
// (a2).  The step itself runs four lanes per env (pob_quad.h).
//
// Algorithm = brax v1 System.step with dynamics_mode "pbd" as restated in DESIGN.md §3
// (brax is not vendored: reference call sites ant_heavenhell.py:108, ant_gather.py:127,
// ant_tag.py:109).  Op order matches oracle/pob_oracle.c expression for expression.
#pragma once
#include "pob_math.h"
#include "pob_sys.h"

struct Body {
  v3 x[POB_NDYN];
  q4 q[POB_NDYN];
  v3 v[POB_NDYN];
  v3 w[POB_NDYN];
};

struct Contacts {
  // [0, 5): ground (CapsulePlane, normal +z, end point S.ground_end[k]),
  // [5, 14): deepest wall contact of capsule i (normal n[i], end point cap_end[i][sel[i]])
  float pen[POB_NGROUND + POB_NDYN];
  v3 n[POB_NDYN];
  bool sel[POB_NDYN];
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

// sphere (centre p, radius r) vs z-rotated box w -> penetration, world normal
POB_D float sphere_box(csys_t &S, int w, v3 p, float r, v3 &n) {
  const float c = S.wall_cos[w], s = S.wall_sin[w];
  const v3 h = SV(S.wall_h[w]);
  v3 d = vsub(p, SV(S.wall_c[w]));
  float lx = FMA(d.y, s, d.x * c), ly = FMA(d.y, c, -(d.x * s)), lz = d.z;
  float qx = clamp_sym(lx, h.x), qy = clamp_sym(ly, h.y), qz = clamp_sym(lz, h.z);
  float ex = lx - qx, ey = ly - qy, ez = lz - qz;
  float d2 = FMA(ez, ez, FMA(ey, ey, ex * ex));
  float pen, nx, ny, nz;
  if (d2 > 0.0f) {
    float dist, inv;
    pob_sqrt_rcp(d2, dist, inv);
    pen = r - dist; nx = ex * inv; ny = ey * inv; nz = ez * inv;
  } else {
    float fx = h.x - fabsf(lx), fy = h.y - fabsf(ly), fz = h.z - fabsf(lz);
    nx = 0.0f; ny = 0.0f; nz = 0.0f;
    if (fx <= fy && fx <= fz) { pen = r + fx; nx = lx < 0.0f ? -1.0f : 1.0f; }
    else if (fy <= fz) { pen = r + fy; ny = ly < 0.0f ? -1.0f : 1.0f; }
    else { pen = r + fz; nz = lz < 0.0f ? -1.0f : 1.0f; }
  }
  n = V(FMA(-ny, s, nx * c), FMA(ny, c, nx * s), nz);
  return pen;
}

// Contact detection of a collide substep: CapsulePlane on the torso and the four feet,
// and for every capsule its deepest sphere-box contact over (wall, segment end).
POB_D void detect(csys_t *Sp, const Body &b, Contacts &ct) {
#pragma unroll
  for (int g = 0; g < POB_NGROUND; ++g) {
    csys_t &S = *launder(Sp);
    const int i = ground_body(g);
    v3 pe = vadd(b.x[i], qrot(SV(S.ground_end[g]), b.q[i]));
    ct.pen[g] = S.ground_r[g] - pe.z;
  }
  // wave-uniform broadphase: bit w set iff some lane's body-centre AABB meets wall w's grown box
  uint32_t near_mask = 0u;
  {
    v3 mn = b.x[0], mx = b.x[0];
#pragma unroll
    for (int i = 1; i < POB_NDYN; ++i) {
      mn = V(fminf(mn.x, b.x[i].x), fminf(mn.y, b.x[i].y), fminf(mn.z, b.x[i].z));
      mx = V(fmaxf(mx.x, b.x[i].x), fmaxf(mx.y, b.x[i].y), fmaxf(mx.z, b.x[i].z));
    }
    csys_t &S = *launder(Sp);
    const int nw = S.n_walls;
    for (int w = 0; w < nw; ++w) {
      const bool near = mn.x <= S.wall_hi[w][0] && mx.x >= S.wall_lo[w][0] && mn.y <= S.wall_hi[w][1] &&
                        mx.y >= S.wall_lo[w][1] && mn.z <= S.wall_hi[w][2] && mx.z >= S.wall_lo[w][2];
      if (__any(near)) near_mask |= 1u << w;
    }
  }
#pragma unroll
  for (int i = 0; i < POB_NDYN; ++i) {
    POB_FENCE();
    csys_t &S = *launder(Sp);
    const int nend = (i == 0) ? 1 : 2;
    v3 pe[2];
#pragma unroll
    for (int q = 0; q < nend; ++q) pe[q] = vadd(b.x[i], qrot(SV(S.cap_end[i][q]), b.q[i]));
    float best = 0.0f;
    v3 bn = V(0.0f, 0.0f, 0.0f);
    bool bsel = false;
    const float r = S.cap_r[i];
    const int nw = S.n_walls;
    for (int w = 0; w < nw; ++w) {
      if (!(near_mask & (1u << w))) continue;  // uniform: no lane can touch wall w
#pragma unroll
      for (int q = 0; q < nend; ++q) {
        v3 n;
        float pen = sphere_box(*launder(Sp), w, pe[q], r, n);
        if (pen > best) { best = pen; bn = n; bsel = q == 1; }
      }
    }
    ct.pen[POB_NGROUND + i] = best;
    ct.n[i] = bn;
    ct.sel[i] = bsel;
  }
}

// contact k: body frame end point, world normal, radius
POB_D void contact_geom(csys_t &S, const Contacts &ct, int k, v3 &e, v3 &n, float &r) {
  if (k < POB_NGROUND) {
    e = SV(S.ground_end[k]);
    n = V(0.0f, 0.0f, 1.0f);
    r = S.ground_r[k];
  } else {
    const int i = k - POB_NGROUND;
    const v3 e0 = SV(S.cap_end[i][0]), e1 = SV(S.cap_end[i][1]);
    e = ct.sel[i] ? e1 : e0;
    n = ct.n[i];
    r = S.cap_r[i];
  }
}

POB_D void contact_velocity(csys_t *Sp, const Body &b, const Contacts &ct, v3 (&dV)[POB_NDYN],
                            v3 (&dW)[POB_NDYN]) {
#pragma unroll
  for (int k = 0; k < POB_NGROUND + POB_NDYN; ++k) {
    POB_FENCE();
    const int i = contact_body(k);
    const float pen = ct.pen[k];
    if (pen > 0.0f) {
      csys_t &S = *launder(Sp);
      v3 e, n;
      float rad;
      contact_geom(S, ct, k, e, n, rad);
      const float im = S.inv_mass[i];
      v3 pe = vadd(b.x[i], qrot(e, b.q[i]));
      v3 cp = vfma(n, -rad, pe);
      v3 rr = vsub(cp, b.x[i]);
      v3 vr = vadd(b.v[i], vcross(b.w[i], rr));
      float vn = vdot(vr, n);
      v3 vt = vfma(n, -vn, vr);
      float lt, ilt;
      pob_sqrt_rcp(vdot(vt, vt), lt, ilt);
      v3 dv = V(0.0f, 0.0f, 0.0f);
      if (lt > 0.0f) {
        float fr = fminf(S.friction * pen * S.inv_h, lt);
        dv = vscl(vt, -(fr * ilt));
      }
      if (vn < 0.0f) dv = vfma(n, -vn, dv);
      float D, iD;
      pob_sqrt_rcp(vdot(dv, dv), D, iD);
      if (D > 0.0f) {
        v3 dh = vscl(dv, iD);
        v3 cd = vcross(rr, dh);
        float w = im + vdot(cd, cd);
        v3 P = vdivs(dv, w);
        dV[i] = vfma(P, im, dV[i]);
        dW[i] = vadd(dW[i], vcross(rr, P));
      }
    }
  }
}

// sys.info(qp).contact at a static state
POB_D void info_contact(csys_t *Sp, const Body &b, v3 (&cvel)[POB_NDYN], v3 (&cang)[POB_NDYN]) {
  Contacts ct;
  detect(Sp, b, ct);
#pragma unroll
  for (int i = 0; i < POB_NDYN; ++i) { cvel[i] = V(0.0f, 0.0f, 0.0f); cang[i] = V(0.0f, 0.0f, 0.0f); }
  contact_velocity(Sp, b, ct, cvel, cang);
}
