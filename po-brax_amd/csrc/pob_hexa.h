// pob_hexa.h -- the PBD Ant step with SIXTEEN lanes per environment (gfx950), for batches
// small enough that one wave per SIMD is all the chip gets (HH B = 4 096 is 512 waves of the
// eight-lane kernel, half the SIMDs idle) and the step time is one wave's dependency chain.
//
// Split: every lane owns ONE body and one side of one joint (lane r = lane & 15 of the env):
//   r = k       P_hip_k   torso (replica x4)   parent side of joint 2k
//   r = 7 - k   C_hip_k   Aux k+1              child side of joint 2k
//   r = 8 + k   P_knee_k  Aux k+1 (replica)    parent side of joint 2k+1
//   r = 15 - k  C_knee_k  lower leg k          child side of joint 2k+1
// so a joint's two sides are one row_half_mirror DPP apart (r <-> 7 - r within each half row),
// an Aux body's two replicas one row_mirror apart (r <-> 15 - r), and the four torso replicas
// form the row's first DPP quad (the torso sums over the hips are quad broadcasts in joint
// order, as in the four- and eight-lane kernels).  Each lane integrates, projects and
// collides its own body only; a joint's scalar work (point constraint, hinge, limit, the
// actuator torque) runs on both of its lanes from the same exchanged operands, so both sides
// hold the same bits.  Every value follows the oracle's op order (oracle/pob_oracle.c; the
// generic joint projection of the eight-lane kernel), so the results are bit-identical to the
// other kernels'.
#pragma once
#include "pob_octet.h"

// per-role table row (16 rows, role r as above), staged in LDS, copied into registers
#define HT_OFFP 0      // joint: off_p (3) off_c (3) axis (3) ref (3) lim_lo lim_hi jdamp strength
#define HT_OFFC 3
#define HT_AXIS 6
#define HT_REF 9
#define HT_LO 12
#define HT_HI 13
#define HT_DAMP 14
#define HT_STRENGTH 15
#define HT_IMP 16      // the joint's parent / child inverse masses
#define HT_IMC 17
#define HT_IM 18       // the lane's body: inverse mass, capsule radius, capsule end e0 (3)
#define HT_R 19
#define HT_E0 20
#define HT_OFF 23      // the lane's joint offset (off_p on the parent side, off_c on the child side)
#define HT_GE 26       // the body's ground contact: end (3), radius, 1.0 if it has one
#define HT_GR 29
#define HT_HASG 30
#define HT_TLO 31      // tan(lim_lo), tan(lim_hi): the actuator gate
#define HT_THI 32
#define HT_ISP 33      // 1.0 on the parent side
#define HT_ISHIP 34    // 1.0 for a hip joint
#define HT_FLOATS POB_HEX_FLOATS
#define HT_TAB_FLOATS (16 * HT_FLOATS + POB_MAXW * POB_WALL_FLOATS)  // + the wall rows
#define HTV(T, f) V((T)[(f)], (T)[(f) + 1], (T)[(f) + 2])

// lane r <-> 7 - r (half row): a joint's two sides
POB_D float hx_pair(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xf, 0xf, true));  // row_half_mirror
}
// lane r <-> 15 - r (row): an Aux body's two replicas
POB_D float hx_mirror(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xf, 0xf, true));  // row_mirror
}
POB_D v3 hx_pair3(v3 a) { return V(hx_pair(a.x), hx_pair(a.y), hx_pair(a.z)); }
POB_D v3 hx_mirror3(v3 a) { return V(hx_mirror(a.x), hx_mirror(a.y), hx_mirror(a.z)); }
POB_D q4 hx_pair4(q4 q) {
  q4 r; r.w = hx_pair(q.w); r.x = hx_pair(q.x); r.y = hx_pair(q.y); r.z = hx_pair(q.z); return r;
}

// Walls a kind's table can hold (pob_system.cpp: the HH T-maze 8, the GA / TAG arenas 4,
// the stock ant none): the sixteen-lane wall loops run over this many rows, and the launch
// checks n_walls against it.
__host__ __device__ constexpr int hex_max_walls(int kind) {
  return kind == POB_ANT ? 0 : (kind == POB_HEAVENHELL ? POB_MAXW : 4);
}

struct HBody {
  v3 x, v, w;
  q4 q;
};

// the body's ground contact (torso and lower legs; pen -1 otherwise) and its wall contacts
// (pob_quad.h QMesh: the segment at detection and the contact-bearing items)
struct HGround {
  float pen;
  v3 pe;  // x + rotate(end, q)
};
// (POB_HEX_POOL, the default since round 6: the wave's contacts in an LDS pool, stored by the
// walk's winner lanes and linked per lane by the owners -- HH B = 4 096 0.0596 -> 0.0563 ms,
// 8 192 0.0699 -> 0.0672, profiles/r7g/ab.txt; 0: the per-lane store with its hand-over loop)
#ifndef POB_HEX_POOL
#define POB_HEX_POOL 1
#endif
struct HMesh {
  v3 a, b;
  uint64_t mc;
  int nct;  // wall contacts of the position pass (the first HMAXC kept in the lane's LDS store)
#if POB_HEX_POOL
  int head;   // the lane's first contact in the wave's pool (POB_HEX_POOL)
  bool povf;  // the wave's contacts overflowed the pool (wave-uniform)
#endif
};
#if POB_HEX_POOL
// the wave's contact pool (pob_mesh.h mesh_wave_walk HAND 2, as the four-lane kernel's fast
// launch): each entry tau, n, dist and the index of the lane's next entry (-1: the last)
#define HPOOL_N 64
struct HPoolSink {
  float *pool;
  int npool;  // (wave-uniform)
  int tail, head, nct;
  uint64_t mc;
  POB_D int store(const bool hit, const float tau, const v3 n, const float dist) {
    const uint64_t m = __ballot(hit);
    const int idx = npool + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    npool += __popcll(m);
    if (hit && idx < HPOOL_N) {
      float *c = pool + 6 * idx;
      c[0] = tau; c[1] = n.x; c[2] = n.y; c[3] = n.z; c[4] = dist;
    }
    return hit ? idx + 1 : 0;  // (past the pool too: the owner still counts the contact and its face)
  }
  POB_D void link(const int, const int bit, const int e) {
    if (e > 0) {
      const int idx = e - 1;
      ++nct;
      mc |= 1ull << bit;  // (the face's contacts are re-walked if the pool overflowed)
      if (idx < HPOOL_N) {
        pool[6 * idx + 5] = __int_as_float(-1);
        if (tail >= 0) pool[6 * tail + 5] = __int_as_float(idx);
        else head = idx;
        tail = idx;
      }
    }
  }
};
#endif
// The position pass's wall contacts (tau, n, pen), kept in the lane's slots of the staging
// region (idle during the substeps; lane-minor: element e of the lane at CS[64 e]) so that the
// velocity pass applies them without evaluating their faces again; a lane with more re-walks
// its contact faces (ms.mc) from the stored segments instead -- the same contacts either way.
#define HMAXC 5
#define HCS_FLOATS (5 * HMAXC)

// Contacts of a collide substep on one lane (oracle order: ground, then walls in wall / face /
// triangle order).  Walls: the broadphase over the walls' grown boxes (registers, HWalls) by
// the body centre, the face items of the lane's body (pob_mesh.h cull), then the wave's face
// walk (pob_mesh.h mesh_wave_walk) with the wall rows from LDS (WT).  The torso is the sphere.
template <int MW, class G>
POB_D void hcontacts_position(G &g, const HCon &SC, const float *HT, const float *WT, const HWalls<MW> &HW,
                              const bool torso, const HBody &b, const v3 px, const q4 pq, HGround &gc, HMesh &ms,
                              v3 &DX, v3 &DA, float *CS, unsigned long long *tacc = nullptr) {
#ifdef POB_EXP_TIMING_SUB
  const unsigned long long _tc0 = __builtin_amdgcn_s_memtime();  // (slot 5: the broadphase + face cull)
#else
  (void)tacc;
#endif
  gc.pe = vadd(b.x, qrot_xy(HTV(HT, HT_GE), b.q));
  gc.pen = HT[HT_HASG] != 0.0f ? HT[HT_GR] - gc.pe.z : -1.0f;
  const float im = HT[HT_IM];
  if (gc.pen > 0.0f) oground_position(g, SC, gc.pen, gc.pe, HT[HT_GR], im, b.x, b.q, pq, px, DX, DA);
  ms.mc = 0ull;
  ms.nct = 0;
#if POB_HEX_POOL
  ms.head = -1;
  ms.povf = false;
#endif
  if (MW == 0) return;
  uint32_t m = 0u;
  {
#ifdef POB_EXP_NO_WALLS
    const int nw = 0;  // timing experiment only
#else
    const int nw = HW.n_walls;
#endif
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      // every wall's box is tested (the table always holds POB_MAXW rows), w < nw a predicate
      const bool near = (b.x.x <= HW.hx[w]) & (b.x.x >= HW.lx[w]) & (b.x.y <= HW.hy[w]) & (b.x.y >= HW.ly[w]);
      m |= (near & (w < nw)) ? 1u << w : 0u;
    }
  }
  if (!__any(m != 0u)) return;
  const v3 rv = qrot_xy(HTV(HT, HT_E0), b.q);
  ms.a = vadd(b.x, rv);
  ms.b = vsub(b.x, rv);
  const float R = HT[HT_R] + POB_MESH_MARGIN;
  uint64_t M = 0ull;
  while (__any(m != 0u)) {
    const bool on = m != 0u;
    const int w = on ? __builtin_ctz(m) : 0;
    m &= m - 1u;
    const MWall W = mwall_row(WT + POB_WALL_FLOATS * w);
    const v3 La = mwall_local(W, HW.cz, ms.a);
    const v3 Lb = torso ? La : mwall_local(W, HW.cz, ms.b);
    const uint32_t fm = mesh_face_mask(La, Lb, W.hx, W.hy, HW.hz, R);
    M |= on ? (uint64_t)fm << (8 * w) : 0ull;
  }
#ifdef POB_EXP_TIMING_SUB
  if (tacc) tacc[5] += __builtin_amdgcn_s_memtime() - _tc0;
#endif
#ifdef POB_EXP_NO_WALK
  return;  // timing experiment only: broadphase and face cull, no face walk
#endif
  // the walk only collects the contacts (its rounds hand each one to its owner lane: a store of
  // five floats); the position responses follow from the store in walk order, one loop over
  // the lanes' contacts instead of the response code in every round's hand-over
  uint64_t Ms[1] = {M};
#if POB_HEX_POOL
  // (CS: the wave's pool)
  HPoolSink sink{CS, 0, -1, -1, 0, 0ull};
#ifdef POB_EXP_TIMING_SUB
  const unsigned long long _tw0 = __builtin_amdgcn_s_memtime();  // (slot 3: the walk alone)
#endif
  mesh_wave_walk<1, false, 2>(g, WT, HW.fc, HW.cz, HW.hz, Ms,
                    [&](const int, v3 &A, v3 &B, float &r, bool &seg) { A = ms.a; B = ms.b; r = HT[HT_R]; seg = !torso; },
                    sink);
#ifdef POB_EXP_TIMING_SUB
  if (tacc) tacc[3] += __builtin_amdgcn_s_memtime() - _tw0;
#endif
  ms.mc = sink.mc;
  ms.nct = sink.nct;
  ms.head = sink.head;
  ms.povf = sink.npool > HPOOL_N;
  const bool ovf = ms.povf && ms.nct > 0;
  {
    int ci = ms.povf ? -1 : ms.head;
#pragma unroll 1
    while (__any(ci >= 0)) {
      if (ci >= 0) {
        const float *c = CS + 6 * ci;
        owall_position(g, SC, HT[HT_R] - c[4], vfma(rv, c[0], b.x), V(c[1], c[2], c[3]), 1e-6f + c[4], im, b.x, b.q,
                       pq, px, DX, DA);
        ci = __float_as_int(c[5]);
      }
    }
  }
#else
  mesh_wave_walk<1, false>(g, WT, HW.fc, HW.cz, HW.hz, Ms,
                    [&](const int, v3 &A, v3 &B, float &r, bool &seg) { A = ms.a; B = ms.b; r = HT[HT_R]; seg = !torso; },
                    [&](const int, const int bit, const float tau, const v3 n, const float dist) {
    ms.mc |= 1ull << bit;
    if (ms.nct < HMAXC) {
      float *c = CS + 64 * 5 * ms.nct;
      c[0] = tau; c[64] = n.x; c[128] = n.y; c[192] = n.z; c[256] = dist;
    }
    ++ms.nct;
  });
  const bool ovf = ms.nct > HMAXC;
  const int nc = ovf ? 0 : ms.nct;
#pragma unroll 1
  for (int i = 0; i < HMAXC; ++i) {
    if (!__any(i < nc)) break;
    if (i < nc) {
      // penetration r - dist; the contact at the triangle point pe - (1e-6 + dist) n
      const float *c = CS + 64 * 5 * i;
      owall_position(g, SC, HT[HT_R] - c[256], vfma(rv, c[0], b.x), V(c[64], c[128], c[192]), 1e-6f + c[256], im, b.x,
                     b.q, pq, px, DX, DA);
    }
  }
#endif
  if (!__any(ovf)) return;
  // (rare) more contacts than the store holds: the contact faces walked again, each contact
  // applied as it comes (the same contacts in the same order)
  uint64_t Mo[1] = {ovf ? ms.mc : 0ull};
  mesh_wave_walk<1, false>(g, WT, HW.fc, HW.cz, HW.hz, Mo,
                    [&](const int, v3 &A, v3 &B, float &r, bool &seg) { A = ms.a; B = ms.b; r = HT[HT_R]; seg = !torso; },
                    [&](const int, const int, const float tau, const v3 n, const float dist) {
    owall_position(g, SC, HT[HT_R] - dist, vfma(rv, tau, b.x), n, 1e-6f + dist, im, b.x, b.q, pq, px, DX, DA);
  });
}

template <int MW, class G>
POB_D void hcontacts_velocity(G &g, const HCon &SC, const float *HT, const float *WT, const HWalls<MW> &HW,
                              const bool torso, const HBody &b, const HGround &gc, const HMesh &ms, v3 &dV, v3 &dW,
                              const float *CS) {
  const float im = HT[HT_IM];
  if (gc.pen > 0.0f)
    ocontact_vel_one(g, SC, true, gc.pen, HTV(HT, HT_GE), V(0.0f, 0.0f, 1.0f), HT[HT_GR], im, b.x, b.q, b.v, b.w, dV, dW);
  if (MW == 0 || !__any(ms.nct != 0)) return;
  const v3 rv = qrot_xy(HTV(HT, HT_E0), b.q);
#if POB_HEX_POOL
  const bool ovf = ms.povf && ms.nct > 0;
  {
    int ci = ms.povf || ms.nct == 0 ? -1 : ms.head;
#pragma unroll 1
    while (__any(ci >= 0)) {
      if (ci >= 0) {
        const float *c = CS + 6 * ci;
        ocontact_vel_pe(g, SC, false, HT[HT_R] - c[4], vfma(rv, c[0], b.x), V(c[1], c[2], c[3]), 1e-6f + c[4], im, b.x,
                        b.v, b.w, dV, dW);
        ci = __float_as_int(c[5]);
      }
    }
  }
#else
  const bool ovf = ms.nct > HMAXC;
  const int n = ovf ? 0 : ms.nct;
#pragma unroll 1
  for (int i = 0; i < HMAXC; ++i) {
    if (!__any(i < n)) break;
    if (i < n) {
      const float *c = CS + 64 * 5 * i;
      ocontact_vel_pe(g, SC, false, HT[HT_R] - c[256], vfma(rv, c[0], b.x), V(c[64], c[128], c[192]), 1e-6f + c[256], im,
                      b.x, b.v, b.w, dV, dW);
    }
  }
#endif
  if (!__any(ovf)) return;
  uint64_t Ms[1] = {ovf ? ms.mc : 0ull};
  mesh_wave_walk<1, false>(g, WT, HW.fc, HW.cz, HW.hz, Ms,
                    [&](const int, v3 &A, v3 &B, float &r, bool &seg) { A = ms.a; B = ms.b; r = HT[HT_R]; seg = !torso; },
                    [&](const int, const int, const float tau, const v3 n, const float dist) {
    ocontact_vel_pe(g, SC, false, HT[HT_R] - dist, vfma(rv, tau, b.x), n, 1e-6f + dist, im, b.x, b.v, b.w, dV, dW);
  });
}

// One XPBD substep on an env's sixteen lanes (see the header comment for the split).
// (HSUB_T: pob_octet.h)
// CS: the lane's wall-contact store (HCS_FLOATS lane-minor slots of LDS, element e at CS[64 e])
template <int MW, class G>
POB_D void hpbd_substep(G &g, csys_t &S, const float *HT, const float *WT, const HWalls<MW> &HW, HBody &b,
                        const float act, v3 &cv, v3 &ca, const bool COLLIDE, float *CS,
                        unsigned long long *tacc = nullptr) {
#ifdef POB_EXP_TIMING_SUB
  unsigned long long _tl = __builtin_amdgcn_s_memtime();
#else
  (void)tacc;
#endif
  const bool isP = HT[HT_ISP] != 0.0f, hip = HT[HT_ISHIP] != 0.0f;
  const bool torso = isP && hip, leg = !isP && !hip;
  const HCon SC{HW.friction, S.inv_h};
  const v3 px = b.x;
  const q4 pq = b.q;
  // 1. acceleration level: the joint's torque tt (actuator + damping) on both of its lanes
  {
    const q4 qo = hx_pair4(b.q);
    const v3 wo = hx_pair3(b.w);
    const q4 qpj = qsel(isP, b.q, qo), qcj = qsel(isP, qo, b.q);
    const v3 wpj = vsel3(isP, b.w, wo), wcj = vsel3(isP, wo, b.w);
    const v3 axis = HTV(HT, HT_AXIS);
    const v3 a = qrot(axis, qpj);
    const bool in = actuator_inside(qpj, qcj, hip, axis, HT[HT_TLO], HT[HT_THI]);
    const v3 t = vscl(a, (in ? act : 0.0f) * HT[HT_STRENGTH]);
    const v3 d = vscl(vsub(wpj, wcj), HT[HT_DAMP]);
    const v3 tt = vadd(t, d);
    const v3 tm = hx_mirror3(tt);  // the other Aux replica's joint torque
    // torso: (((0 - t0) - t2) - t4) - t6 over the row's first quad; Aux: (0 + t_hip) - t_knee;
    // lower leg: 0 + t_knee
    const v3 t0 = quad_bcast3<0>(tt), t2 = quad_bcast3<1>(tt), t4 = quad_bcast3<2>(tt), t6 = quad_bcast3<3>(tt);
    const v3 dwt = vsub(vsub(vsub(vsub(V(0.0f, 0.0f, 0.0f), t0), t2), t4), t6);
    const v3 dwa = vsub(vadd(V(0.0f, 0.0f, 0.0f), hip ? tt : tm), hip ? tm : tt);
    const v3 dwl = vadd(V(0.0f, 0.0f, 0.0f), tt);
    const v3 dw = torso ? dwt : (leg ? dwl : dwa);
    const v3 v = b.v, w = b.w;
    b.v = V(FMA(S.lin_damp, v.x, 0.0f * S.h), FMA(S.lin_damp, v.y, 0.0f * S.h), FMA(S.lin_damp, v.z, S.gz * S.h));
    b.w = V(FMA(S.ang_damp, w.x, dw.x * S.h), FMA(S.ang_damp, w.y, dw.y * S.h), FMA(S.ang_damp, w.z, dw.z * S.h));
    // 2. kinetic
    b.x = vfma(b.v, S.h, b.x);
    const q4 dq = qmul_vq(b.w, b.q);
    q4 q = b.q;
    q.w = FMA(S.half_h, dq.w, q.w); q.x = FMA(S.half_h, dq.x, q.x);
    q.y = FMA(S.half_h, dq.y, q.y); q.z = FMA(S.half_h, dq.z, q.z);
    b.q = g.qnorm(q);
  }
  HSUB_T(0)
  // 3. position projection
  HGround gc;
  HMesh ms;
  {
    v3 DX, DA;
    {
      // the joint (oracle joints_position, the eight-lane kernel's generic form): each lane
      // rotates its own body's vectors, the partner's come over the pair DPP
      const m3 R = qmat(b.q);
      const v3 ro = mrot_xy(R, HTV(HT, HT_OFF));
      const v3 ao = mrot(R, HTV(HT, HT_AXIS)), fo = mrot(R, HTV(HT, HT_REF));
      const v3 xo = hx_pair3(b.x), rx = hx_pair3(ro), ax = hx_pair3(ao), fx = hx_pair3(fo);
      const v3 xpj = vsel3(isP, b.x, xo), xcj = vsel3(isP, xo, b.x);
      const v3 rp = vsel3(isP, ro, rx), rc = vsel3(isP, rx, ro);
      const v3 ap = vsel3(isP, ao, ax), ac = vsel3(isP, ax, ao);
      const v3 fp = vsel3(isP, fo, fx), fc = vsel3(isP, fx, fo);
      const float imp = HT[HT_IMP], imc = HT[HT_IMC];
      const v3 d = vsub(vadd(xcj, rc), vadd(xpj, rp));
      const float L2 = vdot(d, d);
      v3 P = V(0.0f, 0.0f, 0.0f), xp = P, xc = P;
      if (L2 > 0.0f) {
        const v3 ep = vcross(rp, d), ec = vcross(rc, d);
        const float den = FMA(L2, imp + imc, vdot(ep, ep) + vdot(ec, ec));
        const float k = (L2 * HW.s_pos) * g.rcp(den);
        P = vscl(d, k); xp = vscl(ep, k); xc = vscl(ec, k);
      }
      const v3 Pa = vscl(vcross(ap, ac), S.half_s_ang);
      const float psi = pob_atan2f_g(g, vdot(vcross(fp, fc), ap), vdot(fp, fc));
      float dl = 0.0f;
      if (psi < HT[HT_LO]) dl = psi - HT[HT_LO];
      else if (psi > HT[HT_HI]) dl = psi - HT[HT_HI];
      const v3 s = vadd(Pa, vscl(ap, dl * S.half_s_ang));
      const v3 tp = vadd(xp, s), tc = vadd(xc, s);
      // torso: the four hips' parent terms in joint order (the row's first quad)
      const float imp0 = S.inv_mass[0];
      v3 dxt = V(0.0f, 0.0f, 0.0f), dat = dxt;
      dxt = vfma(quad_bcast3<0>(P), imp0, dxt); dat = vadd(dat, quad_bcast3<0>(tp));
      dxt = vfma(quad_bcast3<1>(P), imp0, dxt); dat = vadd(dat, quad_bcast3<1>(tp));
      dxt = vfma(quad_bcast3<2>(P), imp0, dxt); dat = vadd(dat, quad_bcast3<2>(tp));
      dxt = vfma(quad_bcast3<3>(P), imp0, dxt); dat = vadd(dat, quad_bcast3<3>(tp));
      // Aux: the hip's child term, then the knee's parent term (each replica sends its P
      // and its own side's term over the row mirror)
      const v3 Pm = hx_mirror3(P), Tm = hx_mirror3(isP ? tp : tc);
      const float ima = HT[HT_IM];
      const v3 Phip = hip ? P : Pm, Pknee = hip ? Pm : P;
      const v3 Thip = hip ? tc : Tm, Tknee = hip ? Tm : tp;
      const v3 dxa = vfma(Pknee, ima, vfma(Phip, -ima, V(0.0f, 0.0f, 0.0f)));
      const v3 daa = vadd(vsub(V(0.0f, 0.0f, 0.0f), Thip), Tknee);
      // lower leg: the knee's child term
      const v3 dxl = vfma(P, -imc, V(0.0f, 0.0f, 0.0f));
      const v3 dal = vsub(V(0.0f, 0.0f, 0.0f), tc);
      DX = torso ? dxt : (leg ? dxl : dxa);
      DA = torso ? dat : (leg ? dal : daa);
    }
    HSUB_T(1)
    if (COLLIDE) {
      hcontacts_position<MW>(g, SC, HT, WT, HW, torso, b, px, pq, gc, ms, DX, DA, CS
#ifdef POB_EXP_TIMING_SUB
                             , tacc
#endif
      );
      HSUB_T(4)
    }
    b.x = vadd(b.x, DX);
    qadd_half(b.q, qmul_vq(DA, b.q), 1.0f);
  }
  HSUB_T(2)
  // 4. velocity projection
  b.q = g.qnorm(b.q);
  b.v = vscl(vsub(b.x, px), S.inv_h);
  {
    const q4 dq = qmul(b.q, qinv(pq));
    const float k2 = 2.0f * S.inv_h;
    const float kw = dq.w >= 0.0f ? k2 : -k2;
    b.w = V(dq.x * kw, dq.y * kw, dq.z * kw);
  }
  HSUB_T(6)
  // 5. velocity-level contacts (ground first, then wall: the oracle's per-body order)
  if (COLLIDE) {
    v3 dV = V(0.0f, 0.0f, 0.0f), dW = dV;
    hcontacts_velocity<MW>(g, SC, HT, WT, HW, torso, b, gc, ms, dV, dW, CS);
    HSUB_T(7)
    b.v = vadd(b.v, dV); b.w = vadd(b.w, dW);
    cv = vadd(cv, dV);
    ca = vadd(ca, dW);
  }
  HSUB_T(3)
}
