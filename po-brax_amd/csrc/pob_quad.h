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

// The wave's LDS region (QL_FLOATS x 64 floats; the obs / qp staging area between steps):
// * lane-minor per-lane slots of the lane's own bodies (Aux k+1, lower leg): substep-start pose
//   (7 floats each) and Info.contact accumulators (6 each), and the head of the lane's wall
//   contact list (QLL_*; element e of lane t at base[64 e + t]);
// * the torso's pose and accumulators once per lane quad (QLT_*; element e of quad j at
//   base[64 QLL_FLOATS + 16 e + j]): the four lanes' torso replicas are bit-identical, lane
//   k = 0 writes them, all four read (a broadcast);
// * the wave's wall-contact pool (QPOOL_N contacts of 6 floats) of the fast launch: each
//   collide substep's contacts in walk order, a list per lane (round 6: the four-lane kernel's
//   per-lane contact array lived in scratch -- 384 B/lane, reads at 2.25x the algorithmic bytes).
#define QLL_PX(l) (7 * ((l) - 1))       // l = 1, 2
#define QLL_PQ(l) (7 * ((l) - 1) + 3)
#define QLL_CV(l) (14 + 6 * ((l) - 1))
#define QLL_CA(l) (14 + 6 * ((l) - 1) + 3)
#define QLL_HEAD 26
#define QLL_FLOATS 27
#define QLT_PX 0
#define QLT_PQ 3
#define QLT_CV 7
#define QLT_CA 10
#define QLT_FLOATS 13
#define QL_FLOATS 39
#define QPOOL_OFF (QLL_FLOATS * 64 + QLT_FLOATS * 16)
#define QPOOL_N ((QL_FLOATS * 64 - QPOOL_OFF) / 6)
static_assert(QPOOL_N >= 64, "the contact pool holds at least one contact per lane");
// field codes of a body's slots
#define QF_PX 0
#define QF_PQ 1
#define QF_CV 2
#define QF_CA 3
struct QLds {
  float *base;  // the wave's region
  int t;        // the lane
  POB_D static constexpr int lane_off(int l, int f) {
    return f == QF_PX ? QLL_PX(l) : (f == QF_PQ ? QLL_PQ(l) : (f == QF_CV ? QLL_CV(l) : QLL_CA(l)));
  }
  POB_D static constexpr int torso_off(int f) {
    return f == QF_PX ? QLT_PX : (f == QF_PQ ? QLT_PQ : (f == QF_CV ? QLT_CV : QLT_CA));
  }
  // element i of field f of local body l (torso: the quad's slot)
  POB_D float *at(int l, int f, int i) const {
    return l == 0 ? base + 64 * QLL_FLOATS + 16 * (torso_off(f) + i) + (t >> 2) : base + 64 * (lane_off(l, f) + i) + t;
  }
  POB_D v3 get3(int l, int f) const { return V(*at(l, f, 0), *at(l, f, 1), *at(l, f, 2)); }
  POB_D q4 get4(int l, int f) const {
    q4 q; q.w = *at(l, f, 0); q.x = *at(l, f, 1); q.y = *at(l, f, 2); q.z = *at(l, f, 3); return q;
  }
  POB_D void set3(int l, int f, v3 v) const {
    if (l != 0 || (t & 3) == 0) { *at(l, f, 0) = v.x; *at(l, f, 1) = v.y; *at(l, f, 2) = v.z; }
  }
  POB_D void set4(int l, int f, q4 q) const {
    if (l != 0 || (t & 3) == 0) { *at(l, f, 0) = q.w; *at(l, f, 1) = q.x; *at(l, f, 2) = q.y; *at(l, f, 3) = q.z; }
  }
  // body l's (l >= 1) accumulator of another lane of the wave
  POB_D v3 get3_lane(int l, int f, int lane) const {
    const float *p = base + 64 * lane_off(l, f) + lane;
    return V(p[0], p[64], p[128]);
  }
  POB_D float *head() const { return base + 64 * QLL_HEAD + t; }
  POB_D float *pool() const { return base + QPOOL_OFF; }
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

// ---------------------------------------------------------------------- contacts
// Ground (collide_include Ant x Ground: CapsulePlane on the torso and the lower leg):
// [0] torso, [1] lower leg; pe = the sphere centre x + rotate(end, q) at detection.
struct QGround {
  float pen[2];
};
// The lane's bodies' capsule segments at one pose -- a = x + rotate(e0, q), b = x - rotate(e0, q)
// (torso: the sphere centre a) -- for the face cull and the static (sys.info / legacy) walk.
struct QMesh {
  v3 a[QNB], b[QNB];
};
// The lane's wall contacts of a collide substep (pob_mesh.h, brax capsule x TriangulatedBox):
// the detection (before the joint projection, at the pose the position pass projects from)
// walks the lane's face items -- M[l] bit 8 w + f per body l -- with each segment formed from
// that pose when the walk needs it, and keeps the first QK contacts (body, tau, n, dist) in a
// private array in walk order; the position and velocity passes apply them from there.  A lane
// with more keeps its detection-time segments instead (a second private array, written only
// then) and both passes re-walk every face the cull keeps from them (qwalls_rewalk_inl) -- the
// same operations on the same operands: the same contacts in the same order.  Nothing of this
// is live in registers between the passes but the count.
#ifndef QK
#define QK 12  // (8: HH B = 65 536 0.2038 ms with the split launch, 12: 0.1634 -- fewer fix-up waves; 16, 24: the same; profiles/r6c_ab.txt)
#endif
struct QWalls {
  int nct;                // wall contacts of the position pass
  float c[6 * QK];        // the first QK: body, tau, n, dist (the re-walk builds, OVF)
  float seg[6 * QNB];     // nct > QK only: the segments a, b of the three bodies
};
#ifndef POB_QUAD_WAVE_WALK
#define POB_QUAD_WAVE_WALK 1  // 1: the wave-cooperative face walk (pob_mesh.h mesh_wave_walk)
#endif
#if POB_QUAD_WAVE_WALK
#define QWALK mesh_wave_walk
#else
#define QWALK mesh_lane_walk
#endif

// The Ant's capsules (checked by pob_system.cpp) have opposite end points +-e0 in the body
// xy-plane, so one rotation rv = rotate(e0, q) serves both (rotate(-e0) = -rv exactly), and a
// lower leg's ground point is its end 1 (x - rv).  The torso sphere's points are its centre x.
POB_D void qground_detect(csys_t &S, const float *LT, const QBody &b, const v3 rv_leg, QGround &gc, v3 (&pe)[2]) {
  pe[0] = S.torso_point ? b.x[0] : vadd(b.x[0], qrot(qground_end(S, LT, 0), b.q[0]));
  pe[1] = vsub(b.x[2], rv_leg);
  gc.pen[0] = qground_r(S, LT, 0) - pe[0].z;
  gc.pen[1] = qground_r(S, LT, 1) - pe[1].z;
}

// broadphase: bit w set iff wall w's grown box (pob_sys::wall_lo/hi: capsule reach + 2e-3)
// meets the xy AABB of the lane's three body centres -- a wall outside it has every face
// culled for every body of the lane (gap > r + 1e-3), so skipping it changes nothing
POB_D uint32_t qwall_mask(csys_t &S, const QBody &b) {
  float mnx = b.x[0].x, mxx = b.x[0].x, mny = b.x[0].y, mxy = b.x[0].y;
#pragma unroll
  for (int l = 1; l < QNB; ++l) {
    mnx = fminf(mnx, b.x[l].x); mxx = fmaxf(mxx, b.x[l].x);
    mny = fminf(mny, b.x[l].y); mxy = fmaxf(mxy, b.x[l].y);
  }
#ifdef POB_EXP_NO_WALLS
  const int nw = 0;  // timing experiment only
#else
  const int nw = S.n_walls;
#endif
  uint32_t m = 0u;
#pragma unroll
  for (int w = 0; w < POB_MAXW; ++w) {
    // all POB_MAXW boxes loaded at once, w < nw as a predicate
    const float lx = S.wall_lo[w][0], ly = S.wall_lo[w][1], hx = S.wall_hi[w][0], hy = S.wall_hi[w][1];
    const bool near = (mnx <= hx) & (mxx >= lx) & (mny <= hy) & (mxy >= ly);
    m |= (near & (w < nw)) ? 1u << w : 0u;
  }
  return m;
}

// the broadphase with every wall box grown by a further margin (the wave's choice of pass at
// the start of a step: a lane whose grown mask is empty is unlikely to meet a wall's
// broadphase during the step)
POB_D uint32_t qwall_mask_margin(csys_t &S, const QBody &b, const float margin) {
  float mnx = b.x[0].x, mxx = b.x[0].x, mny = b.x[0].y, mxy = b.x[0].y;
#pragma unroll
  for (int l = 1; l < QNB; ++l) {
    mnx = fminf(mnx, b.x[l].x); mxx = fmaxf(mxx, b.x[l].x);
    mny = fminf(mny, b.x[l].y); mxy = fmaxf(mxy, b.x[l].y);
  }
  const int nw = S.n_walls;
  uint32_t m = 0u;
#pragma unroll
  for (int w = 0; w < POB_MAXW; ++w) {
    const float lx = S.wall_lo[w][0] - margin, ly = S.wall_lo[w][1] - margin;
    const float hx = S.wall_hi[w][0] + margin, hy = S.wall_hi[w][1] + margin;
    const bool near = (mnx <= hx) & (mxx >= lx) & (mny <= hy) & (mxy >= ly);
    m |= (near & (w < nw)) ? 1u << w : 0u;
  }
  return m;
}

// the lane's bodies' capsule segments (a, b) (torso: a = b = x)
POB_D void qmesh_segments(csys_t &S, const float *LT, const QBody &b, const v3 rv_leg, QMesh &ms) {
  const v3 rv1 = qrot_xy(qcap_end(S, LT, 1, 0), b.q[1]);
  ms.a[0] = b.x[0]; ms.b[0] = b.x[0];
  ms.a[1] = vadd(b.x[1], rv1); ms.b[1] = vsub(b.x[1], rv1);
  ms.a[2] = vadd(b.x[2], rv_leg); ms.b[2] = vsub(b.x[2], rv_leg);
}
// x + tau rotate(e0, q) of local body l (l = 1, 2; the torso's point is x)
POB_D v3 qseg_point(const float *LT, const int l, const v3 x, const q4 q, const float tau) {
  const float *e = LT + POB_LEG_BODY(l) + 2;
  return vfma(qrot_xy(V(e[0], e[1], e[2]), q), tau, x);
}

// face items of the lane's bodies: M[l] bit 8 w + f for every face f of a wall w that the
// face cull keeps for body l, over the walls of wm (bit 8 l + w: body l's walls; walls walked
// per lane in increasing order)
POB_D void qmesh_items(csys_t &S, const float *LT, const float *WT, const uint32_t wm, const QMesh &ms,
                       uint64_t (&M)[QNB]) {
#pragma unroll
  for (int l = 0; l < QNB; ++l) M[l] = 0ull;
  const float cz = S.wall_cz, hz = S.wall_hz;
  uint32_t m = (wm | (wm >> 8) | (wm >> 16)) & 0xFFu;
  while (__any(m != 0u)) {
    const bool on = m != 0u;
    const int w = on ? __builtin_ctz(m) : 0;
    m &= m - 1u;
    const MWall W = mwall_row(WT + POB_WALL_FLOATS * w);
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      const float R = (l == 0 ? S.cap_r[0] : LT[POB_LEG_BODY(l) + 1]) + POB_MESH_MARGIN;
      const v3 La = mwall_local(W, cz, ms.a[l]);
      const v3 Lb = l == 0 ? La : mwall_local(W, cz, ms.b[l]);
      const uint32_t fm = mesh_face_mask(La, Lb, W.hx, W.hy, hz, R);
      M[l] |= (on && ((wm >> (8 * l + w)) & 1u)) ? (uint64_t)fm << (8 * w) : 0ull;
    }
  }
}

// the walk's view of the lane's bodies: body l's segment, radius and kind (the torso is the
// sphere at its centre).  (Round 4 walked per lane here -- the cooperative walk measured slower
// at four waves per SIMD when its registers pushed the substep's spills up, profiles/r4h; round 5
// made it call-free and spill-free, and the cooperative walk is the four-lane kernel's walk:
// DESIGN.md §4 "Round-5 findings".)
POB_D void qmesh_seg(csys_t &S, const float *LT, const QMesh &ms, const int l, v3 &A, v3 &B, float &r, bool &seg) {
  A = vsel3(l == 0, ms.a[0], vsel3(l == 1, ms.a[1], ms.a[2]));
  B = vsel3(l == 0, ms.b[0], vsel3(l == 1, ms.b[1], ms.b[2]));
  r = l == 0 ? S.cap_r[0] : LT[POB_LEG_BODY(l) + 1];
  seg = l != 0;
}

// body l's value among the lane's three (selects: a runtime index into a register array
// would become a private array in scratch)
POB_D v3 qpick3(const int l, const v3 (&a)[QNB]) { return vsel3(l == 0, a[0], vsel3(l == 1, a[1], a[2])); }
POB_D q4 qpick4(const int l, const q4 (&a)[QNB]) { return qsel(l == 0, a[0], qsel(l == 1, a[1], a[2])); }
POB_D void qput3(const int l, v3 (&a)[QNB], const v3 v) {
  a[0] = vsel3(l == 0, v, a[0]); a[1] = vsel3(l == 1, v, a[1]); a[2] = vsel3(l == 2, v, a[2]);
}

// body l's segment formed from the pose (x, q): qmesh_segments' operations for one body
POB_D void qpose_seg(csys_t &S, const float *LT, const QBody &b, const int l, v3 &A, v3 &B, float &r, bool &seg) {
  const v3 x = qpick3(l, b.x);
  const v3 rv = qrot_xy(qcap_end(S, LT, l == 0 ? 1 : l, 0), qpick4(l, b.q));
  A = l == 0 ? x : vadd(x, rv);
  B = l == 0 ? x : vsub(x, rv);
  r = l == 0 ? S.cap_r[0] : LT[POB_LEG_BODY(l) + 1];
  seg = l != 0;
}

// The face walk of the detection: the cooperative walk (every lane of the wave is active in
// the substeps, step_quad_body) or, in the per-lane build (POB_QUAD_WAVE_WALK 0), each lane's
// own walk out of line (qwalls_walk_ool).  The contacts go to the lane's store.
template <bool LANE>
POB_D void qwalls_walk(csys_t &S, const float *LT, const float *WT, const QBody &b, uint64_t (&M)[QNB], QWalls &ws) {
  GuardBranch g;
#if POB_QUAD_WAVE_WALK
  if (!LANE) {
    mesh_wave_walk<QNB, false>(g, WT, pob_face_table(S), S.wall_cz, S.wall_hz, M,
               [&](const int l, v3 &A, v3 &B, float &r, bool &seg) { qpose_seg(S, LT, b, l, A, B, r, seg); },
               [&](const int l, const int, const float tau, const v3 n, const float dist) {
      if (ws.nct < QK) {
        float *c = ws.c + 6 * ws.nct;
        c[0] = (float)l; c[1] = tau; c[2] = n.x; c[3] = n.y; c[4] = n.z; c[5] = dist;
      }
      ++ws.nct;
    });
    return;
  }
#endif
  mesh_lane_walk<QNB>(g, WT, pob_face_table(S), S.wall_cz, S.wall_hz, M,
             [&](const int l, v3 &A, v3 &B, float &r, bool &seg) { qpose_seg(S, LT, b, l, A, B, r, seg); },
             [&](const int l, const int, const float tau, const v3 n, const float dist) {
    if (ws.nct < QK) {
      float *c = ws.c + 6 * ws.nct;
      c[0] = (float)l; c[1] = tau; c[2] = n.x; c[3] = n.y; c[4] = n.z; c[5] = dist;
    }
    ++ws.nct;
  });
}
// (the per-lane build's walk, out of line: POB_QUAD_WAVE_WALK 0)
__device__ __attribute__((noinline)) int qwalls_walk_ool(csys_t *Sp, const float *LT, const float *WT, v3 x0, v3 x1,
                                                       v3 x2, q4 q0, q4 q1, q4 q2, uint64_t m0, uint64_t m1,
                                                       uint64_t m2, QWalls *ws) {
  csys_t &S = *launder(Sp);
  QBody b;
  b.x[0] = x0; b.x[1] = x1; b.x[2] = x2;
  b.q[0] = q0; b.q[1] = q1; b.q[2] = q2;
  uint64_t M[QNB] = {m0, m1, m2};
  ws->nct = 0;
  qwalls_walk<true>(S, LT, WT, b, M, *ws);
  return ws->nct;
}

// The fast launch's walk (OVF false): the contacts go to the wave's LDS pool (QLds) in walk
// order -- each hand-over step allocates the pool slots of the lanes receiving a contact by
// ballot / mbcnt, and a lane links its contacts into a list (head in its LDS slot, each entry's
// last float = body | (next + 1) << 2) -- so the passes read them from LDS instead of a private
// array in scratch.  A wave whose contacts exceed the pool reports it in ovf (the fix-up launch
// then steps it with the re-walks).
// (POB_QUAD_POOL_DIRECT, the default: the winner lanes store the contacts and the owners only
// link them -- pob_mesh.h mesh_wave_walk HAND 2)
#ifndef POB_QUAD_POOL_DIRECT
#define POB_QUAD_POOL_DIRECT 1
#endif
struct QPoolSink {
  float *pool;
  float *head;
  int npool;  // (wave-uniform)
  int tail, tail_l, nct;
  POB_D int store(const bool hit, const float tau, const v3 n, const float dist) {
    const uint64_t m = __ballot(hit);
    const int idx = npool + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    npool += __popcll(m);
    if (hit && idx < QPOOL_N) {
      float *c = pool + 6 * idx;
      c[0] = tau; c[1] = n.x; c[2] = n.y; c[3] = n.z; c[4] = dist;
    }
    return hit ? idx + 1 : 0;  // (past the pool: counted, never stored -- the wave goes to the fix-up launch)
  }
  POB_D void link(const int l, const int, const int e) {
    if (e > 0) {
      const int idx = e - 1;
      ++nct;
      if (idx < QPOOL_N) {
        pool[6 * idx + 5] = __int_as_float(l);
        if (tail >= 0) pool[6 * tail + 5] = __int_as_float(((idx + 1) << 2) | tail_l);
        else *head = __int_as_float(idx);
        tail = idx;
        tail_l = l;
      }
    }
  }
};
// (POB_QUAD_WALK_GACC, an A/B switch: the walk's range guards branch-free, GuardAcc -- a lane
// that saw an operand outside the fast forms' range sends its wave to the fix-up launch, whose
// exact branch guards give the same bits for every lane that stayed in range.  Measured HH
// B = 65 536 0.1509 -> 0.1546 ms, TAG ±0 (profiles/r7m/ab.txt): off)
#ifndef POB_QUAD_WALK_GACC
#define POB_QUAD_WALK_GACC 0
#endif
POB_D void qwalls_walk_pool(csys_t &S, const float *LT, const float *WT, const QBody &b, uint64_t (&M)[QNB],
                            QWalls &ws, const QLds &L, bool &ovf) {
#if POB_QUAD_WALK_GACC
  GuardAcc g;
#else
  GuardBranch g;
#endif
#if POB_QUAD_POOL_DIRECT
  QPoolSink sink{L.pool(), L.head(), 0, -1, 0, 0};
  mesh_wave_walk<QNB, false, 2>(g, WT, pob_face_table(S), S.wall_cz, S.wall_hz, M,
             [&](const int l, v3 &A, v3 &B, float &r, bool &seg) { qpose_seg(S, LT, b, l, A, B, r, seg); }, sink);
  ws.nct += sink.nct;
  ovf = ovf | (sink.npool > QPOOL_N);
#if POB_QUAD_WALK_GACC
  ovf = ovf | g.bad();
#endif
  return;
#endif
  float *pool = L.pool();
  int npool = 0;  // (wave-uniform)
  int tail = -1, tail_l = 0;
  mesh_wave_walk<QNB, false, 1>(g, WT, pob_face_table(S), S.wall_cz, S.wall_hz, M,
             [&](const int l, v3 &A, v3 &B, float &r, bool &seg) { qpose_seg(S, LT, b, l, A, B, r, seg); },
             [&](const bool want, const int l, const int, const float tau, const v3 n, const float dist) {
    const uint64_t m = __ballot(want);
    if (m == 0ull) return;
    const int idx = npool + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    npool += __popcll(m);
    if (want) {
      if (idx < QPOOL_N) {
        float *c = pool + 6 * idx;
        c[0] = tau; c[1] = n.x; c[2] = n.y; c[3] = n.z; c[4] = dist; c[5] = __int_as_float(l);
        if (tail >= 0) pool[6 * tail + 5] = __int_as_float(((idx + 1) << 2) | tail_l);
        else *L.head() = __int_as_float(idx);
        tail = idx;
        tail_l = l;
      }
      ++ws.nct;
    }
  });
  ovf = ovf | (npool > QPOOL_N);
}

// Wall contact detection of a collide substep, at the pose the position pass projects from
// (after the kinetic update, before the joint projection: the face walk's working set then
// meets only the pose -- the velocities are dead until the velocity projection rewrites them,
// the corrections not yet live).  The contacts (body, tau, n, dist) go to the store in walk
// order (per body the oracle's (wall, face, triangle) order); a lane with more than QK keeps
// its segments for the re-walks of the position and velocity passes (qwalls_rewalk_inl).
// OVF false (the fast wall pass): a lane with more contacts than the store holds only reports
// it in *ovf (the wave then runs the step again in the slow pass, OVF true: the detection-time
// segments kept for the re-walks)
template <bool WALLS, bool OVF = true>
POB_D void qwalls_detect(csys_t *Sp, const float *LT, const float *WT, const QBody &b, QWalls &ws, const QLds &L,
                         bool *ovf = nullptr) {
  ws.nct = 0;
  if (!WALLS) return;
  csys_t &S = *launder(Sp);
  const v3 rv_leg = qrot_xy(qcap_end(S, LT, 2, 0), b.q[2]);
  uint64_t M[QNB];
  {
    QMesh ms;
    qmesh_segments(S, LT, b, rv_leg, ms);
    const uint32_t lw = qwall_mask(S, b);
    qmesh_items(S, LT, WT, lw | (lw << 8) | (lw << 16), ms, M);
  }
#ifdef POB_EXP_NO_WALK
  return;  // timing experiment only: broadphase and face cull, no face walk
#endif
#ifdef POB_EXP_WALK_DEAD
  if (S.n_walls < 64) return;  // timing experiment only: the walk compiled in, never run
#endif
#ifdef POB_EXP_CULL_ONLY
  {  // timing experiment only: the cull's items kept alive, no walk, the passes compiled in
    uint32_t k0 = (uint32_t)M[0], k1 = (uint32_t)M[1], k2 = (uint32_t)M[2];
    asm volatile("" : "+v"(k0), "+v"(k1), "+v"(k2));
    int z = (int)((k0 ^ k1 ^ k2) & 0u);
    asm volatile("" : "+v"(z));
    ws.nct = z;
    return;
  }
#endif
  if (!__any((M[0] | M[1] | M[2]) != 0ull)) return;
#if POB_QUAD_WAVE_WALK
  // (the step kernel runs its substeps on all 64 lanes of every wave: step_quad_body)
  if (!OVF) {
    qwalls_walk_pool(S, LT, WT, b, M, ws, L, *ovf);
    return;
  }
  qwalls_walk<false>(S, LT, WT, b, M, ws);
#else
  ws.nct = qwalls_walk_ool(Sp, LT, WT, b.x[0], b.x[1], b.x[2], b.q[0], b.q[1], b.q[2], M[0], M[1], M[2], &ws);
#endif
#ifdef POB_EXP_NO_APPLY
  {  // timing experiment only: the walk runs, its contacts are not applied
    int z = ws.nct & 0;
    asm volatile("" : "+v"(z));
    ws.nct = z;
  }
#endif
  if (!OVF) {
    *ovf = *ovf | (ws.nct > QK);
    return;
  }
  if (ws.nct > QK) {  // (rare) the detection-time segments for the re-walks
    QMesh ms;
    qmesh_segments(S, LT, b, rv_leg, ms);
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      ws.seg[6 * l] = ms.a[l].x; ws.seg[6 * l + 1] = ms.a[l].y; ws.seg[6 * l + 2] = ms.a[l].z;
      ws.seg[6 * l + 3] = ms.b[l].x; ws.seg[6 * l + 4] = ms.b[l].y; ws.seg[6 * l + 5] = ms.b[l].z;
    }
  }
}

// One wall contact applied at the position level (penetration r - dist, the contact at the
// triangle point pe - (1e-6 + dist) n) / at the velocity level (at the post-projection pose)
template <class G>
POB_D void qwall_pos_one(G &g, csys_t &S, const HCon &SC, const float *LT, const v3 (&x)[QNB], const q4 (&q)[QNB],
                         const v3 (&px)[QNB], const q4 (&pq)[QNB], const int l, const float tau, const v3 n,
                         const float dist, v3 (&DX)[QNB], v3 (&DA)[QNB]) {
  const v3 xl = qpick3(l, x);
  const q4 ql = qpick4(l, q);
  const v3 pe = l == 0 ? xl : qseg_point(LT, l, xl, ql, tau);
  v3 dx = qpick3(l, DX), da = qpick3(l, DA);
  owall_position(g, SC, q_cap_r(S, LT, l) - dist, pe, n, 1e-6f + dist, q_inv_mass(S, LT, l), xl, ql, qpick4(l, pq),
                 qpick3(l, px), dx, da);
  qput3(l, DX, dx);
  qput3(l, DA, da);
}
template <class G>
POB_D void qwall_vel_one(G &g, csys_t &S, const HCon &SC, const float *LT, const v3 (&x)[QNB], const q4 (&q)[QNB],
                         const v3 (&v)[QNB], const v3 (&w)[QNB], const int l, const float tau, const v3 n,
                         const float dist, v3 (&dV)[QNB], v3 (&dW)[QNB]) {
  const v3 xl = qpick3(l, x);
  const v3 pe = l == 0 ? xl : qseg_point(LT, l, xl, qpick4(l, q), tau);
  v3 dv = qpick3(l, dV), dw = qpick3(l, dW);
  ocontact_vel_pe(g, SC, false, q_cap_r(S, LT, l) - dist, pe, n, 1e-6f + dist, q_inv_mass(S, LT, l), xl, qpick3(l, v),
                  qpick3(l, w), dv, dw);
  qput3(l, dV, dv);
  qput3(l, dW, dw);
}

// The re-walk of a lane whose contacts overflowed the store (rare), out of line so that the
// walk's registers stay out of the position and velocity passes: every face the cull keeps
// over every wall, from the detection-time segments (the broadphase only skips walls whose
// faces are all culled), each contact applied in walk order.  State through a private block.
struct QOvf {
  v3 x[QNB], px[QNB], v[QNB], w[QNB], a[QNB], b[QNB], d0[QNB], d1[QNB];
  q4 q[QNB], pq[QNB];
  float fric;
  int on;
};
template <bool VEL>
__device__ __attribute__((noinline)) void qwalls_rewalk(csys_t *Sp, const float *LT, const float *WT, QOvf *st) {
  csys_t &S = *launder(Sp);
  GuardBranch g;
  const HCon SC{st->fric, S.inv_h};
  v3 x[QNB], px[QNB], v[QNB], w[QNB], d0[QNB], d1[QNB];
  q4 q[QNB], pq[QNB];
  QMesh ms;
#pragma unroll
  for (int l = 0; l < QNB; ++l) {
    x[l] = st->x[l]; px[l] = st->px[l]; v[l] = st->v[l]; w[l] = st->w[l]; d0[l] = st->d0[l]; d1[l] = st->d1[l];
    q[l] = st->q[l]; pq[l] = st->pq[l]; ms.a[l] = st->a[l]; ms.b[l] = st->b[l];
  }
  const uint32_t wa = st->on ? (1u << S.n_walls) - 1u : 0u;
  uint64_t M[QNB];
  qmesh_items(S, LT, WT, wa | (wa << 8) | (wa << 16), ms, M);
  QWALK<QNB>(g, WT, pob_face_table(S), S.wall_cz, S.wall_hz, M,
             [&](const int l, v3 &A, v3 &B, float &r, bool &seg) { qmesh_seg(S, LT, ms, l, A, B, r, seg); },
             [&](const int l, const int, const float tau, const v3 n, const float dist) {
    if (VEL) qwall_vel_one(g, S, SC, LT, x, q, v, w, l, tau, n, dist, d0, d1);
    else qwall_pos_one(g, S, SC, LT, x, q, px, pq, l, tau, n, dist, d0, d1);
  });
#pragma unroll
  for (int l = 0; l < QNB; ++l) { st->d0[l] = d0[l]; st->d1[l] = d1[l]; }
}

// The same re-walk inline (POB_QUAD_REWALK_INLINE, the default): the wave-cooperative walk
// with no lane fallback (the step kernel's substeps run on all 64 lanes) and no call -- a call
// site in the pass, however rarely taken, confines every value live across it to the
// callee-saved registers, which spilled the substep's state at every collide substep.  The
// segments come from the store, the substep-start pose (position pass) from LDS.
#ifndef POB_QUAD_REWALK_INLINE
#define POB_QUAD_REWALK_INLINE 1
#endif
template <bool VEL>
POB_D void qwalls_rewalk_inl(csys_t &S, const float *LT, const float *WT, const QBody &b, const QLds &L,
                             const QWalls &ws, const bool ovf, const float fric, v3 (&d0)[QNB], v3 (&d1)[QNB]) {
  GuardBranch g;
  const HCon SC{fric, S.inv_h};
  QMesh ms;
#pragma unroll
  for (int l = 0; l < QNB; ++l) {
    ms.a[l] = V(ws.seg[6 * l], ws.seg[6 * l + 1], ws.seg[6 * l + 2]);
    ms.b[l] = V(ws.seg[6 * l + 3], ws.seg[6 * l + 4], ws.seg[6 * l + 5]);
  }
  const uint32_t wa = ovf ? (1u << S.n_walls) - 1u : 0u;
  uint64_t M[QNB];
  qmesh_items(S, LT, WT, wa | (wa << 8) | (wa << 16), ms, M);
  mesh_wave_walk<QNB, false>(g, WT, pob_face_table(S), S.wall_cz, S.wall_hz, M,
             [&](const int l, v3 &A, v3 &B, float &r, bool &seg) { qmesh_seg(S, LT, ms, l, A, B, r, seg); },
             [&](const int l, const int, const float tau, const v3 n, const float dist) {
    if constexpr (VEL) {
      qwall_vel_one(g, S, SC, LT, b.x, b.q, b.v, b.w, l, tau, n, dist, d0, d1);
    } else {
      v3 px[QNB];
      q4 pq[QNB];
#pragma unroll
      for (int k = 0; k < QNB; ++k) { px[k] = L.get3(k, QF_PX); pq[k] = L.get4(k, QF_PQ); }
      qwall_pos_one(g, S, SC, LT, b.x, b.q, px, pq, l, tau, n, dist, d0, d1);
    }
  });
}

// Position pass of a collide substep: ground contacts (ground first per body, oracle order),
// then the wall contacts from the store in detection order
template <bool WALLS, bool OVF = true>
POB_D void qcontacts_position(csys_t *Sp, const float *LT, const float *WT, QBody &b, const QLds &L, QGround &gc,
                              const QWalls &ws, v3 (&DX)[QNB], v3 (&DA)[QNB], const float fric) {
  csys_t &S = *launder(Sp);
  const HCon SC{fric, S.inv_h};
  GuardBranch g;
  {
    const v3 rv_leg = qrot_xy(qcap_end(S, LT, 2, 0), b.q[2]);
    v3 pe[2];
    qground_detect(S, LT, b, rv_leg, gc, pe);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      POB_FENCE();
      const int l = qcontact_body(c);
      if (gc.pen[c] > 0.0f)
        oground_position(g, SC, gc.pen[c], pe[c], qground_r(S, LT, c), q_inv_mass(S, LT, l), b.x[l], b.q[l],
                         L.get4(l, QF_PQ), L.get3(l, QF_PX), DX[l], DA[l]);
    }
  }
  if (!WALLS || !__any(ws.nct != 0)) return;
  POB_FENCE();
  v3 px[QNB];
  q4 pq[QNB];
#pragma unroll
  for (int l = 0; l < QNB; ++l) { px[l] = L.get3(l, QF_PX); pq[l] = L.get4(l, QF_PQ); }
#if POB_QUAD_WAVE_WALK
  if (!OVF) {  // the fast pass: the lane's list in the wave's pool (a wave with an overflow runs the step again)
    const float *pool = L.pool();
    int ci = ws.nct > 0 ? __float_as_int(*L.head()) : -1;
#pragma unroll 1
    while (__any(ci >= 0)) {
      if (ci >= 0) {
        const float *c = pool + 6 * ci;
        const int meta = __float_as_int(c[5]);
        qwall_pos_one(g, S, SC, LT, b.x, b.q, px, pq, meta & 3, c[0], V(c[1], c[2], c[3]), c[4], DX, DA);
        ci = (meta >> 2) - 1;
      }
    }
    return;
  }
#endif
  const bool ovf = ws.nct > QK;
  const int nc = ovf ? 0 : ws.nct;
#pragma unroll 1
  for (int i = 0; i < QK; ++i) {
    if (!__any(i < nc)) break;
    if (i < nc) {
      const float *c = ws.c + 6 * i;
      qwall_pos_one(g, S, SC, LT, b.x, b.q, px, pq, (int)c[0], c[1], V(c[2], c[3], c[4]), c[5], DX, DA);
    }
  }
  if (!OVF) return;  // (the fast pass: a wave with an overflow runs the step again)
#if POB_QUAD_REWALK_INLINE
#ifndef POB_EXP_NO_REWALK
  if (__any(ovf)) qwalls_rewalk_inl<false>(S, LT, WT, b, L, ws, ovf, fric, DX, DA);  // (timing experiment: off)
#endif
  if (false) {
#else
  if (__any(ovf)) {
#endif
    QOvf st;
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      st.x[l] = b.x[l]; st.q[l] = b.q[l]; st.px[l] = px[l]; st.pq[l] = pq[l]; st.d0[l] = DX[l]; st.d1[l] = DA[l];
      st.a[l] = V(ws.seg[6 * l], ws.seg[6 * l + 1], ws.seg[6 * l + 2]);
      st.b[l] = V(ws.seg[6 * l + 3], ws.seg[6 * l + 4], ws.seg[6 * l + 5]);
    }
    st.fric = fric;
    st.on = ovf ? 1 : 0;
    qwalls_rewalk<false>(Sp, LT, WT, &st);
    // everything live after the call comes back from the block (the callee leaves the pose as
    // it is), so nothing of the pass is live across the call: the call's clobbers then cost no
    // spills of the substep's state (they would fall in every substep, not only on overflow)
#pragma unroll
    for (int l = 0; l < QNB; ++l) { DX[l] = st.d0[l]; DA[l] = st.d1[l]; b.x[l] = st.x[l]; b.q[l] = st.q[l]; }
  }
}

// Velocity pass: ground contacts, then the wall contacts from the store (contact points
// x + tau rotate(e0, q) at the post-projection pose)
template <bool WALLS, bool OVF = true>
POB_D void qcontacts_velocity(csys_t *Sp, const float *LT, const float *WT, QBody &b, const QGround &gc,
                              const QWalls &ws, const QLds &L, v3 (&dV)[QNB], v3 (&dW)[QNB], const float fric) {
  csys_t &S = *launder(Sp);
  const HCon SC{fric, S.inv_h};
  GuardBranch g;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    POB_FENCE();
    const int l = qcontact_body(c);
    if (gc.pen[c] > 0.0f) {
      const v3 e = qground_end(S, LT, c);
      const v3 pe = l == 0 ? vadd(b.x[0], qrot(e, b.q[0])) : vadd(b.x[l], qrot_xy(e, b.q[l]));
      ocontact_vel_pe(g, SC, true, gc.pen[c], pe, V(0.0f, 0.0f, 1.0f), qground_r(S, LT, c), q_inv_mass(S, LT, l), b.x[l],
                      b.v[l], b.w[l], dV[l], dW[l]);
    }
  }
  if (!WALLS || !__any(ws.nct != 0)) return;
#ifdef POB_EXP_NO_VWALK
  return;  // timing experiment only: no velocity-pass wall contacts
#endif
  POB_FENCE();
#if POB_QUAD_WAVE_WALK
  if (!OVF) {
    const float *pool = L.pool();
    int ci = ws.nct > 0 ? __float_as_int(*L.head()) : -1;
#pragma unroll 1
    while (__any(ci >= 0)) {
      if (ci >= 0) {
        const float *c = pool + 6 * ci;
        const int meta = __float_as_int(c[5]);
        qwall_vel_one(g, S, SC, LT, b.x, b.q, b.v, b.w, meta & 3, c[0], V(c[1], c[2], c[3]), c[4], dV, dW);
        ci = (meta >> 2) - 1;
      }
    }
    return;
  }
#endif
  const bool ovf = ws.nct > QK;
  const int nc = ovf ? 0 : ws.nct;
#pragma unroll 1
  for (int i = 0; i < QK; ++i) {
    if (!__any(i < nc)) break;
    if (i < nc) {
      const float *c = ws.c + 6 * i;
      qwall_vel_one(g, S, SC, LT, b.x, b.q, b.v, b.w, (int)c[0], c[1], V(c[2], c[3], c[4]), c[5], dV, dW);
    }
  }
  if (!OVF) return;  // (the fast pass: a wave with an overflow runs the step again)
#if POB_QUAD_REWALK_INLINE
#ifndef POB_EXP_NO_REWALK
  if (__any(ovf)) qwalls_rewalk_inl<true>(S, LT, WT, b, QLds{nullptr, 0}, ws, ovf, fric, dV, dW);
#endif
  if (false) {
#else
  if (__any(ovf)) {
#endif
    QOvf st;
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      st.x[l] = b.x[l]; st.q[l] = b.q[l]; st.v[l] = b.v[l]; st.w[l] = b.w[l]; st.d0[l] = dV[l]; st.d1[l] = dW[l];
      st.a[l] = V(ws.seg[6 * l], ws.seg[6 * l + 1], ws.seg[6 * l + 2]);
      st.b[l] = V(ws.seg[6 * l + 3], ws.seg[6 * l + 4], ws.seg[6 * l + 5]);
    }
    st.fric = fric;
    st.on = ovf ? 1 : 0;
    qwalls_rewalk<true>(Sp, LT, WT, &st);
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      dV[l] = st.d0[l]; dW[l] = st.d1[l];
      b.x[l] = st.x[l]; b.q[l] = st.q[l]; b.v[l] = st.v[l]; b.w[l] = st.w[l];
    }
  }
}

// sys.info(qp).contact and the legacy collisions: detection and the velocity-level response
// (LEGACY: the one-way impulses) at ONE pose, so each contact is applied as it is detected
template <bool WALLS, bool LEGACY>
POB_D void qcontacts_static(csys_t *Sp, const float *LT, const float *WT, const QBody &b, v3 (&dV)[QNB],
                            v3 (&dW)[QNB], const float fric) {
  csys_t &S = *launder(Sp);
  const HCon SC{fric, S.inv_h};
  GuardBranch g;
  const v3 rv_leg = qrot_xy(qcap_end(S, LT, 2, 0), b.q[2]);
  {
    QGround gc;
    v3 pe[2];
    qground_detect(S, LT, b, rv_leg, gc, pe);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      POB_FENCE();
      const int l = qcontact_body(c);
      if (gc.pen[c] > 0.0f) {
        if (LEGACY)
          olegacy_contact(S, gc.pen[c], pe[c], V(0.0f, 0.0f, 1.0f), qground_r(S, LT, c), q_inv_mass(S, LT, l), b.x[l],
                          b.v[l], b.w[l], dV[l], dW[l]);
        else
          ocontact_vel_pe(g, SC, true, gc.pen[c], pe[c], V(0.0f, 0.0f, 1.0f), qground_r(S, LT, c),
                          q_inv_mass(S, LT, l), b.x[l], b.v[l], b.w[l], dV[l], dW[l]);
      }
    }
  }
  if (!WALLS) return;
  POB_FENCE();
  QMesh ms;
  qmesh_segments(S, LT, b, rv_leg, ms);
  uint64_t M[QNB];
  {
    const uint32_t lw = qwall_mask(S, b);
    qmesh_items(S, LT, WT, lw | (lw << 8) | (lw << 16), ms, M);
  }
  mesh_lane_walk<QNB>(g, WT, pob_face_table(S), S.wall_cz, S.wall_hz, M,
                      [&](const int l, v3 &A, v3 &B, float &r, bool &seg) { qmesh_seg(S, LT, ms, l, A, B, r, seg); },
                      [&](const int l, const int, const float tau, const v3 n, const float dist) {
    const v3 x = qpick3(l, b.x);
    const v3 pe = l == 0 ? x : qseg_point(LT, l, x, qpick4(l, b.q), tau);
    const float pen = q_cap_r(S, LT, l) - dist, cd = 1e-6f + dist, iml = q_inv_mass(S, LT, l);
    v3 dv = qpick3(l, dV), dw = qpick3(l, dW);
    if (LEGACY) olegacy_contact(S, pen, pe, n, cd, iml, x, qpick3(l, b.v), qpick3(l, b.w), dv, dw);
    else ocontact_vel_pe(g, SC, false, pen, pe, n, cd, iml, x, qpick3(l, b.v), qpick3(l, b.w), dv, dw);
    qput3(l, dV, dv);
    qput3(l, dW, dw);
  });
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

// One XPBD substep on a lane quad (see the header comment for the split).  CHECK (with WALLS
// false): the substep of the no-wall pass, which still evaluates the wall broadphase of every
// collide substep at the point the wall pass would (qwalls_detect) and reports a lane whose
// mask is not empty in *near -- with every mask empty the wall pass finds no face item, so
// the two passes compute the same bits.
template <bool WALLS, bool CHECK = false, bool OVF = true>
POB_D void qpbd_substep(csys_t *Sp, const float *LT, const float *WT, QBody &b, const float (&act)[QNJ], const QLds &L,
                        const bool COLLIDE, const float fric, bool *near = nullptr, bool *ovf = nullptr) {
#pragma unroll
  for (int l = 0; l < QNB; ++l) { L.set3(l, QF_PX, b.x[l]); L.set4(l, QF_PQ, b.q[l]); }
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
  // 2b. wall contact detection (collide substeps), at the pose the projection starts from
  QWalls ws;
  ws.nct = 0;
  if (COLLIDE) qwalls_detect<WALLS, OVF>(Sp, LT, WT, b, ws, L, ovf);
  if (CHECK && COLLIDE) *near = *near | (qwall_mask(*launder(Sp), b) != 0u);
  // 3. position projection
  QGround gc;
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
    if (COLLIDE) qcontacts_position<WALLS, OVF>(Sp, LT, WT, b, L, gc, ws, DX, DA, fric);
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
    b.v[l] = vscl(vsub(b.x[l], L.get3(l, QF_PX)), S.inv_h);
    q4 dq = qmul(b.q[l], qinv(L.get4(l, QF_PQ)));
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
    qcontacts_velocity<WALLS, OVF>(Sp, LT, WT, b, gc, ws, L, dV, dW, fric);
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      b.v[l] = vadd(b.v[l], dV[l]); b.w[l] = vadd(b.w[l], dW[l]);
      L.set3(l, QF_CV, vadd(L.get3(l, QF_CV), dV[l]));
      L.set3(l, QF_CA, vadd(L.get3(l, QF_CA), dW[l]));
    }
  }
}

// The slow wall pass's substep out of line (POB_QUAD_SLOW_OOL): the step's state through a
// private block, so the substep loop of the fast pass carries neither the re-walks' code nor
// a call's register constraints (a wave runs the slow pass only after a contact-store overflow)
struct QSlow {
  QBody b;
  float act[QNJ];
};
template <bool WALLS>
__device__ __attribute__((noinline)) void qpbd_substep_slow(csys_t *Sp, const float *LT, const float *WT, QSlow *st,
                                                           float *lbase, const int lt, const int collide,
                                                           const float fric) {
  QBody b = st->b;
  float act[QNJ];
#pragma unroll
  for (int j = 0; j < QNJ; ++j) act[j] = st->act[j];
  const QLds L{lbase, lt};
  qpbd_substep<WALLS>(Sp, LT, WT, b, act, L, collide != 0, fric);
  st->b = b;
}

// ------------------------------------------------------------- legacy spring dynamics
// brax <= 0.0.12 spring/impulse step (oracle legacy_substep; pinned by the 20 frames of
// notebooks/ant_tag.ipynb:449) on the same lane quads: kinetic, then spring joints + torque
// actuators as accelerations, then one-way contact impulses.  Every expression follows the
// oracle's generic form (no frame specialisation: this mode is the parity reference for the
// notebook, not the throughput path).

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
                           const QLds &L) {
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
  // collisions: velocity impulses at the post-kinetic pose (oracle legacy_contacts)
  v3 dV[QNB], dW[QNB];
#pragma unroll
  for (int l = 0; l < QNB; ++l) { dV[l] = V(0.0f, 0.0f, 0.0f); dW[l] = V(0.0f, 0.0f, 0.0f); }
  qcontacts_static<WALLS, true>(Sp, LT, WT, b, dV, dW, launder(Sp)->friction);
#pragma unroll
  for (int l = 0; l < QNB; ++l) {
    b.v[l] = vadd(b.v[l], dV[l]); b.w[l] = vadd(b.w[l], dW[l]);
    L.set3(l, QF_CV, vadd(L.get3(l, QF_CV), dV[l]));
    L.set3(l, QF_CA, vadd(L.get3(l, QF_CA), dW[l]));
  }
}
