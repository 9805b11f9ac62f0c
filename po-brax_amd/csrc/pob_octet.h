// pob_octet.h -- the PBD Ant step with EIGHT lanes per environment (gfx950), for batches
// too small to fill the chip with the four-lane kernel (pob_quad.h).
//
// Why: below ~16 K envs the four-lane kernel runs at most one wave per SIMD and its time
// is one wave's dependency chain (a lone wave issues one VALU instruction
// per ~7 cycles; no ILP left to harvest).  Eight lanes per env halve the joint work and
// cut the bodies per lane from three to two, so the chain is shorter, and twice as many
// waves share the SIMDs.
//
// Split: every lane owns ONE joint and its two bodies -- slot 0 = the joint's parent,
// slot 1 = its child:
//   A_k (hip, joint 2k):     slot 0 = torso (replica in the 4 A lanes), slot 1 = Aux k+1
//   B_k (knee, joint 2k+1):  slot 0 = Aux k+1 (replica of A_k's),      slot 1 = lower leg k
// Lane m of the env's 8 (m = lane & 7) is A_m for m < 4 and B_(7-m) for m >= 4, so the A
// lanes form one DPP quad (the torso's sums over the four hips are quad broadcasts, as in
// the four-lane kernel) and A_k <-> B_k is one row_half_mirror DPP move (lane m <-> 7 - m).
// Every lane runs the SAME instruction stream (no role branches): role-dependent values
// come from a per-role table row in LDS and from selects.  The aux body's terms are summed
// in both of its lanes in the oracle's order (hip joint first, then knee joint), from the
// lane's own term and its partner's, so the two replicas stay bit-identical.
// The joint projection is the oracle's generic form (rotation matrices, full vectors).
#pragma once
#include "pob_quad.h"

#define ONB 2  // bodies per lane

struct OBody {
  v3 x[ONB];
  q4 q[ONB];
  v3 v[ONB];
  v3 w[ONB];
};

// per-role table row (8 rows per block: row k = A_k, row 4 + k = B_k), staged in LDS
#define OT_J 0              // joint: off_p(3) off_c(3) axis(3) ref(3) lim_lo lim_hi jdamp strength
#define OT_OFFP 0
#define OT_OFFC 3
#define OT_AXIS 6
#define OT_REF 9
#define OT_LO 12
#define OT_HI 13
#define OT_DAMP 14
#define OT_STRENGTH 15
#define OT_B(s) (16 + 8 * (s))  // slot s body: inv_mass, cap_r, capsule end e0 (3); ends are +-e0
#define OT_G 32                 // ground contact: end (3), radius, slot (0.0f / 1.0f)
#define OT_TLO 37               // tan(lim_lo), tan(lim_hi): the actuator gate
#define OT_THI 38
#define OT_FLOATS POB_OCT_FLOATS
#define OT_TAB_FLOATS (8 * OT_FLOATS + POB_MAXW * POB_WALL_FLOATS)  // + the wall rows
static_assert(OT_TAB_FLOATS % 4 == 0, "the broadphase boxes after the wall rows are read as float4");

#define OTV(T, f) V((T)[(f)], (T)[(f) + 1], (T)[(f) + 2])
// The eight-lane kernel runs at most a few waves per SIMD, so the system table's scalars
// may stay in SGPRs for the whole substep loop (no per-stage re-load, pob_physics.h
// launder), and the lane's role row lives in VGPRs (k_step_oct copies it out of LDS).
#define OLAUNDER(p) (p)

// lane m of an env's octet <-> 7 - m (A_k <-> B_k)
POB_D float oct_swap(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xf, 0xf, true));  // row_half_mirror
}
POB_D v3 oct_swap3(v3 a) { return V(oct_swap(a.x), oct_swap(a.y), oct_swap(a.z)); }
POB_D v3 vsel(bool c, v3 a, v3 b) { return V(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }

// per-lane LDS staging area of the eight-lane kernel (floats per lane): the state load, the
// obs rows and the qp stores go through it
#define OL_FLOATS 26

// ground contact of the lane's ground body (A: torso, B: lower leg) and the wall contacts of
// its two slots (pob_quad.h QMesh: the segments at detection and the contact-bearing items)
struct OGround {
  float pen;
  v3 pe;  // x + rotate(end, q)
};
// The wave's contact pool (per kind, bit 1 << KIND of POB_OCT_POOL_KINDS): the wave's contacts
// in LDS after the lanes' stores -- OPOOL_N entries of tau, n, dist and (next + 1) << 1 | slot --
// stored by the walk's winner lanes and linked per lane by the owners (pob_mesh.h
// mesh_wave_walk HAND 2), the position responses then following the list after the walk
// instead of inside its hand-over.  HH B = 16 384 0.1075 -> 0.0950 ms; TAG B = 12 288 / 16 384
// +0.8 / +1.7 %, GA +1.3 % (profiles/r7i/ab.txt), so HH only.
#ifndef POB_OCT_POOL_KINDS
#define POB_OCT_POOL_KINDS 1
#endif
__host__ __device__ constexpr bool oct_pool(int kind) { return kind >= 0 && ((POB_OCT_POOL_KINDS >> kind) & 1) != 0; }
#define OPOOL_N 64
struct OMesh {
  v3 a[ONB], b[ONB];
  uint64_t mc[ONB];
  int nct;  // wall contacts of the position pass (the first OMAXC kept in the lane's LDS store)
  int head;   // (pool) the lane's first contact
  bool povf;  // (pool) the wave's contacts overflowed it (wave-uniform)
};
struct OPoolSink {
  float *pool;
  int npool;  // (wave-uniform)
  int tail, tail_s, head, nct;
  uint64_t mc0, mc1;
  POB_D int store(const bool hit, const float tau, const v3 n, const float dist) {
    const uint64_t m = __ballot(hit);
    const int idx = npool + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    npool += __popcll(m);
    if (hit && idx < OPOOL_N) {
      float *c = pool + 6 * idx;
      c[0] = tau; c[1] = n.x; c[2] = n.y; c[3] = n.z; c[4] = dist;
    }
    return hit ? idx + 1 : 0;
  }
  POB_D void link(const int s, const int bit, const int e) {
    if (e > 0) {
      const int idx = e - 1;
      ++nct;
      mc0 |= s == 0 ? 1ull << bit : 0ull;
      mc1 |= s == 1 ? 1ull << bit : 0ull;
      if (idx < OPOOL_N) {
        pool[6 * idx + 5] = __int_as_float(s);
        if (tail >= 0) pool[6 * tail + 5] = __int_as_float(((idx + 1) << 1) | tail_s);
        else head = idx;
        tail = idx;
        tail_s = s;
      }
    }
  }
};
// The position pass's wall contacts (slot, tau, n, dist), kept in the lane's LDS store
// (lane-minor: element e at CS[64 e]) so that the velocity pass applies them without evaluating
// their faces again; a lane with more re-walks its contact faces (ms.mc) from its segments,
// which it then leaves in the store too (elements OCS_SEG.., off the registers of the velocity
// projection) -- the same contacts either way.
#define OMAXC 4
#define OCS_SEG (6 * OMAXC)
#define OCS_FLOATS (OCS_SEG + 6 * ONB)

// slot s's capsule end points x +- rotate(e0, q) (torso: e0 = 0, both = x)
POB_D void ocap_points(const float *OT, const OBody &b, int s, v3 &p0, v3 &p1) {
  const v3 rv = qrot_xy(OTV(OT, OT_B(s) + 2), b.q[s]);
  p0 = vadd(b.x[s], rv);
  p1 = vsub(b.x[s], rv);
}

// The walls in registers (the eight- and sixteen-lane kernels): every wall's broadphase box
// (xy), the common z extent and the loop's table scalars, loaded once per launch from the
// kernel's LDS table into VGPRs (the wall rows stay in LDS, read by the per-lane walk).  Read from the system table instead they were ~80 scalar values per collide
// substep -- more than the SGPR budget holds across the substep loop -- so each collide
// substep re-issued ~20 scalar loads and waited for them (SQ_WAIT_ANY was 42 % of a wave's
// cycles at HH B = 4 096 on the sixteen-lane kernel).
#define HW_BOX 0                      // LDS wall table: lo.x lo.y hi.x hi.y per wall,
#define HW_CZ (4 * POB_MAXW)          // then wall_cz, wall_hz, s_pos, friction, n_walls
#define HW_FLOATS (4 * POB_MAXW + 5)
template <int MW>
struct HWalls {
  float lx[MW > 0 ? MW : 1], ly[MW > 0 ? MW : 1], hx[MW > 0 ? MW : 1], hy[MW > 0 ? MW : 1];
  float cz, hz;
  // the table scalars the compiler re-loaded inside the substep loop for want of SGPRs (one
  // waited scalar load per joint projection and per contact): kept in VGPRs as well
  float s_pos, friction;
  int n_walls;
  fcptr_t fc;  // pob_sys::face_c (the walls' face constants, pob_mesh.h)
};
// Fill the wall table's HW_FLOATS entries (lanes 0 .. HW_FLOATS - 1 of the block's first wave
// write one each) and, after the caller's LDS sync, read it into registers.
POB_D void hwalls_stage(csys_t &S, float *tab, const int lane) {
  if (lane < HW_FLOATS) {
    const int w = lane >> 2, c = lane & 3;
    const int e = lane - HW_CZ;
    tab[lane] = e >= 0 ? (e == 0 ? S.wall_cz : e == 1 ? S.wall_hz : e == 2 ? S.s_pos : e == 3 ? S.friction
                                                                                  : __int_as_float(S.n_walls))
                       : (c < 2 ? S.wall_lo[w][c] : S.wall_hi[w][c - 2]);
  }
}
template <int MW>
POB_D void hwalls_load(const float *tab, HWalls<MW> &HW, fcptr_t fc) {
  HW.fc = fc;
#pragma unroll
  for (int w = 0; w < MW; ++w) {
    const float *bx = tab + HW_BOX + 4 * w;
    HW.lx[w] = bx[0]; HW.ly[w] = bx[1]; HW.hx[w] = bx[2]; HW.hy[w] = bx[3];
  }
  HW.cz = tab[HW_CZ]; HW.hz = tab[HW_CZ + 1];
  HW.s_pos = tab[HW_CZ + 2]; HW.friction = tab[HW_CZ + 3];
  HW.n_walls = __float_as_int(tab[HW_CZ + 4]);
}

// Contacts of a collide substep on one lane (oracle order per body: ground, then walls in
// wall / face / triangle order).  Walls: the lane's broadphase mask over its two body centres
// (the boxes from registers, HWalls), the face items per slot (pob_mesh.h cull), then the
// wave's face walk (pob_mesh.h mesh_wave_walk) with the wall rows from LDS (WT).  The torso (A
// slot 0) is the sphere: its segment is the point x (e0 = 0).
POB_D void omesh_seg(const float *OT, const bool isA, const OMesh &ms, const int s, v3 &A, v3 &B, float &r, bool &seg) {
  A = vsel3(s == 0, ms.a[0], ms.a[1]);
  B = vsel3(s == 0, ms.b[0], ms.b[1]);
  r = s == 0 ? OT[OT_B(0) + 1] : OT[OT_B(1) + 1];
  seg = !(isA && s == 0);
}

template <int MW, bool POOL, class G>
POB_D void ocontacts_position(G &g, const HCon &SC, const float *OT, const float *WT, const HWalls<MW> &HW,
                              const bool isA, const OBody &b, const v3 (&pxs)[ONB], const q4 (&pqs)[ONB],
                              OGround &gc, OMesh &ms, v3 (&DX)[ONB], v3 (&DA)[ONB], float *CS) {
  const bool gslot1 = !isA;
  {
    const v3 xg = vsel3(gslot1, b.x[1], b.x[0]);
    const q4 qg = qsel(gslot1, b.q[1], b.q[0]);
    gc.pe = vadd(xg, qrot_xy(OTV(OT, OT_G), qg));
    gc.pen = OT[OT_G + 3] - gc.pe.z;
  }
#pragma unroll
  for (int s = 0; s < ONB; ++s) {
    const bool gs = (s == 1) == gslot1;  // this slot holds the lane's ground body
    if (gs && gc.pen > 0.0f)
      oground_position(g, SC, gc.pen, gc.pe, OT[OT_G + 3], OT[OT_B(s)], b.x[s], b.q[s], pqs[s], pxs[s], DX[s], DA[s]);
  }
  ms.mc[0] = 0ull; ms.mc[1] = 0ull;
  ms.nct = 0;
  if (MW == 0) return;
  v3 rv[ONB];
#pragma unroll
  for (int s = 0; s < ONB; ++s) {
    rv[s] = qrot_xy(OTV(OT, OT_B(s) + 2), b.q[s]);
    ms.a[s] = vadd(b.x[s], rv[s]);
    ms.b[s] = vsub(b.x[s], rv[s]);
  }
  uint32_t lane_mask = 0u;
  {
    const float mnx = fminf(b.x[0].x, b.x[1].x), mxx = fmaxf(b.x[0].x, b.x[1].x);
    const float mny = fminf(b.x[0].y, b.x[1].y), mxy = fmaxf(b.x[0].y, b.x[1].y);
#ifdef POB_EXP_NO_WALLS
    const int nw = 0;  // timing experiment only
#else
    const int nw = HW.n_walls;
#endif
    // the boxes from the LDS table (HW_BOX, after the wall rows) at each collide substep: held
    // in VGPRs across the loop they pushed the two-wave build past 256 registers
    const float *WB = WT + POB_MAXW * POB_WALL_FLOATS + HW_BOX;
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      const float4 bx = *reinterpret_cast<const float4 *>(WB + 4 * w);
      const bool near = (mnx <= bx.z) & (mxx >= bx.x) & (mny <= bx.w) & (mxy >= bx.y);
      lane_mask |= (near & (w < nw)) ? 1u << w : 0u;
    }
  }
  uint64_t M[ONB] = {0ull, 0ull};
  {
    const float R0 = OT[OT_B(0) + 1] + POB_MESH_MARGIN, R1 = OT[OT_B(1) + 1] + POB_MESH_MARGIN;
    uint32_t m = lane_mask;
    while (__any(m != 0u)) {
      const bool on = m != 0u;
      const int w = on ? __builtin_ctz(m) : 0;
      m &= m - 1u;
      const MWall W = mwall_row(WT + POB_WALL_FLOATS * w);
#pragma unroll
      for (int s = 0; s < ONB; ++s) {
        const bool seg = !(isA && s == 0);
        const v3 La = mwall_local(W, HW.cz, ms.a[s]);
        const v3 Lb = seg ? mwall_local(W, HW.cz, ms.b[s]) : La;
        const uint32_t fm = mesh_face_mask(La, Lb, W.hx, W.hy, HW.hz, s == 0 ? R0 : R1);
        M[s] |= on ? (uint64_t)fm << (8 * w) : 0ull;
      }
    }
  }
#ifdef POB_EXP_NO_WALK
  return;  // timing experiment only: broadphase and face cull, no face walk
#endif
  // one position response (slot s, the contact's tau, n, dist)
  auto pos_one = [&](const int s, const float tau, const v3 n, const float dist) {
    const v3 x = vsel3(s == 0, b.x[0], b.x[1]);
    const q4 q = qsel(s == 0, b.q[0], b.q[1]);
    const v3 pe = vfma(vsel3(s == 0, rv[0], rv[1]), tau, x);
    v3 dx = vsel3(s == 0, DX[0], DX[1]), da = vsel3(s == 0, DA[0], DA[1]);
    owall_position(g, SC, (s == 0 ? OT[OT_B(0) + 1] : OT[OT_B(1) + 1]) - dist, pe, n, 1e-6f + dist,
                   s == 0 ? OT[OT_B(0)] : OT[OT_B(1)], x, q, qsel(s == 0, pqs[0], pqs[1]), vsel3(s == 0, pxs[0], pxs[1]),
                   dx, da);
    DX[0] = vsel3(s == 0, dx, DX[0]); DX[1] = vsel3(s == 1, dx, DX[1]);
    DA[0] = vsel3(s == 0, da, DA[0]); DA[1] = vsel3(s == 1, da, DA[1]);
  };
  if constexpr (POOL) {
    float *pool = CS - (int)__lane_id() + OCS_FLOATS * 64;  // (after the lanes' stores)
    OPoolSink sink{pool, 0, -1, 0, -1, 0, 0ull, 0ull};
    mesh_wave_walk<ONB, false, 2>(g, WT, HW.fc, HW.cz, HW.hz, M,
                        [&](const int s, v3 &A, v3 &B, float &r, bool &seg) { omesh_seg(OT, isA, ms, s, A, B, r, seg); },
                        sink);
    ms.mc[0] = sink.mc0; ms.mc[1] = sink.mc1;
    ms.nct = sink.nct;
    ms.head = sink.head;
    ms.povf = sink.npool > OPOOL_N;
    int ci = ms.povf ? -1 : ms.head;
#pragma unroll 1
    while (__any(ci >= 0)) {
      if (ci >= 0) {
        const float *c = pool + 6 * ci;
        const int meta = __float_as_int(c[5]);
        pos_one(meta & 1, c[0], V(c[1], c[2], c[3]), c[4]);
        ci = (meta >> 1) - 1;
      }
    }
    const bool ovf = ms.povf && ms.nct > 0;
    if (__any(ovf)) {
      // (rare) the pool overflowed: the lanes with contacts walk their contact faces again,
      // each response applied as it comes, and keep their segments for the velocity pass
      uint64_t Mo[ONB] = {ovf ? ms.mc[0] : 0ull, ovf ? ms.mc[1] : 0ull};
      mesh_wave_walk<ONB, false>(g, WT, HW.fc, HW.cz, HW.hz, Mo,
                          [&](const int s, v3 &A, v3 &B, float &r, bool &seg) { omesh_seg(OT, isA, ms, s, A, B, r, seg); },
                          [&](const int s, const int, const float tau, const v3 n, const float dist) { pos_one(s, tau, n, dist); });
#pragma unroll
      for (int q = 0; q < ONB; ++q) {
        float *c = CS + 64 * (OCS_SEG + 6 * q);
        c[0] = ms.a[q].x; c[64] = ms.a[q].y; c[128] = ms.a[q].z; c[192] = ms.b[q].x; c[256] = ms.b[q].y; c[320] = ms.b[q].z;
      }
    }
    return;
  }
  mesh_wave_walk<ONB, false>(g, WT, HW.fc, HW.cz, HW.hz, M,
                      [&](const int s, v3 &A, v3 &B, float &r, bool &seg) { omesh_seg(OT, isA, ms, s, A, B, r, seg); },
                      [&](const int s, const int bit, const float tau, const v3 n, const float dist) {
    const v3 x = vsel3(s == 0, b.x[0], b.x[1]);
    const q4 q = qsel(s == 0, b.q[0], b.q[1]);
    const v3 pe = vfma(vsel3(s == 0, rv[0], rv[1]), tau, x);
    v3 dx = vsel3(s == 0, DX[0], DX[1]), da = vsel3(s == 0, DA[0], DA[1]);
    // penetration r - dist; the contact at the triangle point pe - (1e-6 + dist) n
    owall_position(g, SC, (s == 0 ? OT[OT_B(0) + 1] : OT[OT_B(1) + 1]) - dist, pe, n, 1e-6f + dist,
                   s == 0 ? OT[OT_B(0)] : OT[OT_B(1)], x, q, qsel(s == 0, pqs[0], pqs[1]), vsel3(s == 0, pxs[0], pxs[1]),
                   dx, da);
    DX[0] = vsel3(s == 0, dx, DX[0]); DX[1] = vsel3(s == 1, dx, DX[1]);
    DA[0] = vsel3(s == 0, da, DA[0]); DA[1] = vsel3(s == 1, da, DA[1]);
    ms.mc[0] |= s == 0 ? 1ull << bit : 0ull;
    ms.mc[1] |= s == 1 ? 1ull << bit : 0ull;
    if (ms.nct < OMAXC) {
      float *c = CS + 64 * 6 * ms.nct;
      c[0] = (float)s; c[64] = tau; c[128] = n.x; c[192] = n.y; c[256] = n.z; c[320] = dist;
    }
    ++ms.nct;
  });
  if (ms.nct > OMAXC) {
#pragma unroll
    for (int q = 0; q < ONB; ++q) {
      float *c = CS + 64 * (OCS_SEG + 6 * q);
      c[0] = ms.a[q].x; c[64] = ms.a[q].y; c[128] = ms.a[q].z; c[192] = ms.b[q].x; c[256] = ms.b[q].y; c[320] = ms.b[q].z;
    }
  }
}

template <int MW, bool POOL, class G>
POB_D void ocontacts_velocity(G &g, const HCon &SC, const float *OT, const float *WT, const HWalls<MW> &HW,
                              const bool isA, const OBody &b, const OGround &gc, const OMesh &ms, v3 (&dV)[ONB],
                              v3 (&dW)[ONB], const float *CS) {
  const bool gslot1 = !isA;
#pragma unroll
  for (int s = 0; s < ONB; ++s) {
    const bool gs = (s == 1) == gslot1;
    if (gs && gc.pen > 0.0f)
      ocontact_vel_one(g, SC, true, gc.pen, OTV(OT, OT_G), V(0.0f, 0.0f, 1.0f), OT[OT_G + 3], OT[OT_B(s)], b.x[s],
                       b.q[s], b.v[s], b.w[s], dV[s], dW[s]);
  }
  if (MW == 0 || !__any(ms.nct != 0)) return;
  bool ovf;
  if constexpr (POOL) {
    ovf = ms.povf && ms.nct > 0;
    const float *pool = CS - (int)__lane_id() + OCS_FLOATS * 64;
    int ci = ms.povf || ms.nct == 0 ? -1 : ms.head;
#pragma unroll 1
    while (__any(ci >= 0)) {
      if (ci >= 0) {
        const float *c = pool + 6 * ci;
        const int meta = __float_as_int(c[5]);
        const int s = meta & 1;
        const v3 x = vsel3(s == 0, b.x[0], b.x[1]);
        const q4 q = qsel(s == 0, b.q[0], b.q[1]);
        const v3 pe = vfma(qrot_xy(s == 0 ? OTV(OT, OT_B(0) + 2) : OTV(OT, OT_B(1) + 2), q), c[0], x);
        v3 dv = vsel3(s == 0, dV[0], dV[1]), dw = vsel3(s == 0, dW[0], dW[1]);
        ocontact_vel_pe(g, SC, false, (s == 0 ? OT[OT_B(0) + 1] : OT[OT_B(1) + 1]) - c[4], pe, V(c[1], c[2], c[3]),
                        1e-6f + c[4], s == 0 ? OT[OT_B(0)] : OT[OT_B(1)], x, vsel3(s == 0, b.v[0], b.v[1]),
                        vsel3(s == 0, b.w[0], b.w[1]), dv, dw);
        dV[0] = vsel3(s == 0, dv, dV[0]); dV[1] = vsel3(s == 1, dv, dV[1]);
        dW[0] = vsel3(s == 0, dw, dW[0]); dW[1] = vsel3(s == 1, dw, dW[1]);
        ci = (meta >> 1) - 1;
      }
    }
  } else {
  ovf = ms.nct > OMAXC;
  const int nc = ovf ? 0 : ms.nct;
#pragma unroll 1
  for (int i = 0; i < OMAXC; ++i) {
    if (!__any(i < nc)) break;
    if (i < nc) {
      const float *c = CS + 64 * 6 * i;
      const int s = (int)c[0];
      const v3 x = vsel3(s == 0, b.x[0], b.x[1]);
      const q4 q = qsel(s == 0, b.q[0], b.q[1]);
      const v3 pe = vfma(qrot_xy(s == 0 ? OTV(OT, OT_B(0) + 2) : OTV(OT, OT_B(1) + 2), q), c[64], x);
      v3 dv = vsel3(s == 0, dV[0], dV[1]), dw = vsel3(s == 0, dW[0], dW[1]);
      ocontact_vel_pe(g, SC, false, (s == 0 ? OT[OT_B(0) + 1] : OT[OT_B(1) + 1]) - c[320], pe, V(c[128], c[192], c[256]),
                      1e-6f + c[320], s == 0 ? OT[OT_B(0)] : OT[OT_B(1)], x, vsel3(s == 0, b.v[0], b.v[1]),
                      vsel3(s == 0, b.w[0], b.w[1]), dv, dw);
      dV[0] = vsel3(s == 0, dv, dV[0]); dV[1] = vsel3(s == 1, dv, dV[1]);
      dW[0] = vsel3(s == 0, dw, dW[0]); dW[1] = vsel3(s == 1, dw, dW[1]);
    }
  }
  }
  if (!__any(ovf)) return;
  uint64_t M[ONB] = {ovf ? ms.mc[0] : 0ull, ovf ? ms.mc[1] : 0ull};
  mesh_wave_walk<ONB, false>(g, WT, HW.fc, HW.cz, HW.hz, M,
                      [&](const int s, v3 &A, v3 &B, float &r, bool &seg) {
                        const float *c = CS + 64 * (OCS_SEG + 6 * s);
                        A = V(c[0], c[64], c[128]);
                        B = V(c[192], c[256], c[320]);
                        r = s == 0 ? OT[OT_B(0) + 1] : OT[OT_B(1) + 1];
                        seg = !(isA && s == 0);
                      },
                      [&](const int s, const int, const float tau, const v3 n, const float dist) {
    const v3 x = vsel3(s == 0, b.x[0], b.x[1]);
    const q4 q = qsel(s == 0, b.q[0], b.q[1]);
    const v3 pe = vfma(qrot_xy(s == 0 ? OTV(OT, OT_B(0) + 2) : OTV(OT, OT_B(1) + 2), q), tau, x);
    v3 dv = vsel3(s == 0, dV[0], dV[1]), dw = vsel3(s == 0, dW[0], dW[1]);
    ocontact_vel_pe(g, SC, false, (s == 0 ? OT[OT_B(0) + 1] : OT[OT_B(1) + 1]) - dist, pe, n, 1e-6f + dist,
                    s == 0 ? OT[OT_B(0)] : OT[OT_B(1)], x, vsel3(s == 0, b.v[0], b.v[1]), vsel3(s == 0, b.w[0], b.w[1]),
                    dv, dw);
    dV[0] = vsel3(s == 0, dv, dV[0]); dV[1] = vsel3(s == 1, dv, dV[1]);
    dW[0] = vsel3(s == 0, dw, dW[0]); dW[1] = vsel3(s == 1, dw, dW[1]);
  });
}

// timing experiment only (POB_EXP_TIMING_SUB): shader-clock durations of the eight- and
// sixteen-lane substeps'
// phases summed into tacc[0..7] (accel + kinetic, joint, contact position (wall response), velocity
// contacts (wall), contact detection, ground position, velocity projection, ground velocity)
#ifdef POB_EXP_TIMING_SUB
#define HSUB_T(i)                                                  \
  {                                                                \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();   \
    if (tacc) tacc[i] += _t - _tl;                                 \
    _tl = _t;                                                      \
  }
#else
#define HSUB_T(i)
#endif
// the lane's joint, oracle joints_position form: point-to-point impulse P and its angular
// parts xp / xc, hinge alignment + angle limit s
struct OJoint {
  v3 P, xp, xc, s;
};
template <class G>
POB_D void ojoint_position(G &g, csys_t &S, const float s_pos, const float *OT, const OBody &b, OJoint &J) {
  const float imp = OT[OT_B(0)], imc = OT[OT_B(1)];
  const m3 Rp = qmat(b.q[0]), Rc = qmat(b.q[1]);
  // (offsets lie in the body xy-plane for every Ant joint, checked by pob_system.cpp: the
  // products with their zero z drop out, results equal up to the sign of a zero)
  const v3 rp = mrot_xy(Rp, OTV(OT, OT_OFFP)), rc = mrot_xy(Rc, OTV(OT, OT_OFFC));
  const v3 axis = OTV(OT, OT_AXIS), ref = OTV(OT, OT_REF);
  const v3 ap = mrot(Rp, axis), ac = mrot(Rc, axis);
  const v3 fp = mrot(Rp, ref), fc = mrot(Rc, ref);
  v3 d = vsub(vadd(b.x[1], rc), vadd(b.x[0], rp));
  const float L2 = vdot(d, d);
  J.P = V(0.0f, 0.0f, 0.0f); J.xp = J.P; J.xc = J.P;
  if (L2 > 0.0f) {
    const v3 ep = vcross(rp, d), ec = vcross(rc, d);
    const float den = FMA(L2, imp + imc, vdot(ep, ep) + vdot(ec, ec));
    const float k = (L2 * s_pos) * g.rcp(den);  // POB_DIV(L2 * s_pos, den)
    J.P = vscl(d, k); J.xp = vscl(ep, k); J.xc = vscl(ec, k);
  }
  const v3 Pa = vscl(vcross(ap, ac), S.half_s_ang);
  const float psi = pob_atan2f_g(g, vdot(vcross(fp, fc), ap), vdot(fp, fc));
  float dl = 0.0f;
  if (psi < OT[OT_LO]) dl = psi - OT[OT_LO];
  else if (psi > OT[OT_HI]) dl = psi - OT[OT_HI];
  const v3 Pl = vscl(ap, dl * S.half_s_ang);
  J.s = vadd(Pa, Pl);
}

// One XPBD substep on an env octet (isA: this lane is A_k; see the header comment).
// (the substep-start poses px / pq and the Info.contact accumulators cv / ca stay in
// registers: at one or two waves per SIMD there are registers to spare, and an LDS round
// trip would sit on the lone wave's dependency chain)
// G: the range-guard policy (pob_math.h GuardBranch / GuardAcc); HW: the walls and the
// loop's table scalars in registers.
template <int MW, bool POOL = false, class G>
POB_D void opbd_substep(G &g, csys_t *Sp, const float *OT, const float *WT, const HWalls<MW> &HW, const bool isA, OBody &b,
                        const float act, v3 (&cv)[ONB], v3 (&ca)[ONB], const bool COLLIDE, float *CS,
                        unsigned long long *tacc = nullptr) {
#ifdef POB_EXP_TIMING_SUB
  unsigned long long _tl = __builtin_amdgcn_s_memtime();
#else
  (void)tacc;
#endif
  const HCon SC{HW.friction, OLAUNDER(Sp)->inv_h};
  v3 px[ONB];
  q4 pq[ONB];
#pragma unroll
  for (int s = 0; s < ONB; ++s) { px[s] = b.x[s]; pq[s] = b.q[s]; }
  // 1. acceleration level: the lane's joint torque tt (actuator + damping)
  {
    v3 tt;
    {
      const v3 a = qrot(OTV(OT, OT_AXIS), b.q[0]);
      const bool in = actuator_inside(b.q[0], b.q[1], isA, OTV(OT, OT_AXIS), OT[OT_TLO], OT[OT_THI]);
      const v3 t = vscl(a, (in ? act : 0.0f) * OT[OT_STRENGTH]);
      const v3 d = vscl(vsub(b.w[0], b.w[1]), OT[OT_DAMP]);
      tt = vadd(t, d);
    }
    const v3 tpart = oct_swap3(tt);  // the partner's joint torque
    v3 dw[ONB];
    {
      // A slot 0 (torso): (((0 - t0) - t2) - t4) - t6 over the A quad
      const v3 t0 = quad_bcast3<0>(tt), t2 = quad_bcast3<1>(tt), t4 = quad_bcast3<2>(tt), t6 = quad_bcast3<3>(tt);
      const v3 torso = vsub(vsub(vsub(vsub(V(0.0f, 0.0f, 0.0f), t0), t2), t4), t6);
      // aux (A slot 1, B slot 0): (0 + t_hip) - t_knee; B slot 1 (leg): 0 + t_knee
      const v3 thip = vsel3(isA, tt, tpart), tknee = vsel3(isA, tpart, tt);
      const v3 aux = vsub(vadd(V(0.0f, 0.0f, 0.0f), thip), tknee);
      dw[0] = vsel3(isA, torso, aux);
      dw[1] = vsel3(isA, aux, vadd(V(0.0f, 0.0f, 0.0f), tt));
    }
    csys_t &S = *OLAUNDER(Sp);
#pragma unroll
    for (int s = 0; s < ONB; ++s) {
      const v3 v = b.v[s], w = b.w[s];
      b.v[s] = V(FMA(S.lin_damp, v.x, 0.0f * S.h), FMA(S.lin_damp, v.y, 0.0f * S.h), FMA(S.lin_damp, v.z, S.gz * S.h));
      b.w[s] = V(FMA(S.ang_damp, w.x, dw[s].x * S.h), FMA(S.ang_damp, w.y, dw[s].y * S.h),
                 FMA(S.ang_damp, w.z, dw[s].z * S.h));
    }
    // 2. kinetic
#pragma unroll
    for (int s = 0; s < ONB; ++s) {
      b.x[s] = vfma(b.v[s], S.h, b.x[s]);
      q4 dq = qmul_vq(b.w[s], b.q[s]);
      q4 q = b.q[s];
      q.w = FMA(S.half_h, dq.w, q.w); q.x = FMA(S.half_h, dq.x, q.x);
      q.y = FMA(S.half_h, dq.y, q.y); q.z = FMA(S.half_h, dq.z, q.z);
      b.q[s] = g.qnorm(q);
    }
  }
  HSUB_T(0)
  // 3. position projection
  OGround gc;
  OMesh ms;
  {
    v3 DX[ONB], DA[ONB];
    POB_FENCE();
    OJoint J;
    ojoint_position(g, *OLAUNDER(Sp), HW.s_pos, OT, b, J);
    POB_FENCE();
    {
      const float imp = OT[OT_B(0)], imc = OT[OT_B(1)];
      // the aux term this lane contributes: A = hip child term, B = knee parent term
      const v3 tp = vadd(J.xp, J.s), tc = vadd(J.xc, J.s);
      const v3 Pp = oct_swap3(J.P);
      const v3 Tp = oct_swap3(isA ? tc : tp);
      const v3 Phip = vsel3(isA, J.P, Pp), Pknee = vsel3(isA, Pp, J.P);
      const v3 Thip = vsel3(isA, tc, Tp), Tknee = vsel3(isA, Tp, tp);
      // aux (inverse mass im_aux: A's child = B's parent): hip child term, then knee parent term
      const float imaux = isA ? imc : imp;
      const v3 dx_aux = vfma(Pknee, imaux, vfma(Phip, -imaux, V(0.0f, 0.0f, 0.0f)));
      const v3 da_aux = vadd(vsub(V(0.0f, 0.0f, 0.0f), Thip), Tknee);
      // torso (A slot 0): the four hips' parent terms in joint order (A quad)
      const float imp0 = OLAUNDER(Sp)->inv_mass[0];
      v3 dxt = V(0.0f, 0.0f, 0.0f), dat = dxt;
      dxt = vfma(quad_bcast3<0>(J.P), imp0, dxt); dat = vadd(dat, quad_bcast3<0>(tp));
      dxt = vfma(quad_bcast3<1>(J.P), imp0, dxt); dat = vadd(dat, quad_bcast3<1>(tp));
      dxt = vfma(quad_bcast3<2>(J.P), imp0, dxt); dat = vadd(dat, quad_bcast3<2>(tp));
      dxt = vfma(quad_bcast3<3>(J.P), imp0, dxt); dat = vadd(dat, quad_bcast3<3>(tp));
      // leg (B slot 1): knee child term
      const v3 dx_leg = vfma(J.P, -imc, V(0.0f, 0.0f, 0.0f));
      const v3 da_leg = vsub(V(0.0f, 0.0f, 0.0f), tc);
      DX[0] = vsel3(isA, dxt, dx_aux); DA[0] = vsel3(isA, dat, da_aux);
      DX[1] = vsel3(isA, dx_aux, dx_leg); DA[1] = vsel3(isA, da_aux, da_leg);
    }
    HSUB_T(1)
    if (COLLIDE) {
      ocontacts_position<MW, POOL>(g, SC, OT, WT, HW, isA, b, px, pq, gc, ms, DX, DA, CS);
      HSUB_T(4)
    }
#pragma unroll
    for (int s = 0; s < ONB; ++s) {
      b.x[s] = vadd(b.x[s], DX[s]);
      qadd_half(b.q[s], qmul_vq(DA[s], b.q[s]), 1.0f);
    }
  }
  HSUB_T(2)
  // 4. velocity projection
#pragma unroll
  for (int s = 0; s < ONB; ++s) {
    csys_t &S = *OLAUNDER(Sp);
    b.q[s] = g.qnorm(b.q[s]);
    b.v[s] = vscl(vsub(b.x[s], px[s]), S.inv_h);
    q4 dq = qmul(b.q[s], qinv(pq[s]));
    const float k2 = 2.0f * S.inv_h;
    const float kw = dq.w >= 0.0f ? k2 : -k2;
    b.w[s] = V(dq.x * kw, dq.y * kw, dq.z * kw);
  }
  HSUB_T(6)
  // 5. velocity-level contacts
  if (COLLIDE) {
    v3 dV[ONB], dW[ONB];
#pragma unroll
    for (int s = 0; s < ONB; ++s) { dV[s] = V(0.0f, 0.0f, 0.0f); dW[s] = V(0.0f, 0.0f, 0.0f); }
    ocontacts_velocity<MW, POOL>(g, SC, OT, WT, HW, isA, b, gc, ms, dV, dW, CS);
#pragma unroll
    for (int s = 0; s < ONB; ++s) {
      b.v[s] = vadd(b.v[s], dV[s]); b.w[s] = vadd(b.w[s], dW[s]);
      cv[s] = vadd(cv[s], dV[s]);
      ca[s] = vadd(ca[s], dW[s]);
    }
  }
  HSUB_T(3)
}
