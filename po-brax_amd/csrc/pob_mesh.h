// pob_mesh.h -- Ant x Arena contacts on gfx950: brax v1's capsule x TriangulatedBox path
// (capsule_mesh) as restated in DESIGN.md §3 and oracle/pob_oracle.c capsule_wall_mesh.
//
// Every arena wall is a box collider of the frozen Arena body (po_brax/envs/utils.py:6-28,
// add_box_wall_to_body; ant x Arena in collide_include, ant_heavenhell.py:33-34).  brax v1
// meshes a box into 12 triangles and, for every triangle, takes the closest points S (on the
// capsule's segment) and P (on the triangle) by _closest_segment_triangle_points; a triangle
// with |S - P| below the capsule radius is one contact (penetration r - |S - P|, normal
// (S - P) / (1e-6 + |S - P|), position P), and every such contact is applied.  The
// computation runs in the wall's frame (world -> R_z(-theta)(p - c)); a face is the plane
// w = sigma h_k of axis k with face coordinates (a, b, w) = (y, z, x) / (x, z, y) / (x, y, z)
// for k = x / y / z, its rectangle split along the diagonal (-ha, -hb) -> (ha, hb).
//
// Op order, candidate order and tie rules are the oracle's expression for expression (one
// reciprocal per division, FMA chains as spelled there); results are bit-identical.  The
// kernels evaluate a face only when the face cull keeps it (the same cull the oracle applies:
// gap >= r + 1e-3 along some axis between the face rectangle and the segment's bounding box
// means no triangle of the face is within r).
#pragma once
#include <type_traits>
#include "pob_math.h"

#define POB_MESH_MARGIN 1e-3f
// the face constants table (pob_sys::face_c) is read through the constant address space
// (POB_FC_LDS: a generic pointer -- the eight- and sixteen-lane kernels pass their LDS copy of
// the table, the four-lane kernel the device table; the compiler infers each one's address
// space through the inlined walk)
#if defined(POB_MESH_HOST) || defined(POB_FC_LDS)
typedef const float *fcptr_t;
#else
typedef __attribute__((address_space(4))) const float *fcptr_t;
#endif

// one wall: centre x, y (z common), z-rotation cos / sin, half extents x, y (z common)
struct MWall {
  float cx, cy, c, s, hx, hy;
};
POB_D MWall mwall_row(const float *R) {
  const float2 r01 = *reinterpret_cast<const float2 *>(R);
  const float2 r23 = *reinterpret_cast<const float2 *>(R + 2);
  const float2 r45 = *reinterpret_cast<const float2 *>(R + 4);
  MWall W;
  W.cx = r01.x; W.cy = r01.y; W.c = r23.x; W.s = r23.y; W.hx = r45.x; W.hy = r45.y;
  return W;
}
// world point -> wall frame (oracle: d = p - c; (d.y s + d.x c, d.y c - d.x s, d.z))
POB_D v3 mwall_local(const MWall &W, const float cz, const v3 p) {
  const float dx = p.x - W.cx, dy = p.y - W.cy, dz = p.z - cz;
  return V(FMA(dy, W.s, dx * W.c), FMA(dy, W.c, -(dx * W.s)), dz);
}

// The face cull of segment [A, B] (wall frame; A == B for a sphere): bit f (faces -x, +x, -y,
// +y, -z, +z) set iff the face is evaluated.  Per axis k with the segment's extent [lo, hi]:
// the in-plane gap max(lo - h, -h - hi), the + face's gap max(lo - h, h - hi) and the - face's
// max(lo + h, -h - hi) -- the oracle's fmaxf(fminf(..) - w0, w0 - fmaxf(..)) with w0 = +-h.
POB_D uint32_t mesh_face_mask(const v3 A, const v3 B, const float hx, const float hy, const float hz, const float R) {
  const float lo[3] = {fminf(A.x, B.x), fminf(A.y, B.y), fminf(A.z, B.z)};
  const float hi[3] = {fmaxf(A.x, B.x), fmaxf(A.y, B.y), fmaxf(A.z, B.z)};
  const float h[3] = {hx, hy, hz};
  bool in[3], fp[3], fm[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float a1 = lo[k] - h[k], a2 = -h[k] - hi[k];
    in[k] = !(fmaxf(a1, a2) >= R);  // (the oracle's "cull iff gap >= R": NaN keeps the face)
    fp[k] = !(fmaxf(a1, h[k] - hi[k]) >= R);
    fm[k] = !(fmaxf(lo[k] + h[k], a2) >= R);
  }
  uint32_t m = 0u;
  m |= (fm[0] & in[1] & in[2]) ? 1u : 0u;
  m |= (fp[0] & in[1] & in[2]) ? 2u : 0u;
  m |= (fm[1] & in[0] & in[2]) ? 4u : 0u;
  m |= (fp[1] & in[0] & in[2]) ? 8u : 0u;
  m |= (fm[2] & in[0] & in[1]) ? 16u : 0u;
  m |= (fp[2] & in[0] & in[1]) ? 32u : 0u;
  return m;
}

// ---------------------------------------------------------------- brax's closest-point forms
// brax v1's _closest_segment_triangle_points and capsule_mesh as the restatement spells them
// (oracle/pob_oracle.c bseg_make / bseg_seg / btri_point / bpick / bface): three
// segment-segment pairs, the segment-plane point with its closest triangle point, the minimum
// of the four squared distances (ties averaged), the normal (S - P) / (1e-6 + |S - P|), the
// contact at the triangle point.  The same operations on the same operands as the oracle;
// jp.clip as selects (bclamp01 / bclamps: the same bits for -0 and NaN on both sides).
#if defined(POB_MESH_HOST) || defined(POB_MESH_NO_MFENCE)
#define MFENCE() ((void)0)
#else
#define MFENCE() __builtin_amdgcn_sched_barrier(0)
#endif
POB_D float bclamp01(float x) { return x > 0.0f ? (x < 1.0f ? x : 1.0f) : 0.0f; }
POB_D float bclamps(float x, float h) { return x > -h ? (x < h ? x : h) : -h; }

struct F3 {
  float a, b, w;  // face coordinates (a, b in the face plane, w along its normal)
};
POB_D F3 f3(const float a, const float b, const float w) { F3 r; r.a = a; r.b = b; r.w = w; return r; }
POB_D F3 f3sub(const F3 x, const F3 y) { return f3(x.a - y.a, x.b - y.b, x.w - y.w); }
POB_D float f3dot(const F3 x, const F3 y) { return FMA(x.w, y.w, FMA(x.b, y.b, x.a * y.a)); }
POB_D F3 f3fma(const F3 d, const float s, const F3 p) { return f3(FMA(d.a, s, p.a), FMA(d.b, s, p.b), FMA(d.w, s, p.w)); }
POB_D float f3d2(const F3 x, const F3 y) { const F3 d = f3sub(x, y); return f3dot(d, d); }
POB_D F3 f3sel(const bool c, const F3 x, const F3 y) { return f3(c ? x.a : y.a, c ? x.b : y.b, c ? x.w : y.w); }
// wall frame (x, y, z) -> face coordinates of axis k: (y, z, x) / (x, z, y) / (x, y, z)
POB_D F3 fperm(const F3 v, const int k) {
  return f3(k == 0 ? v.b : v.a, k == 2 ? v.b : v.w, k == 0 ? v.a : (k == 1 ? v.b : v.w));
}

// a segment p0 -> p0 + d with brax's derived quantities: len = safe_norm(d), il = 1 / (len +
// 1e-6), dir = d il, hl = len 0.5, mid = p0 + dir hl, idd = 1 / (d.d + 1e-6)
struct BSeg {
  F3 p0, d, dir, mid;
  float hl, il, idd;
};
template <class G>
POB_D BSeg bseg_make(G &g, const F3 p0, const F3 d) {
  BSeg s;
  s.p0 = p0;
  s.d = d;
  const float dd = f3dot(d, d);
  const bool z = (int)(fabsf(d.a) <= 1e-8f) & (int)(fabsf(d.b) <= 1e-8f) & (int)(fabsf(d.w) <= 1e-8f);
  const float len = z ? 0.0f : g.sqrt(z ? 1.0f : dd);
  s.il = g.rcp(len + 1e-6f);
  s.dir = f3(d.a * s.il, d.b * s.il, d.w * s.il);
  s.hl = len * 0.5f;
  s.mid = f3fma(s.dir, s.hl, p0);
  s.idd = g.rcp(dd + 1e-6f);
  return s;
}
POB_D BSeg bseg_perm(const BSeg &s, const int k) {
  BSeg r = s;
  r.p0 = fperm(s.p0, k); r.d = fperm(s.d, k); r.dir = fperm(s.dir, k); r.mid = fperm(s.mid, k);
  return r;
}
// _closest_segment_point(p0, p0 + d, pt)
POB_D F3 bseg_point(const BSeg &s, const F3 pt, float &t) {
  t = bclamp01(f3dot(f3sub(pt, s.p0), s.d) * s.idd);
  return f3fma(s.d, t, s.p0);
}
// _closest_segment_to_segment_points(A, E): S on A (parameter u), P on E; returns |S - P|^2
// and S - P (the candidate's fields)
struct MCand {
  float d2, u, da, db, dw;
};
template <class G>
POB_D void bseg_seg(G &g, const BSeg &A, const BSeg &E, F3 &S, F3 &P, float &u) {
  const F3 trans = f3sub(A.mid, E.mid);
  const float dd = f3dot(A.dir, E.dir), dat = f3dot(A.dir, trans), dbt = f3dot(E.dir, trans);
  const float denom = FMA(-dd, dd, 1.0f);
  const float ota = FMA(dd, dbt, -dat) * g.rcp(denom + 1e-6f);
  const float otb = FMA(ota, dd, dbt);
  const float ta = bclamps(ota, A.hl), tb = bclamps(otb, E.hl);
  const F3 best_a = f3fma(A.dir, ta, A.mid), best_b = f3fma(E.dir, tb, E.mid);
  float s1, s2;
  const F3 new_a = bseg_point(A, best_b, s1);
  const float d1 = f3d2(best_b, new_a);
  const F3 new_b = bseg_point(E, best_a, s2);
  const float d2 = f3d2(best_a, new_b);
  const bool na = d1 < d2;
  S = f3sel(na, new_a, best_a);
  P = f3sel(na, best_b, new_b);
  u = na ? s1 : (A.hl + ta) * A.il;
}
POB_D MCand bcand(const F3 S, const F3 P, const float u) {
  MCand c;
  c.da = S.a - P.a; c.db = S.b - P.b; c.dw = S.w - P.w;
  c.d2 = FMA(c.dw, c.dw, FMA(c.db, c.db, c.da * c.da));
  c.u = u;
  return c;
}
// _closest_triangle_point(V0, V0 + e0, V0 + e1, pt) with the triangle's constants; edges
// s01, s12, s20
struct BTri {
  F3 p0, e0, e1;
  float a, b, c, idet;
  BSeg s01, s12, s20;
};
POB_D F3 btri_point(const BTri &T, const F3 pt) {
  const F3 d = f3sub(pt, T.p0);
  const float e0d = f3dot(T.e0, d), e1d = f3dot(T.e1, d);
  const float u = FMA(T.c, e0d, -(T.b * e1d)) * T.idet, v = FMA(T.a, e1d, -(T.b * e0d)) * T.idet;
  const bool inside = (0.0f <= u) & (u <= 1.0f) & (0.0f <= v) & (v <= 1.0f) & (u + v <= 1.0f);
  F3 cp = f3fma(T.e1, v, f3fma(T.e0, u, T.p0));
  const float d0 = f3d2(cp, pt);
  float t;
  const F3 c1 = bseg_point(T.s01, pt, t);
  const float d1 = f3d2(pt, c1);
  const bool k0 = (d0 < d1) & inside;
  cp = f3sel(k0, cp, c1);
  float md = k0 ? d0 : d1;
  const F3 c2 = bseg_point(T.s12, pt, t);
  const float d2 = f3d2(pt, c2);
  cp = f3sel(d2 < md, c2, cp);
  md = fminf(md, d2);
  const F3 c3 = bseg_point(T.s20, pt, t);
  const float d3 = f3d2(pt, c3);
  return f3sel(d3 < md, c3, cp);
}

// A face (axis k, outward sign sg, plane w = w0, half extents ha, hb) with the capsule's
// segment in face coordinates and the face's constants fc (pob_sys::face_c[wall][k],
// pob_face_consts: its edges' segment terms and triangles' 1 / det -- exactly bseg_make's /
// btri_make's values, formed once per env).  Edges V0 V1 (a), V1 V2 (b), V0 V2 (diagonal),
// V2 V3 (a), V0 V3 (b); triangle t0 = (V0, V1, V2), t1 = (V0, V2, V3) (oracle bface).
struct MFace {
  int k;
  float sg, ha, hb, w0, ha2, hb2;
  BSeg A;          // the capsule's segment
  fcptr_t fc;      // the face's constants (POB_FC_*)
#if defined(POB_MESH_FC_INLINE) || defined(POB_MESH_FC_VEC)
  // (A/B build switches: the constants formed per face evaluation, or the face's row loaded
  // whole -- three 16-B loads -- and each lane's class picked by selects instead of per-lane
  // scattered loads)
  float cv[POB_FACE_FLOATS];
#endif
};
// the face's constants: edge class c's (il, hl, idd), the diagonal's d.d, triangle t's 1 / det
POB_D void mfc_edge(const MFace &F, const int c, float &il, float &hl, float &idd) {
#if defined(POB_MESH_FC_INLINE) || defined(POB_MESH_FC_VEC)
  il = c == 0 ? F.cv[POB_FC_IL(0)] : (c == 1 ? F.cv[POB_FC_IL(1)] : F.cv[POB_FC_IL(2)]);
  hl = c == 0 ? F.cv[POB_FC_HL(0)] : (c == 1 ? F.cv[POB_FC_HL(1)] : F.cv[POB_FC_HL(2)]);
  idd = c == 0 ? F.cv[POB_FC_IDD(0)] : (c == 1 ? F.cv[POB_FC_IDD(1)] : F.cv[POB_FC_IDD(2)]);
#else
  il = F.fc[POB_FC_IL(c)];
  hl = F.fc[POB_FC_HL(c)];
  idd = F.fc[POB_FC_IDD(c)];
#endif
}
POB_D float mfc_ed(const MFace &F) {
#if defined(POB_MESH_FC_INLINE) || defined(POB_MESH_FC_VEC)
  return F.cv[POB_FC_ED];
#else
  return F.fc[POB_FC_ED];
#endif
}
POB_D float mfc_idet(const MFace &F, const int t) {
#if defined(POB_MESH_FC_INLINE) || defined(POB_MESH_FC_VEC)
  return t == 0 ? F.cv[POB_FC_IDET(0)] : F.cv[POB_FC_IDET(1)];
#else
  return F.fc[POB_FC_IDET(t)];
#endif
}
// the capsule's segment in the wall frame (once per wall; oracle capsule_wall_mesh capw)
template <class G>
POB_D BSeg mcap_seg(G &g, const v3 La, const v3 Lb) {
  return bseg_make(g, f3(La.x, La.y, La.z), f3(Lb.x - La.x, Lb.y - La.y, Lb.z - La.z));
}
// fcw: the wall's three axes' constants (pob_sys::face_c[wall])
template <class G>
POB_D MFace mface(G &g, const int f, const BSeg &capw, const float hx, const float hy, const float hz,
                  fcptr_t fcw) {
  MFace F;
  const int k = f >> 1;
  F.k = k;
  F.sg = (f & 1) ? 1.0f : -1.0f;
  F.ha = k == 0 ? hy : hx;
  F.hb = k == 2 ? hy : hz;
  F.w0 = F.sg * (k == 0 ? hx : (k == 1 ? hy : hz));
  F.A = bseg_perm(capw, k);
  F.ha2 = F.ha + F.ha;  // V1 - V0 = (ha - (-ha), ..): exact
  F.hb2 = F.hb + F.hb;
  F.fc = fcw + POB_FACE_FLOATS * k;
#ifdef POB_MESH_FC_VEC
#ifdef POB_MESH_HOST
  for (int i = 0; i < POB_FACE_FLOATS; ++i) F.cv[i] = F.fc[i];
#else
  static_assert(POB_FACE_FLOATS == 12, "three 16-B loads per face row");
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    typedef float f4v __attribute__((ext_vector_type(4)));
#ifdef POB_FC_LDS
    const f4v q = reinterpret_cast<const f4v *>(F.fc)[i];
#else
    const f4v q = reinterpret_cast<const __attribute__((address_space(4))) f4v *>(F.fc)[i];
#endif
    F.cv[4 * i] = q.x; F.cv[4 * i + 1] = q.y; F.cv[4 * i + 2] = q.z; F.cv[4 * i + 3] = q.w;
  }
#endif
#endif
#ifdef POB_MESH_FC_INLINE  // (pob_face_consts' operations in the guard's policy)
  {
    const float dA = F.ha2 * F.ha2, dB = F.hb2 * F.hb2, e_d = FMA(F.hb2, F.hb2, F.ha2 * F.ha2);
    const float dd[3] = {dA, dB, e_d};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float len = g.sqrt(dd[c]);
      F.cv[POB_FC_IL(c)] = g.rcp(len + 1e-6f);
      F.cv[POB_FC_HL(c)] = len * 0.5f;
      F.cv[POB_FC_IDD(c)] = g.rcp(dd[c] + 1e-6f);
    }
    F.cv[POB_FC_ED] = e_d;
    F.cv[POB_FC_IDET(0)] = g.rcp(FMA(dA, e_d, -(dA * dA)));
    F.cv[POB_FC_IDET(1)] = g.rcp(FMA(e_d, dB, -(dB * dB)));
  }
#endif
  (void)g;
  return F;
}
// the segment-plane point's parameter (oracle bface: both triangles, n = (0, 0, sg))
template <class G>
POB_D float mface_tt(G &g, const MFace &F) {
  return bclamp01((F.sg * F.w0 - F.sg * F.A.p0.w) * g.rcp(F.sg * F.A.d.w + 1e-6f));
}
// edge e of the face as a segment: 0 V0 V1, 1 V1 V2, 2 V0 V2, 3 V2 V3, 4 V0 V3, 5 V2 V0, 6 V3 V0:
// p0 = (sa ha, sb hb, w0), d = (ca 2ha, cb 2hb, 0) with signs and classes from bit tables indexed
// by e -- branch-free for a runtime e (the walk's candidate lanes: a chain of compares and
// branches per round before), constant-folded for a constant one; the products with +-1 and 0
// are exact, so the terms are the same bits as the spelled-out selects of round 5
#define ME_PA_NEG 0x55u   // e = 0, 2, 4, 6: p0.a = -ha
#define ME_PB_NEG 0x17u   // e = 0, 1, 2, 4: p0.b = -hb
#define ME_DA_NZ 0x2Du    // e = 0, 2, 3, 5: d.a != 0
#define ME_DA_NEG 0x28u   // e = 3, 5: d.a = -2ha
#define ME_DB_NZ 0x76u    // e = 1, 2, 4, 5, 6: d.b != 0
#define ME_DB_NEG 0x60u   // e = 5, 6: d.b = -2hb
#define ME_CLS 0x1924u    // class (2 bits per e): a-edges 0, b-edges 1, diagonals 2
POB_D BSeg medge(const MFace &F, const int e) {
  const float w0 = F.w0;
  BSeg s;
  const float ca = ((ME_DA_NZ >> e) & 1u) ? (((ME_DA_NEG >> e) & 1u) ? -1.0f : 1.0f) : 0.0f;
  const float cb = ((ME_DB_NZ >> e) & 1u) ? (((ME_DB_NEG >> e) & 1u) ? -1.0f : 1.0f) : 0.0f;
  const float da = ca * F.ha2, db = cb * F.hb2;
  const float pa = ((ME_PA_NEG >> e) & 1u) ? -F.ha : F.ha;
  const float pb = ((ME_PB_NEG >> e) & 1u) ? -F.hb : F.hb;
  const int cls = (int)((ME_CLS >> (2 * e)) & 3u);
  s.p0 = f3(pa, pb, w0);
  s.d = f3(da, db, 0.0f);
  mfc_edge(F, cls, s.il, s.hl, s.idd);
  s.dir = f3(da * s.il, db * s.il, 0.0f);
  s.mid = f3(FMA(s.dir.a, s.hl, pa), FMA(s.dir.b, s.hl, pb), w0);
  return s;
}
// triangle t of the face (oracle btri_make)
POB_D BTri mtri(const MFace &F, const int t) {
  BTri T;
  T.p0 = f3(-F.ha, -F.hb, F.w0);
  T.e0 = t == 0 ? f3(F.ha2, 0.0f, 0.0f) : f3(F.ha2, F.hb2, 0.0f);
  T.e1 = t == 0 ? f3(F.ha2, F.hb2, 0.0f) : f3(0.0f, F.hb2, 0.0f);
  const float dA = F.ha2 * F.ha2, dB = F.hb2 * F.hb2, e_d = mfc_ed(F);
  // a = e0.e0, b = e0.e1, c = e1.e1 with the zero products dropped (exact: +0 terms)
  T.a = t == 0 ? dA : e_d;
  T.b = t == 0 ? dA : dB;
  T.c = t == 0 ? e_d : dB;
  T.idet = mfc_idet(F, t);
  T.s01 = medge(F, t == 0 ? 0 : 2);
  T.s12 = medge(F, t == 0 ? 1 : 3);
  T.s20 = medge(F, t == 0 ? 5 : 6);
  return T;
}
// candidate kk of triangle t (oracle bface order): 0..2 the triangle's edges (t0: V0 V1, V1 V2,
// V0 V2; t1: V0 V2, V2 V3, V0 V3) against the segment, 3 the segment-plane point and its
// closest triangle point; any other kk: none (d2 = +inf).  S, P: the candidate's points (the
// cooperative walk's tie average needs them; zero for none)
template <class G>
POB_D MCand mface_cand(G &g, const MFace &F, const int t, const int kk, F3 &S, F3 &P) {
  MCand c;
  c.d2 = __builtin_inff(); c.u = 0.0f; c.da = 0.0f; c.db = 0.0f; c.dw = 0.0f;
  S = f3(0.0f, 0.0f, 0.0f);
  P = S;
  if (kk < 3) {
    const int e = t == 0 ? kk : (kk == 0 ? 2 : kk + 2);
    float u;
    bseg_seg(g, F.A, medge(F, e), S, P, u);
    c = bcand(S, P, u);
  } else if (kk == 3) {
    const BTri T = mtri(F, t);
    const float tt = mface_tt(g, F);
    S = f3fma(F.A.d, tt, F.A.p0);
    P = btri_point(T, S);
    c = bcand(S, P, tt);
  }
  return c;
}
template <class G>
POB_D MCand mface_cand(G &g, const MFace &F, const int t, const int kk) {
  F3 S, P;
  return mface_cand(g, F, t, kk, S, P);
}
// the triangle's pick with brax's tie rule (oracle bpick): all four candidates, the minimum,
// ties averaged in candidate order (the slow path of a tie: the fast forms take the first
// strict minimum and call this only when two candidates tie at a distance below the radius)
template <class G>
POB_D MCand mtri_pick_ties(G &g, const MFace &F, const int t) {
  F3 sp[4], tp[4];
  float u[4], d2[4];
#pragma unroll
  for (int kk = 0; kk < 3; ++kk) {
    const int e = t == 0 ? kk : (kk == 0 ? 2 : kk + 2);
    bseg_seg(g, F.A, medge(F, e), sp[kk], tp[kk], u[kk]);
    d2[kk] = f3d2(sp[kk], tp[kk]);
  }
  {
    const BTri T = mtri(F, t);
    const float tt = mface_tt(g, F);
    sp[3] = f3fma(F.A.d, tt, F.A.p0);
    tp[3] = btri_point(T, sp[3]);
    u[3] = tt;
    d2[3] = f3d2(sp[3], tp[3]);
  }
  const float mn = fminf(fminf(d2[0], d2[1]), fminf(d2[2], d2[3]));
  F3 S = f3(0.0f, 0.0f, 0.0f), P = S;
  float us = 0.0f, cnt = 0.0f;
  int first = -1;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
    if (d2[kk] == mn) {
      if (first < 0) first = kk;
      S = f3(S.a + sp[kk].a, S.b + sp[kk].b, S.w + sp[kk].w);
      P = f3(P.a + tp[kk].a, P.b + tp[kk].b, P.w + tp[kk].w);
      us += u[kk];
      cnt += 1.0f;
    }
  MCand c;
  c.d2 = __builtin_inff(); c.u = 0.0f; c.da = 0.0f; c.db = 0.0f; c.dw = 0.0f;
  if (first < 0) return c;
  if (cnt > 1.0f) {
    S = f3(S.a / cnt, S.b / cnt, S.w / cnt);
    P = f3(P.a / cnt, P.b / cnt, P.w / cnt);
    c = bcand(S, P, us / cnt);
  } else {
    F3 s1 = sp[0], p1 = tp[0];
#pragma unroll
    for (int kk = 1; kk < 4; ++kk) if (first == kk) { s1 = sp[kk]; p1 = tp[kk]; }
    c = bcand(s1, p1, us);
  }
  return c;
}

// the tie path out of line (rare, ~1 400 instructions: inlined, its registers would set the
// walk's allocation); exact range guards (GuardBranch) whatever the caller's policy -- in range
// the guard policies give the same bits
#ifdef POB_MESH_HOST
POB_D MCand mtri_pick_ties_ool(const int f, const v3 La, const v3 Lb, const float hx, const float hy, const float hz,
                               fcptr_t fcw, const int t) {
  HostGuard g;
  return mtri_pick_ties(g, mface(g, f, mcap_seg(g, La, Lb), hx, hy, hz, fcw), t);
}
#elif defined(POB_MESH_TIES_INLINE)  // A/B build switch: the tie path inline
POB_D MCand mtri_pick_ties_ool(const int f, const v3 La, const v3 Lb, const float hx, const float hy, const float hz,
                               fcptr_t fcw, const int t) {
  GuardBranch g;
  return mtri_pick_ties(g, mface(g, f, mcap_seg(g, La, Lb), hx, hy, hz, fcw), t);
}
#else
__device__ __attribute__((noinline)) MCand mtri_pick_ties_ool(const int f, const v3 La, const v3 Lb, const float hx,
                                                           const float hy, const float hz, fcptr_t fcw,
                                                           const int t) {
  GuardBranch g;
  return mtri_pick_ties(g, mface(g, f, mcap_seg(g, La, Lb), hx, hy, hz, fcw), t);
}
#endif

// the contact of a triangle whose pick is c (oracle capsule_wall_mesh's emission): tau, the
// wall-frame normal (S - P) / (1e-6 + dist) and dist = |S - P| (the caller's penetration is
// r - dist, the contact's offset from the segment point along -n is 1e-6 + dist: the triangle
// point -- both recomputed from dist by the same operations); false when the triangle does
// not penetrate (r - dist <= 0).  d2 = 0 (a segment touching or piercing the triangle: its
// distance is 0 exactly) takes no square root -- kept out of the range guards.
template <class G>
POB_D bool mface_contact(G &g, const int k, const MCand &c, const float r, const float T, float &tau, v3 &nl,
                         float &dist) {
  if (!(c.d2 < T)) return false;
  dist = c.d2 > 0.0f ? g.sqrt(c.d2 > 0.0f ? c.d2 : 1.0f) : 0.0f;
  if (!(r - dist > 0.0f)) return false;
  const float inv = g.rcp(1e-6f + dist);
  const float na = c.da * inv, nb = c.db * inv, nw = c.dw * inv;
  nl = V(k == 0 ? nw : na, k == 0 ? na : (k == 1 ? nw : nb), k == 2 ? nw : nb);
  tau = 1.0f - 2.0f * c.u;
  return true;
}

// a candidate's distance as the reduction's key: NaN as +inf (the oracle's fminf skips NaN and
// its tie mask excludes it; with every distance NaN or +inf there is no contact either way)
POB_D float mcand_key(const float d2) { return d2 < __builtin_inff() ? d2 : __builtin_inff(); }

// first strict minimum over a triangle's candidates, with the tie flag: tie when a later
// candidate equals the running minimum (NaN never enters; +inf ties are below nothing)
POB_D void mpick(MCand &best, bool &tie, const MCand &c) {
  const bool lt = c.d2 < best.d2, eq = c.d2 == best.d2;
  tie = lt ? false : (tie | eq);
  if (lt) best = c;
}

// The contacts of face f (0..5) of a wall with half extents (hx, hy, hz) against the capsule's
// segment (capw: mcap_seg of its wall-frame end points; a sphere has A == B), radius r,
// T = r^2 (1 + 2^-20): for triangle t = 0, 1, hit[t] and its contact (tau, wall-frame normal,
// dist).  tau = 1 - 2u places the segment point on the capsule's segment x + tau rotate(e0, q).
// Exact skips (a candidate whose computed d2 is provably >= T can neither win with a contact
// nor change a winner or a tie below T): an edge whose line the segment's box misses by
// >= R = r + 1e-3 across it, the segment-plane candidate when its point is >= R off the plane
// (its triangle points lie in the plane: w = w0 exactly).  (A NaN bound never skips.)
struct MFaceOut {
  bool hit[2];
  float tau[2], dist[2];
  v3 nl[2];
};
template <class G>
POB_D MFaceOut mesh_face_contacts(G &g, const int f, const v3 La, const v3 Lb, const float hx, const float hy,
                                  const float hz, fcptr_t fcw, const float r, const float T) {
  const MFace F = mface(g, f, mcap_seg(g, La, Lb), hx, hy, hz, fcw);
  const float R = r + POB_MESH_MARGIN;
  const F3 A = F.A.p0;
  const float ha = F.ha, hb = F.hb, w0 = F.w0;
  // the segment's box (its end points A and A + d: the points brax's forms produce lie on it)
  const float e_a = A.a + F.A.d.a, e_b = A.b + F.A.d.b, e_w = A.w + F.A.d.w;
  const float amn = fminf(A.a, e_a), amx = fmaxf(A.a, e_a), bmn = fminf(A.b, e_b), bmx = fmaxf(A.b, e_b);
  const float gw = fmaxf(fminf(A.w, e_w) - w0, w0 - fmaxf(A.w, e_w));
  const bool bottom = !(fmaxf(fmaxf(bmn + hb, -hb - bmx), gw) >= R), top = !(fmaxf(fmaxf(bmn - hb, hb - bmx), gw) >= R);
  const bool right = !(fmaxf(fmaxf(amn - ha, ha - amx), gw) >= R), left = !(fmaxf(fmaxf(amn + ha, -ha - amx), gw) >= R);
  MCand c[2];
  bool tie[2] = {false, false};
#pragma unroll
  for (int t = 0; t < 2; ++t) { c[t].d2 = __builtin_inff(); c[t].u = 0.0f; c[t].da = 0.0f; c[t].db = 0.0f; c[t].dw = 0.0f; }
  F3 S, P;
  float u;
  // t0: V0 V1 (bottom), V1 V2 (right), diagonal; t1: diagonal, V2 V3 (top), V0 V3 (left)
  // (MFENCE: one candidate at a time -- interleaved for ILP they need more registers than the
  // four-lane kernel's budget leaves)
  if (bottom) { bseg_seg(g, F.A, medge(F, 0), S, P, u); mpick(c[0], tie[0], bcand(S, P, u)); }
  MFENCE();
  if (right) { bseg_seg(g, F.A, medge(F, 1), S, P, u); mpick(c[0], tie[0], bcand(S, P, u)); }
  MFENCE();
  bseg_seg(g, F.A, medge(F, 2), S, P, u);
  const MCand dg = bcand(S, P, u);
  mpick(c[0], tie[0], dg);
  mpick(c[1], tie[1], dg);
  MFENCE();
  if (top) { bseg_seg(g, F.A, medge(F, 3), S, P, u); mpick(c[1], tie[1], bcand(S, P, u)); }
  MFENCE();
  if (left) { bseg_seg(g, F.A, medge(F, 4), S, P, u); mpick(c[1], tie[1], bcand(S, P, u)); }
  MFENCE();
  const float tt = mface_tt(g, F);
  const F3 sp = f3fma(F.A.d, tt, F.A.p0);
  if (!(fabsf(sp.w - w0) >= R)) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      mpick(c[t], tie[t], bcand(sp, btri_point(mtri(F, t), sp), tt));
      MFENCE();
    }
  }
  MFaceOut o;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    MCand ct = c[t];
    // (rare: two candidates at one distance; the face is formed again from the end points so
    // that its terms need not stay live through the candidates)
    if (tie[t] && ct.d2 < T) ct = mtri_pick_ties_ool(f, La, Lb, hx, hy, hz, fcw, t);
    o.tau[t] = 0.0f; o.dist[t] = 0.0f; o.nl[t] = V(0.0f, 0.0f, 0.0f);
    o.hit[t] = mface_contact(g, f >> 1, ct, r, T, o.tau[t], o.nl[t], o.dist[t]);
  }
  return o;
}
#ifndef POB_MESH_HOST
// out of line (GuardBranch only: stateless): the face's working set leaves the caller's
// register allocation -- the caller saves its live registers around the call, i.e. only when
// a lane of the wave has a face item (POB_MESH_NOINLINE)
__device__ __attribute__((noinline)) MFaceOut mesh_face_ool(const int f, const v3 La, const v3 Lb, const float hx,
                                                         const float hy, const float hz, fcptr_t fcw,
                                                         const float r, const float T) {
  GuardBranch g;
  return mesh_face_contacts(g, f, La, Lb, hx, hy, hz, fcw, r, T);
}
#endif
#ifndef POB_MESH_NOINLINE
#define POB_MESH_NOINLINE 0
#endif
// emit(tau, n_local, dist) for triangle 0 then 1 when it penetrates
template <class G, class Fn>
POB_D void mesh_face(G &g, const int f, const v3 La, const v3 Lb, const float hx, const float hy, const float hz,
                     fcptr_t fcw, const float r, const float T, Fn &&emit) {
#if POB_MESH_NOINLINE && !defined(POB_MESH_HOST)
  if constexpr (std::is_same<G, GuardBranch>::value) {
    const MFaceOut o = mesh_face_ool(f, La, Lb, hx, hy, hz, fcw, r, T);
    if (o.hit[0]) emit(o.tau[0], o.nl[0], o.dist[0]);
    if (o.hit[1]) emit(o.tau[1], o.nl[1], o.dist[1]);
    return;
  }
#endif
  const MFaceOut o = mesh_face_contacts(g, f, La, Lb, hx, hy, hz, fcw, r, T);
  if (o.hit[0]) emit(o.tau[0], o.nl[0], o.dist[0]);
  if (o.hit[1]) emit(o.tau[1], o.nl[1], o.dist[1]);
}

// wall-frame normal -> world (oracle: (nx c - ny s, ny c + nx s, nz) as fmaf(-ny, s, nx c), ..)
POB_D v3 mwall_world_n(const MWall &W, const v3 nl) {
  return V(FMA(-nl.y, W.s, nl.x * W.c), FMA(nl.y, W.c, nl.x * W.s), nl.z);
}

#ifndef POB_MESH_HOST
// ---------------------------------------------------------------- the wave's face walk
// Walk the lanes' face items (M[s]: bit 8 w + f for face f of wall w of the lane's body slot
// s; slots, then bits, in increasing order: the oracle's contact order per body) and call
// apply(s, bit, tau, n_world, dist) on the owning lane for every penetrating triangle, in
// order.  seg_of(s, A, B, r, seg) gives a slot's segment (world end points), radius and
// whether it is a capsule (false: the torso sphere at A).
//
// A face evaluated on one lane is a few hundred instructions (its ten candidates, both
// triangles' picks and emissions, one after another) and few lanes of a wave hold one at a
// time (0.7 items on the busiest lane per wave and collide substep on HH rollouts,
// scripts/wall_walk_stats.py), so the wave shares them out: each round takes the next items
// of up to eight lanes (a lane's next two of one body when fewer lanes have one) and gives
// each of those faces eight lanes -- lane 4 t + kk of the group computes candidate kk of
// triangle t (mface_cand: the triangle's three edges, the segment-plane point) -- reduces
// each triangle's four candidates to the first strict minimum (DPP over the quad,
// lexicographic (d2, kk), with a tie count: a tie below the radius takes brax's averaging on
// the winner lane), lets the winner compute the contact and hands it to the owner
// (ds_bpermute), which applies its triangles in order.  Needs all 64 lanes active (the DPP
// reduction reads every lane of a quad); with lanes masked off -- the batch's last wave, a
// masked reset -- each lane walks its own items (mesh_lane_walk).
static_assert(POB_MAXW <= 8, "face items pack wall w and face f as bit 8 w + f of a uint64_t");
POB_D float mlane_read(const float v, const int src) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}
POB_D int mlane_read_i(const int v, const int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }
template <int CTRL>
POB_D void mlexmin_dpp(float &d, int &kk) {
  const float od = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(d), CTRL, 0xf, 0xf, true));
  const int ok = __builtin_amdgcn_mov_dpp(kk, CTRL, 0xf, 0xf, true);
  const bool take = (od < d) | ((od == d) & (ok < kk));
  d = take ? od : d;
  kk = take ? ok : kk;
}
template <int CTRL>
POB_D int msum_dpp(const int v) { return v + __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, true); }
// lane j's value within the quad (quad_perm [j, j, j, j])
template <int J>
POB_D float mquad_read(const float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), J * 0x55, 0xf, 0xf, true));
}
// brax's tie rule over the quad's four candidates (oracle bpick with cnt > 1): the points,
// parameters of the candidates at the minimum key summed in candidate order from zero, then
// divided by their count -- every lane of the quad active (DPP reads)
template <int J>
POB_D void mtie_add(const float key, const float dmin, const F3 S, const F3 P, const float u, F3 &Ss, F3 &Ps,
                    float &us, float &cnt) {
  const float kj = mquad_read<J>(key);
  const F3 Sj = f3(mquad_read<J>(S.a), mquad_read<J>(S.b), mquad_read<J>(S.w));
  const F3 Pj = f3(mquad_read<J>(P.a), mquad_read<J>(P.b), mquad_read<J>(P.w));
  const float uj = mquad_read<J>(u);
  if (kj == dmin) {
    Ss = f3(Ss.a + Sj.a, Ss.b + Sj.b, Ss.w + Sj.w);
    Ps = f3(Ps.a + Pj.a, Ps.b + Pj.b, Ps.w + Pj.w);
    us += uj;
    cnt += 1.0f;
  }
}

// mface_cand on a triangle's quad (lane kk of the quad holds candidate kk; every lane of the
// quad active): the segment-plane candidate's three triangle-edge projections (btri_point's
// c1..c3) are computed by the edge lanes beside their own candidates and read by lane 3 over
// DPP -- the same operations on the same operands as btri_point, one divergent path shorter
template <class G>
POB_D MCand mface_cand_quad(G &g, const MFace &F, const int t, const int kk, F3 &S, F3 &P) {
  MCand c;
  c.d2 = __builtin_inff(); c.u = 0.0f; c.da = 0.0f; c.db = 0.0f; c.dw = 0.0f;
  S = f3(0.0f, 0.0f, 0.0f);
  P = S;
  const float tt = mface_tt(g, F);
  const F3 S3 = f3fma(F.A.d, tt, F.A.p0);  // the segment-plane point (lane 3's S)
  F3 cq = S;
  float dq = 0.0f;
  if (kk < 3) {
    const int e = t == 0 ? kk : (kk == 0 ? 2 : kk + 2);
    float u;
    bseg_seg(g, F.A, medge(F, e), S, P, u);
    c = bcand(S, P, u);
    // btri_point's edge kk + 1: s01, s12, s20 = V0 V1, V1 V2, V2 V0 (t0) / V0 V2, V2 V3, V3 V0 (t1)
    const int te = kk < 2 ? e : (t == 0 ? 5 : 6);
    float tq;
    cq = bseg_point(medge(F, te), S3, tq);
    dq = f3d2(S3, cq);
  }
  const F3 c1 = f3(mquad_read<0>(cq.a), mquad_read<0>(cq.b), mquad_read<0>(cq.w));
  const F3 c2 = f3(mquad_read<1>(cq.a), mquad_read<1>(cq.b), mquad_read<1>(cq.w));
  const F3 c3 = f3(mquad_read<2>(cq.a), mquad_read<2>(cq.b), mquad_read<2>(cq.w));
  const float d1 = mquad_read<0>(dq), d2 = mquad_read<1>(dq), d3 = mquad_read<2>(dq);
  if (kk == 3) {
    // btri_point(mtri(F, t), S3) with the edge terms from the quad
    const F3 p0 = f3(-F.ha, -F.hb, F.w0);
    const F3 e0 = t == 0 ? f3(F.ha2, 0.0f, 0.0f) : f3(F.ha2, F.hb2, 0.0f);
    const F3 e1 = t == 0 ? f3(F.ha2, F.hb2, 0.0f) : f3(0.0f, F.hb2, 0.0f);
    const float dA = F.ha2 * F.ha2, dB = F.hb2 * F.hb2, e_d = mfc_ed(F);
    const float ta = t == 0 ? dA : e_d, tb = t == 0 ? dA : dB, tc = t == 0 ? e_d : dB;
    const float idet = mfc_idet(F, t);
    const F3 d = f3sub(S3, p0);
    const float e0d = f3dot(e0, d), e1d = f3dot(e1, d);
    const float u = FMA(tc, e0d, -(tb * e1d)) * idet, v = FMA(ta, e1d, -(tb * e0d)) * idet;
    const bool inside = (0.0f <= u) & (u <= 1.0f) & (0.0f <= v) & (v <= 1.0f) & (u + v <= 1.0f);
    F3 cp = f3fma(e1, v, f3fma(e0, u, p0));
    const float d0 = f3d2(cp, S3);
    const bool k0 = (d0 < d1) & inside;
    cp = f3sel(k0, cp, c1);
    float md = k0 ? d0 : d1;
    cp = f3sel(d2 < md, c2, cp);
    md = fminf(md, d2);
    S = S3;
    P = f3sel(d3 < md, c3, cp);
    c = bcand(S, P, tt);
  }
  return c;
}

// each lane walks its own items, one face per iteration (mesh_face)
template <int NB, class G, class SegOf, class Apply>
POB_D void mesh_lane_walk(G &g, const float *WT, fcptr_t FC, const float cz, const float hz, uint64_t (&M)[NB],
                          SegOf &&seg_of, Apply &&apply) {
  while (true) {
    bool has = false;
    int s = 0;
    uint64_t ml = 0ull;
#pragma unroll
    for (int q = NB - 1; q >= 0; --q) {
      const bool h = M[q] != 0ull;
      s = h ? q : s;
      ml = h ? M[q] : ml;
      has = has | h;
    }
    if (!__any(has)) break;
    const int bit = has ? __builtin_ctzll(ml) : 0;
#pragma unroll
    for (int q = 0; q < NB; ++q) M[q] = (has && s == q) ? (M[q] & (M[q] - 1ull)) : M[q];
    if (has) {
      v3 A, B;
      float r;
      bool seg;
      seg_of(s, A, B, r, seg);
      const MWall W = mwall_row(WT + POB_WALL_FLOATS * (bit >> 3));
      const v3 La = mwall_local(W, cz, A);
      const v3 Lb = seg ? mwall_local(W, cz, B) : La;
      const float T = (r * r) * 1.00000095367431640625f;  // r^2 (1 + 2^-20)
      mesh_face(g, bit & 7, La, Lb, W.hx, W.hy, hz, FC + 3 * POB_FACE_FLOATS * (bit >> 3), r, T,
                [&](const float tau, const v3 nl, const float dist) {
        apply(s, bit, tau, mwall_world_n(W, nl), dist);
      });
    }
  }
}

// (LANE_FALLBACK false: the caller guarantees all 64 lanes active and handles the per-lane
// walk itself -- the four-lane kernel keeps it out of line.  HAND, how the contacts reach their
// owners: 0 apply(s, bit, tau, n, dist) on the owner lane, triangle by triangle; 1 the same
// hand-over with apply(want, s, bit, tau, n, dist) called on every lane (want: the owner's flag)
// -- for a caller that allocates wave-shared storage by ballot; 2 the winners store their
// contacts themselves (apply.store(hit, tau, n, dist) on every lane returns the stored entry + 1,
// 0 for none), each triangle's entry is summed over its quad and the owners read their (at most
// four) entries in one pass and link them in order (apply.link(s, bit, entry)): no hand-over loop)
template <int NB, bool LANE_FALLBACK = true, int HAND = 0, class G, class SegOf, class Apply>
POB_D void mesh_wave_walk(G &g, const float *WT, fcptr_t FC, const float cz, const float hz, uint64_t (&M)[NB],
                          SegOf &&seg_of, Apply &&apply) {
  if constexpr (LANE_FALLBACK) {
#ifdef POB_MESH_LANE_WALK
    if (true) {  // A/B build switch: the per-lane walk everywhere
#else
    if (__ballot(1) != ~0ull) {
#endif
      mesh_lane_walk<NB>(g, WT, FC, cz, hz, M, seg_of, apply);
      return;
    }
  }
  const int lane = (int)__lane_id();
  const int grp = lane >> 3, tri = (lane >> 2) & 1, kk = lane & 3;
  while (true) {
    // the lane's next item (slot s, face bit b1) and the one after it in the same slot (b2)
    bool has = false;
    int s = 0;
    uint64_t ml = 0ull;
#pragma unroll
    for (int q = NB - 1; q >= 0; --q) {
      const bool h = M[q] != 0ull;
      s = h ? q : s;
      ml = h ? M[q] : ml;
      has = has | h;
    }
    const uint64_t req1 = __ballot(has);
    if (req1 == 0ull) break;
    const uint64_t rest = ml & (ml - 1ull);
    const bool has2 = has && rest != 0ull;
    const uint64_t req2 = __ballot(has2);
    const int b1 = has ? __builtin_ctzll(ml) : 0, b2 = has2 ? __builtin_ctzll(rest) : 0;
    // a round's eight groups: the first items of the first eight lanes with one, then (when
    // fewer) the second items of lanes with two -- each lane's items in its order
    const int n1 = __builtin_popcountll(req1), n2 = __builtin_popcountll(req2);
    const uint32_t r1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(req1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)req1, 0u));
    const uint32_t r2 = (uint32_t)n1 +
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(req2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)req2, 0u));
    const bool own1 = has && r1 < 8u, own2 = has2 && r2 < 8u;  // (own2 implies own1: n1 < 8)
    const uint64_t pop = (own1 ? 1ull << b1 : 0ull) | (own2 ? 1ull << b2 : 0ull);
    const int g1 = 8 * (int)r1, g2 = 8 * (int)r2;  // the first lanes of the owner's groups
#pragma unroll
    for (int q = 0; q < NB; ++q) M[q] = s == q ? (M[q] & ~pop) : M[q];
    // group owners: each owner sends its lane number to its groups' first lanes (forward
    // permutes; the other lanes write odd lanes, never read), each group reads its first lane
    const bool gv = grp < n1 + n2;
    const bool second = grp >= n1;
    int ol;
    {
      const int p1 = __builtin_amdgcn_ds_permute((own1 ? g1 : (lane | 1)) << 2, lane);
      const int p2 = __builtin_amdgcn_ds_permute((own2 ? g2 : (lane | 1)) << 2, lane);
      const int o = __builtin_amdgcn_ds_bpermute((lane & ~7) << 2, second ? p2 : p1);
      ol = gv ? (o & 63) : 0;
    }
    v3 A, B;
    float r;
    bool seg;
    seg_of(s, A, B, r, seg);
    const int meta1 = b1 | (seg ? 64 : 0), meta2 = b2 | (seg ? 64 : 0);
    const v3 Ao = V(mlane_read(A.x, ol), mlane_read(A.y, ol), mlane_read(A.z, ol));
    const v3 Bo = V(mlane_read(B.x, ol), mlane_read(B.y, ol), mlane_read(B.z, ol));
    const float ro = mlane_read(r, ol);
    const int ma = mlane_read_i(meta1, ol), mb = mlane_read_i(meta2, ol);
    const int mo = second ? mb : ma;
    const bool sego = (mo & 64) != 0;
    const MWall W = mwall_row(WT + POB_WALL_FLOATS * ((mo >> 3) & 7));
    fcptr_t fcw = FC + 3 * POB_FACE_FLOATS * ((mo >> 3) & 7);
    const v3 La = mwall_local(W, cz, Ao);
    const v3 Lb = sego ? mwall_local(W, cz, Bo) : La;
    const MFace F = mface(g, mo & 7, mcap_seg(g, La, Lb), W.hx, W.hy, hz, fcw);
    F3 Sc, Pc;
    MCand c = mface_cand_quad(g, F, tri, gv ? kk : 7, Sc, Pc);
    c.d2 = mcand_key(c.d2);
    // each triangle's first strict minimum over its quad, and the number of candidates at it
    float dmin = c.d2;
    int kmin = kk;
    mlexmin_dpp<0xB1>(dmin, kmin);  // quad_perm [1, 0, 3, 2]
    mlexmin_dpp<0x4E>(dmin, kmin);  // quad_perm [2, 3, 0, 1]
    const int neq = msum_dpp<0x4E>(msum_dpp<0xB1>(c.d2 == dmin ? 1 : 0));
    const float T = (ro * ro) * 1.00000095367431640625f;
    // (rare) two or more candidates at a minimum below the radius: brax's average of them,
    // gathered over the quad (the same sums as the oracle's bpick, in candidate order)
    const bool tie = gv && neq > 1 && dmin < T;
    if (__any(tie)) {
      F3 Ss = f3(0.0f, 0.0f, 0.0f), Ps = Ss;
      float us = 0.0f, cnt = 0.0f;
      mtie_add<0>(c.d2, dmin, Sc, Pc, c.u, Ss, Ps, us, cnt);
      mtie_add<1>(c.d2, dmin, Sc, Pc, c.u, Ss, Ps, us, cnt);
      mtie_add<2>(c.d2, dmin, Sc, Pc, c.u, Ss, Ps, us, cnt);
      mtie_add<3>(c.d2, dmin, Sc, Pc, c.u, Ss, Ps, us, cnt);
      if (tie && kk == kmin) c = bcand(f3(Ss.a / cnt, Ss.b / cnt, Ss.w / cnt), f3(Ps.a / cnt, Ps.b / cnt, Ps.w / cnt), us / cnt);
    }
    float tau = 0.0f, dst = 0.0f;
    v3 nw = V(0.0f, 0.0f, 0.0f);
    bool hit = false;
    if (gv && kk == kmin) {
      v3 nl;
      hit = mface_contact(g, F.k, c, ro, T, tau, nl, dst);
      if (hit) nw = mwall_world_n(W, nl);
    }
    if constexpr (HAND == 2) {
      // the winners' entries (a lane-order compaction: group, then triangle order -- each owner's
      // contacts in walk order), summed over each triangle's quad (only its winner is nonzero)
      const int e = apply.store(hit, tau, nw, dst);
      const int eq = msum_dpp<0x4E>(msum_dpp<0xB1>(e));
      const int e10 = mlane_read_i(eq, g1), e11 = mlane_read_i(eq, g1 + 4);
      const int e20 = mlane_read_i(eq, g2), e21 = mlane_read_i(eq, g2 + 4);
      if (own1) { apply.link(s, b1, e10); apply.link(s, b1, e11); }
      if (own2) { apply.link(s, b2, e20); apply.link(s, b2, e21); }
    } else {
      // the owners take their items' triangles in order: the winners' lanes first (all four
      // fetches in flight), then each contact
      const int w10 = g1 + mlane_read_i(kmin, g1), w11 = g1 + 4 + mlane_read_i(kmin, g1 + 4);
      const int w20 = g2 + mlane_read_i(kmin, g2), w21 = g2 + 4 + mlane_read_i(kmin, g2 + 4);
      const int nt = __any(own2) ? 4 : 2;
#pragma nounroll
      for (int t = 0; t < nt; ++t) {
        const int wl = t == 0 ? w10 : (t == 1 ? w11 : (t == 2 ? w20 : w21));
        const int h = mlane_read_i(hit ? 1 : 0, wl);
        const float tw = mlane_read(tau, wl), dw = mlane_read(dst, wl);
        const v3 nn = V(mlane_read(nw.x, wl), mlane_read(nw.y, wl), mlane_read(nw.z, wl));
        if constexpr (HAND == 1) apply((t < 2 ? own1 : own2) && h != 0, s, t < 2 ? b1 : b2, tw, nn, dw);
        else if ((t < 2 ? own1 : own2) && h != 0) apply(s, t < 2 ? b1 : b2, tw, nn, dw);
      }
    }
  }
}
#endif  // POB_MESH_HOST
