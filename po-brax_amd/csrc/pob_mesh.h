// pob_mesh.h -- Ant x Arena contacts on gfx950: brax v1's capsule x TriangulatedBox path
// (capsule_mesh) as restated in DESIGN.md §3 and oracle/pob_oracle.c capsule_wall_mesh.
//
// Every arena wall is a box collider of the frozen Arena body (po_brax/envs/utils.py:6-28,
// add_box_wall_to_body; ant x Arena in collide_include, ant_heavenhell.py:33-34).  brax v1
// meshes a box into 12 triangles and, for every triangle, takes the closest points of the
// capsule's segment and the triangle; a triangle closer than the capsule radius is one contact
// (penetration r - |S - P|, normal along S - P), and every such contact is applied.  The
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
#include "pob_math.h"

#define POB_MESH_MARGIN 1e-3f

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

POB_D float clamp01(float x) { return __builtin_amdgcn_fmed3f(x, 0.0f, 1.0f); }

// is (pa, pb) in face triangle t (boundary included)?  (oracle tri_inside)
POB_D bool mtri_inside(const bool t1, const float ha, const float hb, const float pa, const float pb) {
  const float cr = FMA(pa + ha, hb, -((pb + hb) * ha));
  return t1 ? ((pb <= hb) & (pa >= -ha) & (cr <= 0.0f)) : ((pb >= -hb) & (pa <= ha) & (cr >= 0.0f));
}

// running closest candidate: squared distance, segment parameter, S - P (face coordinates)
struct MCand {
  float d2, u, da, db, dw;
};
POB_D void mcand_take(MCand &c, const float u, const float da, const float db, const float dw) {
  const float d2 = FMA(dw, dw, FMA(db, db, da * da));
  if (d2 < c.d2) { c.d2 = d2; c.u = u; c.da = da; c.db = db; c.dw = dw; }
}

// closest point of face triangle t to the plane point (pa, pb) (oracle tri_closest): the point
// if inside, else the first strict minimum over the triangle's edges' nearest points;
// the diagonal D = (2ha, 2hb), inv_dd = 1 / (D . D)
POB_D void mtri_closest(const bool t1, const float ha, const float hb, const float ha2, const float hb2,
                        const float inv_dd, const float pa, const float pb, float &qa, float &qb) {
  if (mtri_inside(t1, ha, hb, pa, pb)) { qa = pa; qb = pb; return; }
  const float s = clamp01(FMA(pb + hb, hb2, (pa + ha) * ha2) * inv_dd);
  const float s2 = 2.0f * s;
  const float da = FMA(s2, ha, -ha), db = FMA(s2, hb, -hb);
  const float ca = clamp_sym(pa, ha), cb = clamp_sym(pb, hb);
  // triangle 0: bottom (ca, -hb), right (ha, cb), diagonal; triangle 1: diagonal, top (ca, hb), left (-ha, cb)
  const float e0a = t1 ? da : ca, e0b = t1 ? db : -hb;
  const float e1a = t1 ? ca : ha, e1b = t1 ? hb : cb;
  const float e2a = t1 ? -ha : da, e2b = t1 ? cb : db;
  float g0 = pa - e0a, h0 = pb - e0b;
  float best = FMA(h0, h0, g0 * g0);
  qa = e0a; qb = e0b;
  const float g1 = pa - e1a, h1 = pb - e1b;
  const float d1 = FMA(h1, h1, g1 * g1);
  if (d1 < best) { best = d1; qa = e1a; qb = e1b; }
  const float g2 = pa - e2a, h2 = pb - e2b;
  const float d2 = FMA(h2, h2, g2 * g2);
  if (d2 < best) { qa = e2a; qb = e2b; }
}

// closest points of the segment A + u D and the edge E0 + t F (in the face plane w = w0):
// the oracle's seg_edge (Ericson's clamped form) as a candidate update
struct MSeg {
  float aa_, ab, aw, Da, Db, Dw, aa, inv_aa;  // A (face coordinates), D = B - A, D . D, 1 / D . D
};
template <class G>
POB_D void mseg_edge(G &g, MCand &c, const MSeg &S, const float e0a, const float e0b, const float w0, const float fa,
                     const float fb, const float ee, const float inv_ee) {
  const float ra = S.aa_ - e0a, rb = S.ab - e0b, rw = S.aw - w0;
  const float f = FMA(fb, rb, fa * ra);
  const float cc = FMA(S.Dw, rw, FMA(S.Db, rb, S.Da * ra));
  const float bb = FMA(S.Db, fb, S.Da * fa);
  const float den = FMA(S.aa, ee, -(bb * bb));
  float u = 0.0f;
  if (den > 0.0f) u = clamp01(FMA(bb, f, -(cc * ee)) * g.rcp(den));
  float t = FMA(bb, u, f) * inv_ee;
  if (t < 0.0f) { t = 0.0f; u = clamp01(-cc * S.inv_aa); }
  else if (t > 1.0f) { t = 1.0f; u = clamp01((bb - cc) * S.inv_aa); }
  const float sa = FMA(u, S.Da, S.aa_), sb = FMA(u, S.Db, S.ab), sw = FMA(u, S.Dw, S.aw);
  mcand_take(c, u, sa - FMA(t, fa, e0a), sb - FMA(t, fb, e0b), sw - w0);
}

// The contacts of face f (0..5) of a wall with half extents (hx, hy, hz) against the segment
// [A, B] (wall frame; seg = false: the point A, the torso sphere), radius r, T = r^2 (1 + 2^-20):
// emit(tau, n_local, pen) for triangle 0 then 1 when it penetrates.  tau = 1 - 2u places the
// contact on the capsule's segment x + tau rotate(e0, q) (A = x + rotate(e0), B = x - rotate(e0)).
// A triangle with d2 >= T has sqrt_rn(d2) >= r (no contact): its square root is skipped.
template <class G, class F>
POB_D void mesh_face(G &g, const int f, const v3 A, const v3 B, const bool seg, const float hx, const float hy,
                     const float hz, const float r, const float T, F &&emit) {
  const int k = f >> 1;
  const float sg = (f & 1) ? 1.0f : -1.0f;
  // face coordinates (a, b, w): k = 0 (y, z, x), 1 (x, z, y), 2 (x, y, z)
  const float ha = k == 0 ? hy : hx, hb = k == 2 ? hy : hz, hw = k == 0 ? hx : (k == 1 ? hy : hz);
  const float w0 = sg * hw;
  MSeg S;
  S.aa_ = k == 0 ? A.y : A.x;
  S.ab = k == 2 ? A.y : A.z;
  S.aw = k == 0 ? A.x : (k == 1 ? A.y : A.z);
  const float Ba = k == 0 ? B.y : B.x, Bb = k == 2 ? B.y : B.z, Bw = k == 0 ? B.x : (k == 1 ? B.y : B.z);
  const float ha2 = 2.0f * ha, hb2 = 2.0f * hb;
  const float e_d = FMA(hb2, hb2, ha2 * ha2), i_d = g.rcp(e_d);
  MCand c[2];
  // end point A (and B) against each triangle
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float qa, qb;
    mtri_closest(t == 1, ha, hb, ha2, hb2, i_d, S.aa_, S.ab, qa, qb);
    c[t].d2 = __builtin_inff(); c[t].u = 0.0f; c[t].da = 0.0f; c[t].db = 0.0f; c[t].dw = 0.0f;
    mcand_take(c[t], 0.0f, S.aa_ - qa, S.ab - qb, S.aw - w0);
  }
  if (seg) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float qa, qb;
      mtri_closest(t == 1, ha, hb, ha2, hb2, i_d, Ba, Bb, qa, qb);
      mcand_take(c[t], 1.0f, Ba - qa, Bb - qb, Bw - w0);
    }
    S.Da = Ba - S.aa_; S.Db = Bb - S.ab; S.Dw = Bw - S.aw;
    S.aa = FMA(S.Dw, S.Dw, FMA(S.Db, S.Db, S.Da * S.Da));
    S.inv_aa = g.rcp(S.aa);
    const float e_a = ha2 * ha2, e_b = hb2 * hb2;
    const float i_a = g.rcp(e_a), i_b = g.rcp(e_b);
    // triangle 0: bottom, right, diagonal; triangle 1: diagonal, top, left (the diagonal's
    // candidate is the same closest pair for both: evaluated once, taken in each order)
    mseg_edge(g, c[0], S, -ha, -hb, w0, ha2, 0.0f, e_a, i_a);
    mseg_edge(g, c[0], S, ha, -hb, w0, 0.0f, hb2, e_b, i_b);
    MCand dg;
    dg.d2 = __builtin_inff(); dg.u = 0.0f; dg.da = 0.0f; dg.db = 0.0f; dg.dw = 0.0f;
    mseg_edge(g, dg, S, -ha, -hb, w0, ha2, hb2, e_d, i_d);
    // (taken on its own squared distance: an untaken dg -- a NaN or overflowing candidate,
    // which the oracle never takes -- keeps d2 = inf, not the 0 of its cleared fields)
#pragma unroll
    for (int t = 0; t < 2; ++t)
      if (dg.d2 < c[t].d2) c[t] = dg;
    mseg_edge(g, c[1], S, ha, hb, w0, -ha2, 0.0f, e_a, i_a);
    mseg_edge(g, c[1], S, -ha, hb, w0, 0.0f, -hb2, e_b, i_b);
    // the segment crossing the face plane inside the triangle
    const float aw = S.aw - w0, bw = Bw - w0;
    if (((aw < 0.0f) & (bw > 0.0f)) | ((aw > 0.0f) & (bw < 0.0f))) {
      const float u = aw * g.rcp(aw - bw);
      const float sa = FMA(u, S.Da, S.aa_), sb = FMA(u, S.Db, S.ab), sw = FMA(u, S.Dw, S.aw);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (mtri_inside(t == 1, ha, hb, sa, sb)) mcand_take(c[t], u, 0.0f, 0.0f, sw - w0);
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (c[t].d2 < T) {
      float dist, inv;
      g.sqrt_rcp(c[t].d2, dist, inv);
      const float pen = r - dist;
      if (pen > 0.0f) {
        float na, nb, nw;
        if (c[t].d2 > 0.0f) { na = c[t].da * inv; nb = c[t].db * inv; nw = c[t].dw * inv; }
        else { na = 0.0f; nb = 0.0f; nw = sg; }
        // face -> wall frame
        const v3 nl = V(k == 0 ? nw : na, k == 0 ? na : (k == 1 ? nw : nb), k == 2 ? nw : nb);
        emit(1.0f - 2.0f * c[t].u, nl, pen);
      }
    }
  }
}

// wall-frame normal -> world (oracle: (nx c - ny s, ny c + nx s, nz) as fmaf(-ny, s, nx c), ..)
POB_D v3 mwall_world_n(const MWall &W, const v3 nl) {
  return V(FMA(-nl.y, W.s, nl.x * W.c), FMA(nl.y, W.c, nl.x * W.s), nl.z);
}
