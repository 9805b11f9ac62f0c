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

// mtri_closest for both triangles of the face at once (mesh_face): the inside tests share the
// diagonal's cross term, the edge points their clamps and the diagonal's closest point -- the
// same operations on the same operands as two mtri_closest calls, each computed once
POB_D void mtri_closest2(const float ha, const float hb, const float ha2, const float hb2, const float inv_dd,
                         const float pa, const float pb, float &qa0, float &qb0, float &qa1, float &qb1) {
  const float cr = FMA(pa + ha, hb, -((pb + hb) * ha));
  const bool in0 = (pb >= -hb) & (pa <= ha) & (cr >= 0.0f);
  const bool in1 = (pb <= hb) & (pa >= -ha) & (cr <= 0.0f);
  const float s = clamp01(FMA(pb + hb, hb2, (pa + ha) * ha2) * inv_dd);
  const float s2 = 2.0f * s;
  const float da = FMA(s2, ha, -ha), db = FMA(s2, hb, -hb);
  const float ca = clamp_sym(pa, ha), cb = clamp_sym(pb, hb);
  // squared distances to the edge points: bottom (ca, -hb), right (ha, cb), diagonal (da, db),
  // top (ca, hb), left (-ha, cb)
  const float gc = pa - ca, gd = pa - da, gr = pa - ha, gl = pa - -ha;
  const float hbt = pb - -hb, hd = pb - db, hcb = pb - cb, htp = pb - hb;
  const float dbot = FMA(hbt, hbt, gc * gc), drt = FMA(hcb, hcb, gr * gr), ddg = FMA(hd, hd, gd * gd);
  const float dtop = FMA(htp, htp, gc * gc), dlf = FMA(hcb, hcb, gl * gl);
  // triangle 0: bottom, right, diagonal; triangle 1: diagonal, top, left (first strict minimum)
  float b0 = dbot, a0 = ca, c0 = -hb;
  if (drt < b0) { b0 = drt; a0 = ha; c0 = cb; }
  if (ddg < b0) { a0 = da; c0 = db; }
  float b1 = ddg, a1 = da, c1 = db;
  if (dtop < b1) { b1 = dtop; a1 = ca; c1 = hb; }
  if (dlf < b1) { a1 = -ha; c1 = cb; }
  qa0 = in0 ? pa : a0; qb0 = in0 ? pb : c0;
  qa1 = in1 ? pa : a1; qb1 = in1 ? pb : c1;
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
#pragma unroll
  for (int t = 0; t < 2; ++t) { c[t].d2 = __builtin_inff(); c[t].u = 0.0f; c[t].da = 0.0f; c[t].db = 0.0f; c[t].dw = 0.0f; }
  // Exact skips: a candidate provably farther than R = r + 1e-3 from the triangle has a computed
  // d2 above T (coordinate errors here are ~1e-6), so it can neither win with a contact nor
  // change a winner without one -- the face cull's argument, per candidate: an end point at
  // |w - w0| >= R from the face plane, an edge whose line the segment's box misses by >= R
  // along one of the two axes across it.  (A NaN bound never skips.)
  const float R = r + POB_MESH_MARGIN;
  // end point A (and B) against each triangle
  if (!(fabsf(S.aw - w0) >= R)) {
    float qa[2], qb[2];
    mtri_closest2(ha, hb, ha2, hb2, i_d, S.aa_, S.ab, qa[0], qb[0], qa[1], qb[1]);
#pragma unroll
    for (int t = 0; t < 2; ++t) mcand_take(c[t], 0.0f, S.aa_ - qa[t], S.ab - qb[t], S.aw - w0);
  }
  if (seg) {
    if (!(fabsf(Bw - w0) >= R)) {
      float qa[2], qb[2];
      mtri_closest2(ha, hb, ha2, hb2, i_d, Ba, Bb, qa[0], qb[0], qa[1], qb[1]);
#pragma unroll
      for (int t = 0; t < 2; ++t) mcand_take(c[t], 1.0f, Ba - qa[t], Bb - qb[t], Bw - w0);
    }
    S.Da = Ba - S.aa_; S.Db = Bb - S.ab; S.Dw = Bw - S.aw;
    S.aa = FMA(S.Dw, S.Dw, FMA(S.Db, S.Db, S.Da * S.Da));
    S.inv_aa = g.rcp(S.aa);
    const float e_a = ha2 * ha2, e_b = hb2 * hb2;
    const float i_a = g.rcp(e_a), i_b = g.rcp(e_b);
    // the segment's box across the edges: gaps to a = +-ha, b = +-hb and to the plane
    const float amn = fminf(S.aa_, Ba), amx = fmaxf(S.aa_, Ba), bmn = fminf(S.ab, Bb), bmx = fmaxf(S.ab, Bb);
    const float gw = fmaxf(fminf(S.aw, Bw) - w0, w0 - fmaxf(S.aw, Bw));
    const bool bottom = !(fmaxf(fmaxf(bmn + hb, -hb - bmx), gw) >= R), top = !(fmaxf(fmaxf(bmn - hb, hb - bmx), gw) >= R);
    const bool right = !(fmaxf(fmaxf(amn - ha, ha - amx), gw) >= R), left = !(fmaxf(fmaxf(amn + ha, -ha - amx), gw) >= R);
    // triangle 0: bottom, right, diagonal; triangle 1: diagonal, top, left (the diagonal's
    // candidate is the same closest pair for both: evaluated once, taken in each order)
    if (bottom) mseg_edge(g, c[0], S, -ha, -hb, w0, ha2, 0.0f, e_a, i_a);
    if (right) mseg_edge(g, c[0], S, ha, -hb, w0, 0.0f, hb2, e_b, i_b);
    MCand dg;
    dg.d2 = __builtin_inff(); dg.u = 0.0f; dg.da = 0.0f; dg.db = 0.0f; dg.dw = 0.0f;
    mseg_edge(g, dg, S, -ha, -hb, w0, ha2, hb2, e_d, i_d);
    // (taken on its own squared distance: an untaken dg -- a NaN or overflowing candidate,
    // which the oracle never takes -- keeps d2 = inf, not the 0 of its cleared fields)
#pragma unroll
    for (int t = 0; t < 2; ++t)
      if (dg.d2 < c[t].d2) c[t] = dg;
    if (top) mseg_edge(g, c[1], S, ha, hb, w0, -ha2, 0.0f, e_a, i_a);
    if (left) mseg_edge(g, c[1], S, -ha, hb, w0, 0.0f, -hb2, e_b, i_b);
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
      // (d2 = 0: the segment touches or pierces the triangle -- common when a leg goes through
      // a wall -- has distance 0 exactly and uses no reciprocal; kept out of the range guards,
      // whose rerun (GuardAcc) would double the wave's step)
      float dist = 0.0f, inv = 0.0f;
      if (c[t].d2 > 0.0f) g.sqrt_rcp(c[t].d2, dist, inv);
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

// ---------------------------------------------------------------- one candidate at a time
// mesh_face's work split into independent pieces, so that the lanes of a wave can evaluate a
// face's candidates side by side (mesh_wave_walk): the face frame, each candidate on its own,
// and the contact of a triangle's winner.  The first strict minimum of mesh_face's sequential
// candidate order is the lexicographic minimum of (d2, position in that order) over the
// candidates (mcand_take never stores a NaN; a candidate it does not take keeps d2 = +inf), so
// the winner, and with it every bit of the contact, is mesh_face's.
struct MFace {
  int k;
  float sg, ha, hb, w0, ha2, hb2, i_d;
  float pa, pb, pw, qa, qb, qw;  // end points A and B in face coordinates (a, b, w)
};
template <class G>
POB_D MFace mface(G &g, const int f, const v3 A, const v3 B, const float hx, const float hy, const float hz) {
  MFace F;
  const int k = f >> 1;
  F.k = k;
  F.sg = (f & 1) ? 1.0f : -1.0f;
  F.ha = k == 0 ? hy : hx;
  F.hb = k == 2 ? hy : hz;
  F.w0 = F.sg * (k == 0 ? hx : (k == 1 ? hy : hz));
  F.pa = k == 0 ? A.y : A.x; F.pb = k == 2 ? A.y : A.z; F.pw = k == 0 ? A.x : (k == 1 ? A.y : A.z);
  F.qa = k == 0 ? B.y : B.x; F.qb = k == 2 ? B.y : B.z; F.qw = k == 0 ? B.x : (k == 1 ? B.y : B.z);
  F.ha2 = 2.0f * F.ha;
  F.hb2 = 2.0f * F.hb;
  F.i_d = g.rcp(FMA(F.hb2, F.hb2, F.ha2 * F.ha2));
  return F;
}

// Candidate kk of triangle t, in mesh_face's order: 0 / 1 the end point A / B, 2..4 the
// triangle's edges (t = 0: bottom, right, diagonal; t = 1: diagonal, top, left), 5 the segment
// crossing the face plane inside the triangle.  Any other kk, or a candidate that does not
// apply (a sphere has its point only; no crossing), stays at d2 = +inf.  The same operations
// on the same operands as mesh_face (its reciprocals 1 / e_a, 1 / e_b, 1 / (D . D) are taken
// here only by the candidates that use them: the same values).
template <class G>
POB_D MCand mface_cand(G &g, const MFace &F, const bool seg, const int t, const int kk) {
  MCand c;
  c.d2 = __builtin_inff(); c.u = 0.0f; c.da = 0.0f; c.db = 0.0f; c.dw = 0.0f;
  if (kk == 0 || (kk == 1 && seg)) {
    const float pa = kk == 0 ? F.pa : F.qa, pb = kk == 0 ? F.pb : F.qb, pw = kk == 0 ? F.pw : F.qw;
    float qa, qb;
    mtri_closest(t == 1, F.ha, F.hb, F.ha2, F.hb2, F.i_d, pa, pb, qa, qb);
    mcand_take(c, kk == 0 ? 0.0f : 1.0f, pa - qa, pb - qb, pw - F.w0);
  } else if (seg && kk >= 2 && kk <= 5) {
    MSeg S;
    S.aa_ = F.pa; S.ab = F.pb; S.aw = F.pw;
    S.Da = F.qa - F.pa; S.Db = F.qb - F.pb; S.Dw = F.qw - F.pw;
    if (kk < 5) {
      S.aa = FMA(S.Dw, S.Dw, FMA(S.Db, S.Db, S.Da * S.Da));
      S.inv_aa = g.rcp(S.aa);
      const bool diag = t == 0 ? kk == 4 : kk == 2;
      const bool first = t == 0 ? kk == 2 : kk == 3;  // bottom (t = 0) / top (t = 1): along a
      const float ha = F.ha, hb = F.hb, ha2 = F.ha2, hb2 = F.hb2;
      // edges: bottom (-ha, -hb) + (2ha, 0), right (ha, -hb) + (0, 2hb), diagonal (-ha, -hb) +
      // (2ha, 2hb), top (ha, hb) + (-2ha, 0), left (-ha, hb) + (0, -2hb)
      const float e0a = diag ? -ha : (t == 0 ? (first ? -ha : ha) : (first ? ha : -ha));
      const float e0b = diag ? -hb : (t == 0 ? -hb : hb);
      const float fa = diag ? ha2 : (first ? (t == 0 ? ha2 : -ha2) : 0.0f);
      const float fb = diag ? hb2 : (first ? 0.0f : (t == 0 ? hb2 : -hb2));
      const float ee = diag ? FMA(hb2, hb2, ha2 * ha2) : (first ? ha2 * ha2 : hb2 * hb2);
      mseg_edge(g, c, S, e0a, e0b, F.w0, fa, fb, ee, diag ? F.i_d : g.rcp(ee));
    } else {
      const float aw = F.pw - F.w0, bw = F.qw - F.w0;
      if (((aw < 0.0f) & (bw > 0.0f)) | ((aw > 0.0f) & (bw < 0.0f))) {
        const float u = aw * g.rcp(aw - bw);
        const float sa = FMA(u, S.Da, S.aa_), sb = FMA(u, S.Db, S.ab), sw = FMA(u, S.Dw, S.aw);
        if (mtri_inside(t == 1, F.ha, F.hb, sa, sb)) mcand_take(c, u, 0.0f, 0.0f, sw - F.w0);
      }
    }
  }
  return c;
}

// mface_cand without branches (the cooperative walk: a wave's lanes hold different kinds, so
// a kind's branch would be executed by the whole wave anyway): every form -- the end point, the
// edge, the crossing -- computed, the lane's kind selected.  The same operations on the same
// operands as mface_cand where its branches are taken; the forms a lane does not need run on
// substituted operands (1 under a reciprocal) that keep the range guards quiet.
template <class G>
POB_D MCand mface_cand_bf(G &g, const MFace &F, const bool seg, const int t, const int kk) {
  const bool t1 = t == 1;
  // end point kk (A for 0, B for 1)
  const bool ep = kk == 0 || (kk == 1 && seg);
  const bool isb = kk == 1;
  const float pa = isb ? F.qa : F.pa, pb = isb ? F.qb : F.pb, pw = isb ? F.qw : F.pw;
  float qa, qb;
  {
    const float ha = F.ha, hb = F.hb;
    const float cr = FMA(pa + ha, hb, -((pb + hb) * ha));
    const bool in = t1 ? ((pb <= hb) & (pa >= -ha) & (cr <= 0.0f)) : ((pb >= -hb) & (pa <= ha) & (cr >= 0.0f));
    const float s_ = clamp01(FMA(pb + hb, F.hb2, (pa + ha) * F.ha2) * F.i_d);
    const float s2 = 2.0f * s_;
    const float da = FMA(s2, ha, -ha), db = FMA(s2, hb, -hb);
    const float ca = clamp_sym(pa, ha), cb = clamp_sym(pb, hb);
    const float e0a = t1 ? da : ca, e0b = t1 ? db : -hb;
    const float e1a = t1 ? ca : ha, e1b = t1 ? hb : cb;
    const float e2a = t1 ? -ha : da, e2b = t1 ? cb : db;
    const float g0 = pa - e0a, h0 = pb - e0b;
    float best = FMA(h0, h0, g0 * g0);
    float ra = e0a, rb = e0b;
    const float g1 = pa - e1a, h1 = pb - e1b;
    const float d1 = FMA(h1, h1, g1 * g1);
    const bool b1 = d1 < best;
    best = b1 ? d1 : best; ra = b1 ? e1a : ra; rb = b1 ? e1b : rb;
    const float g2 = pa - e2a, h2 = pb - e2b;
    const float d2 = FMA(h2, h2, g2 * g2);
    const bool b2 = d2 < best;
    ra = b2 ? e2a : ra; rb = b2 ? e2b : rb;
    qa = in ? pa : ra; qb = in ? pb : rb;
  }
  const float ea_ = pa - qa, eb_ = pb - qb, ew_ = pw - F.w0;
  const float e_d2 = FMA(ew_, ew_, FMA(eb_, eb_, ea_ * ea_));
  // edge kk (2..4) of triangle t
  MSeg S;
  S.aa_ = F.pa; S.ab = F.pb; S.aw = F.pw;
  S.Da = F.qa - F.pa; S.Db = F.qb - F.pb; S.Dw = F.qw - F.pw;
  const bool ed = seg && kk >= 2 && kk <= 4;
  S.aa = FMA(S.Dw, S.Dw, FMA(S.Db, S.Db, S.Da * S.Da));
  S.inv_aa = g.rcp(ed ? S.aa : 1.0f);
  const bool diag = t == 0 ? kk == 4 : kk == 2;
  const bool first = t == 0 ? kk == 2 : kk == 3;
  const float ha = F.ha, hb = F.hb, ha2 = F.ha2, hb2 = F.hb2;
  const float e0a = diag ? -ha : (t == 0 ? (first ? -ha : ha) : (first ? ha : -ha));
  const float e0b = diag ? -hb : (t == 0 ? -hb : hb);
  const float fa = diag ? ha2 : (first ? (t == 0 ? ha2 : -ha2) : 0.0f);
  const float fb = diag ? hb2 : (first ? 0.0f : (t == 0 ? hb2 : -hb2));
  const float ee = diag ? FMA(hb2, hb2, ha2 * ha2) : (first ? ha2 * ha2 : hb2 * hb2);
  const float inv_ee = diag ? F.i_d : g.rcp(ed ? ee : 1.0f);
  float su, sda, sdb, sdw;
  {
    const float ra = S.aa_ - e0a, rb = S.ab - e0b, rw = S.aw - F.w0;
    const float f = FMA(fb, rb, fa * ra);
    const float cc = FMA(S.Dw, rw, FMA(S.Db, rb, S.Da * ra));
    const float bb = FMA(S.Db, fb, S.Da * fa);
    const float den = FMA(S.aa, ee, -(bb * bb));
    const bool dp = den > 0.0f;
    const float u0 = dp ? clamp01(FMA(bb, f, -(cc * ee)) * g.rcp(ed && dp ? den : 1.0f)) : 0.0f;
    const float t0 = FMA(bb, u0, f) * inv_ee;
    const bool tl = t0 < 0.0f, tg = !tl && (t0 > 1.0f);
    const float u = tl ? clamp01(-cc * S.inv_aa) : (tg ? clamp01((bb - cc) * S.inv_aa) : u0);
    const float tt = tl ? 0.0f : (tg ? 1.0f : t0);
    const float sa = FMA(u, S.Da, S.aa_), sb = FMA(u, S.Db, S.ab), sw = FMA(u, S.Dw, S.aw);
    su = u; sda = sa - FMA(tt, fa, e0a); sdb = sb - FMA(tt, fb, e0b); sdw = sw - F.w0;
  }
  const float s_d2 = FMA(sdw, sdw, FMA(sdb, sdb, sda * sda));
  // the crossing (kk 5)
  const float aw = F.pw - F.w0, bw = F.qw - F.w0;
  const bool cr = seg && kk == 5 && (((aw < 0.0f) & (bw > 0.0f)) | ((aw > 0.0f) & (bw < 0.0f)));
  const float cu = aw * g.rcp(cr ? aw - bw : 1.0f);
  const float csa = FMA(cu, S.Da, S.aa_), csb = FMA(cu, S.Db, S.ab), csw = FMA(cu, S.Dw, S.aw);
  const bool cin = cr && (t1 ? ((csb <= hb) & (csa >= -ha) & (FMA(csa + ha, hb, -((csb + hb) * ha)) <= 0.0f))
                             : ((csb >= -hb) & (csa <= ha) & (FMA(csa + ha, hb, -((csb + hb) * ha)) >= 0.0f)));
  const float cdw = csw - F.w0;
  const float c_d2 = FMA(cdw, cdw, FMA(0.0f, 0.0f, 0.0f * 0.0f));
  // the lane's kind (mcand_take's rule: a NaN or +inf d2 is not taken: d2 stays +inf, fields 0)
  MCand c;
  const float d2 = ep ? e_d2 : (ed ? s_d2 : (cin ? c_d2 : __builtin_inff()));
  const bool take = d2 < __builtin_inff();
  c.d2 = take ? d2 : __builtin_inff();
  c.u = take ? (ep ? (isb ? 1.0f : 0.0f) : (ed ? su : cu)) : 0.0f;
  c.da = take ? (ep ? ea_ : (ed ? sda : 0.0f)) : 0.0f;
  c.db = take ? (ep ? eb_ : (ed ? sdb : 0.0f)) : 0.0f;
  c.dw = take ? (ep ? ew_ : (ed ? sdw : cdw)) : 0.0f;
  return c;
}

// the contact of a triangle whose winning candidate is c (mesh_face's emission): tau, the
// wall-frame normal and the penetration; false when the triangle does not penetrate
template <class G>
POB_D bool mface_contact(G &g, const MFace &F, const MCand &c, const float r, const float T, float &tau, v3 &nl,
                         float &pen) {
  if (!(c.d2 < T)) return false;
  float dist = 0.0f, inv = 0.0f;
  if (c.d2 > 0.0f) g.sqrt_rcp(c.d2, dist, inv);  // (d2 = 0: mesh_face)
  pen = r - dist;
  if (!(pen > 0.0f)) return false;
  float na, nb, nw;
  if (c.d2 > 0.0f) { na = c.da * inv; nb = c.db * inv; nw = c.dw * inv; }
  else { na = 0.0f; nb = 0.0f; nw = F.sg; }
  const int k = F.k;
  nl = V(k == 0 ? nw : na, k == 0 ? na : (k == 1 ? nw : nb), k == 2 ? nw : nb);
  tau = 1.0f - 2.0f * c.u;
  return true;
}

#ifndef POB_MESH_HOST
// ---------------------------------------------------------------- the wave's face walk
// Walk the lanes' face items (M[s]: bit 8 w + f for face f of wall w of the lane's body slot
// s; slots, then bits, in increasing order: the oracle's contact order per body) and call
// apply(s, bit, tau, n_world, pen) on the owning lane for every penetrating triangle, in
// order.  seg_of(s, A, B, r, seg) gives a slot's segment (world end points), radius and
// whether it is a capsule (false: the torso sphere at A).
//
// A face costs ~1 000 instructions evaluated on one lane (its twelve candidates and two
// emissions one after another) and few lanes of a wave hold one at a time (0.7 items on the
// busiest lane per wave and collide substep on HH rollouts, scripts/wall_walk_stats.py), so
// the wave shares them out: each round takes the next items of up to four lanes (a lane's
// next two of one body when fewer lanes have one) and gives each of those faces sixteen lanes -- lane 8 t + kk of the group computes candidate kk of
// triangle t -- reduces the candidates to each triangle's winner (DPP, lexicographic (d2, kk)
// minimum over the eight lanes), lets the winner lane compute the contact, and hands it to
// the owner (ds_bpermute), which applies its triangles in order.  Needs all 64 lanes active
// (the DPP reduction reads every lane of a group); with lanes masked off -- the batch's last
// wave, a masked reset -- each lane walks its own items (mesh_lane_walk).
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

// each lane walks its own items, one face per iteration (mesh_face)
template <int NB, class G, class SegOf, class Apply>
POB_D void mesh_lane_walk(G &g, const float *WT, const float cz, const float hz, uint64_t (&M)[NB], SegOf &&seg_of,
                          Apply &&apply) {
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
      mesh_face(g, bit & 7, La, Lb, seg, W.hx, W.hy, hz, r, T, [&](const float tau, const v3 nl, const float pen) {
        apply(s, bit, tau, mwall_world_n(W, nl), pen);
      });
    }
  }
}

template <int NB, class G, class SegOf, class Apply>
POB_D void mesh_wave_walk(G &g, const float *WT, const float cz, const float hz, uint64_t (&M)[NB], SegOf &&seg_of,
                          Apply &&apply) {
#ifdef POB_MESH_LANE_WALK
  if (true) {  // A/B build switch: the per-lane walk everywhere
#else
  if (__ballot(1) != ~0ull) {
#endif
    mesh_lane_walk<NB>(g, WT, cz, hz, M, seg_of, apply);
    return;
  }
  const int lane = (int)__lane_id();
  const int grp = lane >> 4, tri = (lane >> 3) & 1, kk = lane & 7;
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
    // a round's four groups: the first items of the first four lanes with one, then (when
    // fewer) the second items of lanes with two -- each lane's items in its order
    const int n1 = __builtin_popcountll(req1), n2 = __builtin_popcountll(req2);
    const uint32_t r1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(req1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)req1, 0u));
    const uint32_t r2 = (uint32_t)n1 +
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(req2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)req2, 0u));
    const bool own1 = has && r1 < 4u, own2 = has2 && r2 < 4u;  // (own2 implies own1: n1 < 4)
    const uint64_t pop = (own1 ? 1ull << b1 : 0ull) | (own2 ? 1ull << b2 : 0ull);
#pragma unroll
    for (int q = 0; q < NB; ++q) M[q] = s == q ? (M[q] & ~pop) : M[q];
    // group owners (wave-uniform): lane and item of each of the four groups
    int og[4];
    {
      uint64_t m1 = req1, m2 = req2;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool first = q < n1;
        const uint64_t m = first ? m1 : m2;
        og[q] = m != 0ull ? __builtin_ctzll(m) : 0;
        m1 = first ? (m1 & (m1 - 1ull)) : m1;
        m2 = first ? m2 : (m2 & (m2 - 1ull));
      }
    }
    const int ol = grp == 0 ? og[0] : (grp == 1 ? og[1] : (grp == 2 ? og[2] : og[3]));
    const bool gv = grp < n1 + n2;
    const bool second = grp >= n1;
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
    const v3 La = mwall_local(W, cz, Ao);
    const v3 Lb = sego ? mwall_local(W, cz, Bo) : La;
    const MFace F = mface(g, mo & 7, La, Lb, W.hx, W.hy, hz);
    const MCand c = mface_cand_bf(g, F, sego, tri, gv ? kk : 7);
    // each triangle's winner over its eight lanes
    float dmin = c.d2;
    int kmin = kk;
    mlexmin_dpp<0xB1>(dmin, kmin);   // quad_perm [1, 0, 3, 2]
    mlexmin_dpp<0x4E>(dmin, kmin);   // quad_perm [2, 3, 0, 1]
    mlexmin_dpp<0x141>(dmin, kmin);  // row_half_mirror: the other quad of the eight
    float tau = 0.0f, pen = 0.0f;
    v3 nw = V(0.0f, 0.0f, 0.0f);
    bool hit = false;
    if (gv && kk == kmin) {
      v3 nl;
      hit = mface_contact(g, F, c, ro, (ro * ro) * 1.00000095367431640625f, tau, nl, pen);
      if (hit) nw = mwall_world_n(W, nl);
    }
    // the owners take their items' triangles in order: the winners' lanes first (all four
    // fetches in flight), then each contact
    const int g1 = 16 * (int)r1, g2 = 16 * (int)r2;
    const int w10 = g1 + mlane_read_i(kmin, g1), w11 = g1 + 8 + mlane_read_i(kmin, g1 + 8);
    const int w20 = g2 + mlane_read_i(kmin, g2), w21 = g2 + 8 + mlane_read_i(kmin, g2 + 8);
    const int nt = __any(own2) ? 4 : 2;
#pragma nounroll
    for (int t = 0; t < nt; ++t) {
      const int wl = t == 0 ? w10 : (t == 1 ? w11 : (t == 2 ? w20 : w21));
      const int h = mlane_read_i(hit ? 1 : 0, wl);
      const float tw = mlane_read(tau, wl), pw = mlane_read(pen, wl);
      const v3 nn = V(mlane_read(nw.x, wl), mlane_read(nw.y, wl), mlane_read(nw.z, wl));
      if ((t < 2 ? own1 : own2) && h != 0) apply(s, t < 2 ? b1 : b2, tw, nn, pw);
    }
  }
}
#endif  // POB_MESH_HOST
