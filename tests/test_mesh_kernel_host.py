"""CPU: the kernels' capsule x TriangulatedBox code (po-brax_amd/csrc/pob_mesh.h, the device
header itself) compiled for the host against a small shim, bit-compared with the oracle's
independent restatement (oracle/pob_oracle.c capsule_wall_mesh) on random capsule / wall
pairs: the face cull, the per-face closest-point candidates, the contacts' order, tau, normal
and penetration.  (The shim provides the few gfx950 builtins the header uses with their exact
host equivalents: v_med3_f32 -> fminf(fmaxf()), correctly rounded reciprocal / square root ->
IEEE 1/x and sqrtf, as the kernels' fast forms are exact in range.)"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import orc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
MESH_H = os.path.join(ROOT, "po-brax_amd", "csrc", "pob_mesh.h")

SHIM = r"""
#include "pob_sys.h"
#include <math.h>
#include <stdint.h>
#include <string.h>
#define POB_D static inline
#define POB_MESH_HOST 1
struct v3 { float x, y, z; };
struct float2 { float x, y; };
#define FMA(a, b, c) fmaf((a), (b), (c))
POB_D v3 V(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
#define __builtin_inff() INFINITY
struct HostGuard {
  float rcp(float x) { return 1.0f / x; }
  float sqrt(float x) { return sqrtf(x); }
  void sqrt_rcp(float x, float &s, float &i) { s = sqrtf(x); i = 1.0f / s; }
};
"""

DRIVER = r"""
static int g_ties = 0;
// the wall's face constants (pob_sys::face_c[w], as pob_system.cpp builds them)
static void face_table(float hx, float hy, float hz, float *fcw) {
  for (int k = 0; k < 3; ++k) pob_face_consts(k == 0 ? hy : hx, k == 2 ? hy : hz, fcw + POB_FACE_FLOATS * k);
}
extern "C" int host_tie_count(void) { const int n = g_ties; g_ties = 0; return n; }
// the oracle's row: (tau, n, pen = r - dist, cd = 1e-6 + dist), as the kernels' callers form them
static void put(float *out, int n, float tau, v3 nw, float r, float dist) {
  out[6 * n] = tau; out[6 * n + 1] = nw.x; out[6 * n + 2] = nw.y; out[6 * n + 3] = nw.z; out[6 * n + 4] = r - dist;
  out[6 * n + 5] = 1e-6f + dist;
}
// the per-lane form (mesh_face: both triangles, exact candidate skips, tie slow path)
extern "C" int host_mesh_contacts(const float *w, const float *a, const float *b, int seg, float r, float *out) {
  MWall W; W.cx = w[0]; W.cy = w[1]; W.c = w[3]; W.s = w[4]; W.hx = w[5]; W.hy = w[6];
  const float cz = w[2], hz = w[7];
  const v3 La = mwall_local(W, cz, V(a[0], a[1], a[2]));
  const v3 Lb = seg ? mwall_local(W, cz, V(b[0], b[1], b[2])) : La;
  const uint32_t fm = mesh_face_mask(La, Lb, W.hx, W.hy, hz, r + POB_MESH_MARGIN);
  const float T = (r * r) * 1.00000095367431640625f;
  float fcw[3 * POB_FACE_FLOATS];
  face_table(W.hx, W.hy, hz, fcw);
  HostGuard g;
  int n = 0;
  for (int f = 0; f < 6; ++f) {
    if (!((fm >> f) & 1u)) continue;
    mesh_face(g, f, La, Lb, W.hx, W.hy, hz, fcw, r, T, [&](float tau, v3 nl, float dist) {
      put(out, n, tau, mwall_world_n(W, nl), r, dist);
      ++n;
    });
  }
  return n;
}
// the same contacts through the wave walk's decomposition: every candidate on its own, the
// lexicographic (d2, kk) minimum per triangle with the tie count, the winner's contact
extern "C" int host_mesh_contacts_split(const float *w, const float *a, const float *b, int seg, float r, float *out) {
  MWall W; W.cx = w[0]; W.cy = w[1]; W.c = w[3]; W.s = w[4]; W.hx = w[5]; W.hy = w[6];
  const float cz = w[2], hz = w[7];
  const v3 La = mwall_local(W, cz, V(a[0], a[1], a[2]));
  const v3 Lb = seg ? mwall_local(W, cz, V(b[0], b[1], b[2])) : La;
  const uint32_t fm = mesh_face_mask(La, Lb, W.hx, W.hy, hz, r + POB_MESH_MARGIN);
  const float T = (r * r) * 1.00000095367431640625f;
  float fcw[3 * POB_FACE_FLOATS];
  face_table(W.hx, W.hy, hz, fcw);
  HostGuard g;
  int n = 0;
  for (int f = 0; f < 6; ++f) {
    if (!((fm >> f) & 1u)) continue;
    const MFace F = mface(g, f, mcap_seg(g, La, Lb), W.hx, W.hy, hz, fcw);
    for (int t = 0; t < 2; ++t) {
      // (the wave walk's reduction: NaN distances enter as +inf, lexicographic (d2, kk) minimum)
      MCand c[4]; MCand best; int kb = 0;
      F3 S[4], P[4];
      for (int kk = 0; kk < 4; ++kk) {
        c[kk] = mface_cand(g, F, t, kk, S[kk], P[kk]);
        c[kk].d2 = mcand_key(c[kk].d2);
        if (kk == 0 || c[kk].d2 < best.d2 || (c[kk].d2 == best.d2 && kk < kb)) { best = c[kk]; kb = kk; }
      }
      int neq = 0;
      for (int kk = 0; kk < 4; ++kk) neq += c[kk].d2 == best.d2;
      if (neq > 1 && best.d2 < T) {  // (the walk's quad gather: mtie_add over kk = 0..3)
        F3 Ss = f3(0.0f, 0.0f, 0.0f), Ps = Ss;
        float us = 0.0f, cnt = 0.0f;
        const float dmin = best.d2;
        for (int kk = 0; kk < 4; ++kk)
          if (c[kk].d2 == dmin) {
            Ss = f3(Ss.a + S[kk].a, Ss.b + S[kk].b, Ss.w + S[kk].w);
            Ps = f3(Ps.a + P[kk].a, Ps.b + P[kk].b, Ps.w + P[kk].w);
            us += c[kk].u; cnt += 1.0f;
          }
        best = bcand(f3(Ss.a / cnt, Ss.b / cnt, Ss.w / cnt), f3(Ps.a / cnt, Ps.b / cnt, Ps.w / cnt), us / cnt);
        ++g_ties;
      }
      float tau, dist; v3 nl;
      if (mface_contact(g, F.k, best, r, T, tau, nl, dist)) { put(out, n, tau, mwall_world_n(W, nl), r, dist); ++n; }
    }
  }
  return n;
}
"""


@pytest.fixture(scope="module")
def host_mesh(tmp_path_factory):
    d = tmp_path_factory.mktemp("meshhost")
    body = open(MESH_H).read().replace('#include "pob_math.h"', "")
    src = d / "mesh_host.cpp"
    src.write_text(SHIM + body + DRIVER)
    so = d / "mesh_host.so"
    subprocess.check_call(["g++", "-O2", "-mfma", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC",
                           "-I", os.path.dirname(MESH_H), "-shared", "-o", str(so), str(src)])
    lib = C.CDLL(str(so))
    FP = C.POINTER(C.c_float)
    lib.host_mesh_contacts.argtypes = [FP, FP, FP, C.c_int, C.c_float, FP]
    lib.host_mesh_contacts_split.argtypes = [FP, FP, FP, C.c_int, C.c_float, FP]
    return lib


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def test_kernel_mesh_code_equals_oracle_bitwise(host_mesh):
    rng = np.random.default_rng(2024)
    n_contacts = n_cases = 0
    for it in range(20000):
        deg = rng.choice([0.0, 90.0, 180.0, 270.0, rng.uniform(0, 360)])
        a = np.deg2rad(np.float32(deg))
        h = np.array([rng.uniform(0.2, 7.0), rng.uniform(0.2, 0.6), 0.5], np.float32)
        w = np.array([rng.uniform(-8, 8), rng.uniform(-8, 8), 0.5, np.cos(a), np.sin(a), h[0], h[1], h[2]], np.float32)
        R = np.array([[w[3], -w[4], 0], [w[4], w[3], 0], [0, 0, 1]], np.float64)
        loc = rng.uniform(-1.0, 1.0, 3) * h
        k = rng.integers(3)
        loc[k] = np.sign(rng.uniform(-1, 1)) * h[k]
        centre = w[:3] + R @ (loc + rng.normal(0, 0.08, 3))
        seg = rng.uniform() > 0.15
        r = np.float32(0.08 if seg else 0.25)
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        half = rng.uniform(0.0, 0.3) if seg else 0.0
        pa = (centre + half * d).astype(np.float32)
        pb = (centre - half * d).astype(np.float32) if seg else pa.copy()
        ref = orc.mesh_contacts(w, pa, pb, bool(seg), float(r))
        out = np.zeros((12, 6), np.float32)
        n = host_mesh.host_mesh_contacts(_p(w), _p(pa), _p(pb), int(seg), float(r), _p(out))
        got = out[:n]
        assert got.shape == ref.shape and np.array_equal(got.view(np.uint32), ref.view(np.uint32)), \
            (it, deg, w, pa, pb, seg, got, ref)
        out2 = np.zeros((12, 6), np.float32)
        n2 = host_mesh.host_mesh_contacts_split(_p(w), _p(pa), _p(pb), int(seg), float(r), _p(out2))
        assert n2 == n and np.array_equal(out2[:n2].view(np.uint32), ref.view(np.uint32)), (it, "split", out2[:n2], ref)
        n_cases += 1
        n_contacts += n
    assert n_contacts > 2000, n_contacts


def test_kernel_mesh_code_non_finite_segments(host_mesh):
    """Segments with NaN, infinite or overflowing end points (a body whose rotation went NaN
    keeps a finite centre, the out-of-range parity case): no contact where the oracle has none,
    the same contacts where one end point is sound.  (The diagonal candidate shared by both
    triangles must be taken on its own squared distance: a never-taken one is not at 0.)"""
    rng = np.random.default_rng(77)
    bad = [np.nan, np.inf, -np.inf, 1e30, -1e30, 3e19]
    w = np.array([0.0, 0.0, 0.5, 1.0, 0.0, 6.75, 0.5, 0.5], np.float32)
    n_cases = 0
    for it in range(3000):
        pa = np.array([rng.uniform(-7, 7), rng.uniform(-0.7, 0.7), rng.uniform(-0.1, 1.1)], np.float32)
        pb = (pa + rng.normal(0, 0.3, 3)).astype(np.float32)
        for p in (pa, pb):
            for k in range(3):
                if rng.uniform() < 0.3:
                    p[k] = np.float32(bad[rng.integers(len(bad))])
        ref = orc.mesh_contacts(w, pa, pb, True, 0.08)
        out = np.zeros((12, 6), np.float32)
        n = host_mesh.host_mesh_contacts(_p(w), _p(pa), _p(pb), 1, 0.08, _p(out))
        assert n == len(ref) and np.array_equal(out[:n].view(np.uint32), ref.view(np.uint32)), (it, pa, pb, n, ref)
        n2 = host_mesh.host_mesh_contacts_split(_p(w), _p(pa), _p(pb), 1, 0.08, _p(out))
        assert n2 == len(ref) and np.array_equal(out[:n2].view(np.uint32), ref.view(np.uint32)), (it, "split", pa, pb)
        n_cases += 1
    assert n_cases == 3000


def test_kernel_mesh_code_grid_cases_with_ties(host_mesh):
    """Capsules on a 1/16 grid against axis-aligned walls (exact coordinates: segments lying
    over a face's diagonal or parallel to its edges give candidates at the same distance), so
    brax's tie rule (the average of the tied candidates' points) runs on both sides and must
    agree bit for bit."""
    rng = np.random.default_rng(5)
    w = np.array([0.0, 0.0, 0.5, 1.0, 0.0, 1.0, 0.5, 0.5], np.float32)
    host_mesh.host_tie_count()
    n_contacts = 0
    for it in range(20000):
        q = lambda lo, hi: np.float32(rng.integers(int(lo * 16), int(hi * 16) + 1) / 16.0)
        pa = np.array([q(-1.25, 1.25), q(-0.75, 0.75), q(-0.25, 1.25)], np.float32)
        if rng.uniform() < 0.5:  # parallel to an axis or to a face diagonal
            d = np.zeros(3, np.float32)
            ax = rng.integers(3)
            d[ax] = q(-0.5, 0.5)
            if rng.uniform() < 0.5:
                d[(ax + 1) % 3] = d[ax] * (1 if rng.uniform() < 0.5 else -1)
            pb = (pa + d).astype(np.float32)
        else:
            pb = np.array([q(-1.25, 1.25), q(-0.75, 0.75), q(-0.25, 1.25)], np.float32)
        seg = rng.uniform() < 0.85
        r = 0.0625 if seg else 0.25
        ref = orc.mesh_contacts(w, pa, pb, seg, r)
        out = np.zeros((12, 6), np.float32)
        n = host_mesh.host_mesh_contacts(_p(w), _p(pa), _p(pb), int(seg), r, _p(out))
        assert n == len(ref) and np.array_equal(out[:n].view(np.uint32), ref.view(np.uint32)), (it, pa, pb, out[:n], ref)
        n2 = host_mesh.host_mesh_contacts_split(_p(w), _p(pa), _p(pb), int(seg), r, _p(out))
        assert n2 == len(ref) and np.array_equal(out[:n2].view(np.uint32), ref.view(np.uint32)), (it, "split")
        n_contacts += n
    assert n_contacts > 1000
    assert host_mesh.host_tie_count() > 0  # the tie rule was exercised
