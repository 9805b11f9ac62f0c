// pob_kernels.hip -- fused rollout kernels + the C ABI of libpob.so (include/pob.h).
//
// Kernels (batch-major HBM layout; qp stored as float32 or binary16, computed in float32):
//   k_step_quad<KIND,QT> physics (PBD) + per-env POMDP logic + obs + Episode/AutoReset
//                    wrappers, FOUR lanes per environment (pob_quad.h)
//   k_step_mixed<QT> the same body for up to POB_MIX_MAX envs of different kinds in ONE
//                    launch (block ranges select the env; the task tail dispatches on kind)
//   k_reset<KIND,BS,QT> threefry keys -> joint noise -> forward kinematics -> env placement
//                    (HH goal swap / GA top-16-of-156 choice / TAG rejection loop) ->
//                    sys.info contact -> obs; also the masked "reset where done" variants
//   k_default_qp     System.default_qp(joint_angle, joint_velocity)
//   k_split/k_uniform/k_actions/k_advance_key   jax.random on device
//   k_obs_gather     standard_observability_masks column gather
// Reference anchors are given per function; DESIGN.md has the data layout and roofline.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <type_traits>
#include <vector>

#include "../../include/pob.h"

#ifndef POB_QUAD_PRIO  // the four-lane kernel's falling issue priority over the substeps (k_step_quad)
#define POB_QUAD_PRIO 1
#endif
#ifndef POB_OCT_PRIO  // the same in the eight-lane kernel's branch-guard build (two waves per SIMD)
#define POB_OCT_PRIO 1
#endif
#ifndef POB_HEX_PRIO  // the same in the sixteen-lane kernel at two or more waves per SIMD:
#define POB_HEX_PRIO 1  // HH B = 8 192 0.0669 -> 0.0630 ms, TAG 0.0490 -> 0.0461 (profiles/r7ab)
#endif
#include "pob_quad.h"
#include "pob_octet.h"
#include "pob_hexa.h"
#include "pob_physics.h"

namespace pob {
void default_params(pob_params &p);
const char *build_system(int kind, const pob_params &p, pob_sys &s);
int gather_grid(const pob_params &p, float *xyz, int cap);
}  // namespace pob

struct pob_env {
  pob_sys sys;         // host copy
  pob_sys *d_sys = nullptr;  // device copy, read by the kernels through the scalar cache
  pob_params params;
  float *d_grid = nullptr;
  uint32_t *d_scratch = nullptr;  // any-done word for pob_reset_where_done without a flag
  int device = 0;
  int n_cu = 256;  // compute units of the device (SIMDs = 4 x n_cu)
};

#define POB_MIXED (-1)  // KIND of the mixed-launch body: the kind is read from the table
#define POB_F_STAGED (1u << 16)  // internal step flag: coalesced LDS-staged state loads
// (test hook: POB_QUAD_FORCE_FIXUP=1 makes the fast launch hand every wave to the fix-up launch,
// so the parity tests run the fix-up path on every env; an internal flags bit)
#define POB_F_INT_FORCE_FIXUP (1u << 30)
#define POB_F_INTERNAL (POB_F_STAGED | POB_F_INT_FORCE_FIXUP)
#define POB_F_PUBLIC (POB_F_EPISODE | POB_F_AUTORESET | POB_F_ZERO_STEPS_ON_DONE)

// ---------------------------------------------------------------------------- state
#define POB_STATE_FIELDS(X)                                                                    \
  X(pos) X(rot) X(vel) X(ang) X(obs) X(reward) X(done) X(steps) X(truncation) X(m0) X(m1) X(m2) \
  X(rng) X(first_pos) X(first_rot) X(first_vel) X(first_ang) X(first_obs) X(any_done) X(done_u8) X(trunc_i32) \
  X(m0_i32) X(m1_i32) X(any_done_clear) X(obs_masked) X(ovf_mark)

struct StatePtrs {  // device pointers (kernel-argument copy of pob_state)
  float *pos, *rot, *vel, *ang, *obs, *reward, *done, *steps, *truncation, *m0, *m1, *m2;
  uint32_t *rng;
  float *first_pos, *first_rot, *first_vel, *first_ang, *first_obs;
  uint32_t *any_done;
  uint8_t *done_u8;  // typed copies of step outputs (optional, pob.h)
  int32_t *trunc_i32, *m0_i32, *m1_i32;
  uint32_t *any_done_clear;  // pob_reset_where_done zeroes it (optional)
  float *obs_masked;         // obs[:, mask] (optional, ABI v7)
  uint8_t *ovf_mark;         // the split launch's per-wave overflow marks (optional, ABI v8)
};
// obs[:, mask] of a pass's staged observation rows (rows x D floats in LDS at stg), stored
// next to the obs rows: each row's K columns by the wave's lanes (pob_env_set_obs_mask)
POB_D void store_obs_masked(csys_t &S, float *dst, const float *stg, const int rows, const int D, const int lane) {
  const int K = S.obs_mask_n;
  for (int r = 0; r < rows; ++r)
    for (int c = lane; c < K; c += 64) dst[(size_t)r * K + c] = stg[r * D + S.obs_mask[c]];
}
static StatePtrs to_ptrs(const pob_state &s) {
  StatePtrs p;
#define POB_CP(f) p.f = s.f;
  POB_STATE_FIELDS(POB_CP)
#undef POB_CP
  return p;
}

// qp storage: element i of a qp array (pos/rot/vel/ang, first_*) in float32 or binary16.
// The float32 -> binary16 conversion is round-to-nearest-even (v_cvt_f16_f32), the same
// rounding numpy's astype(float16) applies to the oracle's float32 results.
template <typename QT> struct Q;
template <> struct Q<float> {
  static POB_D float ld(const float *p, size_t i) { return p[i]; }
  static POB_D void st(float *p, size_t i, float v) { p[i] = v; }
};
template <> struct Q<__half> {
  static POB_D float ld(const float *p, size_t i) { return __half2float(reinterpret_cast<const __half *>(p)[i]); }
  // The float32 value is pinned in a VGPR first: otherwise the backend may fuse the
  // producing FMA into the conversion (v_fma_mixlo_f16: ONE rounding, straight to binary16),
  // which differs from the spec's float32 result rounded to binary16 exactly when that
  // float32 value is a binary16 tie (measured: 11 of 393 K reset rot elements at B = 10 923)
  static POB_D void st(float *p, size_t i, float v) {
    asm volatile("" : "+v"(v));
    reinterpret_cast<__half *>(p)[i] = __float2half_rn(v);
  }
};
template <typename QT> POB_D v3 ld3(const float *p, size_t i) {
  return V(Q<QT>::ld(p, i), Q<QT>::ld(p, i + 1), Q<QT>::ld(p, i + 2));
}
template <typename QT> POB_D void st3(float *p, size_t i, v3 v) {
  Q<QT>::st(p, i, v.x); Q<QT>::st(p, i + 1, v.y); Q<QT>::st(p, i + 2, v.z);
}
template <typename QT> POB_D q4 ld4(const float *p, size_t i) {
  q4 q; q.w = Q<QT>::ld(p, i); q.x = Q<QT>::ld(p, i + 1); q.y = Q<QT>::ld(p, i + 2); q.z = Q<QT>::ld(p, i + 3);
  return q;
}
template <typename QT> POB_D void st4(float *p, size_t i, q4 q) {
  Q<QT>::st(p, i, q.w); Q<QT>::st(p, i + 1, q.x); Q<QT>::st(p, i + 2, q.y); Q<QT>::st(p, i + 3, q.z);
}
// copy n qp elements (exact in either storage)
template <typename QT> POB_D void cpq(float *dst, const float *src, size_t i, int n) {
  for (int k = 0; k < n; ++k) Q<QT>::st(dst, i + k, Q<QT>::ld(src, i + k));
}
// The same copy by the L lanes of an env's lane group (this lane: j), U loads in flight per
// lane before their stores: a done env's first_qp / first_obs rows cost a few memory round
// trips instead of one per element on one lane (a wave holding a done env was otherwise the
// launch's last by up to 9 us)
template <typename QT, int L, int U>
POB_D void group_cpq(float *dst, const float *src, const size_t i, const int n, const int j) {
  for (int q0 = j; q0 < n; q0 += L * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = q0 + L * u < n ? Q<QT>::ld(src, i + q0 + L * u) : 0.0f;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (q0 + L * u < n) Q<QT>::st(dst, i + q0 + L * u, v[u]);
  }
}
// float rows (obs): dst may be the wave's LDS staging row
template <int L, int U>
POB_D void group_copy(float *dst, const float *src, const int n, const int j) {
  for (int q0 = j; q0 < n; q0 += L * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = q0 + L * u < n ? src[q0 + L * u] : 0.0f;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (q0 + L * u < n) dst[q0 + L * u] = v[u];
  }
}
// a done env's frozen qp rows from first_qp, and (functional mode with distinct first_*
// buffers) the first_qp / first_obs carry-over, by the env's L lanes (j: this lane)
template <typename QT, int L, int U = 4>
POB_D void tail_copies(const StatePtrs &in, const StatePtrs &out, const uint32_t flags, const bool reset_rows,
                       const int b, const int N, const int D, const size_t r3, const size_t r4, const int j) {
  if (reset_rows) {
    group_cpq<QT, L, U>(out.pos, in.first_pos, r3 + 3 * POB_NDYN, 3 * (N - POB_NDYN), j);
    group_cpq<QT, L, U>(out.vel, in.first_vel, r3 + 3 * POB_NDYN, 3 * (N - POB_NDYN), j);
    group_cpq<QT, L, U>(out.ang, in.first_ang, r3 + 3 * POB_NDYN, 3 * (N - POB_NDYN), j);
    group_cpq<QT, L, U>(out.rot, in.first_rot, r4 + 4 * POB_NDYN, 4 * (N - POB_NDYN), j);
  }
  if ((flags & POB_F_AUTORESET) && out.first_pos != in.first_pos) {
    group_cpq<QT, L, U>(out.first_pos, in.first_pos, r3, 3 * N, j);
    group_cpq<QT, L, U>(out.first_vel, in.first_vel, r3, 3 * N, j);
    group_cpq<QT, L, U>(out.first_ang, in.first_ang, r3, 3 * N, j);
    group_cpq<QT, L, U>(out.first_rot, in.first_rot, r4, 4 * N, j);
    group_copy<L, U>(out.first_obs + (size_t)b * D, in.first_obs + (size_t)b * D, D, j);
  }
}

template <int KIND>
POB_D int n_bodies(csys_t &S) {
  return KIND == POB_HEAVENHELL ? 14 : (KIND == POB_TAG ? 12 : (KIND == POB_ANT ? 10 : S.N));
}
template <int KIND>
POB_D int obs_dim(csys_t &S) {
  return KIND == POB_HEAVENHELL ? 114 : (KIND == POB_TAG ? 103 : (KIND == POB_ANT ? 87 : S.D));
}
// obs header shift: the stock ant keeps only the torso z of qp.pos[0] (brax envs/ant.py
// _get_obs: qp.pos[0, 2:]), so its layout is the po-env layout moved left by 2
POB_D constexpr int obs_shift(int kind) { return kind == POB_ANT ? -2 : 0; }

POB_D void load_body(const float *pos, const float *rot, const float *vel, const float *ang, Body &b) {
#pragma unroll
  for (int i = 0; i < POB_NDYN; ++i) {
    b.x[i] = V(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]);
    b.q[i].w = rot[4 * i]; b.q[i].x = rot[4 * i + 1]; b.q[i].y = rot[4 * i + 2]; b.q[i].z = rot[4 * i + 3];
    b.v[i] = V(vel[3 * i], vel[3 * i + 1], vel[3 * i + 2]);
    b.w[i] = V(ang[3 * i], ang[3 * i + 1], ang[3 * i + 2]);
  }
}
template <typename QT>
POB_D void store_body(const Body &b, float *pos, float *rot, float *vel, float *ang, size_t r3, size_t r4) {
#pragma unroll
  for (int i = 0; i < POB_NDYN; ++i) {
    st3<QT>(pos, r3 + 3 * i, b.x[i]);
    st4<QT>(rot, r4 + 4 * i, b.q[i]);
    st3<QT>(vel, r3 + 3 * i, b.v[i]);
    st3<QT>(ang, r3 + 3 * i, b.w[i]);
  }
}

POB_D float clip1(float x) { return x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x); }
POB_D float dist2d(float ax, float ay, float bx, float by) {
  float dx = ax - bx, dy = ay - by;
  return sqrtf(dx * dx + dy * dy);
}

// _get_obs prefix shared by the three envs (ant_heavenhell.py:125-158,
// ant_gather.py:183-213, ant_tag.py:148-181): torso pos(3) rot(4) joint angles(8)
// torso vel(3) ang(3) joint vels(8) clip(contact.vel) (N*3) clip(contact.ang) (N*3).
// Joint angle/vel = sys.joints[0].angle_vel (a3).  sh = -2: stock ant (torso z only).
POB_D void write_obs_common(csys_t &S, int N, const Body &b, const v3 (&cv)[POB_NDYN],
                            const v3 (&ca)[POB_NDYN], float *row, const int sh) {
  if (sh == 0) { row[0] = b.x[0].x; row[1] = b.x[0].y; }
  row[sh + 2] = b.x[0].z;
  row[sh + 3] = b.q[0].w; row[sh + 4] = b.q[0].x; row[sh + 5] = b.q[0].y; row[sh + 6] = b.q[0].z;
#pragma unroll
  for (int j = 0; j < POB_NJ; ++j) {
    const int p = jparent(j), c = jchild(j);
    v3 ap = qrot(SV(S.axis[j]), b.q[p]);
    const v3 ref = SV(S.ref[j]);
    v3 fp = qrot(ref, b.q[p]), fc = qrot(ref, b.q[c]);
    row[sh + 7 + j] = pob_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
    row[sh + 21 + j] = vdot(vsub(b.w[c], b.w[p]), ap);
  }
  row[sh + 15] = b.v[0].x; row[sh + 16] = b.v[0].y; row[sh + 17] = b.v[0].z;
  row[sh + 18] = b.w[0].x; row[sh + 19] = b.w[0].y; row[sh + 20] = b.w[0].z;
  float *o = row + (29 + sh);
#pragma unroll
  for (int i = 0; i < POB_NDYN; ++i) {
    o[3 * i] = clip1(cv[i].x); o[1 + 3 * i] = clip1(cv[i].y); o[2 + 3 * i] = clip1(cv[i].z);
    o[3 * N + 3 * i] = clip1(ca[i].x); o[1 + 3 * N + 3 * i] = clip1(ca[i].y);
    o[2 + 3 * N + 3 * i] = clip1(ca[i].z);
  }
  for (int k = 3 * POB_NDYN; k < 3 * N; ++k) { o[k] = 0.0f; o[3 * N + k] = 0.0f; }
}

// ant_gather.py:152-181 sensor readings, written straight into the obs row.  Scatter
// semantics of XLA-CPU: updates applied in object order (last writer wins) and an
// out-of-span bin -1 wraps to the last slot.
POB_D void ga_readings_begin(csys_t &S, float *o_rd) {
  for (int s = 0; s < 2 * S.ga_n_bins; ++s) o_rd[s] = 0.0f;
}
POB_D float ga_orientation(const q4 rot0) {
  q4 ob; ob.w = 0.0f; ob.x = 1.0f; ob.y = 0.0f; ob.z = 0.0f;
  q4 t = qmul(qmul(rot0, ob), qinv(rot0));
  return pob_atan2f(t.y, t.x);
}
// reading of object k: the slot it writes (-1: none) and the value
POB_D int ga_reading_slot(csys_t &S, int k, float ox, float oy, float dist, float ori, float &inten) {
  float angle = pob_atan2f(ox, oy) - ori;
  bool in_range = dist <= S.ga_sensor_range;
  int bin = (fabsf(angle) <= S.ga_half_span && in_range) ? (int)((angle + S.ga_half_span) / S.ga_bin_res) : -1;
  if (k >= S.ga_n_apples) bin = bin >= 0 ? bin + S.ga_n_apples : -1;
  inten = bin >= 0 ? 1.0f - dist / S.ga_sensor_range : 0.0f;
  int slot = bin < 0 ? bin + 2 * S.ga_n_bins : bin;
  return (slot >= 0 && slot < 2 * S.ga_n_bins) ? slot : -1;
}
POB_D void ga_reading_one(csys_t &S, int k, float ox, float oy, float dist, float ori, float *o_rd) {
  float inten;
  const int slot = ga_reading_slot(S, k, ox, oy, dist, ori, inten);
  if (slot >= 0) o_rd[slot] = inten;
}

// stock ant costs (brax envs/ant.py step [ext]): .5 * sum(action^2) and
// .5e-3 * sum(clip(contact.vel, -1, 1)^2), summed in row-major element order (the frozen
// Ground row adds exact zeros and is skipped)
POB_D float ant_ctrl_cost(const float *a8) {
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < POB_NJ; ++j) s = s + a8[j] * a8[j];
  return 0.5f * s;
}
POB_D float ant_contact_add(float s, v3 c) {
  const float cx = clip1(c.x), cy = clip1(c.y), cz = clip1(c.z);
  s = s + cx * cx; s = s + cy * cy; s = s + cz * cz;
  return s;
}

struct TaskOut {
  float reward, done, trunc, steps, m0, m1, m2;
  uint32_t rng0, rng1;
  float xb, ctrl, contact;  // stock ant inputs: torso x before the step, costs
  float ob0, ob1;           // the task's obs entries (HH heaven direction, TAG target xy)
  // AntGather objects already handled by the env's four lanes (ga_quad_objects)
  bool ga_done_quad, ga_any_a, ga_any_b, ga_all_wait;
  int ga_na, ga_nb;
  // task bodies' input xy loaded before the physics (tp_ok): HH priest, target, hell
  // (rows 10, 11, 12) and TAG target (row 10) -- their loads would otherwise be a memory
  // round trip after the substeps, on the wave's critical path
  bool tp_ok;
  float tp[6];
  float pdone;  // the input done (sixteen-lane kernel: loaded before the physics)
};

// the task bodies' xy (TaskOut::tp) of env row r3
template <int KIND, typename QT>
POB_D void task_prefetch(const StatePtrs &in, const size_t r3, TaskOut &t) {
  using QQ = Q<QT>;
  t.tp_ok = KIND == POB_HEAVENHELL || KIND == POB_TAG;
#pragma unroll
  for (int i = 0; i < 6; ++i) t.tp[i] = 0.0f;
  if (KIND == POB_HEAVENHELL) {
#pragma unroll
    for (int i = 0; i < 3; ++i) { t.tp[2 * i] = QQ::ld(in.pos, r3 + 30 + 3 * i); t.tp[2 * i + 1] = QQ::ld(in.pos, r3 + 31 + 3 * i); }
  } else if (KIND == POB_TAG) {
    t.tp[0] = QQ::ld(in.pos, r3 + 30); t.tp[1] = QQ::ld(in.pos, r3 + 31);
  }
}

// Per-env POMDP logic after the physics (env.step minus System.step) + EpisodeWrapper:
// reward / done / metrics / rng, the task part of the obs, and the task bodies' rows.
// HH ant_heavenhell.py:106-123, GA ant_gather.py:125-150 (+ readings :152-181),
// TAG ant_tag.py:107-146, stock ant brax envs/ant.py step [ext]; EpisodeWrapper.step [ext].
// `pos` is the qp.pos array (QT storage), r3 the env's row offset, `o` its obs row.
template <int KIND, typename QT>
POB_D void task_step(csys_t &S, const StatePtrs &in, const int b, const size_t r3, const int N, const v3 x0,
                     const q4 q0, float *opos, float *o, const uint32_t flags, const int L, TaskOut &t) {
  using QQ = Q<QT>;
  const float tz = x0.z;
  float dead = tz < 0.2f ? 1.0f : 0.0f;
  dead = tz > 1.0f ? 1.0f : dead;
  float reward, done;
  float steps = t.steps, m0 = t.m0, m1 = t.m1, m2 = t.m2;
  uint32_t rng0 = t.rng0, rng1 = t.rng1;
  const int base = 29 + 6 * N;
  if (KIND == POB_HEAVENHELL) {
    // ant_heavenhell.py:106-123
    reward = dead > 0.0f ? S.hh_dying_cost : 0.0f;
    const float *ip = in.pos;
    const float px_ = t.tp_ok ? t.tp[0] : QQ::ld(ip, r3 + 30), py_ = t.tp_ok ? t.tp[1] : QQ::ld(ip, r3 + 31);
    const float tx = t.tp_ok ? t.tp[2] : QQ::ld(ip, r3 + 33), ty = t.tp_ok ? t.tp[3] : QQ::ld(ip, r3 + 34);
    const float hx_ = t.tp_ok ? t.tp[4] : QQ::ld(ip, r3 + 36), hy_ = t.tp_ok ? t.tp[5] : QQ::ld(ip, r3 + 37);
    bool in0 = dist2d(tx, ty, x0.x, x0.y) <= S.hh_visible_radius;    // Target
    bool in1 = dist2d(hx_, hy_, x0.x, x0.y) <= S.hh_visible_radius;  // Hell
    bool in2 = dist2d(px_, py_, x0.x, x0.y) <= S.hh_visible_radius;  // Priest
    if (in0) reward = 1.0f;
    if (in1) reward = -1.0f;
    done = reward != 0.0f ? 1.0f : 0.0f;
    const float sgn = tx > 0.0f ? 1.0f : (tx < 0.0f ? -1.0f : 0.0f);
    t.ob0 = in2 ? sgn : 0.0f;
    m2 = done;  // metrics['hits']
  } else if (KIND == POB_GATHER) {
    // ant_gather.py:125-150 (obs from pre-relocation positions)
    float *rd = o + base;
    int na_hit = 0, nb_hit = 0;
    bool any_a = false, any_b = false, all_wait = true;
    if (t.ga_done_quad) {
      na_hit = t.ga_na; nb_hit = t.ga_nb; any_a = t.ga_any_a; any_b = t.ga_any_b; all_wait = t.ga_all_wait;
    } else {
    ga_readings_begin(S, rd);
    const float ori = ga_orientation(q0);
    for (int k = 0; k < S.n_obj; ++k) {
      const size_t row = r3 + 3 * (11 + k);
      const float ox = QQ::ld(in.pos, row), oy = QQ::ld(in.pos, row + 1), oz = QQ::ld(in.pos, row + 2);
      const float dk = dist2d(x0.x, x0.y, ox, oy);
      ga_reading_one(S, k, ox, oy, dk, ori, rd);
      const bool c = dk <= S.ga_catch_range;
      float nx = ox, ny = oy, nz = oz;
      if (c) { nx = S.ga_waiting[0]; ny = S.ga_waiting[1]; nz = S.ga_waiting[2]; }
      QQ::st(opos, row, nx); QQ::st(opos, row + 1, ny); QQ::st(opos, row + 2, nz);
      if (k < S.ga_n_apples) { any_a |= c; na_hit += c; } else { any_b |= c; nb_hit += c; }
      all_wait &= (nx == S.ga_waiting[0]) & (ny == S.ga_waiting[1]) & (nz == S.ga_waiting[2]);
    }
    }
    reward = dead > 0.0f ? S.ga_dying_cost : 0.0f;
    if (any_a && dead == 0.0f) reward = 1.0f;
    if (any_b && dead == 0.0f) reward = -1.0f;
    done = all_wait ? 1.0f : dead;
    m0 = (float)na_hit; m1 = (float)nb_hit;
  } else if (KIND == POB_ANT) {
    // brax envs/ant.py step (brax <= 0.0.12) [ext]
    const float forward = (x0.x - t.xb) / S.ctrl_dt;
    reward = ((forward - t.ctrl) - t.contact) + 1.0f;
    done = dead;
    m0 = t.ctrl; m1 = t.contact; m2 = forward;  // reward_ctrl_cost / _contact_cost / _forward
  } else {
    // ant_tag.py:107-127, adversary _step_target :129-146
    reward = dead > 0.0f ? S.tag_dying_cost : 0.0f;
    uint32_t n0, n1, c0, c1;
    tf_split(rng0, rng1, 2u, 0u, n0, n1);
    tf_split(rng0, rng1, 2u, 1u, c0, c1);
    uint32_t k20, k21;  // randint(rng1, (), 0, 4) = bits(split(rng1)[1]) % 4
    tf_split(c0, c1, 2u, 1u, k20, k21);
    const int ch = (int)(tf_elem(k20, k21, 1u, 0u) % 4u);
    const float ax = x0.x, ay = x0.y;
    const float tx = t.tp_ok ? t.tp[0] : QQ::ld(in.pos, r3 + 30), ty = t.tp_ok ? t.tp[1] : QQ::ld(in.pos, r3 + 31);
    float vx = ax - tx, vy = ay - ty;
    const float nrm = sqrtf(vx * vx + vy * vy);
    vx = vx / nrm; vy = vy / nrm;
    float cx, cy;
    if (ch == 0) { cx = vy * 1.0f; cy = vx * -1.0f; }
    else if (ch == 1) { cx = vy * -1.0f; cy = vx * 1.0f; }
    else if (ch == 2) { cx = -vx; cy = -vy; }
    else { cx = 0.0f; cy = 0.0f; }
    float nx = cx * S.tag_target_step + tx, ny = cy * S.tag_target_step + ty;
    if (fabsf(nx) > S.tag_cage_xy[0] || fabsf(ny) > S.tag_cage_xy[1]) { nx = tx; ny = ty; }
    QQ::st(opos, r3 + 30, nx); QQ::st(opos, r3 + 31, ny); QQ::st(opos, r3 + 32, 1.0f);
    rng0 = n0; rng1 = n1;
    const bool vis = dist2d(nx, ny, ax, ay) <= S.tag_visible_radius;
    t.ob0 = vis ? nx : 0.0f; t.ob1 = vis ? ny : 0.0f;
    const float tag = dist2d(ax, ay, nx, ny) <= S.tag_tag_radius ? 1.0f : 0.0f;
    m0 = tag;
    if (tag > 0.0f) reward = 1.0f;
    done = (dead != 0.0f || tag != 0.0f) ? 1.0f : 0.0f;
  }
  float trunc = in.truncation ? in.truncation[b] : 0.0f;
  if (flags & POB_F_EPISODE) {  // brax EpisodeWrapper.step [ext]
    steps = steps + 1.0f;
    trunc = steps >= (float)L ? 1.0f - done : 0.0f;
    done = steps >= (float)L ? 1.0f : done;
  }
  t.reward = reward; t.done = done; t.trunc = trunc; t.steps = steps;
  t.m0 = m0; t.m1 = m1; t.m2 = m2; t.rng0 = rng0; t.rng1 = rng1;
}

// AntGather objects (ant_gather.py:125-181) on the env's four quad lanes: lane k takes
// objects k, k + 4, k + 8, k + 12 (n_obj <= 16), so their loads are in flight together and
// the sensor angles / catches / relocations run in parallel; the sensor scatter keeps the
// reference's object order (last writer wins): lane 0 writes the readings of objects
// 0, 1, 2, ... from DPP-gathered (slot, value) pairs.  Counts and flags are reduced over
// the quad.  All four lanes must be active.
#define POB_GA_QUAD_MAX 16
struct GaQuad {
  int slot[4];   // sensor slot written by this lane's object j (-1: none)
  float val[4];  // and the value
};
// The lane's objects' input positions, read from the env's staged pos rows (LDS) during the
// state load, or loaded here when the load was not staged (pre == nullptr).
template <typename QT>
POB_D void ga_quad_prefetch(csys_t &S, const StatePtrs &in, const size_t r3, const float *srow, const int k,
                            v3 (&op)[4]) {
  using QQ = Q<QT>;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int obj = k + 4 * j;
    op[j] = V(0.0f, 0.0f, 0.0f);
    if (obj < S.n_obj) {
      if (srow) op[j] = V(srow[3 * (11 + obj)], srow[3 * (11 + obj) + 1], srow[3 * (11 + obj) + 2]);
      else {
        const size_t row = r3 + 3 * (11 + obj);
        op[j] = V(QQ::ld(in.pos, row), QQ::ld(in.pos, row + 1), QQ::ld(in.pos, row + 2));
      }
    }
  }
}
template <typename QT>
POB_D void ga_quad_objects(csys_t &S, const v3 (&op)[4], const size_t r3, const v3 x0, const q4 q0, const int k,
                           float *opos, GaQuad &g, TaskOut &t) {
  using QQ = Q<QT>;
  const float ori = ga_orientation(q0);
  int na = 0, nb = 0;
  bool any_a = false, any_b = false, all_wait = true;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int obj = k + 4 * j;
    g.slot[j] = -1; g.val[j] = 0.0f;
    if (obj < S.n_obj) {
      const size_t row = r3 + 3 * (11 + obj);
      const float ox = op[j].x, oy = op[j].y, oz = op[j].z;
      const float dk = dist2d(x0.x, x0.y, ox, oy);
      g.slot[j] = ga_reading_slot(S, obj, ox, oy, dk, ori, g.val[j]);
      const bool c = dk <= S.ga_catch_range;
      float nx = ox, ny = oy, nz = oz;
      if (c) { nx = S.ga_waiting[0]; ny = S.ga_waiting[1]; nz = S.ga_waiting[2]; }
      QQ::st(opos, row, nx); QQ::st(opos, row + 1, ny); QQ::st(opos, row + 2, nz);
      if (obj < S.ga_n_apples) { any_a |= c; na += c; } else { any_b |= c; nb += c; }
      all_wait &= (nx == S.ga_waiting[0]) & (ny == S.ga_waiting[1]) & (nz == S.ga_waiting[2]);
    }
  }
  const float fa = (float)na, fb = (float)nb;
  const float flag = (any_a ? 1.0f : 0.0f) + (any_b ? 2.0f : 0.0f) + (all_wait ? 0.0f : 4.0f);
  t.ga_na = (int)(((quad_bcast<0>(fa) + quad_bcast<1>(fa)) + quad_bcast<2>(fa)) + quad_bcast<3>(fa));
  t.ga_nb = (int)(((quad_bcast<0>(fb) + quad_bcast<1>(fb)) + quad_bcast<2>(fb)) + quad_bcast<3>(fb));
  const int f0 = (int)quad_bcast<0>(flag), f1 = (int)quad_bcast<1>(flag), f2 = (int)quad_bcast<2>(flag),
            f3 = (int)quad_bcast<3>(flag);
  const int fo = f0 | f1 | f2 | f3;
  t.ga_any_a = (fo & 1) != 0; t.ga_any_b = (fo & 2) != 0; t.ga_all_wait = (fo & 4) == 0;
  t.ga_done_quad = true;
}
// lane 0 writes the readings of objects 0, 1, 2, ... in order (all four lanes active)
POB_D void ga_quad_scatter(csys_t &S, const GaQuad &g, const int k, float *rd) {
  if (k == 0) ga_readings_begin(S, rd);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float s0 = quad_bcast<0>(__int_as_float(g.slot[j])), v0 = quad_bcast<0>(g.val[j]);
    const float s1 = quad_bcast<1>(__int_as_float(g.slot[j])), v1 = quad_bcast<1>(g.val[j]);
    const float s2 = quad_bcast<2>(__int_as_float(g.slot[j])), v2 = quad_bcast<2>(g.val[j]);
    const float s3 = quad_bcast<3>(__int_as_float(g.slot[j])), v3_ = quad_bcast<3>(g.val[j]);
    if (k == 0) {  // objects 4j, 4j + 1, 4j + 2, 4j + 3
      if (__float_as_int(s0) >= 0) rd[__float_as_int(s0)] = v0;
      if (__float_as_int(s1) >= 0) rd[__float_as_int(s1)] = v1;
      if (__float_as_int(s2) >= 0) rd[__float_as_int(s2)] = v2;
      if (__float_as_int(s3) >= 0) rd[__float_as_int(s3)] = v3_;
    }
  }
}

// task tail of a fixed kind, or (POB_MIXED) of the kind recorded in the env's table
template <int KIND, typename QT>
POB_D void task_dispatch(csys_t &S, const int kind, const StatePtrs &in, const int b, const size_t r3, const int N,
                         const v3 x0, const q4 q0, float *opos, float *o, const uint32_t flags, const int L,
                         TaskOut &t) {
  if (KIND != POB_MIXED) { task_step<KIND, QT>(S, in, b, r3, N, x0, q0, opos, o, flags, L, t); return; }
  if (kind == POB_HEAVENHELL) task_step<POB_HEAVENHELL, QT>(S, in, b, r3, N, x0, q0, opos, o, flags, L, t);
  else if (kind == POB_GATHER) task_step<POB_GATHER, QT>(S, in, b, r3, N, x0, q0, opos, o, flags, L, t);
  else if (kind == POB_TAG) task_step<POB_TAG, QT>(S, in, b, r3, N, x0, q0, opos, o, flags, L, t);
  else task_step<POB_ANT, QT>(S, in, b, r3, N, x0, q0, opos, o, flags, L, t);
}
// the typed copies of the step outputs the caller asked for (pob.h, ABI v5)
POB_D void write_typed(const StatePtrs &out, const int b, const TaskOut &t) {
  if (out.done_u8) out.done_u8[b] = t.done != 0.0f ? 1 : 0;
  if (out.trunc_i32) out.trunc_i32[b] = (int32_t)t.trunc;
  if (out.m0_i32) out.m0_i32[b] = (int32_t)t.m0;
  if (out.m1_i32) out.m1_i32[b] = (int32_t)t.m1;
}
// the task's obs entries into the env's obs row (HH: heaven direction, TAG: target xy; the
// AntGather readings are written by the object pass)
POB_D void task_obs_write(const int kind, float *o, const int base, const TaskOut &t) {
  if (kind == POB_HEAVENHELL) o[base] = t.ob0;
  else if (kind == POB_TAG) { o[base] = t.ob0; o[base + 1] = t.ob1; }
}

// ------------------------------------------------------------------ step, lane quads
// Same fused step with FOUR lanes per env (pob_quad.h): lane k owns the torso (replica)
// and leg k (bodies 2k+1, 2k+2).  39 LDS floats / lane.  Lane 0 runs the per-env POMDP
// tail; every lane writes its bodies' rows, its joints' obs and its cfrc rows.
// gt = the quad-lane index within this env batch (4 b + k).
#ifndef POB_QUAD_MIN_WAVES
#define POB_QUAD_MIN_WAVES 4
#endif
// Per-wave LDS region: the block's per-lane scratch is laid out wave-major (wave w owns
// floats [w * POB_STAGE_FLOATS, (w + 1) * POB_STAGE_FLOATS), element e of its lane t at
// e * 64 + t: conflict-free), so a wave can reuse its whole region as a contiguous staging
// buffer for coalesced state I/O while the other waves of the block still run physics.
#define POB_STAGE_FLOATS (QL_FLOATS * 64)
POB_D void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// envs per obs pass of a wave's staging region (cap floats, rows of D floats, at most maxe):
// a multiple of 4 when it is below maxe, so that every pass's rows start 16-B aligned
POB_D int pass_envs(const int cap, const int D, const int maxe) {
  const int p = cap / D;
  return p >= maxe ? maxe : (p >= 4 ? p & ~3 : p);
}

// Coalesced copy of n_el consecutive qp elements (from element el0) into stg: 16 B (f32)
// / 8 B (f16) vector loads by all 64 lanes.
template <typename QT>
POB_D void stage_load(const float *X, size_t el0, int n_el, float *stg, int lane);
template <>
POB_D void stage_load<float>(const float *X, size_t el0, int n_el, float *stg, int lane) {
  for (int i = 4 * lane; i < n_el; i += 256) {
    const float *p = X + el0 + i;
    if (i + 4 <= n_el) {
      const float4 v = *reinterpret_cast<const float4 *>(p);
      stg[i] = v.x; stg[i + 1] = v.y; stg[i + 2] = v.z; stg[i + 3] = v.w;
    } else {
      for (int q = 0; q < n_el - i; ++q) stg[i + q] = p[q];
    }
  }
}
template <>
POB_D void stage_load<__half>(const float *X, size_t el0, int n_el, float *stg, int lane) {
  const __half *H = reinterpret_cast<const __half *>(X);
  for (int i = 4 * lane; i < n_el; i += 256) {
    const __half *p = H + el0 + i;
    if (i + 4 <= n_el) {
      const uint2 v = *reinterpret_cast<const uint2 *>(p);
      const __half2 a = *reinterpret_cast<const __half2 *>(&v.x), c = *reinterpret_cast<const __half2 *>(&v.y);
      stg[i] = __low2float(a); stg[i + 1] = __high2float(a); stg[i + 2] = __low2float(c); stg[i + 3] = __high2float(c);
    } else {
      for (int q = 0; q < n_el - i; ++q) stg[i + q] = __half2float(p[q]);
    }
  }
}
// All loads of one array issued before any is consumed: MAXI 16-B (8-B for f16) chunks per
// lane in registers (predicated), then written to stg.  Two of these back to back keep two
// arrays' loads in flight at once.
template <typename QT, int MAXI>
struct ChunkLoad {
  float v[MAXI][4];
  // ROWF = elements per env row (N * c), DYNF = those of the dynamic bodies (9 * c): a chunk
  // that lies inside one env's frozen rows is not loaded (the task tail reads frozen rows
  // from memory itself)
  template <int ROWF, int DYNF>
  POB_D void issue(const float *X, size_t el0, int n_el, int lane) {
#pragma unroll
    for (int m = 0; m < MAXI; ++m) {
      const int i = 4 * lane + 256 * m;
      const int o = i % ROWF;
      if (o >= DYNF && o + 4 <= ROWF) continue;
      if (i + 4 <= n_el) {
        if constexpr (sizeof(QT) == 4) {
          const float4 q = *reinterpret_cast<const float4 *>(X + el0 + i);
          v[m][0] = q.x; v[m][1] = q.y; v[m][2] = q.z; v[m][3] = q.w;
        } else {
          const uint2 q = *reinterpret_cast<const uint2 *>(reinterpret_cast<const __half *>(X) + el0 + i);
          const __half2 a = *reinterpret_cast<const __half2 *>(&q.x), c = *reinterpret_cast<const __half2 *>(&q.y);
          v[m][0] = __low2float(a); v[m][1] = __high2float(a); v[m][2] = __low2float(c); v[m][3] = __high2float(c);
        }
      } else if (i < n_el) {
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (q < n_el - i) v[m][q] = Q<QT>::ld(X, el0 + i + q);
      }
    }
  }
  template <int ROWF, int DYNF>
  POB_D void put(float *stg, int n_el, int lane) const {
#pragma unroll
    for (int m = 0; m < MAXI; ++m) {
      const int i = 4 * lane + 256 * m;
      const int o = i % ROWF;
      if (o >= DYNF && o + 4 <= ROWF) continue;
      if (i + 4 <= n_el) { stg[i] = v[m][0]; stg[i + 1] = v[m][1]; stg[i + 2] = v[m][2]; stg[i + 3] = v[m][3]; }
      else if (i < n_el) {
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (q < n_el - i) stg[i + q] = v[m][q];
      }
    }
  }
};

// Coalesced store of the dynamic-body part (first C9 = 9 c elements) of nenv consecutive
// rows of N * c elements, from stg (row-major nenv x C9).
template <typename QT, int C>
POB_D void stage_store_dyn(float *X, size_t el0, int N, int nenv, const float *stg, int lane) {
  constexpr int C9 = POB_NDYN * C;
  if (sizeof(QT) == 4 && (C == 3 || (reinterpret_cast<uintptr_t>(X) & 15) == 0)) {
    // f32: one row (12 or 16 B) per lane and store instruction
    struct alignas(4) f3 { float a, b, c; };
    for (int r = lane; r < nenv * POB_NDYN; r += 64) {
      const int e = r / POB_NDYN, g = r - e * POB_NDYN;
      float *dst = X + el0 + (size_t)e * N * C + g * C;
      const float *src = stg + r * C;
      if constexpr (C == 4) *reinterpret_cast<float4 *>(dst) = *reinterpret_cast<const float4 *>(src);
      else *reinterpret_cast<f3 *>(dst) = f3{src[0], src[1], src[2]};
    }
  } else {
    for (int i = lane; i < nenv * C9; i += 64) {
      const int e = i / C9, j = i - e * C9;
      Q<QT>::st(X, el0 + (size_t)e * N * C + j, stg[i]);
    }
  }
}

// Copy N floats of the system table into LDS with every load of the thread in flight before
// its LDS writes (a strided loop waited for each load in turn: ~10 memory round trips in a
// one-wave block's prologue).  stride = the block size, >= 64.
template <int N>
POB_D void stage_table(float *dst, const __attribute__((address_space(4))) float *src, const int tid,
                       const int stride) {
  constexpr int M = (N + 63) / 64;
  float v[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int i = tid + stride * m;
    v[m] = i < N ? src[i] : 0.0f;
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int i = tid + stride * m;
    if (i < N) dst[i] = v[m];
  }
}
// stage the block table (leg rows, then wall rows) in LDS (all threads of the block;
// before any divergence)
POB_D void stage_leg_table(csys_t *Sp, float *legtab) {
  const __attribute__((address_space(4))) float *src = &Sp->leg[0][0];  // leg[4][..], wall_row[..][8]
  stage_table<POB_TAB_FLOATS>(legtab, src, (int)threadIdx.x, (int)blockDim.x);
  __syncthreads();
}
#ifdef POB_EXP_TIMING
#define POB_TS_WAVES 65536
// per wave: hw id, xcc id, then POB_TS_N stamps (unset stamps are 0)
#ifdef POB_EXP_TIMING_SUB
#define POB_TS_N 16  // + the substep phase sums in stamps 5..12
#else
#define POB_TS_N 10
#endif
#define POB_TS_ROW (POB_TS_N + 4)  // + the wave's start / end on the device-wide 100 MHz clock
__device__ unsigned long long pob_ts_buf[POB_TS_WAVES * POB_TS_ROW];  // timing experiment only
#define POB_TS_DECL() \
  unsigned long long pob_ts[POB_TS_N] = {}; \
  const unsigned long long pob_rt0 = __builtin_amdgcn_s_memrealtime()
#define POB_TS(i) pob_ts[i] = __builtin_amdgcn_s_memtime()
#define POB_TS_WRITE()                                                                   \
  do {                                                                                   \
    POB_TS(POB_TS_N - 1);                                                                \
    if ((threadIdx.x & 63) == 0) {                                                       \
      unsigned hwid, xcc;                                                                \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));                 \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));                 \
      const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);      \
      if (w < POB_TS_WAVES) {                                                            \
        unsigned long long *r = pob_ts_buf + w * POB_TS_ROW;                             \
        r[0] = hwid; r[1] = xcc;                                                         \
        for (int i = 0; i < POB_TS_N; ++i) r[2 + i] = pob_ts[i];                         \
        r[POB_TS_N + 2] = pob_rt0; r[POB_TS_N + 3] = __builtin_amdgcn_s_memrealtime();    \
      }                                                                                  \
    }                                                                                    \
  } while (0)
#else
#define POB_TS_DECL() ((void)0)
#define POB_TS(i) ((void)0)
#define POB_TS_WRITE() ((void)0)
#endif
// dynamic qp rows of a lane quad's wave: the computed state (or the env's first_qp rows when
// the AutoResetWrapper resets it) staged in the wave's LDS region and stored coalesced
template <typename QT>
__device__ __forceinline__ void quad_store_dyn(const StatePtrs &in, const StatePtrs &out, const QBody &bd,
                                               const bool act_lane, const int k, const int le, const int b_first,
                                               const int nenv, const int N, const size_t r3, const size_t r4,
                                               float *stg, const int lane, const bool reset_rows) {
#pragma unroll
  for (int arr = 0; arr < 4; ++arr) {
    const int c = arr == 1 ? 4 : 3;
    if (act_lane) {
#pragma unroll
      for (int l = 0; l < QNB; ++l) {
        if (l == 0 && k != 0) continue;
        const int g = qbody_global(l, k);
        float *o = stg + (le * POB_NDYN + g) * c;
        if (reset_rows) {
          const float *F = arr == 0 ? in.first_pos : (arr == 1 ? in.first_rot : (arr == 2 ? in.first_vel : in.first_ang));
          const size_t src = (arr == 1 ? r4 : r3) + (size_t)g * c;
          for (int q = 0; q < c; ++q) o[q] = Q<QT>::ld(F, src + q);
        } else if (arr == 0) { o[0] = bd.x[l].x; o[1] = bd.x[l].y; o[2] = bd.x[l].z; }
        else if (arr == 1) { o[0] = bd.q[l].w; o[1] = bd.q[l].x; o[2] = bd.q[l].y; o[3] = bd.q[l].z; }
        else if (arr == 2) { o[0] = bd.v[l].x; o[1] = bd.v[l].y; o[2] = bd.v[l].z; }
        else { o[0] = bd.w[l].x; o[1] = bd.w[l].y; o[2] = bd.w[l].z; }
      }
    }
    wave_lds_sync();
    if (arr == 1) stage_store_dyn<QT, 4>(out.rot, (size_t)b_first * N * 4, N, nenv, stg, lane);
    else stage_store_dyn<QT, 3>(arr == 0 ? out.pos : (arr == 2 ? out.vel : out.ang), (size_t)b_first * N * 3, N,
                                nenv, stg, lane);
    wave_lds_sync();
  }
}

// Wall-contact overflow handling of the four-lane kernel (MODE): 0 = in the kernel (the position
// and velocity passes re-walk an overflowing lane's faces); 1 = the fast launch: every wave
// records in ovf_mark[its first env] whether one of its lanes overflowed the contact store (its
// first store clears the mark: AntGather's no-wall pass never reaches the overflow test), and a
// wave that overflowed stores nothing else and exits; 2 = the fix-up launch right after it: only
// the marked waves run, the whole step with the re-walks.  The re-walk code's mere presence in
// the substep loop cost 15 % (HH) through register pressure (profiles/r6a_ab.txt); split, the
// common launch carries none of it.  The marks are a caller-provided scratch array (pob_state
// ovf_mark, ABI v8) outside every output -- round 5's in-band mark (a signalling NaN in the
// wave's first obs element) could be forged by a first_obs row that AUTORESET copies -- and
// every wave of the fast launch writes its mark, so the array needs no initialisation; slices
// of it serve concurrent launches on disjoint state slices (GraphRollout groups).
template <int KIND, typename QT, bool LEG = false, int MODE = 0>
POB_D void step_quad_body(csys_t *Sp, const int B, const StatePtrs &in, const float *__restrict__ act,
                          const StatePtrs &out, const uint32_t flags, const int L, const int gt, float *lds,
                          const float *legtab) {
  csys_t &S = *Sp;
  const int lane = (int)threadIdx.x & 63;
  POB_TS_DECL();  // timing experiment only (POB_EXP_TIMING)
  POB_TS(0);
  float *stg = lds + ((int)threadIdx.x >> 6) * POB_STAGE_FLOATS;  // this wave's region
  const QLds Ls{stg, lane};
  int b = gt >> 2;
  int k = gt & 3;
  const float *LT = legtab + k * POB_LEG_FLOATS;
  const float *WT = legtab + 4 * POB_LEG_FLOATS;
  const int kind = KIND != POB_MIXED ? KIND : S.kind;
  const int N = n_bodies<KIND>(S), D = obs_dim<KIND>(S);
  const int sh = obs_shift(kind);
  bool act_lane = b < B;
  // the wave's 16 envs are consecutive rows of every state array
  int b_first = (gt - lane) >> 2;
  if (b_first >= B) return;  // (wave-uniform: a block's waves past the batch; no barrier follows)
  if (MODE == 2 && out.ovf_mark[b_first] == 0) return;  // (not marked)
  if (MODE == 1 && lane == 0) out.ovf_mark[b_first] = 0;  // (every wave: the passes that finish leave it)
  int nenv = B - b_first < 16 ? B - b_first : 16;
  int le = b - b_first;
  // The physics runs on all 64 lanes (the wave walk's DPP / bpermute rounds need every lane):
  // the lanes past the batch in its last wave replay env B - 1 and store nothing.
  int bl = act_lane ? b : B - 1, lel = bl - b_first;
  size_t r3 = (size_t)bl * N * 3, r4 = (size_t)bl * N * 4;
  // the same indices from an opaque copy of the thread index (after the substep loop: the copies
  // above are then dead across it, instead of held -- in practice spilled -- through it)
  auto rederive = [&]() {
    int g2 = gt;
    asm volatile("" : "+v"(g2));
    b = g2 >> 2;
    k = g2 & 3;
    act_lane = b < B;
    b_first = (g2 - (g2 & 63)) >> 2;
    nenv = B - b_first < 16 ? B - b_first : 16;
    le = b - b_first;
    bl = act_lane ? b : B - 1;
    lel = bl - b_first;
    r3 = (size_t)bl * N * 3;
    r4 = (size_t)bl * N * 4;
  };

  // ---- state load: coalesced vector loads into the wave's region, then every lane
  // picks its bodies (the host sets POB_F_STAGED when the qp pointers are 16-B aligned
  // and 16 envs x N x 4 fit the region); otherwise per-lane loads
  QBody bd;
  constexpr int NMAX = KIND == POB_HEAVENHELL ? 14 : (KIND == POB_TAG ? 12 : (KIND == POB_ANT ? 10 : POB_MAXB));
  constexpr int MAXI = (16 * NMAX * 4 + 255) / 256;  // 16-B chunks per lane of one array
  if ((flags & POB_F_STAGED) && NMAX <= 16 && N == NMAX && 16 * N * 7 <= POB_STAGE_FLOATS) {
    // pairs (pos, rot), (vel, ang): both arrays' loads in flight before either is consumed
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int c0 = 3, c1 = pr == 0 ? 4 : 3;
      const int n0 = nenv * N * c0, n1 = nenv * N * c1;
      ChunkLoad<QT, MAXI> A0, A1;
      // (N == NMAX on this path: HH / TAG / stock ant tables)
      A0.template issue<NMAX * 3, POB_NDYN * 3>(pr == 0 ? in.pos : in.vel, (size_t)b_first * N * c0, n0, lane);
      if (pr == 0) A1.template issue<NMAX * 4, POB_NDYN * 4>(in.rot, (size_t)b_first * N * c1, n1, lane);
      else A1.template issue<NMAX * 3, POB_NDYN * 3>(in.ang, (size_t)b_first * N * c1, n1, lane);
      A0.template put<NMAX * 3, POB_NDYN * 3>(stg, n0, lane);
      if (pr == 0) A1.template put<NMAX * 4, POB_NDYN * 4>(stg + n0, n1, lane);
      else A1.template put<NMAX * 3, POB_NDYN * 3>(stg + n0, n1, lane);
      wave_lds_sync();
      {
#pragma unroll
        for (int l = 0; l < QNB; ++l) {
          const int g = qbody_global(l, k);
          const float *s0 = stg + (lel * N + g) * c0, *s1 = stg + n0 + (lel * N + g) * c1;
          if (pr == 0) {
            bd.x[l] = V(s0[0], s0[1], s0[2]);
            bd.q[l].w = s1[0]; bd.q[l].x = s1[1]; bd.q[l].y = s1[2]; bd.q[l].z = s1[3];
          } else {
            bd.v[l] = V(s0[0], s0[1], s0[2]);
            bd.w[l] = V(s1[0], s1[1], s1[2]);
          }
        }
      }
      wave_lds_sync();
    }
  } else if (flags & POB_F_STAGED) {
#pragma unroll
    for (int arr = 0; arr < 4; ++arr) {
      const int c = arr == 1 ? 4 : 3;
      const float *X = arr == 0 ? in.pos : (arr == 1 ? in.rot : (arr == 2 ? in.vel : in.ang));
      stage_load<QT>(X, (size_t)b_first * N * c, nenv * N * c, stg, lane);
      wave_lds_sync();
      {
#pragma unroll
        for (int l = 0; l < QNB; ++l) {
          const int o = (lel * N + qbody_global(l, k)) * c;
          if (arr == 0) bd.x[l] = V(stg[o], stg[o + 1], stg[o + 2]);
          else if (arr == 1) { bd.q[l].w = stg[o]; bd.q[l].x = stg[o + 1]; bd.q[l].y = stg[o + 2]; bd.q[l].z = stg[o + 3]; }
          else if (arr == 2) bd.v[l] = V(stg[o], stg[o + 1], stg[o + 2]);
          else bd.w[l] = V(stg[o], stg[o + 1], stg[o + 2]);
        }
      }
      wave_lds_sync();
    }
  } else {
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      const int g = qbody_global(l, k);
      bd.x[l] = ld3<QT>(in.pos, r3 + 3 * g);
      bd.q[l] = ld4<QT>(in.rot, r4 + 4 * g);
      bd.v[l] = ld3<QT>(in.vel, r3 + 3 * g);
      bd.w[l] = ld3<QT>(in.ang, r3 + 3 * g);
    }
  }

  POB_TS(1);
  // ---- physics (10 substeps in registers + the lane's LDS slots)
#ifndef POB_QUAD_TWO_PASS
#define POB_QUAD_TWO_PASS 1
#endif
#ifndef POB_QUAD_NEAR_MARGIN
#define POB_QUAD_NEAR_MARGIN 0.5f
#endif
  float jang[QNJ], jvel[QNJ];
  v3 cvl[QNB], cal[QNB];
  TaskOut t;
  t.tp_ok = false;
  {
    float a[QNJ];
#pragma unroll
    for (int jl = 0; jl < QNJ; ++jl) a[jl] = act[(size_t)bl * POB_NJ + 2 * k + jl];
#pragma unroll
    for (int l = 0; l < QNB; ++l) { Ls.set3(l, QF_CV, V(0.0f, 0.0f, 0.0f)); Ls.set3(l, QF_CA, V(0.0f, 0.0f, 0.0f)); }
    const int iters = Sp->substeps / 2;
    const float fric = quad_friction(S);
    // (per kind, bit 1 << KIND: HH 1, GA 2, TAG 4, ant 8, mixed 16 -- the register allocation of
    // each instantiation reacts differently; profiles/r5x_ab.txt: HH B = 65 536 0.1873 ms with
    // neither, TAG 0.1176 with both, GA 0.1147 and mixed fp16 B = 32 768 0.1281 with the
    // re-derivation only; profiles/r5y_ab.txt)
#ifndef POB_QUAD_FAST_PASS
#define POB_QUAD_FAST_PASS 4
#endif
#ifndef POB_QUAD_REDERIVE
#define POB_QUAD_REDERIVE 22
#endif
    constexpr int KBIT = KIND < 0 ? 16 : 1 << KIND;
    constexpr bool FASTP = (POB_QUAD_FAST_PASS & KBIT) != 0, REDER = (POB_QUAD_REDERIVE & KBIT) != 0;
    if (LEG) {
      // legacy spring dynamics: every substep kinetic + springs + contact impulses
#pragma nounroll
      for (int it = 0; it < Sp->substeps; ++it) qlegacy_substep<KIND != POB_ANT>(Sp, LT, WT, bd, a, Ls);
    } else {
#if defined(POB_EXP_NO_COLLIDE)
#pragma nounroll
    for (int it = 0; it < 2 * iters; ++it) qpbd_substep<KIND != POB_ANT>(Sp, LT, WT, bd, a, Ls, false, S.friction);  // timing experiment only
#elif defined(POB_EXP_NO_PHYSICS)
#pragma nounroll
    for (int it = 0; it < 0 * iters; ++it) qpbd_substep<KIND != POB_ANT>(Sp, LT, WT, bd, a, Ls, false, S.friction);  // timing experiment only
#else
    // Two passes (wave-uniform): a wave whose lanes are all clear of the walls' broadphase boxes
    // (grown by POB_QUAD_NEAR_MARGIN) at the start of the step runs the substeps without the
    // wall code and checks the broadphase of every collide substep; if a lane met one, the wave
    // reloads the step's state and runs the wall pass (the no-wall pass is exact when it
    // completes: every wall pass item list would have been empty).  The wall pass's registers
    // and code then cost only the waves near a wall.
    // (AntGather only: its ants start at the arena's centre, so whole waves run the no-wall
    // pass -- 0.272 -> 0.122 ms at B = 65 536; the HH / TAG waves nearly always hold an ant near
    // a wall, and the second copy of the substep loop costs them 5-10 %, profiles/r5m)
    constexpr bool TWO = KIND == POB_GATHER && POB_QUAD_TWO_PASS;
    constexpr bool WALLS = KIND != POB_ANT;
    // Wall passes (POB_QUAD_FAST_PASS, off): a fast pass keeping at most QK wall contacts per
    // lane and collide substep, a wave with more (rare) running the step again in the slow pass
    // with the re-walks.  Measured slower than the one wall pass with the inline re-walk (HH
    // B = 65 536 0.2163 vs 0.1877 ms, TAG 0.1330 vs 0.1221; profiles/r5s_ab.txt): the two loops'
    // live ranges spilled the step's values around them.
    int pass = TWO ? (__any(qwall_mask_margin(S, bd, POB_QUAD_NEAR_MARGIN) != 0u) ? 1 : 0) : 1;
    auto reload = [&]() {
#pragma unroll
      for (int l = 0; l < QNB; ++l) {
        const int g = qbody_global(l, k);
        bd.x[l] = ld3<QT>(in.pos, r3 + 3 * g);
        bd.q[l] = ld4<QT>(in.rot, r4 + 4 * g);
        bd.v[l] = ld3<QT>(in.vel, r3 + 3 * g);
        bd.w[l] = ld3<QT>(in.ang, r3 + 3 * g);
        Ls.set3(l, QF_CV, V(0.0f, 0.0f, 0.0f));
        Ls.set3(l, QF_CA, V(0.0f, 0.0f, 0.0f));
      }
    };
    for (;;) {
    if (pass == 0) {
      bool near = false;
#pragma nounroll
      for (int it = 0; it < 2 * iters; ++it) {
#if POB_QUAD_PRIO == 1
        const int lvl = (it * 4) / (2 * iters);
        if (lvl == 0) __builtin_amdgcn_s_setprio(3);
        else if (lvl == 1) __builtin_amdgcn_s_setprio(2);
        else if (lvl == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
#endif
        qpbd_substep<false, true>(Sp, LT, WT, bd, a, Ls, (it & 1) != 0, fric, &near);
      }
      if (!__any(near)) break;
      // a lane met a wall's broadphase: the step again, from its state, with the walls
      pass = 1;
      reload();
      continue;
    }
#ifndef POB_QUAD_SLOW_OOL
#define POB_QUAD_SLOW_OOL 1  // (with POB_QUAD_FAST_PASS: the slow pass's substep out of line)
#endif
    if (MODE == 1 && WALLS) {
      // the fast launch: the store only; a wave with an overflowing lane leaves the step to the
      // fix-up launch (nothing of its state is written: every output store follows the physics)
      bool ovf = false;
#pragma nounroll
      for (int it = 0; it < 2 * iters; ++it) {
#if POB_QUAD_PRIO == 1
        const int lvl = (it * 4) / (2 * iters);
        if (lvl == 0) __builtin_amdgcn_s_setprio(3);
        else if (lvl == 1) __builtin_amdgcn_s_setprio(2);
        else if (lvl == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
#endif
        qpbd_substep<WALLS, false, false>(Sp, LT, WT, bd, a, Ls, (it & 1) != 0, fric, nullptr, &ovf);
        if (__any(ovf)) break;
      }
      if (__any(ovf) || (flags & POB_F_INT_FORCE_FIXUP)) {
        if (lane == 0) out.ovf_mark[b_first] = 1;
        return;
      }
      break;
    }
    if (pass == 1 && WALLS && FASTP && MODE == 0) {
      bool ovf = false;
#pragma nounroll
      for (int it = 0; it < 2 * iters; ++it) {
        // Issue priority falls with progress, so a SIMD's four waves (one per block) advance
        // together: with the default oldest-first arbitration the first wave finishes early
        // and the last one runs its final substeps alone, at one-wave latency (measured per
        // wave with POB_EXP_TIMING: p0..max of the physics phase 94 K..211 K ticks before,
        // 133 K..182 K with this; kernel 0.120 -> 0.112 ms at B = 65 536).
#if POB_QUAD_PRIO == 1
        const int lvl = (it * 4) / (2 * iters);
        if (lvl == 0) __builtin_amdgcn_s_setprio(3);
        else if (lvl == 1) __builtin_amdgcn_s_setprio(2);
        else if (lvl == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
#endif
        qpbd_substep<WALLS, false, false>(Sp, LT, WT, bd, a, Ls, (it & 1) != 0, fric, nullptr, &ovf);
        if (__any(ovf)) break;
      }
      if (!__any(ovf)) break;
      pass = 2;
      reload();
      continue;
    }
    // the slow wall pass (after an overflow) / the stock ant (no walls)
#pragma nounroll
    for (int it = 0; it < 2 * iters; ++it) {
#if POB_QUAD_PRIO == 1
      const int lvl = (it * 4) / (2 * iters);
      if (lvl == 0) __builtin_amdgcn_s_setprio(3);
      else if (lvl == 1) __builtin_amdgcn_s_setprio(2);
      else if (lvl == 2) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
#endif
#if POB_QUAD_SLOW_OOL
      if (WALLS && FASTP && MODE == 0) {
        QSlow st;
        st.b = bd;
#pragma unroll
        for (int j = 0; j < QNJ; ++j) st.act[j] = a[j];
        qpbd_substep_slow<WALLS>(Sp, LT, WT, &st, Ls.base, Ls.t, (it & 1) != 0 ? 1 : 0, fric);
        bd = st.b;
      } else
#endif
      qpbd_substep<WALLS>(Sp, LT, WT, bd, a, Ls, (it & 1) != 0, fric);
    }
    break;
    }
#endif
    }
    if constexpr (REDER) rederive();
    // the torso's x at the step's start (the reward's displacement): loaded again (the state
    // arrays are not written before the task tail)
    const float xb = ld3<QT>(in.pos, r3).x;
    // joint angle / velocity obs of this lane's joints (a3)
#pragma unroll
    for (int jl = 0; jl < QNJ; ++jl) {
      const int p = jparent(jl), c = jchild(jl);
      v3 ap = qrot(QJV(LT, jl, QJ_AXIS), bd.q[p]);
      const v3 ref = jl == 0 ? V(-1.0f, 0.0f, 0.0f) : V(0.0f, 0.0f, 1.0f);  // the Ant's (pob_system.cpp)
      v3 fp = qrot(ref, bd.q[p]), fc = qrot(ref, bd.q[c]);
      jang[jl] = pob_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
      jvel[jl] = vdot(vsub(bd.w[c], bd.w[p]), ap);
    }
#pragma unroll
    for (int l = 0; l < QNB; ++l) { cvl[l] = Ls.get3(l, QF_CV); cal[l] = Ls.get3(l, QF_CA); }
    if (act_lane && k == 0) {
      float steps = in.steps ? in.steps[b] : 0.0f;
      if ((flags & (POB_F_AUTORESET | POB_F_ZERO_STEPS_ON_DONE)) && in.done[b] != 0.0f) steps = 0.0f;
      t.steps = steps;
      t.m0 = in.m0 ? in.m0[b] : 0.0f; t.m1 = in.m1 ? in.m1[b] : 0.0f; t.m2 = in.m2 ? in.m2[b] : 0.0f;
      t.rng0 = in.rng[2 * b]; t.rng1 = in.rng[2 * b + 1];
      t.xb = xb; t.ctrl = 0.0f; t.contact = 0.0f;
      if (kind == POB_ANT) {
        // full action row; contact rows 0..8 = own slots 0..2, then lanes +1, +2, +3 slots 1..2
        t.ctrl = ant_ctrl_cost(act + (size_t)b * POB_NJ);
        float sc = 0.0f;
#pragma unroll
        for (int l = 0; l < QNB; ++l) sc = ant_contact_add(sc, cvl[l]);
#pragma unroll
        for (int q = 1; q < 4; ++q) {
#pragma unroll
          for (int l = 1; l < QNB; ++l) sc = ant_contact_add(sc, Ls.get3_lane(l, QF_CV, lane + q));
        }
        t.contact = 0.0005f * sc;
      }
    }
  }
  wave_lds_sync();  // every LDS read of the physics slots is done: the region is staging now
  POB_TS(2);

  // ---- obs rows: assembled in the wave's region (P envs per pass), stored coalesced
  float done = 0.0f;
  t.ga_done_quad = false;
  const bool ga_quad = (KIND == POB_GATHER || KIND == POB_MIXED) && kind == POB_GATHER && S.n_obj <= POB_GA_QUAD_MAX;
  GaQuad gq;
  if (ga_quad && act_lane) {
    // functional mode: the object rows of out.pos are written here (the frozen-row copy
    // below skips them)
    v3 gop[4];
    ga_quad_prefetch<QT>(S, in, r3, nullptr, k, gop);
    ga_quad_objects<QT>(S, gop, r3, bd.x[0], bd.q[0], k, out.pos, gq, t);
  }
#ifdef POB_EXP_TIMING_OBS
  POB_TS(3);  // timing experiment: the GA objects apart from the obs rows
#endif
  // The task tail runs once, before the obs passes (it writes no obs row itself: its entries
  // come back in t.ob0 / t.ob1), except for AntGather with more objects than the quad pass
  // handles, whose readings loop writes the row.
  const bool task_in_pass = kind == POB_GATHER && !ga_quad;
  if (act_lane && k == 0 && out.pos != in.pos) {
    // functional mode: carry the frozen rows over before the task tail moves the TAG target
    // or the AntGather objects (the quad object pass has written those rows already)
    for (int i = POB_NDYN; i < N; ++i) {
      if (!(ga_quad && i >= 11)) cpq<QT>(out.pos, in.pos, r3 + 3 * i, 3);
      cpq<QT>(out.vel, in.vel, r3 + 3 * i, 3);
      cpq<QT>(out.ang, in.ang, r3 + 3 * i, 3);
      cpq<QT>(out.rot, in.rot, r4 + 4 * i, 4);
    }
  }
  if (!task_in_pass && act_lane) {
    if (k == 0) {
      task_dispatch<KIND, QT>(S, kind, in, b, r3, N, bd.x[0], bd.q[0], out.pos, nullptr, flags, L, t);
      done = t.done;
    }
    done = quad_bcast<0>(done);  // the quad's four lanes are active together here
  }
#ifdef POB_EXP_TIMING_OBS
  POB_TS(4);
#endif
  const int P = pass_envs(POB_STAGE_FLOATS, D, 16);
  for (int p0 = 0; p0 < nenv; p0 += P) {
    const int pn = nenv - p0 < P ? nenv - p0 : P;
    if (act_lane && le >= p0 && le < p0 + pn) {
      float *o = stg + (le - p0) * D;
#pragma unroll
      for (int jl = 0; jl < QNJ; ++jl) {
        o[sh + 7 + 2 * k + jl] = jang[jl];
        o[sh + 21 + 2 * k + jl] = jvel[jl];
      }
      // cfrc rows: lane k rows 2k+1, 2k+2 (lane 0 also the torso row); the frozen bodies' zero
      // rows split over the four lanes
      float *oc = o + (29 + sh);
#pragma unroll
      for (int l = 0; l < QNB; ++l) {
        if (l == 0 && k != 0) continue;
        const int g = qbody_global(l, k);
        oc[3 * g] = clip1(cvl[l].x); oc[1 + 3 * g] = clip1(cvl[l].y); oc[2 + 3 * g] = clip1(cvl[l].z);
        oc[3 * N + 3 * g] = clip1(cal[l].x); oc[1 + 3 * N + 3 * g] = clip1(cal[l].y); oc[2 + 3 * N + 3 * g] = clip1(cal[l].z);
      }
      for (int q = 3 * POB_NDYN + k; q < 3 * N; q += 4) { oc[q] = 0.0f; oc[3 * N + q] = 0.0f; }
      if (k == 0) {
        if (sh == 0) { o[0] = bd.x[0].x; o[1] = bd.x[0].y; }
        o[sh + 2] = bd.x[0].z;
        o[sh + 3] = bd.q[0].w; o[sh + 4] = bd.q[0].x; o[sh + 5] = bd.q[0].y; o[sh + 6] = bd.q[0].z;
        o[sh + 15] = bd.v[0].x; o[sh + 16] = bd.v[0].y; o[sh + 17] = bd.v[0].z;
        o[sh + 18] = bd.w[0].x; o[sh + 19] = bd.w[0].y; o[sh + 20] = bd.w[0].z;
      }
      if (ga_quad) ga_quad_scatter(S, gq, k, o + 29 + 6 * N);
      if (task_in_pass) {
        if (k == 0) {
          task_dispatch<KIND, QT>(S, kind, in, b, r3, N, bd.x[0], bd.q[0], out.pos, o, flags, L, t);
          done = t.done;
        }
        done = quad_bcast<0>(done);  // the quad's four lanes are active together here
      } else if (k == 0) {
        task_obs_write(kind, o, 29 + 6 * N, t);
      }
      // AutoResetWrapper: the row of a reset env is first_obs, copied by the env's four lanes
      // after every other write of the row (program order within the wave)
      if ((flags & POB_F_AUTORESET) && done != 0.0f) {
        wave_lds_sync();
        group_copy<4, 4>(o, in.first_obs + (size_t)b * D, D, k);
      }
    }
#ifdef POB_EXP_TIMING_OBS
    if (p0 == 0) POB_TS(5);
#endif
    wave_lds_sync();
    float *dst = out.obs + (size_t)(b_first + p0) * D;
    const int n = pn * D;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {  // 16-B stores, then the tail
      const int n4 = n >> 2;
      for (int i = lane; i < n4; i += 64) reinterpret_cast<float4 *>(dst)[i] = reinterpret_cast<const float4 *>(stg)[i];
      for (int i = 4 * n4 + lane; i < n; i += 64) dst[i] = stg[i];
    } else {
      for (int i = lane; i < n; i += 64) dst[i] = stg[i];
    }
    if (out.obs_masked)  // the observation mask's columns of the same rows (ABI v7)
      store_obs_masked(S, out.obs_masked + (size_t)(b_first + p0) * S.obs_mask_n, stg, pn, D, lane);
    wave_lds_sync();
#ifdef POB_EXP_TIMING_OBS
    if (p0 == 0) POB_TS(6);
#endif
  }

#ifdef POB_EXP_TIMING_OBS
  POB_TS(7);
#else
  POB_TS(3);
#endif
  // ---- dynamic qp rows: computed state, or first_qp when the AutoResetWrapper resets (after
  // the obs passes: stored before them, HH B = 65 536 measured 0.0922 -> 0.0943 ms)
  const bool reset_rows = (flags & POB_F_AUTORESET) && done != 0.0f;
  quad_store_dyn<QT>(in, out, bd, act_lane, k, le, b_first, nenv, N, r3, r4, stg, lane, reset_rows);
#ifdef POB_EXP_TIMING_OBS
  POB_TS(8);
#else
  POB_TS(4);
#endif
  // ---- per-env tail: frozen rows, first_* (the env's lanes), scalar outputs (lane 0)
  if (act_lane) tail_copies<QT, 4, 2>(in, out, flags, reset_rows, b, N, D, r3, r4, k);
  if (act_lane && k == 0) {
    out.reward[b] = t.reward;
    out.done[b] = t.done;
    if (out.steps) out.steps[b] = t.steps;
    if (out.truncation) out.truncation[b] = t.trunc;
    if (out.m0) out.m0[b] = t.m0;
    if (out.m1) out.m1[b] = t.m1;
    if (out.m2) out.m2[b] = t.m2;
    out.rng[2 * b] = t.rng0;
    out.rng[2 * b + 1] = t.rng1;
    write_typed(out, b, t);
  }
  if (out.any_done) {
    const unsigned long long m = __ballot(act_lane && k == 0 && done != 0.0f);
    if (m != 0ull && lane == 0) atomicOr(out.any_done, 1u);
  }
  POB_TS_WRITE();
}

// MODE 2 (the fix-up launch): does any wave of the block carry the overflow mark?  (before
// the block's table staging: a block without one exits at once)
POB_D bool quad_block_marked(const int B, const uint8_t *mark, const int bt0) {
  bool any = false;
  for (int w = 0; w < (int)blockDim.x / 64; ++w) {
    const int bf = (bt0 + 64 * w) >> 2;
    if (bf < B) any = any | (mark[bf] != 0);
  }
  return any;
}
template <int KIND, typename QT, int MODE = 0>
__global__ __launch_bounds__(256, POB_QUAD_MIN_WAVES) void k_step_quad(const void *sysp, const int B,
                                                                       const StatePtrs in,
                                                                       const float *__restrict__ act,
                                                                       const StatePtrs out, const uint32_t flags,
                                                                       const int L) {
  __shared__ float lds[QL_FLOATS * 256];
  __shared__ __attribute__((aligned(16))) float legtab[POB_TAB_FLOATS];
  if (MODE == 2 && !quad_block_marked(B, out.ovf_mark, (int)(blockIdx.x * blockDim.x)))
    return;
  stage_leg_table((csys_t *)(size_t)sysp, legtab);
  step_quad_body<KIND, QT, false, MODE>((csys_t *)(size_t)sysp, B, in, act, out, flags, L,
                                        (int)(blockIdx.x * blockDim.x + threadIdx.x), lds, legtab);
}

// AntGather at most three waves per SIMD (B <= 3 x 16 x SIMDs): the same kernel with the
// register budget of three waves -- at four its object / sensor / 211-wide obs passes spill
// (128 B of scratch per lane), and three fit the whole launch anyway (B = 32 768: 0.0998 ->
// 0.0947 ms, interleaved A/B, profiles/r2t)
template <typename QT>
__global__ __launch_bounds__(256, 3) void k_step_quad_ga3(const void *sysp, const int B, const StatePtrs in,
                                                          const float *__restrict__ act, const StatePtrs out,
                                                          const uint32_t flags, const int L) {
  __shared__ float lds[QL_FLOATS * 256];
  __shared__ __attribute__((aligned(16))) float legtab[POB_TAB_FLOATS];
  stage_leg_table((csys_t *)(size_t)sysp, legtab);
  step_quad_body<POB_GATHER, QT>((csys_t *)(size_t)sysp, B, in, act, out, flags, L,
                                 (int)(blockIdx.x * blockDim.x + threadIdx.x), lds, legtab);
}

// The same fused step with the legacy spring dynamics (pob_params.legacy_spring; pob_quad.h
// qlegacy_substep) -- a kernel of its own so the PBD kernels keep their register allocation.
template <int KIND, typename QT>
__global__ __launch_bounds__(256) void k_step_legacy(const void *sysp, const int B, const StatePtrs in,
                                                     const float *__restrict__ act, const StatePtrs out,
                                                     const uint32_t flags, const int L) {
  __shared__ float lds[QL_FLOATS * 256];
  __shared__ __attribute__((aligned(16))) float legtab[POB_TAB_FLOATS];
  stage_leg_table((csys_t *)(size_t)sysp, legtab);
  step_quad_body<KIND, QT, true>((csys_t *)(size_t)sysp, B, in, act, out, flags, L,
                                 (int)(blockIdx.x * blockDim.x + threadIdx.x), lds, legtab);
}

// Mixed launch: segment k owns blocks [blk0_k, blk0_{k+1}); the segment index is
// block-uniform, so every selected table pointer / state pointer stays scalar.
struct MixSeg {
  const void *sysp;
  const float *act;
  StatePtrs in, out;
  int B, blk0;
};
struct MixArgs {
  MixSeg s[POB_MIX_MAX];
  int n;
};
static_assert(POB_MIX_MAX == 4, "pick_state selects among 4 segments");

// force a (block-uniform) pointer into SGPRs: the table pointer feeds scalar loads
POB_D const void *uniform_ptr(const void *p) {
  const uint64_t v = (uint64_t)(size_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const void *)(size_t)(((uint64_t)hi << 32) | lo);
}

#ifndef POB_MIXED_MIN_WAVES
#define POB_MIXED_MIN_WAVES 3  // config 5 runs 2 waves per SIMD: 170 VGPRs, no spills (128: 144 B of scratch, +6 %)
#endif
template <typename QT, int MODE = 0>
__global__ __launch_bounds__(256, POB_MIXED_MIN_WAVES) void k_step_mixed(const MixArgs A, const uint32_t flags,
                                                                        const int L) {
  __shared__ float lds[QL_FLOATS * 256];
  __shared__ __attribute__((aligned(16))) float legtab[POB_TAB_FLOATS];
  const int bx = (int)blockIdx.x;
  int seg = 0;
#pragma unroll
  for (int k = 1; k < POB_MIX_MAX; ++k)
    if (k < A.n && bx >= A.s[k].blk0) seg = k;
  seg = __builtin_amdgcn_readfirstlane(seg);
#define POB_PICK(f) (seg == 0 ? A.s[0].f : (seg == 1 ? A.s[1].f : (seg == 2 ? A.s[2].f : A.s[3].f)))
  StatePtrs in, out;
#define POB_SEL(f) in.f = A.s[0].in.f; out.f = A.s[0].out.f;
  POB_STATE_FIELDS(POB_SEL)
#undef POB_SEL
#pragma unroll
  for (int k = 1; k < POB_MIX_MAX; ++k) {
    if (seg == k) {
#define POB_SEL(f) in.f = A.s[k].in.f; out.f = A.s[k].out.f;
      POB_STATE_FIELDS(POB_SEL)
#undef POB_SEL
    }
  }
  const void *sysp = uniform_ptr(POB_PICK(sysp));
  const float *act = POB_PICK(act);
  const int B = POB_PICK(B), blk0 = POB_PICK(blk0);
#undef POB_PICK
  if (MODE == 2 && !quad_block_marked(B, out.ovf_mark, (bx - blk0) * 256))
    return;
  stage_leg_table((csys_t *)(size_t)sysp, legtab);
  step_quad_body<POB_MIXED, QT, false, MODE>((csys_t *)(size_t)sysp, B, in, act, out, flags, L,
                                (bx - blk0) * 256 + (int)threadIdx.x, lds, legtab);
}

// ------------------------------------------------------------------ step, lane octets
// The same fused step with EIGHT lanes per env (pob_octet.h) for small batches: one wave =
// 8 envs, one wave per block.  Lane m of an env: A_m (m < 4: hip joint m, torso + Aux) or
// B_(7-m) (m >= 4: knee joint, Aux + lower leg).  Lane A_0 runs the per-env POMDP tail.
// (8 AntGather obs rows of the default 8 + 8 objects, 8 x 211 floats, fit: one obs pass)
#define POB_OSTAGE_FLOATS (27 * 64)
static_assert(POB_OSTAGE_FLOATS >= OL_FLOATS * 64, "the octet staging region holds the lanes' LDS slots");
template <int KIND, typename QT, bool GACC>
__global__ __launch_bounds__(64) void k_step_oct(const void *sysp, const int B, const StatePtrs in,
                                                 const float *__restrict__ act, const StatePtrs out,
                                                 const uint32_t flags, const int L) {
  static_assert(KIND != POB_MIXED, "the eight-lane kernel runs one env kind per launch");
  POB_TS_DECL();  // timing experiment only (POB_EXP_TIMING)
  POB_TS(0);
  __shared__ float stg[POB_OSTAGE_FLOATS];
  __shared__ __attribute__((aligned(16))) float otab[OT_TAB_FLOATS + HW_FLOATS];
#ifdef POB_FC_LDS
  __shared__ __attribute__((aligned(16))) float ofc[POB_FC_TAB_FLOATS];  // the walls' face constants
#endif
  csys_t *Sp = (csys_t *)(size_t)sysp;
  csys_t &S = *Sp;
  __shared__ float ocst[OCS_FLOATS * 64 + (oct_pool(KIND) ? 6 * OPOOL_N : 0)];  // the lanes' stores (then the wave's contact pool)
  const int lane = (int)threadIdx.x;
  float *const ocs = ocst + lane;  // the lane's wall-contact store (pob_octet.h)
  const int m = lane & 7;
  const bool isA = m < 4;
  const int k = isA ? m : 7 - m;              // the leg
  const int jown = isA ? 2 * k : 2 * k + 1;    // the lane's joint
  const int g0 = isA ? 0 : 2 * k + 1, g1 = isA ? 2 * k + 1 : 2 * k + 2;  // its slots' bodies
  const Lds Ls{stg, 64, lane};
  const int b_first = (int)blockIdx.x * 8;
  const int b = b_first + (lane >> 3);
  const int nenv = B - b_first < 8 ? B - b_first : 8;
  const int le = lane >> 3;
  const bool act_lane = b < B;
  const int N = n_bodies<KIND>(S), D = obs_dim<KIND>(S);
  constexpr int sh = obs_shift(KIND);
  // the physics runs on all 64 lanes (the wave walk's DPP / bpermute rounds need every lane):
  // the lanes past the batch in its last wave replay env B - 1 and store nothing
  const int bl = act_lane ? b : B - 1, lel = bl - b_first;
  const size_t r3 = (size_t)bl * N * 3, r4 = (size_t)bl * N * 4;
  const bool lane0 = m == 0;  // A_0: the env's POMDP tail

  // ---- state load: coalesced loads of the 8 envs' rows into LDS (pairs of arrays), then
  // every lane picks its two bodies; per-lane loads when the qp pointers are not aligned
  OBody bd;
  v3 gop[4];  // AntGather: this lane's objects' input positions (A lanes)
  bool gop_ok = false;
  constexpr int NMAX = KIND == POB_HEAVENHELL ? 14 : (KIND == POB_TAG ? 12 : (KIND == POB_ANT ? 10 : POB_MAXB));
  if ((flags & POB_F_STAGED) && 8 * N * 7 <= POB_OSTAGE_FLOATS) {
    gop_ok = true;
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int c0 = 3, c1 = pr == 0 ? 4 : 3;
      const int n0 = nenv * N * c0, n1 = nenv * N * c1;
      stage_load<QT>(pr == 0 ? in.pos : in.vel, (size_t)b_first * N * c0, n0, stg, lane);
      stage_load<QT>(pr == 0 ? in.rot : in.ang, (size_t)b_first * N * c1, n1, stg + n0, lane);
      wave_lds_sync();
      if (KIND == POB_GATHER && pr == 0 && act_lane && isA && S.n_obj <= POB_GA_QUAD_MAX)
        ga_quad_prefetch<QT>(S, in, r3, stg + le * N * 3, k, gop);
      {
#pragma unroll
        for (int sl = 0; sl < ONB; ++sl) {
          const int g = sl == 0 ? g0 : g1;
          const float *s0 = stg + (lel * N + g) * c0, *s1 = stg + n0 + (lel * N + g) * c1;
          if (pr == 0) {
            bd.x[sl] = V(s0[0], s0[1], s0[2]);
            bd.q[sl].w = s1[0]; bd.q[sl].x = s1[1]; bd.q[sl].y = s1[2]; bd.q[sl].z = s1[3];
          } else {
            bd.v[sl] = V(s0[0], s0[1], s0[2]);
            bd.w[sl] = V(s1[0], s1[1], s1[2]);
          }
        }
      }
      wave_lds_sync();
    }
  } else {
#pragma unroll
    for (int sl = 0; sl < ONB; ++sl) {
      const int g = sl == 0 ? g0 : g1;
      bd.x[sl] = ld3<QT>(in.pos, r3 + 3 * g);
      bd.q[sl] = ld4<QT>(in.rot, r4 + 4 * g);
      bd.v[sl] = ld3<QT>(in.vel, r3 + 3 * g);
      bd.w[sl] = ld3<QT>(in.ang, r3 + 3 * g);
    }
    // AntGather: the A lanes' object positions ride along with the state loads (one round
    // trip; the registers are free at the octet kernel's occupancy)
    if (KIND == POB_GATHER && act_lane && isA && S.n_obj <= POB_GA_QUAD_MAX) {
      ga_quad_prefetch<QT>(S, in, r3, nullptr, k, gop);
      gop_ok = true;
    }
  }
  (void)NMAX;
  // the action, loaded with the state (its round trip overlaps the table loads)
  const float a_in = act[(size_t)bl * POB_NJ + jown];
  // the role table, staged after the state loads are issued (both in flight together; the
  // block is one wave, so an LDS wait orders the table writes before its reads)
  {
    const __attribute__((address_space(4))) float *src = &Sp->oct[0][0];
    stage_table<8 * OT_FLOATS>(otab, src, (int)threadIdx.x, 64);
    const __attribute__((address_space(4))) float *wsrc = &Sp->wall_row[0][0];
    stage_table<POB_MAXW * POB_WALL_FLOATS>(otab + 8 * OT_FLOATS, wsrc, (int)threadIdx.x, 64);
    hwalls_stage(S, otab + OT_TAB_FLOATS, lane);  // the walls' broadphase boxes, z extent, scalars
#ifdef POB_FC_LDS
    stage_table<POB_FC_TAB_FLOATS>(ofc, &Sp->face_c[0][0][0], (int)threadIdx.x, 64);
#endif
    wave_lds_sync();
  }
  float OT[OT_FLOATS];  // the lane's role row, in registers (constant indices only)
#pragma unroll
  for (int i = 0; i < OT_FLOATS; ++i) OT[i] = otab[(isA ? k : 4 + k) * OT_FLOATS + i];
  const float *WT = otab + 8 * OT_FLOATS;
  constexpr int OMW = hex_max_walls(KIND);
  HWalls<OMW> HW;  // the walls in VGPRs (LDS loads: the compiler keeps them per lane)
#ifdef POB_FC_LDS
  hwalls_load(otab + OT_TAB_FLOATS, HW, ofc);
#else
  hwalls_load(otab + OT_TAB_FLOATS, HW, pob_face_table(S));
#endif
  POB_TS(1);

  // ---- physics (10 substeps in registers)
  float jang = 0.0f, jvel = 0.0f;
  v3 cvl[ONB], cal[ONB];
  TaskOut t;
  t.tp_ok = false;
  if (act_lane && lane0) {
    // the task inputs, loaded before the physics so that their round trip overlaps it (the
    // done test that zeroes steps waits for its load, so it runs after the physics)
    t.steps = in.steps ? in.steps[b] : 0.0f;
    t.pdone = in.done[b];
    t.m0 = in.m0 ? in.m0[b] : 0.0f; t.m1 = in.m1 ? in.m1[b] : 0.0f; t.m2 = in.m2 ? in.m2[b] : 0.0f;
    t.rng0 = in.rng[2 * b]; t.rng1 = in.rng[2 * b + 1];
    task_prefetch<KIND, QT>(in, r3, t);
  }
  {
    const float xb = bd.x[0].x;
    const float a = a_in;
#pragma unroll
    for (int sl = 0; sl < ONB; ++sl) { cvl[sl] = V(0.0f, 0.0f, 0.0f); cal[sl] = V(0.0f, 0.0f, 0.0f); }
    const int iters = Sp->substeps / 2;
#if defined(POB_EXP_NO_COLLIDE)
    GuardBranch gb;
    for (int it = 0; it < 2 * iters; ++it) opbd_substep<OMW, oct_pool(KIND)>(gb, Sp, OT, WT, HW, isA, bd, a, cvl, cal, false, ocs);  // timing experiment only
#elif defined(POB_EXP_NO_PHYSICS)
    GuardBranch gb;
    for (int it = 0; it < 0 * iters; ++it) opbd_substep<OMW, oct_pool(KIND)>(gb, Sp, OT, WT, HW, isA, bd, a, cvl, cal, false, ocs);  // timing experiment only
#else
#ifdef POB_EXP_TIMING_SUB  // timing experiment only: phase durations into stamps 5..12
#define OCT_SUBSTEPS(G)                                                                       \
  _Pragma("nounroll") for (int it = 0; it < 2 * iters; ++it)                                 \
    opbd_substep<OMW, oct_pool(KIND)>(G, Sp, OT, WT, HW, isA, bd, a, cvl, cal, (it & 1) != 0, ocs, pob_ts + 5);
#else
// At two waves per SIMD (the branch-guard build, B > 8 x SIMDs) the four-lane kernel's falling
// issue priority keeps a SIMD's waves together (k_step_quad): HH B = 16 384 -2.2 %, TAG -3 %,
// GA -0.5 % (profiles/r3t/oct_prio_ab.txt); a lone wave per SIMD has no one to yield to.
#define OCT_SUBSTEPS(G)                                                                       \
  _Pragma("nounroll") for (int it = 0; it < 2 * iters; ++it) {                               \
    if (!GACC && POB_OCT_PRIO) {                                                               \
      const int lvl_ = (it * 4) / (2 * iters);                                                 \
      if (lvl_ == 0) __builtin_amdgcn_s_setprio(3);                                            \
      else if (lvl_ == 1) __builtin_amdgcn_s_setprio(2);                                       \
      else if (lvl_ == 2) __builtin_amdgcn_s_setprio(1);                                       \
      else __builtin_amdgcn_s_setprio(0);                                                      \
    }                                                                                          \
    opbd_substep<OMW, oct_pool(KIND)>(G, Sp, OT, WT, HW, isA, bd, a, cvl, cal, (it & 1) != 0, ocs);                \
  }
#endif
    if constexpr (!GACC) {
      GuardBranch gb;
      OCT_SUBSTEPS(gb)
    } else {
      // one wave per SIMD (GACC): the substeps without guard branches (GuardAcc, as in the
      // sixteen-lane kernel); a wave any of whose lanes met an operand outside the fast forms'
      // range reruns them from the loaded state with the branch guards
      const OBody b0 = bd;
      GuardAcc ga;
      OCT_SUBSTEPS(ga)
      if (__builtin_expect(__any(ga.bad()), 0)) {
        bd = b0;
#pragma unroll
        for (int sl = 0; sl < ONB; ++sl) { cvl[sl] = V(0.0f, 0.0f, 0.0f); cal[sl] = V(0.0f, 0.0f, 0.0f); }
        GuardBranch gb;
        OCT_SUBSTEPS(gb)
      }
    }
#undef OCT_SUBSTEPS
#endif
    {  // joint angle / velocity obs of the lane's joint (a3)
      const v3 ap = qrot(OTV(OT, OT_AXIS), bd.q[0]);
      const v3 ref = OTV(OT, OT_REF);
      const v3 fp = qrot(ref, bd.q[0]), fc = qrot(ref, bd.q[1]);
      jang = pob_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
      jvel = vdot(vsub(bd.w[1], bd.w[0]), ap);
    }
    // the lower legs' / auxes' contact velocity sums for the stock ant's contact cost
#pragma unroll
    for (int sl = 0; sl < ONB; ++sl) Ls.set3(3 * sl, cvl[sl]);
    wave_lds_sync();
    if (act_lane && lane0) {
      if ((flags & (POB_F_AUTORESET | POB_F_ZERO_STEPS_ON_DONE)) && t.pdone != 0.0f) t.steps = 0.0f;
      t.xb = xb; t.ctrl = 0.0f; t.contact = 0.0f;
      if (KIND == POB_ANT) {
        // full action row; contact rows 0..8 = torso, then Aux k (lane A_k slot 1) and lower
        // leg k (lane B_k slot 1) for k = 0..3
        t.ctrl = ant_ctrl_cost(act + (size_t)b * POB_NJ);
        float sc = ant_contact_add(0.0f, cvl[0]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sc = ant_contact_add(sc, Ls.get3_lane(3, lane + q));
          sc = ant_contact_add(sc, Ls.get3_lane(3, lane + 7 - q));
        }
        t.contact = 0.0005f * sc;
      }
    }
  }
  wave_lds_sync();  // every LDS read of the physics slots is done: the region is staging now
  POB_TS(2);

  // ---- obs rows: assembled in the wave's region (P envs per pass), stored coalesced
  float done = 0.0f;
  t.ga_done_quad = false;
  const bool ga_quad = KIND == POB_GATHER && S.n_obj <= POB_GA_QUAD_MAX;
  GaQuad gq;
  if (ga_quad && act_lane && isA) {
    if (!gop_ok) ga_quad_prefetch<QT>(S, in, r3, nullptr, k, gop);
    ga_quad_objects<QT>(S, gop, r3, bd.x[0], bd.q[0], k, out.pos, gq, t);
  }
#ifdef POB_EXP_TIMING_OBS
  POB_TS(3);  // timing experiment: the GA objects apart from the obs rows
#endif
  const int P = pass_envs(POB_OSTAGE_FLOATS, D, 8);
  for (int p0 = 0; p0 < nenv; p0 += P) {
    const int pn = nenv - p0 < P ? nenv - p0 : P;
    if (act_lane && le >= p0 && le < p0 + pn) {
      float *o = stg + (le - p0) * D;
      o[sh + 7 + jown] = jang;
      o[sh + 21 + jown] = jvel;
      // cfrc rows: A_0 the torso, A_k Aux k (slot 1), B_k lower leg k (slot 1); the frozen
      // bodies' zero rows split over the eight lanes
      float *oc = o + (29 + sh);
      if (lane0) {
        oc[0] = clip1(cvl[0].x); oc[1] = clip1(cvl[0].y); oc[2] = clip1(cvl[0].z);
        oc[3 * N] = clip1(cal[0].x); oc[1 + 3 * N] = clip1(cal[0].y); oc[2 + 3 * N] = clip1(cal[0].z);
      }
      oc[3 * g1] = clip1(cvl[1].x); oc[1 + 3 * g1] = clip1(cvl[1].y); oc[2 + 3 * g1] = clip1(cvl[1].z);
      oc[3 * N + 3 * g1] = clip1(cal[1].x); oc[1 + 3 * N + 3 * g1] = clip1(cal[1].y);
      oc[2 + 3 * N + 3 * g1] = clip1(cal[1].z);
      for (int q = 3 * POB_NDYN + m; q < 3 * N; q += 8) { oc[q] = 0.0f; oc[3 * N + q] = 0.0f; }
      if (lane0) {
        if (sh == 0) { o[0] = bd.x[0].x; o[1] = bd.x[0].y; }
        o[sh + 2] = bd.x[0].z;
        o[sh + 3] = bd.q[0].w; o[sh + 4] = bd.q[0].x; o[sh + 5] = bd.q[0].y; o[sh + 6] = bd.q[0].z;
        o[sh + 15] = bd.v[0].x; o[sh + 16] = bd.v[0].y; o[sh + 17] = bd.v[0].z;
        o[sh + 18] = bd.w[0].x; o[sh + 19] = bd.w[0].y; o[sh + 20] = bd.w[0].z;
        if (out.pos != in.pos) {  // functional mode: carry the frozen rows over
          for (int i = POB_NDYN; i < N; ++i) {
            if (!(ga_quad && i >= 11)) cpq<QT>(out.pos, in.pos, r3 + 3 * i, 3);
            cpq<QT>(out.vel, in.vel, r3 + 3 * i, 3);
            cpq<QT>(out.ang, in.ang, r3 + 3 * i, 3);
            cpq<QT>(out.rot, in.rot, r4 + 4 * i, 4);
          }
        }
      }
      if (ga_quad && isA) ga_quad_scatter(S, gq, k, o + 29 + 6 * N);
      if (lane0) {
        task_step<KIND, QT>(S, in, b, r3, N, bd.x[0], bd.q[0], out.pos, o, flags, L, t);
        task_obs_write(KIND, o, 29 + 6 * N, t);
        done = t.done;
      }
      {  // the env's done to all eight lanes: A quad from A_0, B quad via A_0 -> B_0 (lane 7)
        const float d1 = quad_bcast<0>(done);
        const float d2 = quad_bcast<3>(oct_swap(d1));
        done = isA ? d1 : d2;
      }
      // AutoResetWrapper: the row of a reset env is first_obs, copied by the env's eight lanes
      // after every other write of the row
      if ((flags & POB_F_AUTORESET) && done != 0.0f) {
        wave_lds_sync();
        group_copy<8, 4>(o, in.first_obs + (size_t)b * D, D, m);
      }
    }
    wave_lds_sync();
    float *dst = out.obs + (size_t)(b_first + p0) * D;
    const int n = pn * D;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
      const int n4 = n >> 2;
      for (int i = lane; i < n4; i += 64) reinterpret_cast<float4 *>(dst)[i] = reinterpret_cast<const float4 *>(stg)[i];
      for (int i = 4 * n4 + lane; i < n; i += 64) dst[i] = stg[i];
    } else {
      for (int i = lane; i < n; i += 64) dst[i] = stg[i];
    }
    if (out.obs_masked)  // the observation mask's columns of the same rows (ABI v7)
      store_obs_masked(S, out.obs_masked + (size_t)(b_first + p0) * S.obs_mask_n, stg, pn, D, lane);
    wave_lds_sync();
  }

#ifdef POB_EXP_TIMING_OBS
  POB_TS(4);
#else
  POB_TS(3);
#endif
  // ---- dynamic qp rows: computed state, or first_qp when the AutoResetWrapper resets
  const bool reset_rows = (flags & POB_F_AUTORESET) && done != 0.0f;
#pragma unroll
  for (int arr = 0; arr < 4; ++arr) {
    const int c = arr == 1 ? 4 : 3;
    if (act_lane) {
#pragma unroll
      for (int sl = 0; sl < ONB; ++sl) {
        if (sl == 0 && !lane0) continue;  // slot 0: the torso (A_0) or an Aux replica
        const int g = sl == 0 ? g0 : g1;
        float *o = stg + (le * POB_NDYN + g) * c;
        if (reset_rows) {
          const float *F = arr == 0 ? in.first_pos : (arr == 1 ? in.first_rot : (arr == 2 ? in.first_vel : in.first_ang));
          const size_t src = (arr == 1 ? r4 : r3) + (size_t)g * c;
          for (int q = 0; q < c; ++q) o[q] = Q<QT>::ld(F, src + q);
        } else if (arr == 0) { o[0] = bd.x[sl].x; o[1] = bd.x[sl].y; o[2] = bd.x[sl].z; }
        else if (arr == 1) { o[0] = bd.q[sl].w; o[1] = bd.q[sl].x; o[2] = bd.q[sl].y; o[3] = bd.q[sl].z; }
        else if (arr == 2) { o[0] = bd.v[sl].x; o[1] = bd.v[sl].y; o[2] = bd.v[sl].z; }
        else { o[0] = bd.w[sl].x; o[1] = bd.w[sl].y; o[2] = bd.w[sl].z; }
      }
    }
    wave_lds_sync();
    if (arr == 1) stage_store_dyn<QT, 4>(out.rot, (size_t)b_first * N * 4, N, nenv, stg, lane);
    else stage_store_dyn<QT, 3>(arr == 0 ? out.pos : (arr == 2 ? out.vel : out.ang), (size_t)b_first * N * 3, N, nenv,
                                stg, lane);
    wave_lds_sync();
  }

#ifndef POB_EXP_TIMING_OBS
  POB_TS(4);
#endif
  // ---- per-env tail: frozen rows, first_* (the env's lanes), scalar outputs (A_0)
  if (act_lane) tail_copies<QT, 8>(in, out, flags, reset_rows, b, N, D, r3, r4, m);
  if (act_lane && lane0) {
    out.reward[b] = t.reward;
    out.done[b] = t.done;
    if (out.steps) out.steps[b] = t.steps;
    if (out.truncation) out.truncation[b] = t.trunc;
    if (out.m0) out.m0[b] = t.m0;
    if (out.m1) out.m1[b] = t.m1;
    if (out.m2) out.m2[b] = t.m2;
    out.rng[2 * b] = t.rng0;
    out.rng[2 * b + 1] = t.rng1;
    write_typed(out, b, t);
  }
  if (out.any_done) {
    const unsigned long long mk = __ballot(act_lane && lane0 && done != 0.0f);
    if (mk != 0ull && lane == 0) atomicOr(out.any_done, 1u);
  }
  POB_TS_WRITE();
}

// ----------------------------------------------------------- step, sixteen lanes per env
// The same fused step with SIXTEEN lanes per env (pob_hexa.h): one wave = 4 envs, one wave per
// block; lane r of an env owns one body and one side of one joint (P_hip_r / C_hip_(7-r) /
// P_knee_(r-8) / C_knee_(15-r)).  Lane 0 (P_hip_0, the torso) runs the per-env POMDP tail.
#define POB_HSTAGE_FLOATS (OL_FLOATS * 64)
static_assert(POB_HSTAGE_FLOATS >= HCS_FLOATS * 64, "the sixteen-lane staging region holds the wall-contact store");
#ifndef POB_HEX_MINW  // experiment: the register budget of this many waves per SIMD
#define POB_HEX_MINW 1
#endif
// PRIO: the falling issue priority over the substeps (POB_HEX_PRIO), launched from two waves
// per SIMD on (at one wave per SIMD it only costs: HH B = 4 096 0.0563 -> 0.0574 ms, profiles/r7ac)
template <int KIND, typename QT, bool GACC, bool PRIO = false>
__global__ __launch_bounds__(64, POB_HEX_MINW) void k_step_hex(const void *sysp, const int B, const StatePtrs in,
                                                 const float *__restrict__ act, const StatePtrs out,
                                                 const uint32_t flags, const int L) {
  static_assert(KIND != POB_MIXED, "the sixteen-lane kernel runs one env kind per launch");
  POB_TS_DECL();  // timing experiment only (POB_EXP_TIMING)
  POB_TS(0);
  __shared__ float stg[POB_HSTAGE_FLOATS];
  __shared__ __attribute__((aligned(16))) float htab[HT_TAB_FLOATS + HW_FLOATS];
#ifdef POB_FC_LDS
  __shared__ __attribute__((aligned(16))) float hfc[POB_FC_TAB_FLOATS];  // the walls' face constants
#endif
  csys_t *Sp = (csys_t *)(size_t)sysp;
  csys_t &S = *Sp;
  const int lane = (int)threadIdx.x;
#if POB_HEX_POOL
  __shared__ float hpool[6 * HPOOL_N];
  float *const hcs = hpool;  // the wave's wall-contact pool (pob_hexa.h POB_HEX_POOL)
#else
  float *const hcs = stg + lane;  // the lane's wall-contact store during the substeps (pob_hexa.h)
#endif
  const int r = lane & 15;
  const bool hip = r < 8, isP = r < 4 || (r >= 8 && r < 12);
  const int k = r < 4 ? r : (r < 8 ? 7 - r : (r < 12 ? r - 8 : 15 - r));  // the leg
  const int jown = hip ? 2 * k : 2 * k + 1;                                 // the lane's joint
  const int g = hip ? (isP ? 0 : 2 * k + 1) : (isP ? 2 * k + 1 : 2 * k + 2);  // its body
  // the lane that writes the body's rows: the torso's lane 0, an Aux's child side, a lower leg
  const bool canon = r == 0 || (hip && !isP) || (!hip && !isP);
  const Lds Ls{stg, 64, lane};
  const int b_first = (int)blockIdx.x * 4;
  const int le = lane >> 4;
  const int b = b_first + le;
  const int nenv = B - b_first < 4 ? B - b_first : 4;
  const bool act_lane = b < B;
  const int N = n_bodies<KIND>(S), D = obs_dim<KIND>(S);
  constexpr int sh = obs_shift(KIND);
  // the physics runs on all 64 lanes (as in the eight-lane kernel): the lanes past the batch
  // in its last wave replay env B - 1 and store nothing
  const int bl = act_lane ? b : B - 1, lel = bl - b_first;
  const size_t r3 = (size_t)bl * N * 3, r4 = (size_t)bl * N * 4;
  const bool lane0 = r == 0;  // P_hip_0: the env's POMDP tail

  // ---- state load: coalesced loads of the 4 envs' rows into LDS (pairs of arrays), then
  // every lane picks its body; per-lane loads when the qp pointers are not aligned
  HBody bd;
  v3 gop[4];  // AntGather: this lane's objects' input positions (torso lanes)
  bool gop_ok = false;
  if ((flags & POB_F_STAGED) && 4 * N * 13 <= POB_HSTAGE_FLOATS) {
    gop_ok = true;
    // all four arrays in one round trip (pos | rot | vel | ang of the wave's envs)
    const int n3 = nenv * N * 3, n4 = nenv * N * 4;
    stage_load<QT>(in.pos, (size_t)b_first * N * 3, n3, stg, lane);
    stage_load<QT>(in.rot, (size_t)b_first * N * 4, n4, stg + n3, lane);
    stage_load<QT>(in.vel, (size_t)b_first * N * 3, n3, stg + n3 + n4, lane);
    stage_load<QT>(in.ang, (size_t)b_first * N * 3, n3, stg + 2 * n3 + n4, lane);
    wave_lds_sync();
    if (KIND == POB_GATHER && act_lane && r < 4 && S.n_obj <= POB_GA_QUAD_MAX)
      ga_quad_prefetch<QT>(S, in, r3, stg + le * N * 3, r, gop);
    {
      const float *sx = stg + (lel * N + g) * 3, *sq = stg + n3 + (lel * N + g) * 4;
      const float *sv = stg + n3 + n4 + (lel * N + g) * 3, *sw = stg + 2 * n3 + n4 + (lel * N + g) * 3;
      bd.x = V(sx[0], sx[1], sx[2]);
      bd.q.w = sq[0]; bd.q.x = sq[1]; bd.q.y = sq[2]; bd.q.z = sq[3];
      bd.v = V(sv[0], sv[1], sv[2]);
      bd.w = V(sw[0], sw[1], sw[2]);
    }
    wave_lds_sync();
  } else {
    bd.x = ld3<QT>(in.pos, r3 + 3 * g);
    bd.q = ld4<QT>(in.rot, r4 + 4 * g);
    bd.v = ld3<QT>(in.vel, r3 + 3 * g);
    bd.w = ld3<QT>(in.ang, r3 + 3 * g);
    // AntGather: lanes 0..3's object positions ride along with the state loads
    if (KIND == POB_GATHER && act_lane && r < 4 && S.n_obj <= POB_GA_QUAD_MAX) {
      ga_quad_prefetch<QT>(S, in, r3, nullptr, r, gop);
      gop_ok = true;
    }
  }
  // the action, loaded with the state (its round trip overlaps the table loads)
  const float a_in = act[(size_t)bl * POB_NJ + jown];
  constexpr int HMW = hex_max_walls(KIND);
  // the role table, staged after the state loads are issued (as in the eight-lane kernel)
  {
    const __attribute__((address_space(4))) float *src = &Sp->hex[0][0];
    stage_table<16 * HT_FLOATS>(htab, src, (int)threadIdx.x, 64);
    const __attribute__((address_space(4))) float *wsrc = &Sp->wall_row[0][0];
    stage_table<POB_MAXW * POB_WALL_FLOATS>(htab + 16 * HT_FLOATS, wsrc, (int)threadIdx.x, 64);
    hwalls_stage(S, htab + HT_TAB_FLOATS, lane);  // the walls' broadphase boxes, z extent, scalars
#ifdef POB_FC_LDS
    stage_table<POB_FC_TAB_FLOATS>(hfc, &Sp->face_c[0][0][0], (int)threadIdx.x, 64);
#endif
    wave_lds_sync();
  }
  float HT[HT_FLOATS];  // the lane's role row, in registers (constant indices only)
#pragma unroll
  for (int i = 0; i < HT_FLOATS; ++i) HT[i] = htab[r * HT_FLOATS + i];
  const float *WT = htab + 16 * HT_FLOATS;
  HWalls<HMW> HW;  // the walls in VGPRs (LDS loads: the compiler keeps them per lane)
#ifdef POB_FC_LDS
  hwalls_load(htab + HT_TAB_FLOATS, HW, hfc);
#else
  hwalls_load(htab + HT_TAB_FLOATS, HW, pob_face_table(S));
#endif
  POB_TS(1);

  // ---- physics (10 substeps in registers)
  float jang = 0.0f, jvel = 0.0f;
  v3 cvl = V(0.0f, 0.0f, 0.0f), cal = cvl;
  TaskOut t;
  t.tp_ok = false;
  if (act_lane && lane0) {
    // the task inputs, loaded before the physics so that their round trip overlaps it (the
    // done test that zeroes steps waits for its load, so it runs after the physics)
    t.steps = in.steps ? in.steps[b] : 0.0f;
    t.pdone = in.done[b];
    t.m0 = in.m0 ? in.m0[b] : 0.0f; t.m1 = in.m1 ? in.m1[b] : 0.0f; t.m2 = in.m2 ? in.m2[b] : 0.0f;
    t.rng0 = in.rng[2 * b]; t.rng1 = in.rng[2 * b + 1];
    task_prefetch<KIND, QT>(in, r3, t);
  }
  {
    const float xb = bd.x.x;
    const float a = a_in;
    const int iters = Sp->substeps / 2;
#if defined(POB_EXP_NO_COLLIDE)
    GuardBranch gb;
    for (int it = 0; it < 2 * iters; ++it) hpbd_substep<hex_max_walls(KIND)>(gb, S, HT, WT, HW, bd, a, cvl, cal, false, hcs);  // timing experiment only
#elif defined(POB_EXP_NO_PHYSICS)
    GuardBranch gb;
    for (int it = 0; it < 0 * iters; ++it) hpbd_substep<hex_max_walls(KIND)>(gb, S, HT, WT, HW, bd, a, cvl, cal, false, hcs);  // timing experiment only
#else
#ifdef POB_HEX_UNROLL2
#define HEX_SUBSTEPS(G)                                                                       \
  _Pragma("nounroll") for (int it = 0; it < iters; ++it) {                                   \
    hpbd_substep<hex_max_walls(KIND)>(G, S, HT, WT, HW, bd, a, cvl, cal, false, hcs);                  \
    hpbd_substep<hex_max_walls(KIND)>(G, S, HT, WT, HW, bd, a, cvl, cal, true, hcs);                   \
  }
#elif defined(POB_EXP_TIMING_SUB)  // timing experiment only: phase durations into stamps 5..12
#define HEX_SUBSTEPS(G)                                                                       \
  _Pragma("nounroll") for (int it = 0; it < 2 * iters; ++it)                                 \
    hpbd_substep<hex_max_walls(KIND)>(G, S, HT, WT, HW, bd, a, cvl, cal, (it & 1) != 0, hcs, pob_ts + 5);
#else
#define HEX_SUBSTEPS(G)                                                                       \
  _Pragma("nounroll") for (int it = 0; it < 2 * iters; ++it) {                               \
    if constexpr (PRIO) {                                                                    \
      const int lvl_ = (it * 4) / (2 * iters);                                               \
      if (lvl_ == 0) __builtin_amdgcn_s_setprio(3);                                          \
      else if (lvl_ == 1) __builtin_amdgcn_s_setprio(2);                                     \
      else if (lvl_ == 2) __builtin_amdgcn_s_setprio(1);                                     \
      else __builtin_amdgcn_s_setprio(0);                                                    \
    }                                                                                        \
    hpbd_substep<hex_max_walls(KIND)>(G, S, HT, WT, HW, bd, a, cvl, cal, (it & 1) != 0, hcs); \
  }
#endif
    if constexpr (!GACC) {
      GuardBranch gb;
      HEX_SUBSTEPS(gb)
    } else {
    // one wave per SIMD (GACC): the substeps without guard branches (GuardAcc, pob_math.h); a wave any of whose lanes
    // met an operand outside the fast forms' range reruns them from the loaded state with
    // the branch guards (bit-identical for every lane that stayed in range)
    const HBody b0 = bd;
    GuardAcc ga;
    HEX_SUBSTEPS(ga)
    if (__builtin_expect(__any(ga.bad()), 0)) {
      bd = b0;
      cvl = V(0.0f, 0.0f, 0.0f); cal = cvl;
      GuardBranch gb;
      HEX_SUBSTEPS(gb)
    }
    }
#endif
    {  // joint angle / velocity obs of the lane's joint (a3), on both of its lanes
      const q4 qo = hx_pair4(bd.q);
      const v3 wo = hx_pair3(bd.w);
      const q4 qp = qsel(isP, bd.q, qo), qc = qsel(isP, qo, bd.q);
      const v3 wp = vsel3(isP, bd.w, wo), wc = vsel3(isP, wo, bd.w);
      const v3 ap = qrot(HTV(HT, HT_AXIS), qp);
      const v3 ref = HTV(HT, HT_REF);
      const v3 fp = qrot(ref, qp), fc = qrot(ref, qc);
      jang = pob_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
      jvel = vdot(vsub(wc, wp), ap);
    }
    // the bodies' contact velocity sums for the stock ant's contact cost
    Ls.set3(0, cvl);
    wave_lds_sync();
    if (act_lane && lane0) {
      if ((flags & (POB_F_AUTORESET | POB_F_ZERO_STEPS_ON_DONE)) && t.pdone != 0.0f) t.steps = 0.0f;
      t.xb = xb; t.ctrl = 0.0f; t.contact = 0.0f;
      if (KIND == POB_ANT) {
        // contact rows 0..8 = torso, then Aux k (lane 7 - k) and lower leg k (lane 15 - k)
        t.ctrl = ant_ctrl_cost(act + (size_t)b * POB_NJ);
        float sc = ant_contact_add(0.0f, cvl);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sc = ant_contact_add(sc, Ls.get3_lane(0, lane + 7 - q));
          sc = ant_contact_add(sc, Ls.get3_lane(0, lane + 15 - q));
        }
        t.contact = 0.0005f * sc;
      }
    }
  }
  wave_lds_sync();  // every LDS read of the physics slots is done: the region is staging now
  POB_TS(2);

  // ---- obs rows: assembled in the wave's region (P envs per pass), stored coalesced
  float done = 0.0f;
  t.ga_done_quad = false;
  const bool ga_quad = KIND == POB_GATHER && S.n_obj <= POB_GA_QUAD_MAX;
  GaQuad gq;
  if (ga_quad && act_lane && r < 4) {
    if (!gop_ok) ga_quad_prefetch<QT>(S, in, r3, nullptr, r, gop);
    ga_quad_objects<QT>(S, gop, r3, bd.x, bd.q, r, out.pos, gq, t);
  }
  const int P = pass_envs(POB_HSTAGE_FLOATS, D, 4);
  for (int p0 = 0; p0 < nenv; p0 += P) {
    const int pn = nenv - p0 < P ? nenv - p0 : P;
    if (act_lane && le >= p0 && le < p0 + pn) {
      float *o = stg + (le - p0) * D;
      if (isP) {
        o[sh + 7 + jown] = jang;
        o[sh + 21 + jown] = jvel;
      }
      // cfrc rows from the body's writing lane; the frozen bodies' zero rows over the 16 lanes
      float *oc = o + (29 + sh);
      if (canon) {
        oc[3 * g] = clip1(cvl.x); oc[1 + 3 * g] = clip1(cvl.y); oc[2 + 3 * g] = clip1(cvl.z);
        oc[3 * N + 3 * g] = clip1(cal.x); oc[1 + 3 * N + 3 * g] = clip1(cal.y); oc[2 + 3 * N + 3 * g] = clip1(cal.z);
      }
      for (int q = 3 * POB_NDYN + r; q < 3 * N; q += 16) { oc[q] = 0.0f; oc[3 * N + q] = 0.0f; }
      if (lane0) {
        if (sh == 0) { o[0] = bd.x.x; o[1] = bd.x.y; }
        o[sh + 2] = bd.x.z;
        o[sh + 3] = bd.q.w; o[sh + 4] = bd.q.x; o[sh + 5] = bd.q.y; o[sh + 6] = bd.q.z;
        o[sh + 15] = bd.v.x; o[sh + 16] = bd.v.y; o[sh + 17] = bd.v.z;
        o[sh + 18] = bd.w.x; o[sh + 19] = bd.w.y; o[sh + 20] = bd.w.z;
        if (out.pos != in.pos) {  // functional mode: carry the frozen rows over
          for (int i = POB_NDYN; i < N; ++i) {
            if (!(ga_quad && i >= 11)) cpq<QT>(out.pos, in.pos, r3 + 3 * i, 3);
            cpq<QT>(out.vel, in.vel, r3 + 3 * i, 3);
            cpq<QT>(out.ang, in.ang, r3 + 3 * i, 3);
            cpq<QT>(out.rot, in.rot, r4 + 4 * i, 4);
          }
        }
      }
      if (ga_quad && r < 4) ga_quad_scatter(S, gq, r, o + 29 + 6 * N);
      if (lane0) {
        task_step<KIND, QT>(S, in, b, r3, N, bd.x, bd.q, out.pos, o, flags, L, t);
        task_obs_write(KIND, o, 29 + 6 * N, t);
        done = t.done;
      }
      done = __shfl(done, lane & ~15);  // the env's done to its sixteen lanes
      // AutoResetWrapper: the row of a reset env is first_obs, copied by the env's sixteen
      // lanes after every other write of the row
      if ((flags & POB_F_AUTORESET) && done != 0.0f) {
        wave_lds_sync();
        group_copy<16, 2>(o, in.first_obs + (size_t)b * D, D, r);
      }
    }
    wave_lds_sync();
    float *dst = out.obs + (size_t)(b_first + p0) * D;
    const int n = pn * D;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
      const int n4 = n >> 2;
      for (int i = lane; i < n4; i += 64) reinterpret_cast<float4 *>(dst)[i] = reinterpret_cast<const float4 *>(stg)[i];
      for (int i = 4 * n4 + lane; i < n; i += 64) dst[i] = stg[i];
    } else {
      for (int i = lane; i < n; i += 64) dst[i] = stg[i];
    }
    if (out.obs_masked)  // the observation mask's columns of the same rows (ABI v7)
      store_obs_masked(S, out.obs_masked + (size_t)(b_first + p0) * S.obs_mask_n, stg, pn, D, lane);
    wave_lds_sync();
  }

  POB_TS(3);
  // ---- dynamic qp rows: computed state, or first_qp when the AutoResetWrapper resets
  const bool reset_rows = (flags & POB_F_AUTORESET) && done != 0.0f;
#pragma unroll
  for (int arr = 0; arr < 4; ++arr) {
    const int c = arr == 1 ? 4 : 3;
    if (act_lane && canon) {
      float *o = stg + (le * POB_NDYN + g) * c;
      if (reset_rows) {
        const float *F = arr == 0 ? in.first_pos : (arr == 1 ? in.first_rot : (arr == 2 ? in.first_vel : in.first_ang));
        const size_t src = (arr == 1 ? r4 : r3) + (size_t)g * c;
        for (int q = 0; q < c; ++q) o[q] = Q<QT>::ld(F, src + q);
      } else if (arr == 0) { o[0] = bd.x.x; o[1] = bd.x.y; o[2] = bd.x.z; }
      else if (arr == 1) { o[0] = bd.q.w; o[1] = bd.q.x; o[2] = bd.q.y; o[3] = bd.q.z; }
      else if (arr == 2) { o[0] = bd.v.x; o[1] = bd.v.y; o[2] = bd.v.z; }
      else { o[0] = bd.w.x; o[1] = bd.w.y; o[2] = bd.w.z; }
    }
    wave_lds_sync();
    if (arr == 1) stage_store_dyn<QT, 4>(out.rot, (size_t)b_first * N * 4, N, nenv, stg, lane);
    else stage_store_dyn<QT, 3>(arr == 0 ? out.pos : (arr == 2 ? out.vel : out.ang), (size_t)b_first * N * 3, N, nenv,
                                stg, lane);
    wave_lds_sync();
  }

  POB_TS(4);
  // ---- per-env tail: frozen rows, first_* (the env's lanes), scalar outputs (lane 0)
  if (act_lane) tail_copies<QT, 16>(in, out, flags, reset_rows, b, N, D, r3, r4, r);
  if (act_lane && lane0) {
    out.reward[b] = t.reward;
    out.done[b] = t.done;
    if (out.steps) out.steps[b] = t.steps;
    if (out.truncation) out.truncation[b] = t.trunc;
    if (out.m0) out.m0[b] = t.m0;
    if (out.m1) out.m1[b] = t.m1;
    if (out.m2) out.m2[b] = t.m2;
    out.rng[2 * b] = t.rng0;
    out.rng[2 * b + 1] = t.rng1;
    write_typed(out, b, t);
  }
  if (out.any_done) {
    const unsigned long long mk = __ballot(act_lane && lane0 && done != 0.0f);
    if (mk != 0ull && lane == 0) atomicOr(out.any_done, 1u);
  }
  POB_TS_WRITE();
}


// ----------------------------------------------------------------------------- reset
// System.default_qp forward kinematics (a4): child.rot = parent.rot * axis_angle(axis, q),
// child.pos = anchor - R(child) off_c with anchor = parent.pos + R(parent) off_p; then the
// ant tree is lifted so that its lowest collider point is at z = 0.
POB_D void fk(csys_t &S, const float (&qpos)[POB_NJ], const float (&qvel)[POB_NJ], Body &b) {
  b.x[0] = V(0.0f, 0.0f, 0.0f);
  b.q[0].w = 1.0f; b.q[0].x = 0.0f; b.q[0].y = 0.0f; b.q[0].z = 0.0f;
  b.v[0] = V(0.0f, 0.0f, 0.0f); b.w[0] = V(0.0f, 0.0f, 0.0f);
#pragma unroll
  for (int j = 0; j < POB_NJ; ++j) {
    const int p = jparent(j), c = jchild(j);
    float s, co;
    pob_sincosf(qpos[j] * 0.5f, &s, &co);
    const v3 axis = SV(S.axis[j]);
    q4 loc; loc.w = co; loc.x = axis.x * s; loc.y = axis.y * s; loc.z = axis.z * s;
    b.q[c] = qmul(b.q[p], loc);
    v3 anchor = vadd(b.x[p], qrot(SV(S.off_p[j]), b.q[p]));
    b.x[c] = vsub(anchor, qrot(SV(S.off_c[j]), b.q[c]));
    b.w[c] = vscl(qrot(axis, b.q[p]), qvel[j]);  // default_qp: own joint only, no linear velocity
    b.v[c] = V(0.0f, 0.0f, 0.0f);
  }
  float zmin = 3.0e38f;
#pragma unroll
  for (int i = 0; i < POB_NDYN; ++i) {
#pragma unroll
    for (int q = 0; q < (i == 0 ? 1 : 2); ++q) {
      float z = vadd(b.x[i], qrot(SV(S.cap_end[i][q]), b.q[i])).z - S.cap_r[i];
      if (z < zmin) zmin = z;
    }
  }
#pragma unroll
  for (int i = 0; i < POB_NDYN; ++i) b.x[i].z = b.x[i].z - zmin;
}

enum { RESET_FULL = 0, RESET_GYM = 1, RESET_OWN = 2 };

// jax.random.choice(key, grid, (K,), replace=False) = first K of a stable argsort of
// random_bits(split(key)[1], (n,)) (one shuffle round for n <= ~1600): choice_topk_quad.

// Env.reset with FOUR lanes per env (the step kernel's split, pob_quad.h): lane k of the
// env's quad owns the torso (replica) and leg k.  A masked reset (gym / randomized
// autoreset) typically has one done env per wave, so its cost is one env's latency: the
// quad splits the forward kinematics (two joints per lane instead of eight), the contact
// detection and solve (three bodies per lane) and the obs (two joints per lane).
// Op order per value = oracle/pob_oracle.c (reset + sys.info + _get_obs).
struct QReset {
  QBody bd;
  v3 cv[QNB], ca[QNB];    // sys.info(qp).contact of the local bodies (the reset obs' cfrc)
  float jang[QNJ], jvel[QNJ];
  float ax, ay;           // HH / TAG: ant xy offset (also shifts the Ground row)
  float tx, ty;           // TAG target xy
  int hh_first;           // HH: goal order of choice(rng3, hhp[:2], 2)
  uint32_t rng0, rng1;    // new info['rng']
#ifdef POB_EXP_TIMING
  unsigned long long ts[4];  // timing experiment only: stamps inside qreset_compute
#endif
};

// minimum over the env's lane quad (exact and order-free; all four lanes active)
POB_D float quad_min(float x) {
  const float a = fminf(quad_bcast<0>(x), quad_bcast<1>(x));
  const float b = fminf(quad_bcast<2>(x), quad_bcast<3>(x));
  return fminf(a, b);
}

// choice_topk on an env's lane quad: lane k inserts the keys of grid indices i = k (mod 4)
// into its own sorted list (its LDS column, stable: equal keys keep index order), then lane
// 0 merges the four lists by (key, index) -- the first K of the stable argsort of all n
// keys, as choice_topk -- into out[o * OS] (o = 0..K-1).
template <int BS>
POB_D void choice_topk_quad(uint32_t k0, uint32_t k1, int n, int K, int k, uint32_t *lds_key, int *lds_idx, int *out,
                            int OS) {
  const int t = threadIdx.x;
  uint32_t s0, s1;
  tf_split(k0, k1, 2u, 1u, s0, s1);
  int cnt = 0;
  for (int i = k; i < n; i += 4) {
    const uint32_t key = tf_elem(s0, s1, (uint32_t)n, (uint32_t)i);
    if (cnt == K && key >= lds_key[(K - 1) * BS + t]) continue;
    int pos = cnt < K ? cnt : K - 1;
    while (pos > 0 && lds_key[(pos - 1) * BS + t] > key) {
      lds_key[pos * BS + t] = lds_key[(pos - 1) * BS + t];
      lds_idx[pos * BS + t] = lds_idx[(pos - 1) * BS + t];
      --pos;
    }
    lds_key[pos * BS + t] = key;
    lds_idx[pos * BS + t] = i;
    if (cnt < K) ++cnt;
  }
  wave_lds_sync();
  if (k == 0) {
    int head[4], len[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      head[q] = 0;
      const int nq = (n - q + 3) / 4;
      len[q] = nq < K ? nq : K;
    }
    for (int m = 0; m < K; ++m) {
      int best = -1;
      uint32_t bk = 0u;
      int bi = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (head[q] < len[q]) {
          const uint32_t kq = lds_key[head[q] * BS + t + q];
          const int iq = lds_idx[head[q] * BS + t + q];
          if (best < 0 || kq < bk || (kq == bk && iq < bi)) { best = q; bk = kq; bi = iq; }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) head[q] += (q == best) ? 1 : 0;
      out[m * OS] = bi;
    }
  }
  wave_lds_sync();
}

// choice_topk for ONE env by the whole wave (all 64 lanes active; k0, k1 wave-uniform): the
// first K of the stable argsort of random_bits(split(key)[1], (n,)), n <= 2 * 64 * POB_CW_SLOTS.
//  1. lane l hashes pairs p = l + 64 m: one threefry2x32 call gives elements p and p + h
//     (h = ceil(n / 2); tf_elem's pairing);
//  2. candidates: the keys <= T0 for the smallest T0 in 2^30 - 1, 2^31 - 1, 2^32 - 1 with at
//     least K of them (for n = 156, K = 16 the first bound holds but with probability ~1e-5:
//     about n / 4 = 39 candidates), compacted into LDS as (key, index) pairs;
//  3. each candidate's rank by (key, index) among the candidates -- which is its rank among
//     all n keys, since every non-candidate is larger -- and the candidates of rank < K are
//     written to out[rank * OS].
// One env's choice is a short, wave-parallel chain (~2 threefry calls per lane, one ballot
// round, ~40 broadcast LDS reads) instead of a lane quad hashing n / 4 keys in a row and
// merging four sorted lists: an AntGather reset wave spent ~66 us in that (profiles/r3c).
#define POB_CW_SLOTS 8
#define GA_OBJ_F 5  // k_reset's per-object table: x, y, z, reading intensity, reading slot
POB_D void choice_topk_wave(uint32_t k0, uint32_t k1, int n, int K, uint2 *lcand, int *out, int OS) {
  const int lane = (int)(threadIdx.x & 63);
  uint32_t s0, s1;
  tf_split(k0, k1, 2u, 1u, s0, s1);
  const int h = (n + 1) >> 1;
  const int ns = (h + 63) >> 6;  // pair slots in use (wave-uniform)
  uint32_t ka[POB_CW_SLOTS], kb[POB_CW_SLOTS];
  bool va[POB_CW_SLOTS], vb[POB_CW_SLOTS];
#pragma unroll
  for (int m = 0; m < POB_CW_SLOTS; ++m) {
    const int p = lane + 64 * m;
    va[m] = m < ns && p < h;
    vb[m] = va[m] && p + h < n;
    ka[m] = 0u; kb[m] = 0u;
    if (va[m]) threefry2x32(s0, s1, (uint32_t)p, vb[m] ? (uint32_t)(p + h) : 0u, ka[m], kb[m]);
  }
  uint32_t T = 0x3FFFFFFFu;
  for (;;) {  // wave-uniform, at most three rounds
    int cnt = 0;
#pragma unroll
    for (int m = 0; m < POB_CW_SLOTS; ++m) {
      if (m < ns) {
        cnt += __popcll(__ballot(va[m] && ka[m] <= T));
        cnt += __popcll(__ballot(vb[m] && kb[m] <= T));
      }
    }
    if (cnt >= K || T == 0xFFFFFFFFu) break;
    T = (T << 1) | 1u;
  }
  int nc = 0;
#pragma unroll
  for (int m = 0; m < POB_CW_SLOTS; ++m) {
    if (m < ns) {
      const bool sa = va[m] && ka[m] <= T, sb = vb[m] && kb[m] <= T;
      const uint64_t ma = __ballot(sa);
      const uint64_t mb = __ballot(sb);
      const int pa = nc + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, 0u));
      nc += __popcll(ma);
      const int pb = nc + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
      nc += __popcll(mb);
      const int p = lane + 64 * m;
      if (sa) lcand[pa] = make_uint2(ka[m], (uint32_t)p);
      if (sb) lcand[pb] = make_uint2(kb[m], (uint32_t)(p + h));
    }
  }
  wave_lds_sync();
  for (int e = lane; e < nc; e += 64) {
    const uint2 ce = lcand[e];
    int rank = 0;
#pragma unroll 4
    for (int f = 0; f < nc; ++f) {
      const uint2 cf = lcand[f];
      rank += (cf.x < ce.x || (cf.x == ce.x && cf.y < ce.y)) ? 1 : 0;
    }
    if (rank < K) out[rank * OS] = (int)ce.y;
  }
  wave_lds_sync();
}

template <int KIND, int BS>
POB_D void qreset_compute(csys_t *Sp, const float *LT, const float *WT, const int k, uint32_t k0, uint32_t k1,
                          QReset &R, uint32_t *lds_key, int *lds_idx, const bool wave_choice, float *ga_obj,
                          const bool objects_by_wave = false) {
  csys_t &S = *Sp;
  // random_split(rng, 5) (HH, TAG) | 4 (GA) | 3 (stock ant, brax envs/ant.py reset)
  const uint32_t ns = KIND == POB_GATHER ? 4u : (KIND == POB_ANT ? 3u : 5u);
  uint32_t r[5][2];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    if (i < (int)ns) tf_split(k0, k1, ns, (uint32_t)i, r[i][0], r[i][1]);
    else { r[i][0] = 0u; r[i][1] = 0u; }
  }
#ifdef POB_EXP_TIMING
  R.ts[0] = __builtin_amdgcn_s_memtime();
#endif
  // System.default_qp forward kinematics of this lane's leg (joints 2k, 2k + 1), the torso
  // at the origin (oracle fk / kernel fk op order)
  QBody &b = R.bd;
  b.x[0] = V(0.0f, 0.0f, 0.0f);
  b.q[0].w = 1.0f; b.q[0].x = 0.0f; b.q[0].y = 0.0f; b.q[0].z = 0.0f;
  b.v[0] = V(0.0f, 0.0f, 0.0f); b.w[0] = V(0.0f, 0.0f, 0.0f);
#pragma unroll
  for (int jl = 0; jl < QNJ; ++jl) {
    const int j = 2 * k + jl, p = jparent(jl), c = jchild(jl);
    const float qpos = S.default_angle[j] + tf_uniform(r[1][0], r[1][1], 8u, (uint32_t)j, -0.1f, 0.1f);
    const float qvel = tf_uniform(r[2][0], r[2][1], 8u, (uint32_t)j, -0.1f, 0.1f);
    float sn, co;
    pob_sincosf(qpos * 0.5f, &sn, &co);
    const v3 axis = QJV(LT, jl, QJ_AXIS);
    q4 loc; loc.w = co; loc.x = axis.x * sn; loc.y = axis.y * sn; loc.z = axis.z * sn;
    b.q[c] = qmul(b.q[p], loc);
    const v3 anchor = vadd(b.x[p], qrot(QJV(LT, jl, QJ_OFFP), b.q[p]));
    b.x[c] = vsub(anchor, qrot(QJV(LT, jl, QJ_OFFC), b.q[c]));
    // default_qp's joint velocity: the child's own joint only (axis * qvel rotated by the
    // parent), no linear velocity (oracle orc_default_qp)
    b.w[c] = vscl(qrot(axis, b.q[p]), qvel);
    b.v[c] = V(0.0f, 0.0f, 0.0f);
  }
  // lift: the lowest capsule point of the whole ant at z = 0
  float zmin = vadd(b.x[0], qrot(qcap_end(S, LT, 0, 0), b.q[0])).z - q_cap_r(S, LT, 0);
#pragma unroll
  for (int l = 1; l < QNB; ++l) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float z = vadd(b.x[l], qrot(qcap_end(S, LT, l, q), b.q[l])).z - q_cap_r(S, LT, l);
      zmin = z < zmin ? z : zmin;
    }
  }
  zmin = quad_min(zmin);
#pragma unroll
  for (int l = 0; l < QNB; ++l) b.x[l].z = b.x[l].z - zmin;
#ifdef POB_EXP_TIMING
  R.ts[1] = __builtin_amdgcn_s_memtime();
#endif
  R.ax = 0.0f; R.ay = 0.0f; R.tx = 0.0f; R.ty = 0.0f; R.hh_first = 0;
  if (KIND == POB_HEAVENHELL) {
    // ant_heavenhell.py:87-103
    R.ax = tf_uniform(r[3][0], r[3][1], 2u, 0u, -0.5f, 0.5f);
    R.ay = tf_uniform(r[3][0], r[3][1], 2u, 1u, 0.5f, 1.5f);
    uint32_t s0, s1, y0, y1;  // choice(rng3, hhp[:2], 2, replace=False)
    tf_split(r[3][0], r[3][1], 2u, 1u, s0, s1);
    threefry2x32(s0, s1, 0u, 1u, y0, y1);
    R.hh_first = (y1 < y0) ? 1 : 0;
    R.rng0 = r[0][0]; R.rng1 = r[0][1];
  } else if (KIND == POB_GATHER) {
    // ant_gather.py:109-123: the env's chosen grid indices go to lds_idx's env row block
    if (!wave_choice)  // (else k_reset ran choice_topk_wave for this env already)
      choice_topk_quad<BS>(r[3][0], r[3][1], S.n_grid, S.n_obj, k, lds_key, lds_idx,
                           lds_idx + POB_MAXOBJ * BS + (threadIdx.x >> 2), BS / 4);
    R.rng0 = k0; R.rng1 = k1;  // ant_gather.py:106 stores the input key
    // the objects' positions and sensor readings (ant_gather.py:118-123, _get_readings), object
    // o on quad lane o % 4, into the env's LDS table (GA_OBJ: x, y, z, intensity, slot)
    // (objects_by_wave: k_reset computes the table with one lane per object instead)
    float *eo = ga_obj + (threadIdx.x >> 2) * GA_OBJ_F * POB_MAXOBJ;
    const float ori = ga_orientation(b.q[0]);
    for (int o = k; o < (objects_by_wave ? 0 : S.n_obj); o += 4) {
      const int g = lds_idx[POB_MAXOBJ * BS + o * (BS / 4) + (threadIdx.x >> 2)];
      const float ox = S.grid[3 * g], oy = S.grid[3 * g + 1];
      float inten;
      const int slot = ga_reading_slot(S, o, ox, oy, dist2d(b.x[0].x, b.x[0].y, ox, oy), ori, inten);
      eo[o] = ox; eo[POB_MAXOBJ + o] = oy; eo[2 * POB_MAXOBJ + o] = o < S.ga_n_apples ? 1.0f : S.grid[3 * g + 2];
      eo[3 * POB_MAXOBJ + o] = inten; eo[4 * POB_MAXOBJ + o] = __int_as_float(slot);
    }
  } else if (KIND == POB_ANT) {
    R.rng0 = r[0][0]; R.rng1 = r[0][1];  // (not part of the stock ant's State)
  } else {
    // ant_tag.py:63-105 (all four lanes run the same rejection loop)
    const float lo0 = -S.tag_cage_xy[0], lo1 = -S.tag_cage_xy[1];
    R.ax = tf_uniform(r[3][0], r[3][1], 2u, 0u, lo0, S.tag_cage_xy[0]);
    R.ay = tf_uniform(r[3][0], r[3][1], 2u, 1u, lo1, S.tag_cage_xy[1]);
    uint32_t q0 = r[4][0], q1 = r[4][1];
    float tx = tf_uniform(q0, q1, 2u, 0u, lo0, S.tag_cage_xy[0]);
    float ty = tf_uniform(q0, q1, 2u, 1u, lo1, S.tag_cage_xy[1]);
    for (int it = 0; it < 100000 && dist2d(tx, ty, R.ax, R.ay) <= S.tag_min_spawn_distance; ++it) {
      uint32_t n0, n1;
      tf_split(q0, q1, 2u, 1u, n0, n1);
      q0 = n0; q1 = n1;
      tx = tf_uniform(q0, q1, 2u, 0u, lo0, S.tag_cage_xy[0]);
      ty = tf_uniform(q0, q1, 2u, 1u, lo1, S.tag_cage_xy[1]);
    }
    R.tx = tx; R.ty = ty;
    R.rng0 = r[0][0]; R.rng1 = r[0][1];
  }
  if (KIND == POB_HEAVENHELL || KIND == POB_TAG) {
#pragma unroll
    for (int l = 0; l < QNB; ++l) { b.x[l].x = b.x[l].x + R.ax; b.x[l].y = b.x[l].y + R.ay; }
  }
#ifdef POB_EXP_TIMING
  R.ts[2] = __builtin_amdgcn_s_memtime();
#endif
  // sys.info(qp).contact: contact detection + velocity-level solve at the static qp
#pragma unroll
  for (int l = 0; l < QNB; ++l) { R.cv[l] = V(0.0f, 0.0f, 0.0f); R.ca[l] = V(0.0f, 0.0f, 0.0f); }
  if (S.legacy) qcontacts_static<KIND != POB_ANT, true>(Sp, LT, WT, b, R.cv, R.ca, S.friction);  // the colliders' impulses
  else qcontacts_static<KIND != POB_ANT, false>(Sp, LT, WT, b, R.cv, R.ca, S.friction);
#ifdef POB_EXP_TIMING
  R.ts[3] = __builtin_amdgcn_s_memtime();
#endif
  // joint angle / velocity obs of this lane's joints (a3)
#pragma unroll
  for (int jl = 0; jl < QNJ; ++jl) {
    const int p = jparent(jl), c = jchild(jl);
    const v3 ap = qrot(QJV(LT, jl, QJ_AXIS), b.q[p]);
    const v3 ref = jl == 0 ? V(-1.0f, 0.0f, 0.0f) : V(0.0f, 0.0f, 1.0f);  // the Ant's (pob_system.cpp)
    const v3 fp = qrot(ref, b.q[p]), fc = qrot(ref, b.q[c]);
    R.jang[jl] = pob_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
    R.jvel[jl] = vdot(vsub(b.w[c], b.w[p]), ap);
  }
}

// Row writers: lane k writes its bodies' parts of one env row of each output array (float32
// values; the storage conversion happens in the coalesced copy); the frozen rows are split
// over the quad; lane 0 then writes the task rows (program order: after the frozen fill).
enum { RROW_POS = 0, RROW_ROT = 1, RROW_VEL = 2, RROW_ANG = 3, RROW_OBS = 4 };
template <int KIND, int BS>
// quad_all = false: the frozen bodies' constant parts (identity rotations, zero velocities,
// zero contact-force obs) and AntGather's object rows and sensor readings are left to the
// caller (k_reset's masked path writes them with the whole wave); every element this
// function writes is disjoint from them.
POB_D void qreset_row(csys_t &S, const QReset &R, const int k, const int arr, float *row, const float *ga_obj,
                      const bool quad_all = true) {
  const int N = n_bodies<KIND>(S);
  const QBody &b = R.bd;
  if (arr == RROW_POS) {
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      if (l == 0 && k != 0) continue;
      const int g = qbody_global(l, k);
      row[3 * g] = b.x[l].x; row[3 * g + 1] = b.x[l].y; row[3 * g + 2] = b.x[l].z;
    }
    for (int i = POB_NDYN + k; i < N; i += 4) {
      // (the task bodies written whole below are skipped: every element of the row is written
      // by one lane once, so the row may go straight to global memory, k_reset's masked path)
      if (KIND == POB_HEAVENHELL && (i == 11 || i == 12)) continue;
      if (KIND == POB_TAG && i == 10) continue;
      if (KIND == POB_GATHER && i >= 11 && i < 11 + S.n_obj) continue;
      row[3 * i] = S.frozen_pos[i][0]; row[3 * i + 1] = S.frozen_pos[i][1]; row[3 * i + 2] = S.frozen_pos[i][2];
    }
    if (KIND == POB_GATHER && quad_all) {  // object o on quad lane o % 4
      const float *eo = ga_obj + (threadIdx.x >> 2) * GA_OBJ_F * POB_MAXOBJ;
      for (int o = k; o < S.n_obj; o += 4) {
        float *d = row + 3 * (11 + o);
        d[0] = eo[o]; d[1] = eo[POB_MAXOBJ + o]; d[2] = eo[2 * POB_MAXOBJ + o];
      }
    }
    if (k == 0) {
      if (KIND == POB_HEAVENHELL || KIND == POB_TAG) {  // Ground is in ant_indices
        row[27] = S.frozen_pos[9][0] + R.ax; row[28] = S.frozen_pos[9][1] + R.ay;
      }
      if (KIND == POB_HEAVENHELL) {
        row[33] = S.hh_hhp[R.hh_first][0]; row[34] = S.hh_hhp[R.hh_first][1]; row[35] = 1.0f;
        row[36] = S.hh_hhp[1 - R.hh_first][0]; row[37] = S.hh_hhp[1 - R.hh_first][1]; row[38] = 1.0f;
      } else if (KIND == POB_TAG) {
        row[30] = R.tx; row[31] = R.ty; row[32] = 0.5f;
      }
    }
  } else if (arr == RROW_ROT) {
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      if (l == 0 && k != 0) continue;
      const int g = qbody_global(l, k);
      row[4 * g] = b.q[l].w; row[4 * g + 1] = b.q[l].x; row[4 * g + 2] = b.q[l].y; row[4 * g + 3] = b.q[l].z;
    }
    if (quad_all)
      for (int i = POB_NDYN + k; i < N; i += 4) { row[4 * i] = 1.0f; row[4 * i + 1] = 0.0f; row[4 * i + 2] = 0.0f; row[4 * i + 3] = 0.0f; }
  } else if (arr == RROW_VEL || arr == RROW_ANG) {
    const v3 *v = arr == RROW_VEL ? b.v : b.w;
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      if (l == 0 && k != 0) continue;
      const int g = qbody_global(l, k);
      row[3 * g] = v[l].x; row[3 * g + 1] = v[l].y; row[3 * g + 2] = v[l].z;
    }
    if (quad_all)
      for (int i = 3 * POB_NDYN + k; i < 3 * N; i += 4) row[i] = 0.0f;
  } else {
    const int sh = obs_shift(KIND);
#pragma unroll
    for (int jl = 0; jl < QNJ; ++jl) {
      row[sh + 7 + 2 * k + jl] = R.jang[jl];
      row[sh + 21 + 2 * k + jl] = R.jvel[jl];
    }
    float *oc = row + (29 + sh);
#pragma unroll
    for (int l = 0; l < QNB; ++l) {
      if (l == 0 && k != 0) continue;
      const int g = qbody_global(l, k);
      oc[3 * g] = clip1(R.cv[l].x); oc[1 + 3 * g] = clip1(R.cv[l].y); oc[2 + 3 * g] = clip1(R.cv[l].z);
      oc[3 * N + 3 * g] = clip1(R.ca[l].x); oc[1 + 3 * N + 3 * g] = clip1(R.ca[l].y); oc[2 + 3 * N + 3 * g] = clip1(R.ca[l].z);
    }
    if (quad_all)
      for (int q = 3 * POB_NDYN + k; q < 3 * N; q += 4) { oc[q] = 0.0f; oc[3 * N + q] = 0.0f; }
    if (k == 0) {
      if (sh == 0) { row[0] = b.x[0].x; row[1] = b.x[0].y; }
      row[sh + 2] = b.x[0].z;
      row[sh + 3] = b.q[0].w; row[sh + 4] = b.q[0].x; row[sh + 5] = b.q[0].y; row[sh + 6] = b.q[0].z;
      row[sh + 15] = b.v[0].x; row[sh + 16] = b.v[0].y; row[sh + 17] = b.v[0].z;
      row[sh + 18] = b.w[0].x; row[sh + 19] = b.w[0].y; row[sh + 20] = b.w[0].z;
      const int base = 29 + 6 * N;
      if (KIND == POB_HEAVENHELL) {
        row[base] = 0.0f;  // priest_in_range = 0 at reset
      } else if (KIND == POB_GATHER && quad_all) {
        // the scatter readings[slot] = intensity in object order (a later object wins a slot)
        float *rd = row + base;
        ga_readings_begin(S, rd);
        const float *eo = ga_obj + (threadIdx.x >> 2) * GA_OBJ_F * POB_MAXOBJ;
        for (int o = 0; o < S.n_obj; ++o) {
          const int slot = __float_as_int(eo[4 * POB_MAXOBJ + o]);
          if (slot >= 0) rd[slot] = eo[3 * POB_MAXOBJ + o];
        }
      } else if (KIND == POB_TAG) {
        const bool vis = dist2d(R.tx, R.ty, b.x[0].x, b.x[0].y) <= S.tag_visible_radius;
        row[base] = vis ? R.tx : 0.0f; row[base + 1] = vis ? R.ty : 0.0f;
      }
    }
  }
}

// Coalesced store of staged rows (row r of W elements at stg + r * WP) to
// X[(b0 + r) * W ...] (and FX, when given) for the rows whose bit is set in `rows`.
template <typename QT>
POB_D void reset_store_rows(float *X, float *FX, const size_t b0, const int W, const int nrows, const int WP,
                            const float *stg, const uint32_t rows, const int lane) {
  if (4 * __popc(rows) < nrows) {
    // a masked reset (typically one done env per wave): the set rows only, each stored by the
    // whole wave (a few iterations instead of a pass over all 16 rows' elements)
    for (uint32_t m = rows; m != 0u; m &= m - 1u) {
      const int rr = __builtin_ctz(m);
      for (int e0 = lane; e0 < W; e0 += 64) {
        const float v = stg[rr * WP + e0];
        Q<QT>::st(X, (b0 + rr) * W + e0, v);
        if (FX) Q<QT>::st(FX, (b0 + rr) * W + e0, v);
      }
    }
    return;
  }
  int r = 0, e = lane;
  while (e >= W) { e -= W; ++r; }
  for (int i = lane; i < nrows * W; i += 64) {
    if ((rows >> r) & 1u) {
      const float v = stg[r * WP + e];
      Q<QT>::st(X, b0 * W + i, v);
      if (FX) Q<QT>::st(FX, b0 * W + i, v);
    }
    e += 64;
    while (e >= W) { e -= W; ++r; }
  }
}

// gym mode: this batch is rows [first, first + B) of a global batch of `total` envs (index
// sharding over ranks, sharding.py): keys = split(gym_key, total + 1)[1 + first + b], and
// the gym key advances to split(gym_key, total + 1)[0] when *any_flag (the GLOBAL any-done,
// all-reduced across ranks by the caller) is set.
// One wave per block = 16 envs x 4 lanes.  Every env's reset is computed in registers by
// its quad, then each output array is staged row by row in LDS (16 rows of WP floats,
// dynamic shared memory) and stored coalesced -- to the state and, in a full reset, to
// first_qp / first_obs at the same time (no read-back).  Masked modes store only the rows
// of done envs; a wave without one exits at once.
template <int KIND, int BS, typename QT>
__global__ __launch_bounds__(BS) void k_reset(const void *sysp, const int B, const int mode,
                                              const uint32_t *__restrict__ keys, const uint32_t *gym_in,
                                              uint32_t *gym_out, const uint32_t *any_flag, const StatePtrs s,
                                              const int total, const int first, const int WP) {
  static_assert(BS == 64, "k_reset stages one wave's rows per block");
  POB_TS_DECL();  // timing experiment only (POB_EXP_TIMING; waves with nothing to reset exit unrecorded)
  POB_TS(0);
  __shared__ __attribute__((aligned(16))) uint32_t lds_key[KIND == POB_GATHER ? POB_MAXOBJ * BS : 1];
  // per-lane sorted lists, then the merged choice per env (POB_MAXOBJ x 16 envs)
  __shared__ int lds_idx[KIND == POB_GATHER ? POB_MAXOBJ * BS + POB_MAXOBJ * (BS / 4) : 1];
  __shared__ __attribute__((aligned(16))) float legtab[POB_TAB_FLOATS];
  // AntGather: each env's objects (x, y, z, reading intensity, reading slot), POB_MAXOBJ each
  __shared__ float ga_obj[KIND == POB_GATHER ? (BS / 4) * GA_OBJ_F * POB_MAXOBJ : 1];
  extern __shared__ float stg[];  // 16 rows of WP floats
  csys_t *Sp = (csys_t *)(size_t)sysp;
  csys_t &S = *Sp;
  const int lane = (int)threadIdx.x;
  const int k = lane & 3;
  const int e0 = (int)blockIdx.x * (BS / 4);  // first env of this wave
  const int b = e0 + (lane >> 2);
  // the next step's any-done word (gym wrapper, double-buffered): the step before this launch
  // used the other word, and the next launch on the stream reads this one after it is zero
  if (s.any_done_clear && blockIdx.x == 0 && lane == 0) *s.any_done_clear = 0u;
  bool active = b < B;
  // the env's done flag is loaded together with the any-done word and the gym key (one round
  // trip, not two: the key's hash below would otherwise wait for a load issued after the
  // any-done test)
  const float dn = active && mode != RESET_FULL ? s.done[b] : 1.0f;
  uint32_t gk0 = 0u, gk1 = 0u;
  if (mode == RESET_GYM) { gk0 = gym_in[0]; gk1 = gym_in[1]; }
  if (mode == RESET_GYM) {
    const bool any = *any_flag != 0u;
    if (b == 0 && k == 0 && gym_out) {
      uint32_t g0 = gk0, g1 = gk1;
      if (any) tf_split(gk0, gk1, (uint32_t)total + 1u, 0u, g0, g1);
      gym_out[0] = g0; gym_out[1] = g1;
    }
    if (!any) return;  // block-uniform
  }
  active = active && dn != 0.0f;
  const uint64_t lanes = __ballot(active && k == 0);
  if (lanes == 0ull) return;  // block-uniform (a masked reset with no done env in this wave)
  // the system table's loads are issued here and land in LDS after the key hashes below
  constexpr int TPL = (POB_TAB_FLOATS + BS - 1) / BS;
  float tabv[TPL];
  {
    const __attribute__((address_space(4))) float *src = &Sp->leg[0][0];
#pragma unroll
    for (int i = 0; i < TPL; ++i) {
      const int j = lane + BS * i;
      tabv[i] = j < POB_TAB_FLOATS ? src[j] : 0.0f;
    }
  }
  // keys of the envs to reset only (a gym key is a threefry hash: a wave without a done env
  // computes none)
  uint32_t k0 = 0u, k1 = 0u;
  if (active) {
    if (mode == RESET_FULL) { k0 = keys[2 * b]; k1 = keys[2 * b + 1]; }
    else if (mode == RESET_GYM)
      tf_split(gk0, gk1, (uint32_t)total + 1u, (uint32_t)(first + b) + 1u, k0, k1);
    else { k0 = s.rng[2 * b]; k1 = s.rng[2 * b + 1]; }
  }
  POB_TS(1);
  uint32_t rows = 0u;  // bit e: env e0 + e is reset
#pragma unroll
  for (int e = 0; e < 16; ++e) rows |= (uint32_t)((lanes >> (4 * e)) & 1ull) << e;
#pragma unroll
  for (int i = 0; i < TPL; ++i) {
    const int j = lane + BS * i;
    if (j < POB_TAB_FLOATS) legtab[j] = tabv[i];
  }
  __syncthreads();
  const float *LT = legtab + k * POB_LEG_FLOATS;
  const float *WT = legtab + 4 * POB_LEG_FLOATS;
  // AntGather's object choice, one env at a time by the whole wave (ant_gather.py:118)
  const bool wave_choice = KIND == POB_GATHER && S.n_grid <= 2 * 64 * POB_CW_SLOTS &&
                           S.n_grid <= POB_MAXOBJ * BS / 2;  // (key, index) pairs in lds_key
  if (wave_choice) {
    for (uint32_t m = rows; m != 0u; m &= m - 1u) {
      const int e = __builtin_ctz(m);
      const uint32_t a0 = __builtin_amdgcn_readlane(k0, 4 * e), a1 = __builtin_amdgcn_readlane(k1, 4 * e);
      uint32_t c0, c1;
      tf_split(a0, a1, 4u, 3u, c0, c1);  // rng3 of random_split(rng, 4) (ant_gather.py:110)
      choice_topk_wave(c0, c1, S.n_grid, S.n_obj, (uint2 *)lds_key, lds_idx + POB_MAXOBJ * BS + e, BS / 4);
    }
  }
  QReset R;
  // a masked reset with few done envs in the wave (the gym step's case: about one) writes the
  // rows straight from registers, and the per-object work takes one lane per object
  const int nenv = B - e0 < BS / 4 ? B - e0 : BS / 4;
  const bool few = mode != RESET_FULL && 4 * __popc(rows) < nenv;
  const bool objects_by_wave = KIND == POB_GATHER && few && wave_choice && S.n_obj <= BS;
  if (active) qreset_compute<KIND, BS>(Sp, LT, WT, k, k0, k1, R, lds_key, lds_idx, wave_choice, ga_obj, objects_by_wave);
  if (objects_by_wave) {
    // ant_gather.py:118-123: object o of env e on lane o (the quad's loop ran four in a row)
    const float ori_l = active ? ga_orientation(R.bd.q[0]) : 0.0f;
    const float tx_l = active ? R.bd.x[0].x : 0.0f, ty_l = active ? R.bd.x[0].y : 0.0f;
    for (uint32_t m = rows; m != 0u; m &= m - 1u) {
      const int e = __builtin_ctz(m);
      const float ori = __shfl(ori_l, 4 * e), tx = __shfl(tx_l, 4 * e), ty = __shfl(ty_l, 4 * e);
      if (lane < S.n_obj) {  // (S.n_obj <= BS: checked above)
        const int o = lane;
        const int g = lds_idx[POB_MAXOBJ * BS + o * (BS / 4) + e];
        const float ox = S.grid[3 * g], oy = S.grid[3 * g + 1];
        float inten;
        const int slot = ga_reading_slot(S, o, ox, oy, dist2d(tx, ty, ox, oy), ori, inten);
        float *eo = ga_obj + e * GA_OBJ_F * POB_MAXOBJ;
        eo[o] = ox; eo[POB_MAXOBJ + o] = oy; eo[2 * POB_MAXOBJ + o] = o < S.ga_n_apples ? 1.0f : S.grid[3 * g + 2];
        eo[3 * POB_MAXOBJ + o] = inten; eo[4 * POB_MAXOBJ + o] = __int_as_float(slot);
      }
    }
  }
  if (KIND == POB_GATHER) wave_lds_sync();  // the objects' table, read by other lanes
  POB_TS(2);
#ifdef POB_EXP_TIMING
  {  // the first active lane's stamps inside the compute (stamps 4..7 of the wave's row)
    const int src = __builtin_ctzll(lanes);
    for (int i = 0; i < 4; ++i)
      pob_ts[4 + i] = ((unsigned long long)__shfl((int)(R.ts[i] >> 32), src) << 32) |
                      (unsigned int)__shfl((int)(unsigned int)R.ts[i], src);
  }
#endif
  const int N = n_bodies<KIND>(S), D = obs_dim<KIND>(S);
  const bool full = mode == RESET_FULL && s.first_pos;
  float *myrow = stg + (lane >> 2) * WP;
  // A masked reset with few done envs in the wave (the gym step's case: about one) writes each
  // env's rows straight from its quad's registers to global memory: no LDS staging, no wave
  // syncs between the arrays (the five staged passes were a quarter of the reset wave's life,
  // 7.7 K of 28.5 K ticks at HH B = 65 536).  float32 qp storage only (binary16 rows take the
  // staged path and its converting stores).
  if (std::is_same<QT, float>::value && few) {
    if (active) {
#pragma unroll 1
      for (int arr = 0; arr < 5; ++arr) {
        const int W = arr == RROW_OBS ? D : (arr == RROW_ROT ? 4 * N : 3 * N);
        float *X = arr == RROW_POS ? s.pos : (arr == RROW_ROT ? s.rot : (arr == RROW_VEL ? s.vel : (arr == RROW_ANG ? s.ang : s.obs)));
        qreset_row<KIND, BS>(S, R, k, arr, X + (size_t)b * W, ga_obj, false);
      }
    }
    // the frozen bodies' constant parts, by the whole wave (AntGather: 288 floats per env,
    // 72 single-float stores per lane of the env's quad): identity rotations, zero linear /
    // angular velocities, zero contact-force obs
    const int nf = N - POB_NDYN, sh = obs_shift(KIND);
    for (uint32_t m = rows; m != 0u; m &= m - 1u) {
      const size_t rb = (size_t)(e0 + __builtin_ctz(m));
      float *rot = s.rot + rb * 4 * N + 4 * POB_NDYN;
      float *vel = s.vel + rb * 3 * N + 3 * POB_NDYN, *ang = s.ang + rb * 3 * N + 3 * POB_NDYN;
      float *oc = s.obs + rb * D + 29 + sh + 3 * POB_NDYN;
      for (int i = lane; i < 4 * nf; i += 64) rot[i] = (i & 3) == 0 ? 1.0f : 0.0f;
      for (int i = lane; i < 3 * nf; i += 64) { vel[i] = 0.0f; ang[i] = 0.0f; oc[i] = 0.0f; oc[3 * N + i] = 0.0f; }
      if (KIND == POB_GATHER) {
        // the objects' pos rows (object o on lane o) and the sensor readings (slot r on lane r:
        // the scatter's last writer in object order, 0 where no object lands)
        const float *eo = ga_obj + __builtin_ctz(m) * GA_OBJ_F * POB_MAXOBJ;
        for (int o = lane; o < S.n_obj; o += 64) {
          float *d = s.pos + rb * 3 * N + 3 * (11 + o);
          d[0] = eo[o]; d[1] = eo[POB_MAXOBJ + o]; d[2] = eo[2 * POB_MAXOBJ + o];
        }
        for (int r = lane; r < 2 * S.ga_n_bins; r += 64) {
          float v = 0.0f;
          for (int o = 0; o < S.n_obj; ++o)
            if (__float_as_int(eo[4 * POB_MAXOBJ + o]) == r) v = eo[3 * POB_MAXOBJ + o];
          s.obs[rb * D + 29 + 6 * N + r] = v;
        }
      }
    }
  } else {
#pragma unroll 1
  for (int arr = 0; arr < 5; ++arr) {
    const int W = arr == RROW_OBS ? D : (arr == RROW_ROT ? 4 * N : 3 * N);
    float *X = arr == RROW_POS ? s.pos : (arr == RROW_ROT ? s.rot : (arr == RROW_VEL ? s.vel : (arr == RROW_ANG ? s.ang : s.obs)));
    float *FX = !full ? nullptr
                      : (arr == RROW_POS ? s.first_pos
                                         : (arr == RROW_ROT ? s.first_rot
                                                            : (arr == RROW_VEL ? s.first_vel
                                                                               : (arr == RROW_ANG ? s.first_ang : s.first_obs))));
    if (active) qreset_row<KIND, BS>(S, R, k, arr, myrow, ga_obj);
    wave_lds_sync();
    if (arr == RROW_OBS) reset_store_rows<float>(X, FX, (size_t)e0, W, nenv, WP, stg, rows, lane);
    else reset_store_rows<QT>(X, FX, (size_t)e0, W, nenv, WP, stg, rows, lane);
    wave_lds_sync();
  }
  }
  POB_TS(3);
  POB_TS(8);  // (marks the row as a reset wave's: the step kernels do not set stamp 8)
  POB_TS_WRITE();
  if (s.obs_masked) {
    // obs[:, mask] of the rows this launch resets (ABI v8; the step kernels fuse the same
    // gather): from the staged rows still in LDS, or -- rows written straight from registers --
    // read back from memory after this wave's stores (workgroup scope: the same CU's L1)
    const bool direct = std::is_same<QT, float>::value && few;
    if (direct) __threadfence_block();
    const int K = S.obs_mask_n;
    for (uint32_t m = rows; m != 0u; m &= m - 1u) {
      const int e = __builtin_ctz(m);
      const size_t rb = (size_t)(e0 + e);
      for (int c = lane; c < K; c += 64) {
        const int col = S.obs_mask[c];
        s.obs_masked[rb * K + c] = direct ? s.obs[rb * D + col] : stg[e * WP + col];
      }
    }
  }
  if (!active || k != 0) return;
  if (mode == RESET_FULL) {
    s.rng[2 * b] = R.rng0; s.rng[2 * b + 1] = R.rng1;
    s.reward[b] = 0.0f; s.done[b] = 0.0f;
    if (s.steps) s.steps[b] = 0.0f;
    if (s.truncation) s.truncation[b] = 0.0f;
    if (s.m0) s.m0[b] = 0.0f;
    if (s.m1) s.m1[b] = 0.0f;
    if (s.m2) s.m2[b] = 0.0f;
  } else if (mode == RESET_GYM) {
    if (s.steps) s.steps[b] = 0.0f;
  }
}

// LDS row pitch of k_reset's staging area: the widest row (obs or rot), odd so that the
// envs' rows start in distinct banks
static int reset_pitch(const pob_sys &S) {
  const int w = S.D > 4 * S.N ? S.D : 4 * S.N;
  return w | 1;
}

__global__ void k_any_done(const float *done, int B, uint32_t *flag) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const bool d = b < B && done[b] != 0.0f;
  const unsigned long long m = __ballot(d);
  if (m != 0ull && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

template <int KIND>
__global__ void k_default_qp(const void *sysp, int B, const float *qpos, const float *qvel, float *pos, float *rot,
                             float *vel, float *ang) {
  csys_t &S = *(csys_t *)(size_t)sysp;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int N = n_bodies<KIND>(S);
  float qp[POB_NJ], qv[POB_NJ];
#pragma unroll
  for (int j = 0; j < POB_NJ; ++j) { qp[j] = qpos[(size_t)b * POB_NJ + j]; qv[j] = qvel[(size_t)b * POB_NJ + j]; }
  Body bd;
  fk(S, qp, qv, bd);
  const size_t r3 = (size_t)b * N * 3, r4 = (size_t)b * N * 4;
  store_body<float>(bd, pos, rot, vel, ang, r3, r4);
  for (int i = POB_NDYN; i < N; ++i) {
#pragma unroll
    for (int c = 0; c < 3; ++c) { pos[r3 + 3 * i + c] = S.frozen_pos[i][c]; vel[r3 + 3 * i + c] = 0.0f; ang[r3 + 3 * i + c] = 0.0f; }
    rot[r4 + 4 * i] = 1.0f; rot[r4 + 4 * i + 1] = 0.0f; rot[r4 + 4 * i + 2] = 0.0f; rot[r4 + 4 * i + 3] = 0.0f;
  }
}

// --------------------------------------------------------------------------- random
__global__ void k_split(const uint32_t *key, int num, int first, int count, uint32_t *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  uint32_t o0, o1;
  tf_split(key[0], key[1], (uint32_t)num, (uint32_t)(first + i), o0, o1);
  out[2 * i] = o0; out[2 * i + 1] = o1;
}
// vmap(split)(keys, num): out[b, i] = split(keys[b], num)[i]
__global__ void k_split_batch(const uint32_t *keys, int B, int num, uint32_t *out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * num) return;
  const int b = t / num, i = t - b * num;
  uint32_t o0, o1;
  tf_split(keys[2 * b], keys[2 * b + 1], (uint32_t)num, (uint32_t)i, o0, o1);
  out[2 * t] = o0; out[2 * t + 1] = o1;
}
__global__ void k_uniform(const uint32_t *key, int n, int first, int count, float lo, float hi, float *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  out[i] = tf_uniform(key[0], key[1], (uint32_t)n, (uint32_t)(first + i), lo, hi);
}
// act = uniform(split(key)[1], (total, A), -1, 1)[first:first+B]
__global__ void k_actions(const uint32_t *key, int total, int first, int B, int A, float *act) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * A) return;
  uint32_t s0, s1;
  tf_split(key[0], key[1], 2u, 1u, s0, s1);
  act[i] = tf_uniform(s0, s1, (uint32_t)total * (uint32_t)A, (uint32_t)first * (uint32_t)A + (uint32_t)i, -1.0f, 1.0f);
}
__global__ void k_advance_key(uint32_t *key) {
  uint32_t o0, o1;
  tf_split(key[0], key[1], 2u, 0u, o0, o1);
  key[0] = o0; key[1] = o1;
}
__global__ void k_obs_gather(const float *obs, int B, int D, const int32_t *idx, int K, float *out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * K) return;
  const int b = t / K, k = t - b * K;
  out[t] = obs[(size_t)b * D + idx[k]];
}

// ============================================================================ C ABI
static thread_local char g_err[512] = "";
static int fail(int code, const char *msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}
static int hip_check(hipError_t e, const char *what) {
  if (e == hipSuccess) return POB_OK;
  snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
  return POB_EHIP;
}
static inline dim3 grid_for(int n, int bs) { return dim3((unsigned)((n + bs - 1) / bs)); }

// host-side launch helpers (kind / storage dispatch)
template <typename QT>
static void launch_reset(const pob_sys &S, dim3 g, hipStream_t st, const void *sp, int B, int mode,
                         const uint32_t *keys, const uint32_t *gin, uint32_t *gout, const uint32_t *flag,
                         const StatePtrs &p, int total = 0, int first = 0) {
  if (total <= 0) total = B;
  const int WP = reset_pitch(S);
  const size_t shm = sizeof(float) * 16 * (size_t)WP;  // 16 envs per block
  switch (S.kind) {
    case POB_HEAVENHELL: hipLaunchKernelGGL((k_reset<POB_HEAVENHELL, 64, QT>), g, dim3(64), shm, st, sp, B, mode, keys, gin, gout, flag, p, total, first, WP); break;
    case POB_GATHER: hipLaunchKernelGGL((k_reset<POB_GATHER, 64, QT>), g, dim3(64), shm, st, sp, B, mode, keys, gin, gout, flag, p, total, first, WP); break;
    case POB_TAG: hipLaunchKernelGGL((k_reset<POB_TAG, 64, QT>), g, dim3(64), shm, st, sp, B, mode, keys, gin, gout, flag, p, total, first, WP); break;
    default: hipLaunchKernelGGL((k_reset<POB_ANT, 64, QT>), g, dim3(64), shm, st, sp, B, mode, keys, gin, gout, flag, p, total, first, WP); break;
  }
}
// eight lanes per env up to this batch (the POB_OCTET_MAX_B environment variable, read at
// every launch, overrides it; 0 disables the eight-lane kernel)
static int octet_max_batch() {
  const char *e = getenv("POB_OCTET_MAX_B");
  return e ? atoi(e) : 16384;
}
// sixteen lanes per env (POB_HEXA_MAX_B overrides the per-kind limit below; 0 disables).
// Round 3 (the spring contact model): one wave per SIMD, B <= 4 envs x 4 SIMDs x n_cu (4 096
// on 256 CUs).  At two waves per SIMD the eight-lane
// kernel (one wave per SIMD up to B = 8 192) is faster: interleaved A/B, kernel ms
// (profiles/r3k/kernel_select.txt)
//                B:  5 120           6 144           7 168           8 192
//   HH  hex / oct:   0.0371/0.0366   0.0379/0.0365   0.0384/0.0372   0.0388/0.0373
//   TAG hex / oct:   0.0358/0.0346   0.0376/0.0348   0.0369/0.0350   0.0372/0.0354
// while at B = 4 096 the sixteen-lane kernel is 19 % faster (HH 0.0295 / 0.0363).
// Round 5 (brax's spelling: the wall walk dominates small batches): per kind, interleaved A/B
// (profiles/r6h_ab.txt, r6i_ab.txt), hex / oct kernel ms --
//   HH   B = 6 144 0.0715 / 0.0998, 8 192 0.0750 / 0.1009, 12 288 0.1036 / 0.1098, 16 384 0.1178 / 0.1149
//   TAG  B = 6 144 0.0502 / 0.0488, 8 192 0.0514 / 0.0541, 12 288 0.0751 / 0.0645
//   GA   B = 6 144 0.0374 / 0.0356, 8 192 0.0381 / 0.0369
// so the sixteen-lane kernel ran HH up to 3 waves per SIMD (48 x CUs: 12 288), TAG up to 2
// (8 192), GA and the stock ant up to 1.  Round 6 (the eight-lane kernel's contact pool for HH,
// profiles/r7k): HH B = 12 288 hex / oct 0.0924 / 0.0891, 8 192 0.0662 / 0.0803; TAG 6 144
// 0.0476 / 0.0457, 8 192 0.0490 / 0.0500 -- so HH up to 2 waves per SIMD too (32 x CUs).
static int hexa_max_batch(int n_cu, int kind) {
  const char *e = getenv("POB_HEXA_MAX_B");
  if (e) return atoi(e);
  return (kind == POB_HEAVENHELL || kind == POB_TAG ? 32 : 16) * n_cu;
}
template <typename QT, bool GACC>
static void launch_step_hex_g(int kind, hipStream_t st, const void *sp, int B, const StatePtrs &pi, const float *act,
                              const StatePtrs &po, uint32_t flags, int L, int n_cu) {
  const dim3 g((unsigned)((B + 3) / 4)), b(64);
  if (POB_HEX_PRIO && (B + 3) / 4 > 4 * n_cu) {  // two or more waves per SIMD (HH and TAG run that far)
    if (kind == POB_HEAVENHELL) {
      hipLaunchKernelGGL((k_step_hex<POB_HEAVENHELL, QT, GACC, true>), g, b, 0, st, sp, B, pi, act, po, flags, L);
      return;
    }
    if (kind == POB_TAG) {
      hipLaunchKernelGGL((k_step_hex<POB_TAG, QT, GACC, true>), g, b, 0, st, sp, B, pi, act, po, flags, L);
      return;
    }
  }
  switch (kind) {
    case POB_HEAVENHELL: hipLaunchKernelGGL((k_step_hex<POB_HEAVENHELL, QT, GACC>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
    case POB_GATHER: hipLaunchKernelGGL((k_step_hex<POB_GATHER, QT, GACC>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
    case POB_TAG: hipLaunchKernelGGL((k_step_hex<POB_TAG, QT, GACC>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
    default: hipLaunchKernelGGL((k_step_hex<POB_ANT, QT, GACC>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
  }
}
// Up to one wave per SIMD (B <= the SIMD count x 4 envs) the wave's dependency chain is the
// step time and the guard branches split it (GuardAcc, measured HH B=4 096 -3.5 %).  With two
// or more waves per SIMD the spring-model build measured the accumulator's VALU operations as
// the larger cost (B = 8 192: TAG / GA +1 %); with brax's spelling the accumulator wins there
// too for HH and TAG (HH B = 8 192 -1.7 %, 12 288 -2.4 %, TAG 8 192 -1 %; profiles/r6p), so
// HH and TAG take it at every batch, GA and the stock ant up to one wave per SIMD.
// POB_HEX_GACC=0/1 forces either.
template <typename QT>
static void launch_step_hex(int kind, int n_cu, hipStream_t st, const void *sp, int B, const StatePtrs &pi,
                            const float *act, const StatePtrs &po, uint32_t flags, int L) {
  const char *f = getenv("POB_HEX_GACC");
  const bool acc = f ? atoi(f) != 0 : (kind == POB_HEAVENHELL || kind == POB_TAG || (B + 3) / 4 <= 4 * n_cu);
  if (acc) launch_step_hex_g<QT, true>(kind, st, sp, B, pi, act, po, flags, L, n_cu);
  else launch_step_hex_g<QT, false>(kind, st, sp, B, pi, act, po, flags, L, n_cu);
}
template <typename QT, bool GACC>
static void launch_step_oct_g(int kind, hipStream_t st, const void *sp, int B, const StatePtrs &pi, const float *act,
                              const StatePtrs &po, uint32_t flags, int L) {
  const dim3 g((unsigned)((B + 7) / 8)), b(64);
  switch (kind) {
    case POB_HEAVENHELL: hipLaunchKernelGGL((k_step_oct<POB_HEAVENHELL, QT, GACC>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
    case POB_GATHER: hipLaunchKernelGGL((k_step_oct<POB_GATHER, QT, GACC>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
    case POB_TAG: hipLaunchKernelGGL((k_step_oct<POB_TAG, QT, GACC>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
    default: hipLaunchKernelGGL((k_step_oct<POB_ANT, QT, GACC>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
  }
}
// As for the sixteen-lane kernel: branch-free guards (GuardAcc) while the waves fit one per
// SIMD (B <= 8 envs x the SIMD count), the branch guards above.  POB_OCT_GACC=0/1 forces either.
template <typename QT>
static void launch_step_oct(int kind, int n_cu, hipStream_t st, const void *sp, int B, const StatePtrs &pi,
                            const float *act, const StatePtrs &po, uint32_t flags, int L) {
  const char *f = getenv("POB_OCT_GACC");
  const bool acc = f ? atoi(f) != 0 : (B + 7) / 8 <= 4 * n_cu;
  if (acc) launch_step_oct_g<QT, true>(kind, st, sp, B, pi, act, po, flags, L);
  else launch_step_oct_g<QT, false>(kind, st, sp, B, pi, act, po, flags, L);
}
// The fast + fix-up launches per kind (bit 1 << kind, mixed 16): HH B = 65 536 0.1877 ->
// 0.1634 ms, TAG 0.1192 -> 0.1055, GA 0.1148 -> 0.1145, mixed fp16 B = 32 768 0.1281 -> 0.1316
// (profiles/r6b_ab.txt, r6c_ab.txt); since round 6's LDS contact pool (no scratch in the fast
// launch) the mixed launch too: fp16 B = 32 768 0.1231 -> 0.1149 ms (profiles/r7h).
// POB_QUAD_SPLIT=0 / 1 forces the one-launch form / the split.
#ifndef POB_QUAD_SPLIT_KINDS
#define POB_QUAD_SPLIT_KINDS 23
#endif
static bool quad_split_launch(int kind) {
  const char *f = getenv("POB_QUAD_SPLIT");
  if (f) return atoi(f) != 0;
  return ((POB_QUAD_SPLIT_KINDS >> (kind < 0 ? 4 : kind)) & 1) != 0;
}
static uint32_t quad_force_fixup() {
  const char *f = getenv("POB_QUAD_FORCE_FIXUP");
  return f && atoi(f) != 0 ? POB_F_INT_FORCE_FIXUP : 0u;
}
template <typename QT>
static void launch_step_quad(int kind, bool legacy, int n_cu, hipStream_t st, const void *sp, int B,
                             const StatePtrs &pi, const float *act, const StatePtrs &po, uint32_t flags, int L) {
  // Batches of at most one wave per CU launch one-wave blocks, so each wave gets a CU (its
  // scalar unit, LDS and instruction cache) to itself instead of four waves sharing 1/4 of
  // the CUs; larger batches use 256-thread blocks (the kernel is block-size agnostic)
  const int bs = 4 * B <= 64 * 256 ? 64 : 256;
  const dim3 g = grid_for(4 * B, bs), b(bs);
  if (legacy) {
    switch (kind) {
      case POB_HEAVENHELL: hipLaunchKernelGGL((k_step_legacy<POB_HEAVENHELL, QT>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
      case POB_GATHER: hipLaunchKernelGGL((k_step_legacy<POB_GATHER, QT>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
      case POB_TAG: hipLaunchKernelGGL((k_step_legacy<POB_TAG, QT>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
      default: hipLaunchKernelGGL((k_step_legacy<POB_ANT, QT>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
    }
    return;
  }
  if (kind == POB_GATHER && (size_t)4 * B <= (size_t)3 * 64 * 4 * n_cu) {
    hipLaunchKernelGGL((k_step_quad_ga3<QT>), g, b, 0, st, sp, B, pi, act, po, flags, L);
    return;
  }
  // walls: the fast launch, then the fix-up launch of its overflowing waves (MODE 1 / 2 above;
  // without the caller's mark array the one-launch form)
  const bool split = quad_split_launch(kind) && po.ovf_mark != nullptr;
  flags |= split ? quad_force_fixup() : 0u;
  switch (kind) {
    case POB_HEAVENHELL:
      if (split) {
        hipLaunchKernelGGL((k_step_quad<POB_HEAVENHELL, QT, 1>), g, b, 0, st, sp, B, pi, act, po, flags, L);
        hipLaunchKernelGGL((k_step_quad<POB_HEAVENHELL, QT, 2>), g, b, 0, st, sp, B, pi, act, po, flags, L);
      } else {
        hipLaunchKernelGGL((k_step_quad<POB_HEAVENHELL, QT>), g, b, 0, st, sp, B, pi, act, po, flags, L);
      }
      break;
    case POB_GATHER:
      if (split) {
        hipLaunchKernelGGL((k_step_quad<POB_GATHER, QT, 1>), g, b, 0, st, sp, B, pi, act, po, flags, L);
        hipLaunchKernelGGL((k_step_quad<POB_GATHER, QT, 2>), g, b, 0, st, sp, B, pi, act, po, flags, L);
      } else {
        hipLaunchKernelGGL((k_step_quad<POB_GATHER, QT>), g, b, 0, st, sp, B, pi, act, po, flags, L);
      }
      break;
    case POB_TAG:
      if (split) {
        hipLaunchKernelGGL((k_step_quad<POB_TAG, QT, 1>), g, b, 0, st, sp, B, pi, act, po, flags, L);
        hipLaunchKernelGGL((k_step_quad<POB_TAG, QT, 2>), g, b, 0, st, sp, B, pi, act, po, flags, L);
      } else {
        hipLaunchKernelGGL((k_step_quad<POB_TAG, QT>), g, b, 0, st, sp, B, pi, act, po, flags, L);
      }
      break;
    default: hipLaunchKernelGGL((k_step_quad<POB_ANT, QT>), g, b, 0, st, sp, B, pi, act, po, flags, L); break;
  }
}
extern "C" {

int pob_abi_version(void) { return POB_ABI_VERSION; }
const char *pob_last_error(void) { return g_err; }

int pob_default_params(pob_params *p) {
  if (!p) return fail(POB_EINVAL, "params is NULL");
  pob::default_params(*p);
  return POB_OK;
}

// Device tables of destroyed envs.  pob_env_destroy never calls the HIP runtime: a handle
// may be dropped while some stream is being captured into a hipGraph (a Python finaliser run
// by the garbage collector in the middle of a capture), and hipFree there invalidates the
// capture (hipErrorStreamCaptureInvalidated).  The tables (~4 KB per env) are freed by the
// next pob_env_create, which cannot itself run inside a capture (it allocates).
static std::mutex g_grave_mu;
static std::vector<void *> g_grave;

static void drain_grave() {
  std::vector<void *> dead;
  {
    std::lock_guard<std::mutex> lk(g_grave_mu);
    dead.swap(g_grave);
  }
  for (void *p : dead) (void)hipFree(p);
}

int pob_env_create(int kind, const pob_params *p, pob_env **out) {
  if (!out) return fail(POB_EINVAL, "out is NULL");
  *out = nullptr;
  drain_grave();
  pob_params prm;
  if (p) prm = *p; else pob::default_params(prm);
  pob_env *e = new (std::nothrow) pob_env();
  if (!e) return fail(POB_ENOMEM, "out of host memory");
  e->params = prm;
  if (const char *msg = pob::build_system(kind, prm, e->sys)) { delete e; return fail(POB_EINVAL, msg); }
  int rc = hip_check(hipGetDevice(&e->device), "hipGetDevice");
  if (!rc) rc = hip_check(hipDeviceGetAttribute(&e->n_cu, hipDeviceAttributeMultiprocessorCount, e->device),
                          "hipDeviceGetAttribute(CUs)");
  if (rc) { delete e; return rc; }
  rc = hip_check(hipMalloc(&e->d_scratch, 64), "hipMalloc(scratch)");
  if (rc) { delete e; return rc; }
  if (kind == POB_GATHER) {
    static float tmp[3 * 4096];
    const int n = pob::gather_grid(prm, tmp, 4096);
    rc = hip_check(hipMalloc(&e->d_grid, sizeof(float) * 3 * n), "hipMalloc(grid)");
    if (!rc) rc = hip_check(hipMemcpy(e->d_grid, tmp, sizeof(float) * 3 * n, hipMemcpyHostToDevice), "hipMemcpy(grid)");
    if (rc) { (void)hipFree(e->d_scratch); delete e; return rc; }
    e->sys.grid = e->d_grid;
  }
  rc = hip_check(hipMalloc(&e->d_sys, sizeof(pob_sys)), "hipMalloc(sys)");
  if (!rc) rc = hip_check(hipMemcpy(e->d_sys, &e->sys, sizeof(pob_sys), hipMemcpyHostToDevice), "hipMemcpy(sys)");
  if (rc) { if (e->d_grid) (void)hipFree(e->d_grid); (void)hipFree(e->d_scratch); delete e; return rc; }
  *out = e;
  return POB_OK;
}

void pob_env_destroy(pob_env *e) {
  if (!e) return;
  {
    std::lock_guard<std::mutex> lk(g_grave_mu);
    for (void *p : {(void *)e->d_grid, (void *)e->d_scratch, (void *)e->d_sys})
      if (p) g_grave.push_back(p);
  }
  delete e;
}

int pob_release_deferred(void) {
  size_t n;
  {
    std::lock_guard<std::mutex> lk(g_grave_mu);
    n = g_grave.size();
  }
  drain_grave();
  return (int)n;
}

int pob_env_dims(const pob_env *e, int *n, int *d, int *a) {
  if (!e) return fail(POB_EINVAL, "env is NULL");
  if (n) *n = e->sys.N;
  if (d) *d = e->sys.D;
  if (a) *a = POB_NJ;
  return POB_OK;
}

int pob_env_default_angle(const pob_env *e, float *out8) {
  if (!e || !out8) return fail(POB_EINVAL, "NULL argument");
  for (int j = 0; j < POB_NJ; ++j) out8[j] = e->sys.default_angle[j];
  return POB_OK;
}

static int check_state(const pob_state *s, bool need_rng) {
  if (!s) return fail(POB_EINVAL, "state is NULL");
  if (!s->pos || !s->rot || !s->vel || !s->ang || !s->obs || !s->reward || !s->done)
    return fail(POB_EINVAL, "state: qp/obs/reward/done pointers are required");
  if (need_rng && !s->rng) return fail(POB_EINVAL, "state: rng pointer is required");
  return POB_OK;
}

int pob_reset(pob_env *e, int B, const uint32_t *keys, const pob_state *out, void *stream) {
  if (!e) return fail(POB_EINVAL, "env is NULL");
  if (B <= 0) return fail(POB_EINVAL, "batch size must be positive");
  if (!keys) return fail(POB_EINVAL, "keys is NULL");
  if (int rc = check_state(out, true)) return rc;
  if (out->first_pos && (!out->first_rot || !out->first_vel || !out->first_ang || !out->first_obs))
    return fail(POB_EINVAL, "state: first_* pointers must be all set or all NULL");
  if (out->obs_masked && e->sys.obs_mask_n == 0) return fail(POB_EINVAL, "obs_masked given but the env has no observation mask");
  hipStream_t st = (hipStream_t)stream;
  const StatePtrs p = to_ptrs(*out);
  if (e->sys.qp_f16)
    launch_reset<__half>(e->sys, grid_for(B, 16), st, e->d_sys, B, RESET_FULL, keys, nullptr, nullptr, nullptr, p);
  else
    launch_reset<float>(e->sys, grid_for(B, 16), st, e->d_sys, B, RESET_FULL, keys, nullptr, nullptr, nullptr, p);
  return hip_check(hipGetLastError(), "k_reset launch");
}

// The coalesced LDS-staged state load (POB_F_STAGED) is opt-in (POB_STAGE=1, read at every
// launch): since the quad / octet / hexa kernels hold every body in its owner lane, per-lane
// loads of the owned rows (one round trip, no LDS pass, frozen rows never read) are as fast
// or faster at every batch size and kind -- HH B = 65 536 0.0935 -> 0.0914 ms, GA B = 16 384
// 0.0766 -> 0.0728 ms, GA B = 65 536 0.132 -> 0.125 ms (profiles/r2q).  Staging needs 16-B
// aligned qp rows and 16 envs' rows of the widest array (rot) to fit the wave's region.
static bool can_stage(const pob_env *e, const pob_state *in) {
  const char *ev = getenv("POB_STAGE");
  if (!ev || atoi(ev) == 0) return false;
  const uintptr_t m = (uintptr_t)in->pos | (uintptr_t)in->rot | (uintptr_t)in->vel | (uintptr_t)in->ang;
  return (m & 15u) == 0 && 16 * e->sys.N * 4 <= POB_STAGE_FLOATS;
}

static int check_step(const pob_env *e, int B, const pob_state *in, const float *act, const pob_state *out,
                      uint32_t flags, int episode_length) {
  if (!e) return fail(POB_EINVAL, "env is NULL");
  if (B <= 0) return fail(POB_EINVAL, "batch size must be positive");
  if (!act) return fail(POB_EINVAL, "action is NULL");
  if (int rc = check_state(in, true)) return rc;
  if (int rc = check_state(out, true)) return rc;
  if (flags & ~(uint32_t)POB_F_PUBLIC) return fail(POB_EINVAL, "unknown step flag bits");
  if ((flags & POB_F_EPISODE) && episode_length <= 0) return fail(POB_EINVAL, "episode_length must be positive");
  if ((flags & POB_F_AUTORESET) &&
      (!in->first_pos || !in->first_rot || !in->first_vel || !in->first_ang || !in->first_obs ||
       !out->first_pos || !out->first_rot || !out->first_vel || !out->first_ang || !out->first_obs))
    return fail(POB_EINVAL, "AUTORESET needs first_qp/first_obs in both states");
  if ((flags & POB_F_EPISODE) && (!out->steps || !out->truncation)) return fail(POB_EINVAL, "EPISODE needs steps/truncation");
  if (out->obs_masked && e->sys.obs_mask_n == 0) return fail(POB_EINVAL, "obs_masked given but the env has no observation mask");
  return POB_OK;
}

int pob_step(pob_env *e, int B, const pob_state *in, const float *act, const pob_state *out, uint32_t flags,
             int episode_length, void *stream) {
  if (int rc = check_step(e, B, in, act, out, flags, episode_length)) return rc;
  flags &= ~POB_F_INTERNAL;
  if (can_stage(e, in)) flags |= POB_F_STAGED;
  hipStream_t st = (hipStream_t)stream;
  const StatePtrs pi = to_ptrs(*in), po = to_ptrs(*out);
  const void *sp = (const void *)e->d_sys;
  const bool hex = e->sys.oct_ok && !e->sys.legacy && B <= hexa_max_batch(e->n_cu, e->sys.kind) &&  // legacy: lane quads only
                   e->sys.n_walls <= hex_max_walls(e->sys.kind);
  const bool oct = e->sys.oct_ok && !e->sys.legacy && B <= octet_max_batch() &&
                   e->sys.n_walls <= hex_max_walls(e->sys.kind);
  if (hex && e->sys.qp_f16) launch_step_hex<__half>(e->sys.kind, e->n_cu, st, sp, B, pi, act, po, flags, episode_length);
  else if (hex) launch_step_hex<float>(e->sys.kind, e->n_cu, st, sp, B, pi, act, po, flags, episode_length);
  else if (oct && e->sys.qp_f16) launch_step_oct<__half>(e->sys.kind, e->n_cu, st, sp, B, pi, act, po, flags, episode_length);
  else if (oct) launch_step_oct<float>(e->sys.kind, e->n_cu, st, sp, B, pi, act, po, flags, episode_length);
  else if (e->sys.qp_f16) launch_step_quad<__half>(e->sys.kind, e->sys.legacy, e->n_cu, st, sp, B, pi, act, po, flags, episode_length);
  else launch_step_quad<float>(e->sys.kind, e->sys.legacy, e->n_cu, st, sp, B, pi, act, po, flags, episode_length);
  return hip_check(hipGetLastError(), "k_step launch");
}

int pob_step_mixed(int n, pob_env *const *envs, const int *B, const pob_state *in, const float *const *act,
                   const pob_state *out, uint32_t flags, int episode_length, void *stream) {
  if (n < 1 || n > POB_MIX_MAX) return fail(POB_EINVAL, "mixed step: 1 <= n <= POB_MIX_MAX envs");
  if (!envs || !B || !in || !act || !out) return fail(POB_EINVAL, "NULL argument");
  MixArgs A;
  memset(&A, 0, sizeof(A));
  A.n = n;
  flags &= ~POB_F_INTERNAL;
  bool stage = true, marks = true;
  long long blk = 0;
  for (int k = 0; k < n; ++k) {
    const pob_env *e = envs[k];
    if (int rc = check_step(e, B[k], &in[k], act[k], &out[k], flags, episode_length)) return rc;
    if (e->sys.qp_f16 != envs[0]->sys.qp_f16) return fail(POB_EINVAL, "mixed step: envs must share qp_storage");
    if (e->sys.legacy) return fail(POB_EINVAL, "mixed step: legacy-spring envs step through pob_step");
    if (e->device != envs[0]->device) return fail(POB_EINVAL, "mixed step: envs must live on one device");
    stage = stage && can_stage(e, &in[k]);
    marks = marks && out[k].ovf_mark != nullptr;
    MixSeg &s = A.s[k];
    s.sysp = e->d_sys; s.act = act[k]; s.in = to_ptrs(in[k]); s.out = to_ptrs(out[k]);
    s.B = B[k]; s.blk0 = (int)blk;
    blk += (4LL * B[k] + 255) / 256;
    if (blk > INT_MAX) return fail(POB_EINVAL, "mixed step: batch too large");
  }
  for (int k = n; k < POB_MIX_MAX; ++k) { A.s[k] = A.s[n - 1]; A.s[k].blk0 = INT_MAX; }
  if (stage) flags |= POB_F_STAGED;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)blk);
  if (quad_split_launch(POB_MIXED) && marks) {  // the fast launch, then the fix-up launch of its overflowing waves
    flags |= quad_force_fixup();
    if (envs[0]->sys.qp_f16) {
      hipLaunchKernelGGL((k_step_mixed<__half, 1>), g, dim3(256), 0, st, A, flags, episode_length);
      hipLaunchKernelGGL((k_step_mixed<__half, 2>), g, dim3(256), 0, st, A, flags, episode_length);
    } else {
      hipLaunchKernelGGL((k_step_mixed<float, 1>), g, dim3(256), 0, st, A, flags, episode_length);
      hipLaunchKernelGGL((k_step_mixed<float, 2>), g, dim3(256), 0, st, A, flags, episode_length);
    }
  } else if (envs[0]->sys.qp_f16) {
    hipLaunchKernelGGL((k_step_mixed<__half>), g, dim3(256), 0, st, A, flags, episode_length);
  } else {
    hipLaunchKernelGGL((k_step_mixed<float>), g, dim3(256), 0, st, A, flags, episode_length);
  }
  return hip_check(hipGetLastError(), "k_step_mixed launch");
}

int pob_reset_where_done(pob_env *e, int B, int mode, const uint32_t *gym_in, uint32_t *gym_out, const pob_state *s,
                         void *stream) {
  return pob_reset_where_done_shard(e, B, B, 0, mode, gym_in, gym_out, s, stream);
}

int pob_reset_where_done_shard(pob_env *e, int B, int total, int first, int mode, const uint32_t *gym_in,
                               uint32_t *gym_out, const pob_state *s, void *stream) {
  if (!e) return fail(POB_EINVAL, "env is NULL");
  if (B <= 0) return fail(POB_EINVAL, "batch size must be positive");
  if (first < 0 || total < B || (long long)first + B > total || total >= INT_MAX)
    return fail(POB_EINVAL, "shard [first, first + B) must lie in [0, total)");
  if (int rc = check_state(s, true)) return rc;
  if (mode != POB_RESET_GYM && mode != POB_RESET_OWN) return fail(POB_EINVAL, "unknown reset mode");
  if (mode == POB_RESET_GYM && (!gym_in || !gym_out)) return fail(POB_EINVAL, "gym mode needs gym_key_in/out");
  // block 0 writes gym_out and clears *any_done_clear while every block reads gym_in / *any_done
  if (mode == POB_RESET_GYM && gym_out < gym_in + 2 && gym_in < gym_out + 2)
    return fail(POB_EINVAL, "gym_key_in and gym_key_out must not overlap");
  if (s->any_done_clear && s->any_done_clear == s->any_done)
    return fail(POB_EINVAL, "any_done_clear must not alias any_done");
  if (s->obs_masked && e->sys.obs_mask_n == 0) return fail(POB_EINVAL, "obs_masked given but the env has no observation mask");
  hipStream_t st = (hipStream_t)stream;
  const StatePtrs p = to_ptrs(*s);
  const uint32_t *flag = s->any_done;
  if (mode == POB_RESET_GYM && !flag) {
    int rc = hip_check(hipMemsetAsync(e->d_scratch, 0, 16, st), "hipMemsetAsync");
    if (rc) return rc;
    hipLaunchKernelGGL(k_any_done, grid_for(B, 256), dim3(256), 0, st, s->done, B, e->d_scratch);
    flag = e->d_scratch;
  }
  const int kmode = mode == POB_RESET_GYM ? RESET_GYM : RESET_OWN;
  if (e->sys.qp_f16)
    launch_reset<__half>(e->sys, grid_for(B, 16), st, e->d_sys, B, kmode, nullptr, gym_in, gym_out, flag, p, total,
                         first);
  else
    launch_reset<float>(e->sys, grid_for(B, 16), st, e->d_sys, B, kmode, nullptr, gym_in, gym_out, flag, p, total,
                        first);
  return hip_check(hipGetLastError(), "k_reset(where done) launch");
}

int pob_default_qp(pob_env *e, int B, const float *qpos, const float *qvel, float *pos, float *rot, float *vel,
                   float *ang, void *stream) {
  if (!e) return fail(POB_EINVAL, "env is NULL");
  if (B <= 0) return fail(POB_EINVAL, "batch size must be positive");
  if (!qpos || !qvel || !pos || !rot || !vel || !ang) return fail(POB_EINVAL, "NULL argument");
  hipStream_t st = (hipStream_t)stream;
  switch (e->sys.kind) {
    case POB_HEAVENHELL: hipLaunchKernelGGL((k_default_qp<POB_HEAVENHELL>), grid_for(B, 64), dim3(64), 0, st, (const void *)e->d_sys, B, qpos, qvel, pos, rot, vel, ang); break;
    case POB_GATHER: hipLaunchKernelGGL((k_default_qp<POB_GATHER>), grid_for(B, 64), dim3(64), 0, st, (const void *)e->d_sys, B, qpos, qvel, pos, rot, vel, ang); break;
    case POB_TAG: hipLaunchKernelGGL((k_default_qp<POB_TAG>), grid_for(B, 64), dim3(64), 0, st, (const void *)e->d_sys, B, qpos, qvel, pos, rot, vel, ang); break;
    default: hipLaunchKernelGGL((k_default_qp<POB_ANT>), grid_for(B, 64), dim3(64), 0, st, (const void *)e->d_sys, B, qpos, qvel, pos, rot, vel, ang); break;
  }
  return hip_check(hipGetLastError(), "k_default_qp launch");
}

int pob_random_split(const uint32_t *key, int num, int first, int count, uint32_t *out, void *stream) {
  if (!key || !out) return fail(POB_EINVAL, "NULL argument");
  if (num <= 0 || first < 0 || count < 0 || first + count > num) return fail(POB_EINVAL, "bad split range");
  if (count == 0) return POB_OK;
  hipLaunchKernelGGL(k_split, grid_for(count, 256), dim3(256), 0, (hipStream_t)stream, key, num, first, count, out);
  return hip_check(hipGetLastError(), "k_split launch");
}

int pob_random_split_batch(const uint32_t *keys, int B, int num, uint32_t *out, void *stream) {
  if (!keys || !out) return fail(POB_EINVAL, "NULL argument");
  if (B < 0 || num <= 0 || (long long)B * num >= INT_MAX) return fail(POB_EINVAL, "bad batched split shape");
  if (B == 0) return POB_OK;
  hipLaunchKernelGGL(k_split_batch, grid_for(B * num, 256), dim3(256), 0, (hipStream_t)stream, keys, B, num, out);
  return hip_check(hipGetLastError(), "k_split_batch launch");
}

int pob_random_uniform(const uint32_t *key, int n, int first, int count, float lo, float hi, float *out, void *stream) {
  if (!key || !out) return fail(POB_EINVAL, "NULL argument");
  if (n <= 0 || first < 0 || count < 0 || first + count > n) return fail(POB_EINVAL, "bad uniform range");
  if (count == 0) return POB_OK;
  hipLaunchKernelGGL(k_uniform, grid_for(count, 256), dim3(256), 0, (hipStream_t)stream, key, n, first, count, lo, hi, out);
  return hip_check(hipGetLastError(), "k_uniform launch");
}

int pob_random_actions(uint32_t *key_io, int total, int first, int B, int A, float *act, void *stream) {
  if (!key_io || !act) return fail(POB_EINVAL, "NULL argument");
  if (B <= 0 || A <= 0 || first < 0 || first + B > total) return fail(POB_EINVAL, "bad action shard");
  if ((long long)total * A >= 4294967295LL) return fail(POB_EINVAL, "too many action elements");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_actions, grid_for(B * A, 256), dim3(256), 0, st, key_io, total, first, B, A, act);
  hipLaunchKernelGGL(k_advance_key, dim3(1), dim3(1), 0, st, key_io);
  return hip_check(hipGetLastError(), "k_actions launch");
}

int pob_env_set_obs_mask(pob_env *e, const int32_t *idx, int K) {
  if (!e) return fail(POB_EINVAL, "env is NULL");
  if (K < 0 || K > POB_MAX_OBS_MASK) return fail(POB_EINVAL, "obs mask: K out of range");
  if (K > 0 && !idx) return fail(POB_EINVAL, "obs mask: idx is NULL");
  for (int i = 0; i < K; ++i)
    if (idx[i] < 0 || idx[i] >= e->sys.D) return fail(POB_EINVAL, "obs mask: index out of range for the observation");
  e->sys.obs_mask_n = K;
  for (int i = 0; i < POB_MAX_OBS_MASK; ++i) e->sys.obs_mask[i] = (int16_t)(i < K ? idx[i] : 0);
  return hip_check(hipMemcpy(e->d_sys, &e->sys, sizeof(pob_sys), hipMemcpyHostToDevice), "hipMemcpy(sys)");
}

int pob_obs_gather(const float *obs, int B, int D, const int32_t *idx, int K, float *out, void *stream) {
  if (!obs || !idx || !out) return fail(POB_EINVAL, "NULL argument");
  if (B <= 0 || D <= 0 || K <= 0) return fail(POB_EINVAL, "bad shape");
  hipLaunchKernelGGL(k_obs_gather, grid_for(B * K, 256), dim3(256), 0, (hipStream_t)stream, obs, B, D, idx, K, out);
  return hip_check(hipGetLastError(), "k_obs_gather launch");
}

}  // extern "C"

#ifdef POB_EXP_TIMING
// timing experiment only: per wave [HW_ID, XCC_ID, t0..t5] of the last step launch
extern "C" __attribute__((visibility("default"))) int pob_debug_timing(unsigned long long *host, int waves) {
  if (waves > POB_TS_WAVES) waves = POB_TS_WAVES;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(pob_ts_buf), sizeof(unsigned long long) * POB_TS_ROW * waves) == hipSuccess ? 0 : -1;
}
#endif
