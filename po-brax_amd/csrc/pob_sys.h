// pob_sys.h -- static system tables of one env instance (host-built, passed to every
// kernel by value as a kernel argument, so the wave reads them through the scalar cache).
//
// Built by pob_system.cpp from the constructor kwargs exactly as brax.System(cfg) is built
// from extend_ant_cfg(...) in the reference (ant_heavenhell.py:13-39, ant_gather.py:17-39,
// ant_tag.py:13-25, envs/utils.py:6-119).  The ant's TOPOLOGY is compile-time (8 revolute
// joints, parent(j) = j odd ? j : 0, child(j) = j + 1; ground contacts on bodies
// 0,2,4,6,8); every number (offsets, axes, limits, masses, capsules, walls) is data.
#pragma once
#include <stddef.h>
#include <stdint.h>

#define POB_NDYN 9      // dynamic ant bodies
#define POB_NJ 8        // revolute joints == actuators == action dim
#define POB_NGROUND 5   // collide_include Ant x Ground pairs
#define POB_MAXW 8      // walls (HH T-maze: 8, arenas: 4)
#define POB_MAXB 43     // bodies (GA: 11 + up to 32 objects)
#define POB_MAXOBJ 32   // GA apples + bombs
#define POB_MAXBINS 32  // GA 2 * n_bins

// per-leg table of the four-lanes-per-env kernel (pob_quad.h), leg k = joints 2k, 2k+1,
// bodies 2k+1, 2k+2, ground collider k+1; staged in LDS once per block
#define POB_LEG_JOINT(jl) (16 * (jl))   // off_p(3) off_c(3) axis(3) tan_lo tan_hi 0 lim_lo lim_hi jdamp strength
#define POB_LEG_BODY(l) (32 + 8 * ((l) - 1))  // inv_mass cap_r cap_end[2][3]   (l = 1, 2)
#define POB_LEG_GROUND 48               // ground_end(3) ground_r
#define POB_LEG_FLOATS 52
// wall rows staged behind the leg table: centre x, y, cos, sin, half-extent x, y (every
// wall shares centre z and half-extent z: pob_sys::wall_cz / wall_hz).  4 leg rows + 8 wall
// rows = 1 KiB, which keeps the quad kernel's LDS at 40 KiB per block (4 blocks per CU).
#define POB_WALL_FLOATS 6
#define POB_TAB_FLOATS (4 * POB_LEG_FLOATS + POB_MAXW * POB_WALL_FLOATS)
// per-role rows of the eight-lanes-per-env kernel (pob_octet.h: OT_* offsets)
#define POB_OCT_FLOATS 40
// per-role rows of the sixteen-lanes-per-env kernel (pob_hexa.h: HT_* offsets)
#define POB_HEX_FLOATS 36

#define POB_MAX_OBS_MASK 256  // >= the largest observation (AntGather: 211)

// Per (wall, face axis k) constants of the capsule x TriangulatedBox forms (pob_mesh.h): a
// face of axis k has half extents (ha, hb) = (hy, hz) / (hx, hz) / (hx, hy) and edges of
// three classes -- along a (length 2 ha), along b (2 hb), the diagonal -- each with brax's
// segment terms il = 1 / (len + 1e-6), hl = len / 2, idd = 1 / (d.d + 1e-6) (oracle bseg_make
// of the edge: d.d is exactly the one nonzero square, or the FMA of the two for the diagonal),
// then e_d = d.d of the diagonal and the two triangles' 1 / det (oracle btri_make).  The
// same IEEE operations as the oracle's per-face evaluation (sqrt, division and fma are
// correctly rounded here and there), formed once per env instead of per face evaluation.
#define POB_FACE_FLOATS 12
#define POB_FC_TAB_FLOATS (POB_MAXW * 3 * POB_FACE_FLOATS)  // pob_sys::face_c
#define POB_FC_IL(c) (3 * (c))
#define POB_FC_HL(c) (3 * (c) + 1)
#define POB_FC_IDD(c) (3 * (c) + 2)
#define POB_FC_ED 9
#define POB_FC_IDET(t) (10 + (t))
static inline void pob_face_consts(const float ha, const float hb, float *o) {
  const float ha2 = ha + ha, hb2 = hb + hb;
  const float dA = ha2 * ha2, dB = hb2 * hb2;
  const float e_d = __builtin_fmaf(hb2, hb2, ha2 * ha2);
  const float dd[3] = {dA, dB, e_d};
  for (int c = 0; c < 3; ++c) {
    const float len = __builtin_sqrtf(dd[c]);
    o[POB_FC_IL(c)] = 1.0f / (len + 1e-6f);
    o[POB_FC_HL(c)] = len * 0.5f;
    o[POB_FC_IDD(c)] = 1.0f / (dd[c] + 1e-6f);
  }
  o[POB_FC_ED] = e_d;
  // t0 = (V0, V1, V2): a = dA, b = dA, c = e_d; t1 = (V0, V2, V3): a = e_d, b = dB, c = dB
  o[POB_FC_IDET(0)] = 1.0f / __builtin_fmaf(dA, e_d, -(dA * dA));
  o[POB_FC_IDET(1)] = 1.0f / __builtin_fmaf(e_d, dB, -(dB * dB));
}

struct pob_sys {
  int kind, N, D, n_obj;
  int substeps, n_walls, n_grid;
  int ga_n_apples, ga_n_bins;
  // integrator (dt_sub = dt / substeps)
  float h, half_h, inv_h, lin_damp, ang_damp, gz;
  float inv_mass[POB_NDYN];
  // joints: parent/child offsets, hinge axis and reference direction (body frame),
  // limits (rad), angular damping, actuator strength, default angle
  float off_p[POB_NJ][3], off_c[POB_NJ][3], axis[POB_NJ][3], ref[POB_NJ][3];
  float lim_lo[POB_NJ], lim_hi[POB_NJ], jdamp[POB_NJ], strength[POB_NJ], default_angle[POB_NJ];
  float tan_lo[POB_NJ], tan_hi[POB_NJ];  // torque actuator gate (pob_math.h actuator_inside)
  // one capsule per dynamic body: segment end points (body frame) and radius; body 0's
  // segment is degenerate (a sphere: one end point)
  float cap_end[POB_NDYN][2][3], cap_r[POB_NDYN];
  float ground_end[POB_NGROUND][3], ground_r[POB_NGROUND];
  // walls: box centre (world), half extents, z-rotation cos/sin
  float wall_c[POB_MAXW][3], wall_h[POB_MAXW][3], wall_cos[POB_MAXW], wall_sin[POB_MAXW];
  // broadphase: world AABB of each wall grown by (capsule reach + radius + margin); a
  // lane skips a wall when none of its body centres falls inside it (exact: every triangle of
  // a culled wall is farther than r from the capsule, no contact)
  float wall_lo[POB_MAXW][3], wall_hi[POB_MAXW][3];
  float wall_cz, wall_hz;  // the common centre z / half-extent z of every wall
  alignas(16) float face_c[POB_MAXW][3][POB_FACE_FLOATS];  // pob_face_consts of every wall's three axes (rows of 48 B, 16-B aligned)
  float friction, s_pos, half_s_ang;
  // legacy spring dynamics (pob_params.legacy_spring; brax <= 0.0.12): joint stiffness, spring
  // damping, limit strength, Baumgarte rate (baumgarte_erp * substeps / dt)
  int legacy;
  float k_spring, c_spring, k_limit, erp;
  // default_qp rows of the frozen bodies (index >= 9)
  float frozen_pos[POB_MAXB][3];
  // env parameters (float32 as the reference's jnp scalars)
  float hh_hhp[2][2], hh_priest[2], hh_visible_radius, hh_dying_cost;
  float ga_catch_range, ga_sensor_range, ga_half_span, ga_bin_res, ga_dying_cost, ga_waiting[3];
  float tag_tag_radius, tag_visible_radius, tag_target_step, tag_min_spawn_distance;
  float tag_cage_xy[2], tag_dying_cost;
  float leg[4][POB_LEG_FLOATS];  // gathered copies of the per-leg rows above
  float wall_row[POB_MAXW][POB_WALL_FLOATS];  // the walls again, one row each (follows leg)
  float oct[8][POB_OCT_FLOATS];  // eight-lane kernel: rows A_0..A_3 (hips), B_0..B_3 (knees)
  float hex[16][POB_HEX_FLOATS];  // sixteen-lane kernel: role rows (pob_hexa.h)
  int oct_ok;         // the Ant pattern the eight-lane kernel assumes holds (torso sphere)
  float ctrl_dt;      // sys.config.dt (float32 proto field): stock ant forward reward
  int qp_f16;         // qp stored as binary16 (pob_params.qp_storage)
  int torso_point;    // body 0's capsule end and ground end are the body origin (the Ant torso
                      // sphere): its contact points are x itself, no rotation needed
  const float *grid;  // GA object grid (n_grid, 3), device memory owned by the env
  // observation mask (pob_env_set_obs_mask, ABI v7): the step kernels also store
  // obs[:, obs_mask[0 .. obs_mask_n)] into pob_state.obs_masked
  int obs_mask_n;
  int16_t obs_mask[POB_MAX_OBS_MASK];
};
static_assert(offsetof(pob_sys, wall_row) == offsetof(pob_sys, leg) + sizeof(float) * 4 * POB_LEG_FLOATS,
              "the block table (leg rows, wall rows) is staged as one contiguous copy");
