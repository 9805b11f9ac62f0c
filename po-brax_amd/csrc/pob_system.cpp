// pob_system.cpp -- builds the static tables of one env (the brax.System(cfg) step).
//
// What the reference does at construction (all [ext] brax v1 unless a file is cited):
//   * extend_ant_cfg adds walls / spheres to brax.envs.ant._SYSTEM_CONFIG
//     (ant_heavenhell.py:13-39, ant_gather.py:17-39, ant_tag.py:13-25);
//   * draw_t_maze / draw_arena / add_box_wall_to_body compute the wall boxes
//     (envs/utils.py:6-28, 60-83, 87-119);
//   * brax.System derives joint axes from the euler `rotation`, capsule end points from
//     the collider rotation, and integrator constants from dt / substeps;
//   * ActionRepeatWrapper multiplies dt and substeps by action_repeat (wrappers.py:16-24).
// Config floats live in float32 protobuf fields, so they are rounded to float32 before
// any double-precision derivation, and every derived constant is rounded once at the end.
#include <cmath>
#include <cstring>

#include "pob_sys.h"
#include "../../include/pob.h"

namespace pob {

static double f32d(double x) { return (double)(float)x; }

static void d_euler_to_quat(const double e[3], double q[4]) {
  double c1 = cos(e[0] * M_PI / 360), c2 = cos(e[1] * M_PI / 360), c3 = cos(e[2] * M_PI / 360);
  double s1 = sin(e[0] * M_PI / 360), s2 = sin(e[1] * M_PI / 360), s3 = sin(e[2] * M_PI / 360);
  q[0] = c1 * c2 * c3 - s1 * s2 * s3;
  q[1] = s1 * c2 * c3 + c1 * s2 * s3;
  q[2] = c1 * s2 * c3 - s1 * c2 * s3;
  q[3] = c1 * c2 * s3 + s1 * s2 * c3;
}
static void d_rotate(const double v[3], const double q[4], double r[3]) {
  double s = q[0], u[3] = {q[1], q[2], q[3]};
  double t = u[0] * v[0] + u[1] * v[1] + u[2] * v[2];
  double c = s * s - (u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
  double cr[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]};
  for (int i = 0; i < 3; ++i) r[i] = 2 * (t * u[i]) + c * v[i] + 2 * s * cr[i];
}

// brax ant (brax.envs.ant._SYSTEM_CONFIG as serialised in notebooks/ant_tag.ipynb:449)
static const double kMass[POB_NDYN] = {10, 1, 1, 1, 1, 1, 1, 1, 1};
static const double kCapsule[POB_NDYN][3] = {  // radius, length, end
    {0.25, 0.5, 1},  {0.08, 0.44284272, 0}, {0.08, 0.7256854, -1},
    {0.08, 0.44284272, 0}, {0.08, 0.7256854, -1}, {0.08, 0.44284272, 0},
    {0.08, 0.7256854, -1}, {0.08, 0.44284272, 0}, {0.08, 0.7256854, -1}};
static const double kCapsuleRot[POB_NDYN][3] = {
    {0, 0, 0},   {90, -45, 0},  {90, -45, 0},  {90, 45, 0},  {90, 45, 0},
    {-90, 45, 0}, {-90, 45, 0}, {-90, -45, 0}, {-90, -45, 0}};
static const double kJoint[POB_NJ][11] = {  // parent_offset(3) child_offset(3) rotation(3) min max
    {0.2, 0.2, 0, -0.1, -0.1, 0, 0, -90, 0, -30, 30},
    {0.1, 0.1, 0, -0.2, -0.2, 0, 0, 0, 135, 30, 70},
    {-0.2, 0.2, 0, 0.1, -0.1, 0, 0, -90, 0, -30, 30},
    {-0.1, 0.1, 0, 0.2, -0.2, 0, 0, 0, 45, -70, -30},
    {-0.2, -0.2, 0, 0.1, 0.1, 0, 0, -90, 0, -30, 30},
    {-0.1, -0.1, 0, 0.2, 0.2, 0, 0, 0, 135, -70, -30},
    {0.2, -0.2, 0, -0.1, 0.1, 0, 0, -90, 0, -30, 30},
    {0.1, -0.1, 0, -0.2, 0.2, 0, 0, 0, 45, 30, 70}};
static const int kGroundBody[POB_NGROUND] = {0, 2, 4, 6, 8};  // collide_include Ant x Ground

// envs/utils.py:6-28: box from `from` to `to` in xy, halfsize (|v|/2, width, half_height),
// rotation.z = arccos(x_hat . v / |v|) in degrees, on the frozen Arena body (z = 0.5).
static void add_box_wall(pob_sys &s, double fx, double fy, double tx, double ty, double half_h,
                         double width) {
  int w = s.n_walls++;
  double vx = tx - fx, vy = ty - fy;
  double len = sqrt(vx * vx + vy * vy);
  double zr = acos((1.0 * vx + 0.0 * vy) / len) * 180.0 / M_PI;
  double mx = f32d((fx + tx) / 2), my = f32d((fy + ty) / 2);
  double ang = f32d(zr) * M_PI / 180.0;
  s.wall_c[w][0] = (float)mx; s.wall_c[w][1] = (float)my; s.wall_c[w][2] = 0.5f;
  s.wall_h[w][0] = (float)f32d(len / 2); s.wall_h[w][1] = (float)f32d(width);
  s.wall_h[w][2] = (float)f32d(half_h);
  s.wall_cos[w] = (float)cos(ang);
  s.wall_sin[w] = (float)sin(ang);
}

// grid of AntGather object slots (ant_gather.py:88-91); returns count, fills xyz
int gather_grid(const pob_params &p, float *xyz, int cap) {
  int n = 0;
  float cx = p.ga_cage_xy[0], cy = p.ga_cage_xy[1];
  for (float gy = -cy; gy < cy + 1.0f; gy += 1.0f)
    for (float gx = -cx; gx < cx + 1.0f; gx += 1.0f)
      if (sqrtf(gx * gx + gy * gy) > p.ga_robot_object_spacing) {
        if (n < cap) { xyz[3 * n] = gx; xyz[3 * n + 1] = gy; xyz[3 * n + 2] = 0.0f; }
        ++n;
      }
  return n;
}

void default_params(pob_params &p) {
  memset(&p, 0, sizeof(p));
  p.hh_heaven_hell[0][0] = -5.25f; p.hh_heaven_hell[0][1] = 7.0f;
  p.hh_heaven_hell[1][0] = 5.25f;  p.hh_heaven_hell[1][1] = 7.0f;
  p.hh_priest[0] = 0.0f; p.hh_priest[1] = 7.0f;
  p.hh_visible_radius = 2.0f; p.hh_dying_cost = -2.0f;
  p.ga_n_apples = 8; p.ga_n_bombs = 8;
  p.ga_cage_xy[0] = 6.0f; p.ga_cage_xy[1] = 6.0f;
  p.ga_robot_object_spacing = 2.0f; p.ga_catch_range = 1.0f; p.ga_n_bins = 10;
  p.ga_sensor_range = 6.0f; p.ga_sensor_span = 3.14159265358979323846f; p.ga_dying_cost = -10.0f;
  p.tag_tag_radius = 1.5f; p.tag_visible_radius = 3.0f; p.tag_target_step = 0.5f;
  p.tag_min_spawn_distance = 5.0f; p.tag_cage_xy[0] = 4.5f; p.tag_cage_xy[1] = 4.5f;
  p.tag_dying_cost = -1.0f;
  p.action_repeat = 1;
  p.solver_scale_pos = 0.6f; p.solver_scale_ang = 0.2f;
  p.legacy_spring = 0;
}

// Returns an error message or nullptr.  grid (GA) is filled separately by the caller.
const char *build_system(int kind, const pob_params &p, pob_sys &s) {
  memset(&s, 0, sizeof(s));
  if (kind < 0 || kind > 3) return "unknown env kind";
  if (p.action_repeat < 1) return "action_repeat must be >= 1";
  if (p.qp_storage != POB_QP_F32 && p.qp_storage != POB_QP_F16) return "unknown qp_storage";
  s.kind = kind;
  s.qp_f16 = p.qp_storage == POB_QP_F16;
  const int ar = p.action_repeat;
  const double dt = f32d(0.05) * ar;
  const int sub = 10 * ar;
  const double hd = dt / sub;
  s.ctrl_dt = (float)dt;
  s.substeps = sub;
  s.h = (float)hd; s.half_h = 0.5f * s.h; s.inv_h = (float)(1.0 / hd);
  s.lin_damp = (float)exp(0.0 * hd);
  s.ang_damp = (float)exp(f32d(-0.05) * hd);
  s.gz = (float)f32d(-9.8);
  s.friction = 1.0f;
  s.s_pos = p.solver_scale_pos;
  s.half_s_ang = 0.5f * p.solver_scale_ang;
  if (p.legacy_spring != 0 && p.legacy_spring != 1) return "legacy_spring must be 0 or 1";
  // legacy spring config (notebooks/ant_tag.ipynb:449: stiffness 18000, springDamping 80, no
  // limitStrength = stiffness, baumgarteErp 0.1); oracle orc_env_create
  s.legacy = p.legacy_spring;
  s.k_spring = 18000.0f; s.c_spring = 80.0f; s.k_limit = 18000.0f;
  s.erp = (float)(f32d(0.1) * sub / dt);
  for (int i = 0; i < POB_NDYN; ++i) s.inv_mass[i] = 1.0f / (float)kMass[i];
  for (int j = 0; j < POB_NJ; ++j) {
    const double *J = kJoint[j];
    for (int c = 0; c < 3; ++c) { s.off_p[j][c] = (float)J[c]; s.off_c[j][c] = (float)J[3 + c]; }
    double q[4], ex[3] = {1, 0, 0}, ez[3] = {0, 0, 1}, a[3], r[3];
    d_euler_to_quat(J + 6, q);
    d_rotate(ex, q, a);
    d_rotate(ez, q, r);
    // components that are zero up to the euler rounding (cos 90 deg = 6e-17) are exactly
    // zero (oracle: same rule), so the hinge frames are the exact vectors pob_quad.h assumes
    for (int c = 0; c < 3; ++c) {
      if (fabs(a[c]) < 1e-9) a[c] = 0.0;
      if (fabs(r[c]) < 1e-9) r[c] = 0.0;
    }
    for (int c = 0; c < 3; ++c) { s.axis[j][c] = (float)a[c]; s.ref[j][c] = (float)r[c]; }
    s.lim_lo[j] = (float)(J[9] * M_PI / 180.0);
    s.lim_hi[j] = (float)(J[10] * M_PI / 180.0);
    s.tan_lo[j] = (float)tan((double)s.lim_lo[j]);  // oracle orc_env_create: the same host libm
    s.tan_hi[j] = (float)tan((double)s.lim_hi[j]);
    if (!(s.lim_lo[j] > (float)(-M_PI / 2) && s.lim_hi[j] < (float)(M_PI / 2) && s.lim_lo[j] <= s.lim_hi[j]))
      return "joint limits outside (-90, 90) degrees (the actuator gate assumes them)";
    s.default_angle[j] = (float)((J[9] + J[10]) * M_PI / 360.0);
    s.jdamp[j] = 20.0f; s.strength[j] = 350.0f;
  }
  int g = 0;
  for (int i = 0; i < POB_NDYN; ++i) {
    double q[4], ez[3] = {0, 0, 1}, a[3];
    d_euler_to_quat(kCapsuleRot[i], q);
    d_rotate(ez, q, a);
    double r = f32d(kCapsule[i][0]), len = f32d(kCapsule[i][1]);
    double seg = len / 2 - r;
    for (int c = 0; c < 3; ++c)
      if (fabs(a[c]) < 1e-9) a[c] = 0.0;  // as the joint frames (oracle: same rule)
    int end = (int)kCapsule[i][2];
    s.cap_r[i] = (float)r;
    if ((i == 0) != (seg == 0.0)) return "ant topology: only the torso capsule is a sphere";
    for (int c = 0; c < 3; ++c) {
      s.cap_end[i][0][c] = (float)(a[c] * seg);
      s.cap_end[i][1][c] = (float)(-a[c] * seg);
    }
    if (g < POB_NGROUND && kGroundBody[g] == i) {
      double sg = (end == 0) ? 1.0 : (double)end;
      for (int c = 0; c < 3; ++c) s.ground_end[g][c] = (float)(a[c] * seg * sg);
      s.ground_r[g] = (float)r;
      ++g;
    }
  }
  if (kind == POB_HEAVENHELL) {
    s.N = 14; s.D = 29 + 6 * 14 + 1;
    double tx = fmax(p.hh_heaven_hell[0][0], fmax(p.hh_heaven_hell[1][0], p.hh_priest[0])) + 1.0;
    double ty = fmax(p.hh_heaven_hell[0][1], fmax(p.hh_heaven_hell[1][1], p.hh_priest[1])) + 1.0;
    const double hw = 2.0, r = 0.5;  // draw_t_maze(hallway_width=2, r=0.5), boxes not halved
    const double P[8][2] = {{-tx - r, ty + r}, {tx + r, ty + r},      {tx + r, ty - hw - r},
                            {hw + r, ty - hw - r}, {hw + r, -r},      {-hw - r, -r},
                            {-hw - r, ty - hw - r}, {-tx - r, ty - hw - r}};
    for (int i = 0; i < 8; ++i) add_box_wall(s, P[i][0], P[i][1], P[(i + 1) % 8][0], P[(i + 1) % 8][1], 0.5, r);
    s.frozen_pos[10][0] = p.hh_priest[0]; s.frozen_pos[10][1] = p.hh_priest[1]; s.frozen_pos[10][2] = 1.0f;
    s.frozen_pos[11][2] = 0.5f; s.frozen_pos[12][2] = 0.5f; s.frozen_pos[13][2] = 0.5f;
    for (int k = 0; k < 2; ++k) { s.hh_hhp[k][0] = p.hh_heaven_hell[k][0]; s.hh_hhp[k][1] = p.hh_heaven_hell[k][1]; }
    s.hh_priest[0] = p.hh_priest[0]; s.hh_priest[1] = p.hh_priest[1];
    s.hh_visible_radius = p.hh_visible_radius; s.hh_dying_cost = p.hh_dying_cost;
  } else if (kind == POB_GATHER) {
    const int no = p.ga_n_apples + p.ga_n_bombs;
    if (p.ga_n_apples < 0 || p.ga_n_bombs < 0 || no < 1 || no > POB_MAXOBJ) return "n_apples + n_bombs must be in [1, 32]";
    if (p.ga_n_bins < 1 || 2 * p.ga_n_bins > POB_MAXBINS) return "n_bins must be in [1, 16]";
    s.n_obj = no; s.ga_n_apples = p.ga_n_apples; s.ga_n_bins = p.ga_n_bins;
    s.N = 11 + no; s.D = 29 + 6 * s.N + 2 * p.ga_n_bins;
    const double x = p.ga_cage_xy[0] + 1.0, y = p.ga_cage_xy[1] + 1.0, r = 0.5 / 2;
    const double P[4][2] = {{x + r, y + r}, {x + r, -y - r}, {-x - r, -y - r}, {-x - r, y + r}};
    for (int i = 0; i < 4; ++i) add_box_wall(s, P[i][0], P[i][1], P[(i + 1) % 4][0], P[(i + 1) % 4][1], 0.5, r);
    s.frozen_pos[10][2] = 0.5f;
    for (int i = 0; i < no; ++i) s.frozen_pos[11 + i][2] = 0.25f;
    static float tmp[3 * 4096];
    s.n_grid = gather_grid(p, tmp, 4096);
    if (s.n_grid < no) return "object grid smaller than n_apples + n_bombs";
    if (s.n_grid > 1625) return "object grid too large (one threefry shuffle round needs n <= 1625)";
    for (int c = 0; c < 3; ++c) s.ga_waiting[c] = tmp[3 * (s.n_grid - 1) + c] + p.ga_sensor_range * 2.0f;
    s.ga_catch_range = p.ga_catch_range; s.ga_sensor_range = p.ga_sensor_range;
    s.ga_half_span = (float)((double)p.ga_sensor_span / 2.0);
    s.ga_bin_res = (float)((2.0 * ((double)p.ga_sensor_span / 2.0)) / p.ga_n_bins);
    s.ga_dying_cost = p.ga_dying_cost;
  } else if (kind == POB_ANT) {
    // stock brax ant (envs/ant.py, brax <= 0.0.12): the 9 ant bodies + Ground, no arena;
    // obs = torso z, rot, joint angles (13) | torso vel, ang, joint vels (14) | cfrc (60)
    s.N = 10; s.D = 27 + 6 * 10;
  } else {
    s.N = 12; s.D = 29 + 6 * 12 + 2;
    const double x = p.tag_cage_xy[0] + 1.0, y = p.tag_cage_xy[1] + 1.0, r = 0.5 / 2;
    const double P[4][2] = {{x + r, y + r}, {x + r, -y - r}, {-x - r, -y - r}, {-x - r, y + r}};
    for (int i = 0; i < 4; ++i) add_box_wall(s, P[i][0], P[i][1], P[(i + 1) % 4][0], P[(i + 1) % 4][1], 0.5, r);
    s.frozen_pos[10][2] = 0.5f; s.frozen_pos[11][2] = 0.5f;
    s.tag_tag_radius = p.tag_tag_radius; s.tag_visible_radius = p.tag_visible_radius;
    s.tag_target_step = p.tag_target_step; s.tag_min_spawn_distance = p.tag_min_spawn_distance;
    s.tag_cage_xy[0] = p.tag_cage_xy[0]; s.tag_cage_xy[1] = p.tag_cage_xy[1];
    s.tag_dying_cost = p.tag_dying_cost;
  }
  // per-leg gathered table (pob_quad.h): the same numbers, laid out per leg
  for (int k = 0; k < 4; ++k) {
    float *L = s.leg[k];
    for (int jl = 0; jl < 2; ++jl) {
      const int j = 2 * k + jl;
      float *J = L + POB_LEG_JOINT(jl);
      for (int c = 0; c < 3; ++c) {
        J[c] = s.off_p[j][c]; J[3 + c] = s.off_c[j][c]; J[6 + c] = s.axis[j][c];
      }
      J[9] = s.tan_lo[j]; J[10] = s.tan_hi[j]; J[11] = 0.0f;  // (the kernels use the Ant's fixed references)
      J[12] = s.lim_lo[j]; J[13] = s.lim_hi[j]; J[14] = s.jdamp[j]; J[15] = s.strength[j];
    }
    for (int l = 1; l <= 2; ++l) {
      const int i = 2 * k + l;
      float *Bd = L + POB_LEG_BODY(l);
      Bd[0] = s.inv_mass[i]; Bd[1] = s.cap_r[i];
      for (int q = 0; q < 2; ++q)
        for (int c = 0; c < 3; ++c) Bd[2 + 3 * q + c] = s.cap_end[i][q][c];
    }
    for (int c = 0; c < 3; ++c) L[POB_LEG_GROUND + c] = s.ground_end[k + 1][c];
    L[POB_LEG_GROUND + 3] = s.ground_r[k + 1];
  }
  s.wall_cz = 0.5f; s.wall_hz = 0.5f;
  for (int w = 0; w < s.n_walls; ++w) {
    if (s.wall_c[w][2] != s.wall_cz || s.wall_h[w][2] != s.wall_hz) return "walls: centre z / half height differ";
    // pob_mesh.h mface forms the face edges' lengths without brax's safe_norm zero test
    if (!(s.wall_h[w][0] > 1e-6f && s.wall_h[w][1] > 1e-6f && s.wall_h[w][2] > 1e-6f)) return "walls: degenerate box";
    for (int k = 0; k < 3; ++k)  // face axis k: (ha, hb) = (hy, hz) / (hx, hz) / (hx, hy)
      pob_face_consts(s.wall_h[w][k == 0 ? 1 : 0], s.wall_h[w][k == 2 ? 1 : 2], s.face_c[w][k]);
    float *R = s.wall_row[w];
    R[0] = s.wall_c[w][0]; R[1] = s.wall_c[w][1]; R[2] = s.wall_cos[w];
    R[3] = s.wall_sin[w]; R[4] = s.wall_h[w][0]; R[5] = s.wall_h[w][1];
  }
  // broadphase boxes: wall AABB + the largest distance from a body centre to any point of
  // its capsule (|end| + r) + 1e-3 margin: a wall outside a lane's box is farther than r + 1e-3
  // from every capsule of the lane, so none of its triangles can be in contact (pob_mesh.h)
  double reach = 0.0;
  for (int i = 0; i < POB_NDYN; ++i)
    for (int q = 0; q < 2; ++q) {
      const float *e = s.cap_end[i][q];
      reach = fmax(reach, sqrt((double)e[0] * e[0] + (double)e[1] * e[1] + (double)e[2] * e[2]) + s.cap_r[i]);
    }
  reach += 1e-3;
  for (int w = 0; w < s.n_walls; ++w) {
    const double c = fabs((double)s.wall_cos[w]), sn = fabs((double)s.wall_sin[w]);
    const double ex[3] = {c * s.wall_h[w][0] + sn * s.wall_h[w][1], sn * s.wall_h[w][0] + c * s.wall_h[w][1],
                          (double)s.wall_h[w][2]};
    for (int k = 0; k < 3; ++k) {
      s.wall_lo[w][k] = (float)(s.wall_c[w][k] - ex[k] - reach);
      s.wall_hi[w][k] = (float)(s.wall_c[w][k] + ex[k] + reach);
    }
  }
  // joint frames the step kernel specialises (pob_quad.h qjoint_position): every offset lies in
  // the body xy-plane; hips (joints 0, 2, 4, 6): axis = +z, reference = -x; knees: axis in the
  // xy-plane, reference = +z
  for (int j = 0; j < POB_NJ; ++j) {
    bool ok = s.off_p[j][2] == 0.0f && s.off_c[j][2] == 0.0f;
    if (j % 2 == 0)
      ok = ok && s.axis[j][0] == 0.0f && s.axis[j][1] == 0.0f && s.axis[j][2] == 1.0f && s.ref[j][0] == -1.0f &&
           s.ref[j][1] == 0.0f && s.ref[j][2] == 0.0f;
    else
      ok = ok && s.axis[j][2] == 0.0f && s.ref[j][0] == 0.0f && s.ref[j][1] == 0.0f && s.ref[j][2] == 1.0f;
    if (!ok) return "joint frames differ from the Ant's (the step kernel assumes them)";
  }
  // capsules the contact passes specialise: end points in the body xy-plane, the two ends of
  // a capsule opposite (one rotation serves both), a lower leg's ground point = its end 1
  for (int i = 1; i < POB_NDYN; ++i)
    for (int c = 0; c < 3; ++c)
      if (s.cap_end[i][0][2] != 0.0f || s.cap_end[i][1][c] != -s.cap_end[i][0][c])
        return "capsules differ from the Ant's (the step kernel assumes them)";
  for (int g = 1; g < POB_NGROUND; ++g)
    for (int c = 0; c < 3; ++c)
      if (s.ground_end[g][c] != s.cap_end[2 * g][1][c]) return "ground contact points differ from the Ant's";
  s.torso_point = 1;
  for (int q = 0; q < 2; ++q)
    for (int c = 0; c < 3; ++c) s.torso_point &= s.cap_end[0][q][c] == 0.0f;
  for (int c = 0; c < 3; ++c) s.torso_point &= s.ground_end[0][c] == 0.0f;
  // eight-lane kernel rows (pob_octet.h): role A_k = joint 2k (torso, Aux k+1), B_k = joint
  // 2k+1 (Aux k+1, lower leg k); per slot the body's inverse mass, radius and capsule end e0
  // (ends +-e0; the torso sphere: 0); the lane's ground contact (A: torso, B: lower leg)
  for (int r = 0; r < 8; ++r) {
    const int k = r & 3;
    const bool A = r < 4;
    const int j = A ? 2 * k : 2 * k + 1;
    const int body[2] = {A ? 0 : 2 * k + 1, A ? 2 * k + 1 : 2 * k + 2};
    float *O = s.oct[r];
    for (int i = 0; i < POB_OCT_FLOATS; ++i) O[i] = 0.0f;
    for (int c = 0; c < 3; ++c) {
      O[c] = s.off_p[j][c]; O[3 + c] = s.off_c[j][c]; O[6 + c] = s.axis[j][c]; O[9 + c] = s.ref[j][c];
    }
    O[12] = s.lim_lo[j]; O[13] = s.lim_hi[j]; O[14] = s.jdamp[j]; O[15] = s.strength[j];
    for (int sl = 0; sl < 2; ++sl) {
      float *Bd = O + 16 + 8 * sl;
      Bd[0] = s.inv_mass[body[sl]]; Bd[1] = s.cap_r[body[sl]];
      for (int c = 0; c < 3; ++c) Bd[2 + c] = s.cap_end[body[sl]][0][c];
    }
    const int g = A ? 0 : k + 1;
    for (int c = 0; c < 3; ++c) O[32 + c] = s.ground_end[g][c];
    O[35] = s.ground_r[g];
    O[36] = A ? 0.0f : 1.0f;
    O[37] = s.tan_lo[j]; O[38] = s.tan_hi[j];
  }
  // sixteen-lane kernel rows (pob_hexa.h): role r = k (P_hip_k: torso), 7 - k (C_hip_k: Aux),
  // 8 + k (P_knee_k: Aux), 15 - k (C_knee_k: lower leg); the joint's row plus the lane's body
  for (int r = 0; r < 16; ++r) {
    const bool hip = r < 8, isP = r < 4 || (r >= 8 && r < 12);
    const int k = r < 4 ? r : (r < 8 ? 7 - r : (r < 12 ? r - 8 : 15 - r));
    const int j = hip ? 2 * k : 2 * k + 1;
    const int body = hip ? (isP ? 0 : 2 * k + 1) : (isP ? 2 * k + 1 : 2 * k + 2);
    float *H = s.hex[r];
    for (int i = 0; i < POB_HEX_FLOATS; ++i) H[i] = 0.0f;
    for (int c = 0; c < 3; ++c) {
      H[c] = s.off_p[j][c]; H[3 + c] = s.off_c[j][c]; H[6 + c] = s.axis[j][c]; H[9 + c] = s.ref[j][c];
      H[20 + c] = s.cap_end[body][0][c];
      H[23 + c] = isP ? s.off_p[j][c] : s.off_c[j][c];
    }
    H[12] = s.lim_lo[j]; H[13] = s.lim_hi[j]; H[14] = s.jdamp[j]; H[15] = s.strength[j];
    H[16] = s.inv_mass[hip ? 0 : 2 * k + 1]; H[17] = s.inv_mass[hip ? 2 * k + 1 : 2 * k + 2];
    H[18] = s.inv_mass[body]; H[19] = s.cap_r[body];
    const int g = body == 0 ? 0 : (body == 2 * k + 2 ? k + 1 : -1);  // ground collider of the body
    if (g >= 0) {
      for (int c = 0; c < 3; ++c) H[26 + c] = s.ground_end[g][c];
      H[29] = s.ground_r[g]; H[30] = 1.0f;
    }
    H[31] = s.tan_lo[j]; H[32] = s.tan_hi[j];
    H[33] = isP ? 1.0f : 0.0f; H[34] = hip ? 1.0f : 0.0f;
  }
  s.oct_ok = s.torso_point;
  return nullptr;
}

}  // namespace pob
