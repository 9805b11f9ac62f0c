/* pob_oracle.c -- CPU restatement of the po-brax rollout hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see pob_oracle.h).  Written for clarity: AoS per env,
 * plain loops, one helper per brax.math primitive.  Every floating-point expression
 * is spelled in a fixed evaluation order and compiled with -ffp-contract=off so that
 * the HIP kernels (written independently against the same spec) must
 * agree with it bit for bit; transcendental functions use the fixed polynomial forms
 * below (orc_atan2f / orc_sincosf) for the same reason.
 *
 * Reference anchors (file:line in /root/reference):
 *   RNG            more_jp.py:57-77 ; ant_heavenhell.py:88-99 ; ant_gather.py:110-118 ;
 *                  ant_tag.py:63-105,129-146  -> jax.random threefry (pre-partitionable)
 *   walls          envs/utils.py:6-28 (add_box_wall_to_body), :60-83 (draw_arena),
 *                  :87-119 (draw_t_maze)
 *   HH             ant_heavenhell.py:13-39 (config), :75-103 (reset), :106-123 (step),
 *                  :125-158 (obs)
 *   GA             ant_gather.py:17-39, :85-91 (grid), :93-123 (reset), :125-150 (step),
 *                  :152-181 (readings), :183-213 (obs)
 *   TAG            ant_tag.py:13-25, :63-105 (reset), :107-127 (step), :129-146 (adversary),
 *                  :148-181 (obs)
 *   wrappers       envs/__init__.py:50-72 (create chain), envs/wrappers.py:16-24,
 *                  :245-262 (gym autoreset); brax EpisodeWrapper / AutoResetWrapper [ext]
 *   physics        brax v1 System.step / info / default_qp [ext] -- restated, DESIGN.md §3
 *
 * PARITY UNPINNED where no reference artefact reaches: the PBD solver (brax v1 is not vendored;
 * no recorded PBD trajectory exists) and every wall contact -- the default spelling MV_BRAX is
 * brax v1's capsule_mesh as recalled, its triangulation / winding / edge loop / frame choices
 * measured against the 1-ulp noise floor but not pinned.  Pinned: threefry
 * (public KATs), FK / reset / the shared actuator gate and kinetic step (the notebook's 21
 * legacy frames), the Config tables, the POMDP logic line by line.
 */
#include "pob_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NDYN 9
#define NJ 8
#define MAXB 27
#define MAXW 8
#define MAXOBJ 64

/* Algorithmic FLOP counter (built with -DORC_COUNT_FLOPS, single-threaded): every
 * float add/sub/mul/div/sqrt/min/max of the restated algorithm counts 1; comparisons,
 * selects and negations count 0.  Only executed branches are counted (an inactive contact
 * costs nothing), which is the algorithmic work, not the SIMT work the GPU issues. */
#ifdef ORC_COUNT_FLOPS
static long long g_flops = 0;
/* 0: every capsule x wall x end pair (the reference's algorithm: brax evaluates all static
 *    collider pairs); 1: only the pairs the HIP step kernel evaluates (per-lane xy
 *    broadphase of pob_quad.h qdetect, and the square root / normal only when
 *    d2 < r^2 (1 + 2^-20)) -- same results, fewer operations */
static int g_flop_mode = 0;
#define FL(n) (g_flops += (n))
#else
#define FL(n) ((void)0)
#endif
long long orc_flops_read_and_reset(void) {
#ifdef ORC_COUNT_FLOPS
  long long f = g_flops; g_flops = 0; return f;
#else
  return -1;
#endif
}
int orc_flops_set_mode(int mode) {
#ifdef ORC_COUNT_FLOPS
  g_flop_mode = mode; return 0;
#else
  (void)mode; return -1;
#endif
}

/* ----------------------------------------------------------------------------- math */
typedef struct { float x, y, z; } v3;
typedef struct { float w, x, y, z; } q4;

static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { FL(3); return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { FL(3); return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vscl(v3 a, float s) { FL(3); return V(a.x * s, a.y * s, a.z * s); }
static inline v3 vdivs(v3 a, float s) { FL(4); float inv = 1.0f / s; return V(a.x * inv, a.y * inv, a.z * inv); }
/* vector / quaternion helpers as fused multiply-add chains: fmaf() is correctly rounded
 * (FMA3 with -mfma, libm otherwise) and matches the kernels' v_fma_f32 bit for bit.  FL()
 * counts algorithmic flops (an FMA = 2). */
static inline float vdot(v3 a, v3 b) { FL(5); return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 vcross(v3 a, v3 b) {
  FL(9);
  return V(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
/* brax.math.rotate: r = 2*(u.v)u + (s^2 - u.u) v + 2 s (u x v) */
static inline v3 qrot(v3 v, q4 q) {
  FL(2 + 1 + 12 + 6); /* w*w, c-sub, s2, r (12), + s2*cr (6); vdot x2 and vcross count themselves */
  v3 u = V(q.x, q.y, q.z);
  float t2 = 2.0f * vdot(u, v);
  float c = fmaf(q.w, q.w, -vdot(u, u));
  float s2 = 2.0f * q.w;
  v3 cr = vcross(u, v);
  return V(fmaf(t2, u.x, fmaf(c, v.x, s2 * cr.x)), fmaf(t2, u.y, fmaf(c, v.y, s2 * cr.y)),
           fmaf(t2, u.z, fmaf(c, v.z, s2 * cr.z)));
}
/* rotation matrix of q from the same formula (R v = (s^2 - u.u) v + 2 (u.v) u + 2 s u x v):
 * the joint projection rotates three vectors per body through it */
typedef struct { float m00, m01, m02, m10, m11, m12, m20, m21, m22; } m3;
static inline m3 qmat(q4 q) {
  FL(5 + 2 + 4 + 3 + 18);
  const float c = fmaf(q.w, q.w, -fmaf(q.z, q.z, fmaf(q.y, q.y, q.x * q.x)));
  const float x2 = 2.0f * q.x, y2 = 2.0f * q.y, z2 = 2.0f * q.z, s2 = 2.0f * q.w;
  const float sx = s2 * q.x, sy = s2 * q.y, sz = s2 * q.z;
  m3 r;
  r.m00 = fmaf(x2, q.x, c); r.m11 = fmaf(y2, q.y, c); r.m22 = fmaf(z2, q.z, c);
  r.m01 = fmaf(x2, q.y, -sz); r.m10 = fmaf(x2, q.y, sz);
  r.m02 = fmaf(x2, q.z, sy); r.m20 = fmaf(x2, q.z, -sy);
  r.m12 = fmaf(y2, q.z, -sx); r.m21 = fmaf(y2, q.z, sx);
  return r;
}
static inline v3 mrot(const m3 *R, v3 v) {
  FL(15);
  return V(fmaf(R->m02, v.z, fmaf(R->m01, v.y, R->m00 * v.x)), fmaf(R->m12, v.z, fmaf(R->m11, v.y, R->m10 * v.x)),
           fmaf(R->m22, v.z, fmaf(R->m21, v.y, R->m20 * v.x)));
}
/* brax.math.quat_mul */
static inline q4 qmul(q4 u, q4 v) {
  FL(28);
  q4 r;
  r.w = fmaf(-u.z, v.z, fmaf(-u.y, v.y, fmaf(-u.x, v.x, u.w * v.w)));
  r.x = fmaf(-u.z, v.y, fmaf(u.y, v.z, fmaf(u.x, v.w, u.w * v.x)));
  r.y = fmaf(u.z, v.x, fmaf(u.y, v.w, fmaf(-u.x, v.z, u.w * v.y)));
  r.z = fmaf(u.z, v.w, fmaf(-u.y, v.x, fmaf(u.x, v.y, u.w * v.z)));
  return r;
}
/* quat_mul([0, a], q) with the zero terms dropped */
static inline q4 qmul_vq(v3 a, q4 q) {
  FL(20);
  q4 r;
  r.w = fmaf(-a.z, q.z, fmaf(-a.y, q.y, -(a.x * q.x)));
  r.x = fmaf(-a.z, q.y, fmaf(a.y, q.z, a.x * q.w));
  r.y = fmaf(a.z, q.x, fmaf(a.y, q.w, -(a.x * q.z)));
  r.z = fmaf(a.z, q.w, fmaf(-a.y, q.x, a.x * q.y));
  return r;
}
static inline q4 qinv(q4 q) { q4 r = {q.w, -q.x, -q.y, -q.z}; return r; }
/* a * s + b, fused per component */
static inline v3 vfma(v3 a, float s, v3 b) {
  FL(6);
  return V(fmaf(a.x, s, b.x), fmaf(a.y, s, b.y), fmaf(a.z, s, b.z));
}
/* x + rotate(v, q) with the translation folded into the rotation's fused chain */
static inline v3 qrot_add(v3 v, q4 q, v3 x) {
  FL(2 + 1 + 12 + 6 + 3);
  v3 u = V(q.x, q.y, q.z);
  float t2 = 2.0f * vdot(u, v);
  float c = fmaf(q.w, q.w, -vdot(u, u));
  float s2 = 2.0f * q.w;
  v3 cr = vcross(u, v);
  return V(fmaf(t2, u.x, fmaf(c, v.x, fmaf(s2, cr.x, x.x))), fmaf(t2, u.y, fmaf(c, v.y, fmaf(s2, cr.y, x.y))),
           fmaf(t2, u.z, fmaf(c, v.z, fmaf(s2, cr.z, x.z))));
}
/* world point of a body-frame contact point: x + rotate(e, q) (rotation first, then the
 * translation: the kernels share one rotation between a capsule's end points +-e) */
static inline v3 cpoint(v3 e, q4 q, v3 x) { return vadd(x, qrot(e, q)); }
/* Substep quaternion normalisation: with e = |q|^2 - 1 (exact, Sterbenz),
 * 1/|q| = 1 - e/2 + 3e^2/8 - 5e^3/16 + O(e^4) (truncation <= 35/128 e^4 < 2^-27 for
 * |e| <= 2^-6; rollouts stay below 2.4e-3); 1 / sqrt(|q|^2) outside that range.
 * Same rule in the HIP kernels (pob_math.h qnormalize). */
static inline q4 qnormalize(q4 q) {
  FL(15);
  float n2 = fmaf(q.z, q.z, fmaf(q.y, q.y, fmaf(q.x, q.x, q.w * q.w)));
  float e = n2 - 1.0f;
  float inv = fmaf(fmaf(fmaf(-0.3125f, e, 0.375f), e, -0.5f), e, 1.0f);
  if (!(fabsf(e) <= 0x1p-6f)) inv = 1.0f / sqrtf(n2);
  q4 r = {q.w * inv, q.x * inv, q.y * inv, q.z * inv};
  return r;
}

/* atan2f: branch-free octant reduction t = min(|x|,|y|) * (1 / max(|x|,|y|)), atan t =
 * t P(t^2) (degree-7 minimax on [0, 1], 7.2e-8 relative), pi/2 - r, pi - r and the sign of y
 * by selects; <= 4 ulp against atan2.  Same form in the HIP kernels (pob_math.h). */
static float orc_atan2f(float y, float x) {
  FL(24);
  const float ax = fabsf(x), ay = fabsf(y);
  const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  float t = mn * (1.0f / mx);
  t = mx > 0.0f ? t : 0.0f;
  const float s = t * t;
  float p = fmaf(s, -0.0047533135f, 0.024452504f);
  p = fmaf(p, s, -0.059750218f);
  p = fmaf(p, s, 0.09932368f);
  p = fmaf(p, s, -0.14026737f);
  p = fmaf(p, s, 0.19971494f);
  p = fmaf(p, s, -0.33332205f);
  p = fmaf(p, s, 0.99999994f);
  float r = t * p;
  r = ay > ax ? 1.5707964f - r : r;
  r = x < 0.0f ? 3.1415927f - r : r;
  r = copysignf(r, y);
  return r + (x * 0.0f + y * 0.0f);
}
/* Test hook for the spec's elementary functions (tests/test_oracle_golden.py):
 * op 0: out[i] = orc_atan2f(a[i], b[i]); op 1: the substep normalisation of the quaternions
 * a[4i..4i+3] into out[4i..4i+3]. */
void orc_math_check(int op, int n, const float *a, const float *b, float *out) {
  for (int i = 0; i < n; ++i) {
    if (op == 0) out[i] = orc_atan2f(a[i], b[i]);
    else {
      q4 q = {a[4 * i], a[4 * i + 1], a[4 * i + 2], a[4 * i + 3]};
      q4 r = qnormalize(q);
      out[4 * i] = r.w; out[4 * i + 1] = r.x; out[4 * i + 2] = r.y; out[4 * i + 3] = r.z;
    }
  }
}
/* Cephes-form sinf/cosf with Cody-Waite reduction by pi/4. */
static void orc_sincosf(float x, float *s, float *c) {
  FL(26);
  float sgn_s = 1.0f, sgn_c = 1.0f;
  if (x < 0.0f) { x = -x; sgn_s = -1.0f; }
  int j = (int)(1.27323954473516f * x);
  float y = (float)j;
  if (j & 1) { j += 1; y += 1.0f; }
  j &= 7;
  if (j > 3) { sgn_s = -sgn_s; sgn_c = -sgn_c; j -= 4; }
  if (j > 1) sgn_c = -sgn_c;
  float xr = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
  float z = xr * xr;
  float ps = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * xr + xr;
  float pc = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) *
                 z * z - 0.5f * z + 1.0f;
  if (j == 1 || j == 2) { *s = sgn_s * pc; *c = sgn_c * ps; }
  else { *s = sgn_s * ps; *c = sgn_c * pc; }
}

/* ------------------------------------------------------------------------ threefry */
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

void orc_threefry2x32(const uint32_t key[2], uint32_t x0, uint32_t x1, uint32_t out[2]) {
  static const int R[2][4] = {{13, 15, 26, 6}, {17, 29, 16, 24}};
  uint32_t ks[3] = {key[0], key[1], key[0] ^ key[1] ^ 0x1BD11BDAu};
  uint32_t a = x0 + ks[0], b = x1 + ks[1];
  for (int i = 0; i < 5; ++i) {
    for (int k = 0; k < 4; ++k) {
      a += b;
      b = rotl32(b, R[i & 1][k]);
      b ^= a;
    }
    a += ks[(i + 1) % 3];
    b += ks[(i + 2) % 3] + (uint32_t)(i + 1);
  }
  out[0] = a; out[1] = b;
}

/* element j of threefry_2x32(key, iota(n)) */
static uint32_t tf_elem(const uint32_t key[2], uint32_t n, uint32_t j) {
  uint32_t h = (n + 1) / 2, o[2];
  if (j < h) {
    uint32_t x1 = j + h; if (x1 >= n) x1 = 0; /* odd-size zero pad */
    orc_threefry2x32(key, j, x1, o); return o[0];
  }
  orc_threefry2x32(key, j - h, j, o); return o[1];
}

void orc_split(const uint32_t key[2], int n, uint32_t *out) {
  for (int i = 0; i < 2 * n; ++i) out[i] = tf_elem(key, 2u * (uint32_t)n, (uint32_t)i);
}
static void split_k(const uint32_t key[2], int n, int i, uint32_t out[2]) {
  out[0] = tf_elem(key, 2u * (uint32_t)n, 2u * (uint32_t)i);
  out[1] = tf_elem(key, 2u * (uint32_t)n, 2u * (uint32_t)i + 1u);
}
static inline float bits_to_unit(uint32_t b) {
  union { uint32_t u; float f; } c; c.u = (b >> 9) | 0x3F800000u; return c.f - 1.0f;
}
void orc_uniform(const uint32_t key[2], int n, const float *lo, const float *hi, int lohi_n,
                 float *out) {
  for (int i = 0; i < n; ++i) {
    float l = lo[lohi_n > 1 ? i : 0], h = hi[lohi_n > 1 ? i : 0];
    float f = bits_to_unit(tf_elem(key, (uint32_t)n, (uint32_t)i));
    float v = f * (h - l) + l;
    out[i] = v > l ? v : l;
  }
}
int orc_randint(const uint32_t key[2], int lo, int hi) {
  uint32_t k[4]; orc_split(key, 2, k);
  uint32_t span = (uint32_t)(hi - lo);
  uint32_t hb = tf_elem(k, 1, 0), lb = tf_elem(k + 2, 1, 0);
  uint32_t m = (65536u % span); m = (m * m) % span;
  uint32_t off = ((hb % span) * m + (lb % span)) % span;
  return lo + (int)off;
}
/* first k of jax _shuffle(key, arange(n)) (rounds = ceil(3 ln n / ln(2^32-1))). */
void orc_choice_idx(const uint32_t key[2], int n, int k, int *out) {
  int rounds = (int)ceil(3.0 * log(n > 1 ? (double)n : 1.0) / log(4294967295.0));
  int *x = (int *)malloc(sizeof(int) * n), *t = (int *)malloc(sizeof(int) * n);
  uint32_t *sk = (uint32_t *)malloc(sizeof(uint32_t) * n);
  uint32_t kk[2] = {key[0], key[1]};
  for (int i = 0; i < n; ++i) x[i] = i;
  for (int r = 0; r < rounds; ++r) {
    uint32_t s[4]; orc_split(kk, 2, s);
    kk[0] = s[0]; kk[1] = s[1];
    for (int i = 0; i < n; ++i) sk[i] = tf_elem(s + 2, (uint32_t)n, (uint32_t)i);
    /* stable sort of x by sk (insertion sort keeps stability) */
    for (int i = 0; i < n; ++i) t[i] = i;
    for (int i = 1; i < n; ++i) {
      int v = t[i], j = i - 1;
      while (j >= 0 && sk[t[j]] > sk[v]) { t[j + 1] = t[j]; --j; }
      t[j + 1] = v;
    }
    int *nx = (int *)malloc(sizeof(int) * n);
    for (int i = 0; i < n; ++i) nx[i] = x[t[i]];
    memcpy(x, nx, sizeof(int) * n); free(nx);
  }
  for (int i = 0; i < k; ++i) out[i] = x[i];
  free(x); free(t); free(sk);
}

/* ------------------------------------------------------------------ system tables */
struct orc_env {
  int kind, N, D, n_obj;
  /* integrator */
  float h, half_h, inv_h, lin_damp, ang_damp, g[3];
  int substeps;
  float mass[NDYN], inv_mass[NDYN];
  /* joints (ant tree; parent(j) = j odd ? j : 0, child(j) = j+1) */
  v3 off_p[NJ], off_c[NJ], axis[NJ], ref[NJ];
  float lim_lo[NJ], lim_hi[NJ], jdamp[NJ], strength[NJ];
  float tan_lo[NJ], tan_hi[NJ]; /* actuator gate (actuator_inside) */
  float default_angle[NJ];
  /* legacy spring dynamics (brax <= 0.0.12 config: notebooks/ant_tag.ipynb:449) */
  int legacy;
  float k_spring, c_spring, k_limit, erp;
  /* colliders: one capsule per ant body */
  v3 cap_end[NDYN][2]; int cap_nend[NDYN]; float cap_r[NDYN];
  int n_ground; int ground_body[NDYN]; v3 ground_end[NDYN]; float ground_r[NDYN];
  int n_walls; v3 wall_c[MAXW], wall_h[MAXW]; float wall_cos[MAXW], wall_sin[MAXW];
  float friction, s_pos, half_s_ang;
  /* frozen/default bodies (default_qp rows for bodies >= 9) */
  float frozen_pos[MAXB][3];
  /* env params */
  orc_params p;
  /* GA */
  int n_grid; float grid[400][3]; float waiting[3];
  /* stock ant: control dt (sys.config.dt as a float32 proto field) */
  float ctrl_dt;
};

void orc_default_params(orc_params *p) {
  memset(p, 0, sizeof(*p));
  p->hh_heaven_hell[0][0] = -5.25f; p->hh_heaven_hell[0][1] = 7.0f;
  p->hh_heaven_hell[1][0] = 5.25f; p->hh_heaven_hell[1][1] = 7.0f;
  p->hh_priest[0] = 0.0f; p->hh_priest[1] = 7.0f;
  p->hh_visible_radius = 2.0f; p->hh_dying_cost = -2.0f;
  p->ga_n_apples = 8; p->ga_n_bombs = 8;
  p->ga_cage_xy[0] = 6.0f; p->ga_cage_xy[1] = 6.0f;
  p->ga_robot_object_spacing = 2.0f; p->ga_catch_range = 1.0f; p->ga_n_bins = 10;
  p->ga_sensor_range = 6.0f; p->ga_sensor_span = 3.14159265358979323846f; p->ga_dying_cost = -10.0f;
  p->tag_tag_radius = 1.5f; p->tag_visible_radius = 3.0f; p->tag_target_step = 0.5f;
  p->tag_min_spawn_distance = 5.0f; p->tag_cage_xy[0] = 4.5f; p->tag_cage_xy[1] = 4.5f;
  p->tag_dying_cost = -1.0f;
  p->action_repeat = 1;
  p->solver_scale_pos = 0.6f; p->solver_scale_ang = 0.2f;
  p->legacy_spring = 0;
  p->wall_contact = 0;
}

/* double-precision config maths (System construction time) */
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

/* brax ant (bodies, joints) as carried by notebooks/ant_tag.ipynb:449 */
static const double ANT_MASS[NDYN] = {10, 1, 1, 1, 1, 1, 1, 1, 1};
static const double ANT_CAP[NDYN][3] = { /* radius, length, end */
    {0.25, 0.5, 1}, {0.08, 0.44284272, 0}, {0.08, 0.7256854, -1}, {0.08, 0.44284272, 0},
    {0.08, 0.7256854, -1}, {0.08, 0.44284272, 0}, {0.08, 0.7256854, -1},
    {0.08, 0.44284272, 0}, {0.08, 0.7256854, -1}};
static const double ANT_CAPROT[NDYN][3] = {{0, 0, 0},   {90, -45, 0}, {90, -45, 0},
                                           {90, 45, 0}, {90, 45, 0},  {-90, 45, 0},
                                           {-90, 45, 0}, {-90, -45, 0}, {-90, -45, 0}};
static const double ANT_JOINT[NJ][11] = { /* off_p(3) off_c(3) rot(3) lo hi */
    {0.2, 0.2, 0, -0.1, -0.1, 0, 0, -90, 0, -30, 30},
    {0.1, 0.1, 0, -0.2, -0.2, 0, 0, 0, 135, 30, 70},
    {-0.2, 0.2, 0, 0.1, -0.1, 0, 0, -90, 0, -30, 30},
    {-0.1, 0.1, 0, 0.2, -0.2, 0, 0, 0, 45, -70, -30},
    {-0.2, -0.2, 0, 0.1, 0.1, 0, 0, -90, 0, -30, 30},
    {-0.1, -0.1, 0, 0.2, 0.2, 0, 0, 0, 135, -70, -30},
    {0.2, -0.2, 0, -0.1, 0.1, 0, 0, -90, 0, -30, 30},
    {0.1, -0.1, 0, -0.2, 0.2, 0, 0, 0, 45, 30, 70}};

static double f32d(double x) { return (double)(float)x; }

/* utils.py:6-28 add_box_wall_to_body: from->to in xy, z rotation = arccos(x.v/|v|) */
static void add_box_wall(orc_env *e, double fx, double fy, double tx, double ty, double half_h,
                         double width) {
  int w = e->n_walls++;
  double vx = tx - fx, vy = ty - fy;
  double len = sqrt(vx * vx + vy * vy);
  double zr = acos((1.0 * vx + 0.0 * vy) / len) * 180.0 / M_PI;
  /* proto floats: position/rotation/halfsize stored as float32 */
  double mx = f32d((fx + tx) / 2), my = f32d((fy + ty) / 2);
  double rz = f32d(zr);
  double ang = rz * M_PI / 180.0;
  e->wall_c[w] = V((float)mx, (float)my, 0.5f); /* Arena body at z = 0.5 */
  e->wall_h[w] = V((float)f32d(len / 2), (float)f32d(width), (float)f32d(half_h));
  e->wall_cos[w] = (float)cos(ang);
  e->wall_sin[w] = (float)sin(ang);
}

orc_env *orc_env_create(int kind, const orc_params *pin) {
  orc_env *e = (orc_env *)calloc(1, sizeof(orc_env));
  orc_params p; if (pin) p = *pin; else orc_default_params(&p);
  e->kind = kind; e->p = p;
  int ar = p.action_repeat > 0 ? p.action_repeat : 1;
  double dt = f32d(0.05) * ar; int sub = 10 * ar; /* wrappers.py:21-23 */
  double hd = dt / sub;
  e->ctrl_dt = (float)dt;
  e->substeps = sub;
  e->h = (float)hd; e->half_h = 0.5f * e->h; e->inv_h = (float)(1.0 / hd);
  e->lin_damp = (float)exp(0.0 * hd);
  e->ang_damp = (float)exp(f32d(-0.05) * hd);
  e->g[0] = 0.0f; e->g[1] = 0.0f; e->g[2] = (float)f32d(-9.8);
  e->friction = 1.0f;
  e->s_pos = p.solver_scale_pos;
  e->half_s_ang = 0.5f * p.solver_scale_ang;
  /* legacy: stiffness 18000, springDamping 80, limit strength = stiffness (limitStrength
   * unset), baumgarteErp 0.1 scaled by substeps / dt (brax Collider [ext]) */
  e->legacy = p.legacy_spring != 0;
  e->k_spring = 18000.0f; e->c_spring = 80.0f; e->k_limit = 18000.0f;
  e->erp = (float)(f32d(0.1) * sub / dt);
  for (int i = 0; i < NDYN; ++i) { e->mass[i] = (float)ANT_MASS[i]; e->inv_mass[i] = 1.0f / e->mass[i]; }
  for (int j = 0; j < NJ; ++j) {
    const double *J = ANT_JOINT[j];
    e->off_p[j] = V((float)J[0], (float)J[1], (float)J[2]);
    e->off_c[j] = V((float)J[3], (float)J[4], (float)J[5]);
    double q[4], ex[3] = {1, 0, 0}, ez[3] = {0, 0, 1}, a[3], r[3];
    d_euler_to_quat(J + 6, q);
    d_rotate(ex, q, a); d_rotate(ez, q, r);
    /* components that are zero up to the euler rounding (|c| < 1e-9, e.g. cos 90 deg) are
     * exactly zero: the hinge frames are then the exact axis-aligned / in-plane vectors the
     * kernels exploit (pob_system.cpp does the same) */
    for (int c = 0; c < 3; ++c) { if (fabs(a[c]) < 1e-9) a[c] = 0.0; if (fabs(r[c]) < 1e-9) r[c] = 0.0; }
    e->axis[j] = V((float)a[0], (float)a[1], (float)a[2]);
    e->ref[j] = V((float)r[0], (float)r[1], (float)r[2]);
    e->lim_lo[j] = (float)(J[9] * M_PI / 180.0);
    e->lim_hi[j] = (float)(J[10] * M_PI / 180.0);
    e->tan_lo[j] = (float)tan((double)e->lim_lo[j]);
    e->tan_hi[j] = (float)tan((double)e->lim_hi[j]);
    e->default_angle[j] = (float)((J[9] + J[10]) * M_PI / 360.0);
    e->jdamp[j] = 20.0f; e->strength[j] = 350.0f;
  }
  for (int i = 0; i < NDYN; ++i) {
    double q[4], ez[3] = {0, 0, 1}, a[3];
    d_euler_to_quat(ANT_CAPROT[i], q);
    d_rotate(ez, q, a);
    double r = f32d(ANT_CAP[i][0]), len = f32d(ANT_CAP[i][1]);
    double seg = len / 2 - r;
    for (int c = 0; c < 3; ++c) if (fabs(a[c]) < 1e-9) a[c] = 0.0; /* as the joint frames */
    e->cap_r[i] = (float)r;
    int end = (int)ANT_CAP[i][2];
    if (seg == 0.0) { e->cap_nend[i] = 1; e->cap_end[i][0] = V(0, 0, 0); }
    else {
      e->cap_nend[i] = 2;
      e->cap_end[i][0] = V((float)(a[0] * seg), (float)(a[1] * seg), (float)(a[2] * seg));
      e->cap_end[i][1] = V((float)(-a[0] * seg), (float)(-a[1] * seg), (float)(-a[2] * seg));
    }
    /* collide_include Ant x Ground: Torso + 4 lower legs; CapsulePlane uses `end` */
    if (i == 0 || i == 2 || i == 4 || i == 6 || i == 8) {
      int k = e->n_ground++;
      e->ground_body[k] = i; e->ground_r[k] = (float)r;
      double s = (end == 0) ? 1.0 : (double)end;
      e->ground_end[k] = V((float)(a[0] * seg * s), (float)(a[1] * seg * s), (float)(a[2] * seg * s));
    }
  }
  memset(e->frozen_pos, 0, sizeof(e->frozen_pos));
  if (kind == ORC_HH) {
    e->N = 14; e->D = 29 + 2 * 3 * 14 + 1;
    double tx = fmax(p.hh_heaven_hell[0][0], fmax(p.hh_heaven_hell[1][0], p.hh_priest[0])) + 1.0;
    double ty = fmax(p.hh_heaven_hell[0][1], fmax(p.hh_heaven_hell[1][1], p.hh_priest[1])) + 1.0;
    double hw = 2.0, r = 0.5;
    double P[8][2] = {{-tx - r, ty + r}, {tx + r, ty + r}, {tx + r, ty - hw - r},
                      {hw + r, ty - hw - r}, {hw + r, -r}, {-hw - r, -r},
                      {-hw - r, ty - hw - r}, {-tx - r, ty - hw - r}};
    for (int i = 0; i < 8; ++i) add_box_wall(e, P[i][0], P[i][1], P[(i + 1) % 8][0], P[(i + 1) % 8][1], 0.5, r);
    e->frozen_pos[10][0] = p.hh_priest[0]; e->frozen_pos[10][1] = p.hh_priest[1]; e->frozen_pos[10][2] = 1.0f;
    e->frozen_pos[11][2] = 0.5f; e->frozen_pos[12][2] = 0.5f; e->frozen_pos[13][2] = 0.5f;
  } else if (kind == ORC_GA) {
    int no = p.ga_n_apples + p.ga_n_bombs;
    e->n_obj = no;
    e->N = 11 + no; e->D = 29 + 2 * 3 * e->N + 2 * p.ga_n_bins;
    double x = p.ga_cage_xy[0] + 1.0, y = p.ga_cage_xy[1] + 1.0, r = 0.5 / 2;
    double P[4][2] = {{x + r, y + r}, {x + r, -y - r}, {-x - r, -y - r}, {-x - r, y + r}};
    for (int i = 0; i < 4; ++i) add_box_wall(e, P[i][0], P[i][1], P[(i + 1) % 4][0], P[(i + 1) % 4][1], 0.5, r);
    e->frozen_pos[10][2] = 0.5f;
    for (int i = 0; i < no; ++i) e->frozen_pos[11 + i][2] = 0.25f;
    /* ant_gather.py:88-91: meshgrid('xy') over arange(-cx, cx+1) x arange(-cy, cy+1) */
    int n = 0;
    float cx = p.ga_cage_xy[0], cy = p.ga_cage_xy[1];
    for (float gy = -cy; gy < cy + 1.0f; gy += 1.0f)
      for (float gx = -cx; gx < cx + 1.0f; gx += 1.0f) {
        if (sqrtf(gx * gx + gy * gy) > p.ga_robot_object_spacing) {
          e->grid[n][0] = gx; e->grid[n][1] = gy; e->grid[n][2] = 0.0f; ++n;
        }
      }
    e->n_grid = n;
    for (int c = 0; c < 3; ++c) e->waiting[c] = e->grid[n - 1][c] + p.ga_sensor_range * 2.0f;
  } else if (kind == ORC_ANT) {
    /* stock brax ant (brax <= 0.0.12 envs/ant.py, registered at po_brax/envs/__init__.py:30):
     * bodies 0-8 + Ground, no arena; obs 13 qpos + 14 qvel + 60 cfrc = 87 */
    e->N = 10; e->D = 87;
  } else {
    e->N = 12; e->D = 29 + 2 * 3 * 12 + 2;
    double x = p.tag_cage_xy[0] + 1.0, y = p.tag_cage_xy[1] + 1.0, r = 0.5 / 2;
    double P[4][2] = {{x + r, y + r}, {x + r, -y - r}, {-x - r, -y - r}, {-x - r, y + r}};
    for (int i = 0; i < 4; ++i) add_box_wall(e, P[i][0], P[i][1], P[(i + 1) % 4][0], P[(i + 1) % 4][1], 0.5, r);
    e->frozen_pos[10][2] = 0.5f; e->frozen_pos[11][2] = 0.5f;
  }
  return e;
}
void orc_env_destroy(orc_env *e) { free(e); }
void orc_env_dims(const orc_env *e, int *n, int *d, int *a) { *n = e->N; *d = e->D; *a = NJ; }

/* -------------------------------------------------------------------- body state */
typedef struct { v3 x[NDYN]; q4 q[NDYN]; v3 v[NDYN]; v3 w[NDYN]; } body_t;

static inline int jparent(int j) { return (j & 1) ? j : 0; }
static inline int jchild(int j) { return j + 1; }

/* ----------------------------------------------------------------- default_qp (a4) */
void orc_default_qp(const orc_env *e, const float *qpos, const float *qvel, float *pos, float *rot,
                    float *vel, float *ang) {
  body_t b;
  b.x[0] = V(0, 0, 0); b.q[0].w = 1.0f; b.q[0].x = b.q[0].y = b.q[0].z = 0.0f;
  b.v[0] = V(0, 0, 0); b.w[0] = V(0, 0, 0);
  for (int j = 0; j < NJ; ++j) {
    int p = jparent(j), c = jchild(j);
    float s, co; orc_sincosf(qpos[j] * 0.5f, &s, &co);
    q4 loc = {co, e->axis[j].x * s, e->axis[j].y * s, e->axis[j].z * s};
    b.q[c] = qmul(b.q[p], loc);
    v3 anchor = vadd(b.x[p], qrot(e->off_p[j], b.q[p]));
    b.x[c] = vsub(anchor, qrot(e->off_c[j], b.q[c]));
    /* joint velocity: the child's angular velocity is its own joint's axis (parent frame) * qvel,
     * rotated to the world; no accumulation down the tree, zero linear velocity (brax
     * System.default_qp [ext]; pinned by the notebook trajectory, tests/test_oracle_golden.py) */
    b.w[c] = vscl(qrot(e->axis[j], b.q[p]), qvel[j]);
    b.v[c] = V(0, 0, 0);
  }
  float zmin = 3.0e38f;
  for (int i = 0; i < NDYN; ++i)
    for (int k = 0; k < e->cap_nend[i]; ++k) {
      float z = vadd(b.x[i], qrot(e->cap_end[i][k], b.q[i])).z - e->cap_r[i];
      if (z < zmin) zmin = z;
    }
  for (int i = 0; i < e->N; ++i) {
    float *P = pos + 3 * i, *R = rot + 4 * i, *Vv = vel + 3 * i, *A = ang + 3 * i;
    if (i < NDYN) {
      P[0] = b.x[i].x; P[1] = b.x[i].y; P[2] = b.x[i].z - zmin;
      R[0] = b.q[i].w; R[1] = b.q[i].x; R[2] = b.q[i].y; R[3] = b.q[i].z;
      Vv[0] = b.v[i].x; Vv[1] = b.v[i].y; Vv[2] = b.v[i].z;
      A[0] = b.w[i].x; A[1] = b.w[i].y; A[2] = b.w[i].z;
    } else {
      P[0] = e->frozen_pos[i][0]; P[1] = e->frozen_pos[i][1]; P[2] = e->frozen_pos[i][2];
      R[0] = 1.0f; R[1] = R[2] = R[3] = 0.0f;
      Vv[0] = Vv[1] = Vv[2] = 0.0f; A[0] = A[1] = A[2] = 0.0f;
    }
  }
}

/* ------------------------------------------------------------------------- contacts */
/* A contact: body, penetration, world normal, radius, and where on the body it sits.  Ground
 * contacts (CapsulePlane) sit at the body-frame end point e; wall contacts (Ant x Arena) at
 * the point x + tau * rotate(e0, q) of the capsule's segment (e0 = the capsule's end 0, the
 * segment is x + [-1, 1] * rotate(e0, q); the torso is a sphere, e0 = 0).  Contacts are kept
 * in the order ground (collider order), then per capsule its wall contacts in (wall, face,
 * triangle) order; each body's corrections are accumulated in that order. */
#define MAXCT (NDYN + NDYN * MAXW * 12)
typedef struct {
  int count;
  int body[MAXCT], ground[MAXCT];
  float pen[MAXCT], r[MAXCT], tau[MAXCT];
  v3 n[MAXCT], e[MAXCT];
} contacts_t;

/* world point of contact k at the body pose (x, q) */
static inline v3 contact_point(const orc_env *e, const body_t *b, const contacts_t *ct, int k) {
  const int i = ct->body[k];
  if (ct->ground[k]) return cpoint(ct->e[k], b->q[i], b->x[i]);
  FL(6);
  const v3 rv = qrot(e->cap_end[i][0], b->q[i]);
  return V(fmaf(rv.x, ct->tau[k], b->x[i].x), fmaf(rv.y, ct->tau[k], b->x[i].y), fmaf(rv.z, ct->tau[k], b->x[i].z));
}

/* sphere (centre p, radius r) vs the z-rotated box w; returns penetration, world normal
 * (wall_contact = 1 only: the round-1..3 model) */
static float sphere_box(const orc_env *e, int w, v3 p, float r, v3 *n) {
  float c = e->wall_cos[w], s = e->wall_sin[w];
  v3 h = e->wall_h[w];
  v3 d = vsub(p, e->wall_c[w]);
  FL(6 + 6 + 3 + 5); /* local x/y, clamp, e, d2 */
  float lx = fmaf(d.y, s, d.x * c), ly = fmaf(d.y, c, -(d.x * s)), lz = d.z;
  float qx = fminf(fmaxf(lx, -h.x), h.x), qy = fminf(fmaxf(ly, -h.y), h.y), qz = fminf(fmaxf(lz, -h.z), h.z);
  float ex = lx - qx, ey = ly - qy, ez = lz - qz;
  float d2 = fmaf(ez, ez, fmaf(ey, ey, ex * ex));
  float pen, nx, ny, nz;
  if (d2 > 0.0f) {
    FL(5);
    float dist = sqrtf(d2);
    float inv = 1.0f / dist;
    pen = r - dist; nx = ex * inv; ny = ey * inv; nz = ez * inv;
  } else {
    FL(4);
    float fx = h.x - fabsf(lx), fy = h.y - fabsf(ly), fz = h.z - fabsf(lz);
    nx = 0.0f; ny = 0.0f; nz = 0.0f;
    if (fx <= fy && fx <= fz) { pen = r + fx; nx = lx < 0.0f ? -1.0f : 1.0f; }
    else if (fy <= fz) { pen = r + fy; ny = ly < 0.0f ? -1.0f : 1.0f; }
    else { pen = r + fz; nz = lz < 0.0f ? -1.0f : 1.0f; }
  }
  FL(6);
  *n = V(fmaf(-ny, s, nx * c), fmaf(ny, c, nx * s), nz);
  return pen;
}

/* ---- brax v1 capsule x TriangulatedBox (capsule_mesh) [ext, recalled; DESIGN.md §3] ----
 * brax v1 routes capsule x box pairs through its mesh path: the box collider becomes a
 * TriangulatedBox (6 faces x 2 triangles) and capsule_mesh returns, for EVERY triangle, the
 * closest points between the capsule's segment and the triangle, penetration r - |S - P| and
 * the normal along S - P; the collider applies every penetrating one.  Restated here in the
 * wall's own frame (the Arena is frozen at the identity rotation; each wall is a box rotated
 * about z): local = R_z(-theta)(p - c), the same transform as the sphere-box model.  A face is
 * the plane w = sigma h_k of axis k in face coordinates (a, b, w) = (y, z, x), (x, z, y),
 * (x, y, z) for k = x, y, z; its rectangle [-ha, ha] x [-hb, hb] is split along the diagonal
 * V0 = (-ha, -hb) -> V2 = (ha, hb): triangle 0 = (V0, V1 = (ha, -hb), V2), triangle 1 =
 * (V0, V2, V3 = (-ha, hb)).  Faces in the order -x, +x, -y, +y, -z, +z.
 *
 * Closest points of segment S(u) = A + u D (u in [0, 1]) and triangle T: the minimum of the
 * convex |S(u) - T| is attained at an end point (closest triangle point to A or B), at a
 * closest pair of the segment and a triangle edge, or where the segment crosses the
 * triangle's plane inside T -- the candidates below, taken in that order, the first strict
 * minimum of the squared distance winning (brax's _closest_segment_triangle_points tests
 * the same three kinds).  Degenerate contact (S on the triangle, |S - P| = 0): the normal is
 * the face's outward normal and the penetration r.
 *
 * Face cull (part of this restatement, applied identically by the kernels): a face whose
 * rectangle is separated from the segment's axis-aligned bounding box (face coordinates) by
 * a gap >= r + 1e-3 along some axis is not evaluated -- every point pair is then at least
 * r + 1e-3 apart, and the float evaluation of its triangles (errors ~1e-6 at these
 * coordinates) could not produce a penetrating contact.  orc_set_face_cull(0) and the FLOP
 * counter's reference mode evaluate every face; the results are identical (tests). */
#define WALL_CULL_MARGIN 1e-3f
static int g_face_cull = 1;
void orc_set_face_cull(int on) { g_face_cull = on != 0; }

static long long g_cst[16];
static int g_cst_on = 0;
void orc_contact_stats_enable(int on) { g_cst_on = on != 0; }
void orc_contact_stats(long long out[16]) {
  for (int i = 0; i < 16; ++i) { out[i] = g_cst[i]; g_cst[i] = 0; }
}
#define CST(i, v) do { if (g_cst_on) g_cst[i] += (v); } while (0)

static inline float clamp01(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }
typedef struct { float a, b, w; } f3; /* face coordinates */

/* is (pa, pb) in face triangle t (boundary included)? */
static inline int tri_inside(int t, float ha, float hb, float pa, float pb) {
  FL(4);
  const float cr = fmaf(pa + ha, hb, -((pb + hb) * ha)); /* >= 0: on or below the diagonal */
  return t == 0 ? (pb >= -hb && pa <= ha && cr >= 0.0f) : (pb <= hb && pa >= -ha && cr <= 0.0f);
}
/* closest point (qa, qb) of face triangle t to the face-plane point (pa, pb): the point itself
 * when inside, else the nearest of the triangle's edges' nearest points (edge order: triangle
 * 0 bottom, right, diagonal; triangle 1 diagonal, top, left; first strict minimum) */
static void tri_closest(int t, float ha, float hb, float pa, float pb, float *qa, float *qb) {
  if (tri_inside(t, ha, hb, pa, pb)) { *qa = pa; *qb = pb; return; }
  FL(4 + 1 + 8 + 6 + 6);
  /* diagonal V0 -> V2, D = (2ha, 2hb): s = clamp01(((p - V0) . D) / (D . D)) */
  const float ha2 = 2.0f * ha, hb2 = 2.0f * hb;
  const float s = clamp01(fmaf(pb + hb, hb2, (pa + ha) * ha2) * (1.0f / fmaf(hb2, hb2, ha2 * ha2)));
  const float s2 = 2.0f * s;
  const float da = fmaf(s2, ha, -ha), db = fmaf(s2, hb, -hb);
  float ea[3], eb[3];
  if (t == 0) {
    ea[0] = fminf(fmaxf(pa, -ha), ha); eb[0] = -hb;  /* bottom V0 -> V1 */
    ea[1] = ha; eb[1] = fminf(fmaxf(pb, -hb), hb);   /* right V1 -> V2 */
    ea[2] = da; eb[2] = db;
  } else {
    ea[0] = da; eb[0] = db;
    ea[1] = fminf(fmaxf(pa, -ha), ha); eb[1] = hb;   /* top V2 -> V3 */
    ea[2] = -ha; eb[2] = fminf(fmaxf(pb, -hb), hb);  /* left V3 -> V0 */
  }
  float best = 0.0f;
  for (int k = 0; k < 3; ++k) {
    const float ga = pa - ea[k], gb = pb - eb[k];
    const float d2 = fmaf(gb, gb, ga * ga);
    if (k == 0 || d2 < best) { best = d2; *qa = ea[k]; *qb = eb[k]; }
  }
}

typedef struct { float d2, u; f3 d; } cand_t; /* squared distance, segment parameter, S - P */
static inline void cand_take(cand_t *c, float u, f3 d) {
  FL(5);
  const float d2 = fmaf(d.w, d.w, fmaf(d.b, d.b, d.a * d.a));
  if (d2 < c->d2) { c->d2 = d2; c->u = u; c->d = d; }
}
/* closest points of the segment A + u D and the edge E0 + t F (F in the face plane, F.w = 0):
 * Ericson's clamped form; ee = F . F, inv_ee = 1 / ee, aa = D . D > 0, inv_aa = 1 / aa */
static void seg_edge(cand_t *c, f3 A, f3 D, float aa, float inv_aa, float e0a, float e0b, float w0, float fa, float fb,
                     float ee, float inv_ee) {
  FL(3 + 3 + 5 + 3 + 3 + 2 + 3);
  const f3 r = {A.a - e0a, A.b - e0b, A.w - w0};
  const float f = fmaf(fb, r.b, fa * r.a);
  const float cc = fmaf(D.w, r.w, fmaf(D.b, r.b, D.a * r.a));
  const float bb = fmaf(D.b, fb, D.a * fa);
  const float den = fmaf(aa, ee, -(bb * bb));
  float u = 0.0f;
  if (den > 0.0f) { FL(4); u = clamp01(fmaf(bb, f, -(cc * ee)) * (1.0f / den)); }
  float t = fmaf(bb, u, f) * inv_ee;
  if (t < 0.0f) { FL(1); t = 0.0f; u = clamp01(-cc * inv_aa); }
  else if (t > 1.0f) { FL(2); t = 1.0f; u = clamp01((bb - cc) * inv_aa); }
  FL(6 + 4 + 3);
  const f3 S = {fmaf(u, D.a, A.a), fmaf(u, D.b, A.b), fmaf(u, D.w, A.w)};
  const f3 d = {S.a - fmaf(t, fa, e0a), S.b - fmaf(t, fb, e0b), S.w - w0};
  cand_take(c, u, d);
}

/* closest points of the segment [A, B] (or the point A when !seg) and face triangle t of the
 * face w = w0 with half extents (ha, hb) */
static cand_t seg_tri(int t, float ha, float hb, float w0, f3 A, f3 B, int seg, f3 D, float aa, float inv_aa) {
  cand_t c; c.d2 = INFINITY; c.u = 0.0f; c.d.a = c.d.b = c.d.w = 0.0f;
  float qa, qb;
  tri_closest(t, ha, hb, A.a, A.b, &qa, &qb);
  FL(3);
  { const f3 d = {A.a - qa, A.b - qb, A.w - w0}; c.d2 = INFINITY; cand_take(&c, 0.0f, d); }
  if (!seg) return c;
  tri_closest(t, ha, hb, B.a, B.b, &qa, &qb);
  FL(3);
  { const f3 d = {B.a - qa, B.b - qb, B.w - w0}; cand_take(&c, 1.0f, d); }
  /* the edges (edge vectors from the face's constant tables: 2ha, 2hb) */
  const float ha2 = 2.0f * ha, hb2 = 2.0f * hb;
  FL(1 + 1 + 3);
  const float e_a = ha2 * ha2, e_b = hb2 * hb2, e_d = fmaf(hb2, hb2, ha2 * ha2);
  const float i_a = 1.0f / e_a, i_b = 1.0f / e_b, i_d = 1.0f / e_d;
  if (t == 0) {
    seg_edge(&c, A, D, aa, inv_aa, -ha, -hb, w0, ha2, 0.0f, e_a, i_a);  /* bottom V0 -> V1 */
    seg_edge(&c, A, D, aa, inv_aa, ha, -hb, w0, 0.0f, hb2, e_b, i_b);   /* right V1 -> V2 */
    seg_edge(&c, A, D, aa, inv_aa, -ha, -hb, w0, ha2, hb2, e_d, i_d);   /* diagonal V0 -> V2 */
  } else {
    seg_edge(&c, A, D, aa, inv_aa, -ha, -hb, w0, ha2, hb2, e_d, i_d);   /* diagonal V0 -> V2 */
    seg_edge(&c, A, D, aa, inv_aa, ha, hb, w0, -ha2, 0.0f, e_a, i_a);   /* top V2 -> V3 */
    seg_edge(&c, A, D, aa, inv_aa, -ha, hb, w0, 0.0f, -hb2, e_b, i_b);  /* left V3 -> V0 */
  }
  /* the segment crossing the face plane inside the triangle */
  FL(2);
  const float aw = A.w - w0, bw = B.w - w0;
  if ((aw < 0.0f && bw > 0.0f) || (aw > 0.0f && bw < 0.0f)) {
    FL(3 + 6 + 1);
    const float u = aw * (1.0f / (aw - bw));
    const f3 S = {fmaf(u, D.a, A.a), fmaf(u, D.b, A.b), fmaf(u, D.w, A.w)};
    if (tri_inside(t, ha, hb, S.a, S.b)) { const f3 d = {0.0f, 0.0f, S.w - w0}; cand_take(&c, u, d); }
  }
  return c;
}

/* ---- brax v1's own spelling of capsule_mesh [ext, recalled] (deviation table).
 * The exact form above computes the closest points exactly (up to rounding); brax v1 spells
 * them with regularised divisions and another candidate set.  g_mesh_variant selects, per
 * deviation, brax's form (oracle/brax_mesh_study.py measures each one's effect on a step);
 * the restatement adopts all three (the default):
 *   MV_EPS_NORMAL  normal = (S - P) / (1e-6 + dist)  (capsule_mesh), so a touching or
 *                  piercing segment (S == P) gives the zero normal, a nearly touching one a
 *                  short normal (the exact form: the unit normal, the face's outward normal
 *                  at S == P).  dist = |S - P| (capsule_mesh's jp.safe_norm(penetration_vec,
 *                  axis=1) tests jnp.allclose over all twelve triangles at once, which a box
 *                  never meets: the plain norm)
 *   MV_POS_TRI     the contact position is the triangle point P = S - (1e-6 + dist) n
 *                  (capsule_mesh: pos = triangle_p; the exact form: the capsule's surface point
 *                  S - r n)
 *   MV_FORM        the closest points by brax's _closest_segment_triangle_points: three
 *                  segment-segment pairs (_closest_segment_to_segment_points: directions
 *                  d / (len + 1e-6), mid-point parameters, the (denom + 1e-6) line solution,
 *                  both clipped, then each re-projected onto the other segment by
 *                  _closest_segment_point with (d.d + 1e-6)), the segment-plane point
 *                  (_closest_segment_point_plane: (d - n.a) / (n.(b - a) + 1e-6), clipped) and
 *                  its barycentric closest triangle point (_closest_triangle_point), the
 *                  minimum of the four squared distances, ties averaged.
 * Frames and shared terms: the capsule's segment quantities (length, direction, mid point,
 * 1 / (d.d + 1e-6)) are formed once per wall in the wall frame (x, y, z order) and permuted
 * into face coordinates; a face's edges are exact constants of its half extents.  Triangles
 * (p0, p1, p2): t0 = (V0, V1, V2), t1 = (V0, V2, V3) of the face rectangle V0 = (-ha, -hb),
 * V1 = (ha, -hb), V2 = (ha, hb), V3 = (-ha, hb) (the restatement's triangulation; brax's
 * TriangulatedBox vertex order is not recoverable here).  Divisions are a * (1 / b) (the
 * spec's rule; brax divides: <= 1 ulp apart). */
#define MV_EPS_NORMAL 1
#define MV_POS_TRI 4
#define MV_FORM 8
#define MV_BRAX (MV_EPS_NORMAL | MV_POS_TRI | MV_FORM)
/* (the default, MV_BRAX: brax's spelling as recalled -- parity-unpinned, see the file header) */
static int g_mesh_variant = MV_BRAX;
void orc_set_mesh_variant(int v) { g_mesh_variant = v; }
int orc_get_mesh_variant(void) { return g_mesh_variant; }

static inline f3 F3(float a, float b, float w) { f3 r = {a, b, w}; return r; }
static inline f3 f3sub(f3 x, f3 y) { FL(3); return F3(x.a - y.a, x.b - y.b, x.w - y.w); }
static inline float f3dot(f3 x, f3 y) { FL(5); return fmaf(x.w, y.w, fmaf(x.b, y.b, x.a * y.a)); }
/* p + d s, fused per component */
static inline f3 f3fma(f3 d, float s, f3 p) { FL(6); return F3(fmaf(d.a, s, p.a), fmaf(d.b, s, p.b), fmaf(d.w, s, p.w)); }
static inline float bdist2(f3 x, f3 y) { const f3 d = f3sub(x, y); return f3dot(d, d); }
/* jp.clip as selects (the same bits on every target, -0 and NaN included: NaN clips to the
 * lower bound, -0 to +0 / -h) */
static inline float bclamp01(float x) { return x > 0.0f ? (x < 1.0f ? x : 1.0f) : 0.0f; }
static inline float bclamps(float x, float h) { return x > -h ? (x < h ? x : h) : -h; }

/* a segment p0 -> p0 + d with brax's derived quantities: len = jp.safe_norm(d) (0 when every
 * |d_i| <= 1e-8), il = 1 / (len + 1e-6), dir = d il, hl = len 0.5, mid = p0 + dir hl,
 * idd = 1 / (d.d + 1e-6) */
typedef struct { f3 p0, d, dir, mid; float hl, il, idd; } bseg_t;
static bseg_t bseg_make(f3 p0, f3 d) {
  bseg_t s;
  s.p0 = p0; s.d = d;
  const float dd = f3dot(d, d);
  FL(1 + 2 + 3 + 1 + 2);
  const float len = (fabsf(d.a) <= 1e-8f && fabsf(d.b) <= 1e-8f && fabsf(d.w) <= 1e-8f) ? 0.0f : sqrtf(dd);
  s.il = 1.0f / (len + 1e-6f);
  s.dir = F3(d.a * s.il, d.b * s.il, d.w * s.il);
  s.hl = len * 0.5f;
  s.mid = f3fma(s.dir, s.hl, p0);
  s.idd = 1.0f / (dd + 1e-6f);
  return s;
}
/* wall-frame (x, y, z) -> face coordinates (a, b, w) of axis k */
static inline f3 fperm(f3 v, int k) { return k == 0 ? F3(v.b, v.w, v.a) : (k == 1 ? F3(v.a, v.w, v.b) : v); }
static inline bseg_t bseg_perm(const bseg_t *s, int k) {
  bseg_t r = *s;
  r.p0 = fperm(s->p0, k); r.d = fperm(s->d, k); r.dir = fperm(s->dir, k); r.mid = fperm(s->mid, k);
  return r;
}
/* _closest_segment_point(p0, p0 + d, pt): t = clip((pt - p0).d / (d.d + 1e-6), 0, 1) */
static inline f3 bseg_point(const bseg_t *s, f3 pt, float *tp) {
  FL(1);
  const float t = bclamp01(f3dot(f3sub(pt, s->p0), s->d) * s->idd);
  *tp = t;
  return f3fma(s->d, t, s->p0);
}
/* _closest_segment_to_segment_points(A, E) -> (best_a, best_b); *u = best_a's parameter on A */
static float bseg_seg(const bseg_t *A, const bseg_t *E, f3 *pa, f3 *pb, float *u) {
  const f3 trans = f3sub(A->mid, E->mid);
  const float dd = f3dot(A->dir, E->dir), dat = f3dot(A->dir, trans), dbt = f3dot(E->dir, trans);
  FL(2 + 1 + 3 + 2 + 4 + 2);
  const float denom = fmaf(-dd, dd, 1.0f);
  const float ota = fmaf(dd, dbt, -dat) * (1.0f / (denom + 1e-6f));
  const float otb = fmaf(ota, dd, dbt);
  const float ta = bclamps(ota, A->hl), tb = bclamps(otb, E->hl);
  f3 best_a = f3fma(A->dir, ta, A->mid), best_b = f3fma(E->dir, tb, E->mid);
  float s1, s2;
  const f3 new_a = bseg_point(A, best_b, &s1);
  const float d1 = bdist2(best_b, new_a);
  const f3 new_b = bseg_point(E, best_a, &s2);
  const float d2 = bdist2(best_a, new_b);
  float ua = (A->hl + ta) * A->il;
  if (d1 < d2) { best_a = new_a; ua = s1; }
  else best_b = new_b;
  *pa = best_a; *pb = best_b; *u = ua;
  return bdist2(best_a, best_b);
}
/* _closest_triangle_point(p0, p0 + e0, p0 + e1, pt): barycentric (u, v) with the triangle's
 * constants a = e0.e0, b = e0.e1, c = e1.e1, idet = 1 / (a c - b b); else the edges' closest
 * points (p0 p1, p1 p2, p2 p0 given as segments) */
typedef struct { f3 p0, e0, e1; float a, b, c, idet; bseg_t s01, s12, s20; } btri_t;
static f3 btri_point(const btri_t *T, f3 pt) {
  const f3 d = f3sub(pt, T->p0);
  const float e0d = f3dot(T->e0, d), e1d = f3dot(T->e1, d);
  FL(3 + 3 + 1);
  const float u = fmaf(T->c, e0d, -(T->b * e1d)) * T->idet, v = fmaf(T->a, e1d, -(T->b * e0d)) * T->idet;
  const int inside = 0.0f <= u && u <= 1.0f && 0.0f <= v && v <= 1.0f && u + v <= 1.0f;
  f3 cp = f3fma(T->e1, v, f3fma(T->e0, u, T->p0));
  const float d0 = bdist2(cp, pt);
  float t;
  const f3 c1 = bseg_point(&T->s01, pt, &t);
  const float d1 = bdist2(pt, c1);
  float md = d0;
  if (!(d0 < d1 && inside)) { cp = c1; md = d1; }
  const f3 c2 = bseg_point(&T->s12, pt, &t);
  const float d2 = bdist2(pt, c2);
  FL(2);
  if (d2 < md) cp = c2;
  md = fminf(md, d2);
  const f3 c3 = bseg_point(&T->s20, pt, &t);
  const float d3 = bdist2(pt, c3);
  if (d3 < md) cp = c3;
  return cp;
}
static btri_t btri_make(f3 p0, f3 p1, f3 p2) {
  btri_t T;
  T.p0 = p0; T.e0 = f3sub(p1, p0); T.e1 = f3sub(p2, p0);
  T.a = f3dot(T.e0, T.e0); T.b = f3dot(T.e0, T.e1); T.c = f3dot(T.e1, T.e1);
  FL(3 + 1);
  T.idet = 1.0f / fmaf(T.a, T.c, -(T.b * T.b));
  T.s01 = bseg_make(p0, f3sub(p1, p0)); T.s12 = bseg_make(p1, f3sub(p2, p1)); T.s20 = bseg_make(p2, f3sub(p0, p2));
  return T;
}
/* the minimum of the four squared distances, ties averaged (jp.amin, mask, sum / sum(mask)); a
 * triangle whose distances are all NaN has no candidate (d2 = +inf: the exact form's rule) */
static cand_t bpick(const f3 sp[4], const f3 tp[4], const float u[4], const float d2[4]) {
  FL(3);
  const float mn = fminf(fminf(d2[0], d2[1]), fminf(d2[2], d2[3]));
  f3 S = F3(0.0f, 0.0f, 0.0f), P = S;
  float us = 0.0f, cnt = 0.0f;
  int first = -1;
  for (int k = 0; k < 4; ++k)
    if (d2[k] == mn) {
      if (first < 0) first = k;
      FL(7);
      S = F3(S.a + sp[k].a, S.b + sp[k].b, S.w + sp[k].w);
      P = F3(P.a + tp[k].a, P.b + tp[k].b, P.w + tp[k].w);
      us += u[k]; cnt += 1.0f;
    }
  cand_t c; c.d2 = INFINITY; c.u = 0.0f; c.d.a = c.d.b = c.d.w = 0.0f;
  if (first < 0) return c;
  if (cnt > 1.0f) {
    FL(7);
    S = F3(S.a / cnt, S.b / cnt, S.w / cnt); P = F3(P.a / cnt, P.b / cnt, P.w / cnt); us /= cnt;
    c.d = f3sub(S, P); c.d2 = f3dot(c.d, c.d);
  } else {
    c.d = f3sub(sp[first], tp[first]); c.d2 = d2[first];
  }
  c.u = us;
  return c;
}
/* both triangles of face (axis k, outward sign sg, plane w = w0, half extents ha, hb) against
 * the capsule segment A (face coordinates): _closest_segment_triangle_points per triangle */
static void bface(float ha, float hb, float w0, float sg, const bseg_t *A, cand_t c[2]) {
  const f3 V0 = F3(-ha, -hb, w0), V1 = F3(ha, -hb, w0), V2 = F3(ha, hb, w0), V3 = F3(-ha, hb, w0);
  /* the segment-plane point (both triangles: p0 = V0, n = (0, 0, sg); n's zero products drop
   * out exactly) */
  FL(1 + 1 + 1 + 1 + 2);
  const float tt = bclamp01((sg * w0 - sg * A->p0.w) * (1.0f / (sg * A->d.w + 1e-6f)));
  const f3 sp4 = f3fma(A->d, tt, A->p0);
  /* the edges as segments: t0 (V0 V1), (V1 V2), (V0 V2); t1 (V0 V2), (V2 V3), (V0 V3) */
  const bseg_t E01 = bseg_make(V0, f3sub(V1, V0)), E12 = bseg_make(V1, f3sub(V2, V1));
  const bseg_t E02 = bseg_make(V0, f3sub(V2, V0)), E23 = bseg_make(V2, f3sub(V3, V2));
  const bseg_t E03 = bseg_make(V0, f3sub(V3, V0));
  f3 sp[4], tp[4];
  float u[4], d2[4];
  f3 sdg, tdg;
  float udg;
  const float ddg = bseg_seg(A, &E02, &sdg, &tdg, &udg);
  for (int t = 0; t < 2; ++t) {
    if (t == 0) {
      d2[0] = bseg_seg(A, &E01, &sp[0], &tp[0], &u[0]);
      d2[1] = bseg_seg(A, &E12, &sp[1], &tp[1], &u[1]);
      sp[2] = sdg; tp[2] = tdg; u[2] = udg; d2[2] = ddg;
    } else {
      sp[0] = sdg; tp[0] = tdg; u[0] = udg; d2[0] = ddg;
      d2[1] = bseg_seg(A, &E23, &sp[1], &tp[1], &u[1]);
      d2[2] = bseg_seg(A, &E03, &sp[2], &tp[2], &u[2]);
    }
    const btri_t T = t == 0 ? btri_make(V0, V1, V2) : btri_make(V0, V2, V3);
    sp[3] = sp4; u[3] = tt;
    tp[3] = btri_point(&T, sp4);
    d2[3] = bdist2(sp4, tp[3]);
    c[t] = bpick(sp, tp, u, d2);
  }
}

/* ---- the choices of the brax spelling that nothing pins (round 6; DESIGN.md §3, "unpinned
 * choices").  brax v1's TriangulatedBox vertex order and face triangulation are not
 * recoverable without brax, and the restatement evaluates in the wall's own frame where brax
 * evaluates in the world frame.  Each choice is a variant bit on top of the adopted spelling
 * (MV_BRAX), measured by oracle/brax_mesh_study.py --unpinned:
 *   MV_DIAG    the face's other diagonal (V1 - V3): t0 = (V1, V2, V3), t1 = (V1, V3, V0)
 *   MV_NFLIP   the winding reversed: each triangle's vertices in the opposite order, so
 *              brax's face normal (the segment-plane candidate's n, which enters through
 *              n.(b - a) + 1e-6) points into the box
 *   MV_EDGE    _closest_segment_triangle_points' segment-segment edges as the loop p0 p1,
 *              p1 p2, p2 p0 (the restatement: p0 p1, p1 p2, p0 p2 -- the diagonal then shared
 *              by the face's two triangles)
 *   MV_WORLD   the world frame: the face's vertices and its normal rotated by the wall's z
 *              rotation and translated by its centre, the capsule's segment from its world end
 *              points, the generic 3-D forms throughout, the normal (S - P) / (1e-6 + |S - P|)
 *              in world coordinates
 *   MV_GENERIC the variant path with none of the above (bit-identical to bface: a self-check)
 * The default stays MV_BRAX (the kernels' spelling). */
#define MV_DIAG 16
#define MV_NFLIP 32
#define MV_EDGE 64
#define MV_WORLD 128
#define MV_GENERIC 256
#define MV_VARPATH (MV_DIAG | MV_NFLIP | MV_EDGE | MV_WORLD | MV_GENERIC)

/* both triangles of a face given by its corners V[0..3] (V0 V1 V2 V3 of bface, in the frame of
 * evaluation) and its outward normal n (same frame) against the capsule segment A */
static void bface_var(const f3 V[4], f3 nout, int mv, const bseg_t *A, cand_t c[2]) {
  static const int TRI[2][2][3] = {{{0, 1, 2}, {0, 2, 3}}, {{1, 2, 3}, {1, 3, 0}}};
  const f3 n = (mv & MV_NFLIP) ? F3(-nout.a, -nout.b, -nout.w) : nout;
  for (int t = 0; t < 2; ++t) {
    const int *id = TRI[(mv & MV_DIAG) ? 1 : 0][t];
    const f3 p0 = V[id[0]], p1 = V[(mv & MV_NFLIP) ? id[2] : id[1]], p2 = V[(mv & MV_NFLIP) ? id[1] : id[2]];
    /* _closest_segment_point_plane(a, b, p0, n): t = (p0.n - n.a) / (n.(b - a) + 1e-6), clipped */
    FL(1 + 1 + 1);
    const float tt = bclamp01((f3dot(p0, n) - f3dot(n, A->p0)) * (1.0f / (f3dot(n, A->d) + 1e-6f)));
    f3 sp[4], tp[4];
    float u[4], d2[4];
    const bseg_t Ea = bseg_make(p0, f3sub(p1, p0)), Eb = bseg_make(p1, f3sub(p2, p1));
    const bseg_t Ec = (mv & MV_EDGE) ? bseg_make(p2, f3sub(p0, p2)) : bseg_make(p0, f3sub(p2, p0));
    d2[0] = bseg_seg(A, &Ea, &sp[0], &tp[0], &u[0]);
    d2[1] = bseg_seg(A, &Eb, &sp[1], &tp[1], &u[1]);
    d2[2] = bseg_seg(A, &Ec, &sp[2], &tp[2], &u[2]);
    const btri_t T = btri_make(p0, p1, p2);
    sp[3] = f3fma(A->d, tt, A->p0);
    u[3] = tt;
    tp[3] = btri_point(&T, sp[3]);
    d2[3] = bdist2(sp[3], tp[3]);
    c[t] = bpick(sp, tp, u, d2);
  }
}

/* component k of the wall-local vector (x, y, z) */
static inline float comp(v3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }
/* wall-local (x, y, z) -> world: R_z(theta) l + c (the inverse of capsule_wall_mesh's map) */
static inline v3 wall_to_world(const orc_env *e, int w, v3 l, int point) {
  const float c = e->wall_cos[w], s = e->wall_sin[w];
  v3 r = V(fmaf(-l.y, s, l.x * c), fmaf(l.y, c, l.x * s), l.z);
  if (point) r = vadd(r, e->wall_c[w]);
  return r;
}

/* the mesh contacts of capsule i (world end points pa, pb; pb unused for the torso) against
 * wall w, appended to ct */
static void capsule_wall_mesh(const orc_env *e, int i, int w, v3 pa, v3 pb, contacts_t *ct) {
  const float c = e->wall_cos[w], s = e->wall_sin[w];
  const v3 h = e->wall_h[w];
  const float r = e->cap_r[i];
  const int seg = e->cap_nend[i] == 2;
  FL(3 + 6 + (seg ? 9 : 0));
  const v3 da = vsub(pa, e->wall_c[w]);
  const v3 La = V(fmaf(da.y, s, da.x * c), fmaf(da.y, c, -(da.x * s)), da.z);
  v3 Lb = La;
  if (seg) { const v3 db = vsub(pb, e->wall_c[w]); Lb = V(fmaf(db.y, s, db.x * c), fmaf(db.y, c, -(db.x * s)), db.z); }
  const float R = r + WALL_CULL_MARGIN;
  const int mv = g_mesh_variant;
  /* brax form: the capsule's segment quantities once per wall, in the wall frame (x, y, z) */
  bseg_t capw;
  if (mv & MV_FORM) capw = bseg_make(F3(La.x, La.y, La.z), f3sub(F3(Lb.x, Lb.y, Lb.z), F3(La.x, La.y, La.z)));
  /* (MV_WORLD: the segment from the world end points) */
  bseg_t capworld;
  if (mv & MV_WORLD) {
    const v3 wb = seg ? pb : pa;
    capworld = bseg_make(F3(pa.x, pa.y, pa.z), f3sub(F3(wb.x, wb.y, wb.z), F3(pa.x, pa.y, pa.z)));
  }
  CST(0, 1);
  int n_hit = 0;
  for (int f = 0; f < 6; ++f) {
    const int k = f >> 1, ka = k == 0 ? 1 : 0, kb = k == 2 ? 1 : 2;
    const float sg = (f & 1) ? 1.0f : -1.0f;
    const float ha = comp(h, ka), hb = comp(h, kb), w0 = sg * comp(h, k);
    const f3 A = {comp(La, ka), comp(La, kb), comp(La, k)};
    const f3 B = {comp(Lb, ka), comp(Lb, kb), comp(Lb, k)};
#ifdef ORC_COUNT_FLOPS
    const int cull = g_face_cull && g_flop_mode == 1;
#else
    const int cull = g_face_cull;
#endif
    if (cull) {
      FL(6);
      const float gw = fmaxf(fminf(A.w, B.w) - w0, w0 - fmaxf(A.w, B.w));
      const float ga = fmaxf(fminf(A.a, B.a) - ha, -ha - fmaxf(A.a, B.a));
      const float gb = fmaxf(fminf(A.b, B.b) - hb, -hb - fmaxf(A.b, B.b));
      if (gw >= R || ga >= R || gb >= R) continue;
    }
    CST(1, 1);
    cand_t cds[2];
    if ((mv & MV_FORM) && (mv & MV_VARPATH)) {
      /* the unpinned choices (variant path): the face's corners in face coordinates, or in
       * the world frame */
      f3 Vc[4] = {F3(-ha, -hb, w0), F3(ha, -hb, w0), F3(ha, hb, w0), F3(-ha, hb, w0)};
      f3 nrm = F3(0.0f, 0.0f, sg);
      if (mv & MV_WORLD) {
        for (int q = 0; q < 4; ++q) {
          float l[3];
          l[ka] = Vc[q].a; l[kb] = Vc[q].b; l[k] = Vc[q].w;
          const v3 wv = wall_to_world(e, w, V(l[0], l[1], l[2]), 1);
          Vc[q] = F3(wv.x, wv.y, wv.z);
        }
        float l[3] = {0.0f, 0.0f, 0.0f};
        l[k] = sg;
        const v3 wn = wall_to_world(e, w, V(l[0], l[1], l[2]), 0);
        nrm = F3(wn.x, wn.y, wn.z);
        bface_var(Vc, nrm, mv, &capworld, cds);
      } else {
        const bseg_t capf = bseg_perm(&capw, k);
        bface_var(Vc, nrm, mv, &capf, cds);
      }
    } else if (mv & MV_FORM) {
      const bseg_t capf = bseg_perm(&capw, k);
      bface(ha, hb, w0, sg, &capf, cds);
    } else {
      f3 D = {0.0f, 0.0f, 0.0f};
      float aa = 0.0f, inv_aa = 0.0f;
      if (seg) {
        FL(3 + 5 + 1);
        D.a = B.a - A.a; D.b = B.b - A.b; D.w = B.w - A.w;
        aa = fmaf(D.w, D.w, fmaf(D.b, D.b, D.a * D.a));
        inv_aa = 1.0f / aa;
      }
      for (int t = 0; t < 2; ++t) cds[t] = seg_tri(t, ha, hb, w0, A, B, seg, D, aa, inv_aa);
    }
    for (int t = 0; t < 2; ++t) {
      const cand_t cd = cds[t];
      FL(1);
      const float dist = sqrtf(cd.d2);
      const float pen = r - dist;
      if (!(pen > 0.0f)) continue;
      f3 nf;
      float cdist; /* |S - P| + 1e-6 (or |S - P|): the contact position's offset from S along -n */
      if (mv & MV_EPS_NORMAL) {
        FL(5);
        cdist = 1e-6f + dist;
        const float inv = 1.0f / cdist;
        nf.a = cd.d.a * inv; nf.b = cd.d.b * inv; nf.w = cd.d.w * inv;
        if (!(cd.d2 > 0.0f)) CST(6, 1);
      } else if (cd.d2 > 0.0f) { FL(4); cdist = dist; const float inv = 1.0f / dist; nf.a = cd.d.a * inv; nf.b = cd.d.b * inv; nf.w = cd.d.w * inv; }
      else { cdist = 0.0f; nf.a = 0.0f; nf.b = 0.0f; nf.w = sg; CST(6, 1); }
      /* back to wall-local (x, y, z), then to the world (MV_WORLD: world already) */
      float nl[3]; nl[ka] = nf.a; nl[kb] = nf.b; nl[k] = nf.w;
      FL(6 + 1);
      const int m = ct->count++;
      ct->body[m] = i; ct->ground[m] = 0; ct->pen[m] = pen; ct->r[m] = (mv & MV_POS_TRI) ? cdist : r;
      ct->tau[m] = 1.0f - 2.0f * cd.u;
      if ((mv & MV_WORLD) && (mv & MV_FORM)) ct->n[m] = V(nf.a, nf.b, nf.w);
      else ct->n[m] = V(fmaf(-nl[1], s, nl[0] * c), fmaf(nl[1], c, nl[0] * s), nl[2]);
      ct->e[m] = V(0.0f, 0.0f, 0.0f);
      ++n_hit;
      if (g_cst_on) {
        /* the segment point inside the box? */
        const float u = cd.u;
        const v3 S = V(fmaf(u, Lb.x - La.x, La.x), fmaf(u, Lb.y - La.y, La.y), fmaf(u, Lb.z - La.z, La.z));
        if (fabsf(S.x) < h.x && fabsf(S.y) < h.y && fabsf(S.z) < h.z) CST(5, 1);
      }
    }
  }
  CST(2, n_hit);
}

/* Test hook (tests/test_contact_mesh.py): the mesh contacts of one capsule against one wall
 * box.  wall = (cx, cy, cz, cos, sin, hx, hy, hz), the capsule's world end points a, b (seg = 0:
 * the sphere at a) and radius r; out[6 k ..] = (tau, nx, ny, nz, pen, cd) of contact k in
 * (face, triangle) order, cd = the contact position's offset from the segment point along -n;
 * returns the count (<= 12). */
int orc_mesh_contacts(const float *wall, const float *a, const float *b, int seg, float r, float *out) {
  orc_env *e = (orc_env *)calloc(1, sizeof(orc_env));
  e->n_walls = 1;
  e->wall_c[0] = V(wall[0], wall[1], wall[2]);
  e->wall_cos[0] = wall[3]; e->wall_sin[0] = wall[4];
  e->wall_h[0] = V(wall[5], wall[6], wall[7]);
  e->cap_r[0] = r; e->cap_nend[0] = seg ? 2 : 1;
  contacts_t *ct = (contacts_t *)malloc(sizeof(contacts_t));
  ct->count = 0;
  capsule_wall_mesh(e, 0, 0, V(a[0], a[1], a[2]), V(b[0], b[1], b[2]), ct);
  for (int k = 0; k < ct->count; ++k) {
    out[6 * k] = ct->tau[k]; out[6 * k + 1] = ct->n[k].x; out[6 * k + 2] = ct->n[k].y;
    out[6 * k + 3] = ct->n[k].z; out[6 * k + 4] = ct->pen[k]; out[6 * k + 5] = ct->r[k];
  }
  const int n = ct->count;
  free(ct); free(e);
  return n;
}

#ifdef ORC_COUNT_FLOPS
/* FLOP-count mode 1 only (no effect on any result).  The HIP kernel's per-lane broadphase
 * (pob_quad.h qdetect, boxes from pob_system.cpp): lane k of an env holds the torso, Aux
 * k+1 and lower leg k; it walks wall w iff the xy AABB of those three body centres meets
 * the wall's xy box grown by the largest capsule reach (|end| + r) + 1e-3. */
static void kernel_wall_masks(const orc_env *e, const body_t *b, uint32_t mask[4]) {
  double reach = 0.0;
  for (int i = 0; i < NDYN; ++i)
    for (int q = 0; q < e->cap_nend[i]; ++q) {
      const v3 c = e->cap_end[i][q];
      reach = fmax(reach, sqrt((double)c.x * c.x + (double)c.y * c.y + (double)c.z * c.z) + e->cap_r[i]);
    }
  reach += 1e-3;
  for (int k = 0; k < 4; ++k) {
    const int l[3] = {0, 2 * k + 1, 2 * k + 2};
    float mnx = b->x[0].x, mxx = mnx, mny = b->x[0].y, mxy = mny;
    for (int t = 1; t < 3; ++t) {
      mnx = fminf(mnx, b->x[l[t]].x); mxx = fmaxf(mxx, b->x[l[t]].x);
      mny = fminf(mny, b->x[l[t]].y); mxy = fmaxf(mxy, b->x[l[t]].y);
    }
    mask[k] = 0u;
    for (int w = 0; w < e->n_walls; ++w) {
      const double c = fabs((double)e->wall_cos[w]), sn = fabs((double)e->wall_sin[w]);
      const double ex = c * e->wall_h[w].x + sn * e->wall_h[w].y, ey = sn * e->wall_h[w].x + c * e->wall_h[w].y;
      const float lox = (float)(e->wall_c[w].x - ex - reach), hix = (float)(e->wall_c[w].x + ex + reach);
      const float loy = (float)(e->wall_c[w].y - ey - reach), hiy = (float)(e->wall_c[w].y + ey + reach);
      if (mnx <= hix && mxx >= lox && mny <= hiy && mxy >= loy) mask[k] |= 1u << w;
    }
  }
}
/* operations of one broadphase-surviving sphere-box pair in the kernel (wall_contact = 1):
 * centre offset, local frame, clamp, distance^2 always; square root, normal and its rotation
 * only when d2 < r^2 (1 + 2^-20) (or the sphere centre is inside) */
static long long pair_flops_executed(const orc_env *e, int w, v3 p, float r) {
  const float c = e->wall_cos[w], s = e->wall_sin[w];
  const v3 h = e->wall_h[w];
  const float dx = p.x - e->wall_c[w].x, dy = p.y - e->wall_c[w].y, dz = p.z - e->wall_c[w].z;
  const float lx = fmaf(dy, s, dx * c), ly = fmaf(dy, c, -(dx * s)), lz = dz;
  const float ex = lx - fminf(fmaxf(lx, -h.x), h.x), ey = ly - fminf(fmaxf(ly, -h.y), h.y);
  const float ez = lz - fminf(fmaxf(lz, -h.z), h.z);
  const float d2 = fmaf(ez, ez, fmaf(ey, ey, ex * ex));
  const float T = (r * r) * 1.00000095367431640625f;
  long long f = 3 + 6 + 6 + 3 + 5;
  if (!(d2 >= T)) f += (d2 > 0.0f ? 5 : 4) + 6;
  return f;
}
#endif

#ifdef ORC_COUNT_FLOPS
/* Statistics hook (FLOP build, mode 1, single-threaded; no effect on results): per env and
 * collide substep, the face items of each body -- the faces the face cull keeps over the walls
 * of the four-lane kernel's broadphase mask of a lane holding the body (the torso: of lane 0) --
 * into buf[(env * nsub + substep) * 9 + body] (scripts/wall_walk_stats.py) */
static int *g_items_buf = NULL;
static int g_items_nsub = 0, g_items_env = 0, g_items_sub = 0;
void orc_items_record(int *buf, int nsub) { g_items_buf = buf; g_items_nsub = nsub; }
static int face_items(const orc_env *e, int i, int w, v3 pa, v3 pb) {
  const float c = e->wall_cos[w], s = e->wall_sin[w];
  const v3 h = e->wall_h[w];
  const v3 da = vsub(pa, e->wall_c[w]), db = vsub(pb, e->wall_c[w]);
  const v3 La = V(fmaf(da.y, s, da.x * c), fmaf(da.y, c, -(da.x * s)), da.z);
  const v3 Lb = V(fmaf(db.y, s, db.x * c), fmaf(db.y, c, -(db.x * s)), db.z);
  const float R = e->cap_r[i] + WALL_CULL_MARGIN;
  int n = 0;
  for (int f = 0; f < 6; ++f) {
    const int k = f >> 1, ka = k == 0 ? 1 : 0, kb = k == 2 ? 1 : 2;
    const float w0 = ((f & 1) ? 1.0f : -1.0f) * comp(h, k), ha = comp(h, ka), hb = comp(h, kb);
    const float Aw = comp(La, k), Bw = comp(Lb, k), Aa = comp(La, ka), Ba = comp(Lb, ka), Ab = comp(La, kb), Bb = comp(Lb, kb);
    const float gw = fmaxf(fminf(Aw, Bw) - w0, w0 - fmaxf(Aw, Bw));
    const float ga = fmaxf(fminf(Aa, Ba) - ha, -ha - fmaxf(Aa, Ba));
    const float gb = fmaxf(fminf(Ab, Bb) - hb, -hb - fmaxf(Ab, Bb));
    if (!(gw >= R || ga >= R || gb >= R)) ++n;
  }
  return n;
}
#endif

/* contact detection for the collide substep: ground (CapsulePlane on the torso and the four
 * lower legs), then per capsule its Ant x Arena contacts (wall_contact 0: every penetrating
 * triangle of every wall; 1: the deepest sphere-box contact over end points x walls). */
static void detect(const orc_env *e, const body_t *b, contacts_t *ct) {
  int k = 0;
  for (int g = 0; g < e->n_ground; ++g, ++k) {
    int i = e->ground_body[g];
    v3 pe = cpoint(e->ground_end[g], b->q[i], b->x[i]);
    FL(1);
    ct->pen[k] = e->ground_r[g] - pe.z;
    ct->n[k] = V(0.0f, 0.0f, 1.0f);
    ct->e[k] = e->ground_end[g]; ct->r[k] = e->ground_r[g]; ct->body[k] = i; ct->ground[k] = 1; ct->tau[k] = 0.0f;
  }
  ct->count = k;
#ifdef ORC_COUNT_FLOPS
  uint32_t lane_mask[4] = {0u, 0u, 0u, 0u};
  if (g_flop_mode == 1) kernel_wall_masks(e, b, lane_mask);
#endif
  if (e->n_walls > 0) CST(7, 1);
#ifdef ORC_COUNT_FLOPS
  if (g_flop_mode == 1 && g_items_buf && g_items_sub < g_items_nsub) {
    v3 sa[NDYN], sb[NDYN];
    for (int i = 0; i < NDYN; ++i) {
      sa[i] = cpoint(e->cap_end[i][0], b->q[i], b->x[i]);
      sb[i] = cpoint(e->cap_end[i][e->cap_nend[i] - 1], b->q[i], b->x[i]);
    }
    for (int i = 0; i < NDYN; ++i) {
      const uint32_t lm = lane_mask[i == 0 ? 0 : (i - 1) / 2];
      int n = 0;
      for (int w = 0; w < e->n_walls; ++w)
        if ((lm >> w) & 1u) n += face_items(e, i, w, sa[i], sb[i]);
      g_items_buf[((size_t)g_items_env * g_items_nsub + g_items_sub) * NDYN + i] = n;
    }
    ++g_items_sub;
  }
#endif
  for (int i = 0; i < NDYN; ++i) {
    v3 pe[2]; /* the capsule's end points in world (independent of the wall) */
    for (int q = 0; q < e->cap_nend[i]; ++q) pe[q] = cpoint(e->cap_end[i][q], b->q[i], b->x[i]);
#ifdef ORC_COUNT_FLOPS
    const uint32_t lmask = i == 0 ? (lane_mask[0] | lane_mask[1] | lane_mask[2] | lane_mask[3]) : lane_mask[(i - 1) / 2];
#endif
    if (e->p.wall_contact == 0) {
      const int before = ct->count;
      for (int w = 0; w < e->n_walls; ++w) {
#ifdef ORC_COUNT_FLOPS
        const long long f0 = g_flops;
#endif
        capsule_wall_mesh(e, i, w, pe[0], pe[e->cap_nend[i] - 1], ct);
#ifdef ORC_COUNT_FLOPS
        if (g_flop_mode == 1 && !((lmask >> w) & 1u)) g_flops = f0;  /* culled by the kernel's broadphase */
#endif
      }
      const int nh = ct->count - before;
      if (e->n_walls > 0) {
        CST(3, nh > 0);
        if (g_cst_on && nh > g_cst[4]) g_cst[4] = nh;
        CST(8 + (nh < 7 ? nh : 7), 1);
      }
      continue;
    }
    float best = 0.0f; v3 bn = V(0, 0, 0); float btau = 1.0f;
    for (int w = 0; w < e->n_walls; ++w)
      for (int q = 0; q < e->cap_nend[i]; ++q) {
#ifdef ORC_COUNT_FLOPS
        const long long f0 = g_flops;
#endif
        v3 n; float pen = sphere_box(e, w, pe[q], e->cap_r[i], &n);
#ifdef ORC_COUNT_FLOPS
        if (g_flop_mode == 1) g_flops = f0 + (((lmask >> w) & 1u) ? pair_flops_executed(e, w, pe[q], e->cap_r[i]) : 0);
#endif
        if (pen > best) { best = pen; bn = n; btau = q == 0 ? 1.0f : -1.0f; }
      }
    if (best > 0.0f) {
      const int m = ct->count++;
      ct->pen[m] = best; ct->n[m] = bn; ct->tau[m] = btau; ct->e[m] = V(0, 0, 0);
      ct->r[m] = e->cap_r[i]; ct->body[m] = i; ct->ground[m] = 0;
    }
  }
}

/* position-level contact projection (normal + static friction) into DX / DA (DA: the
 * body's accumulated angular correction vector, turned into a rotation update once at the
 * end of the projection) */
static void contact_position(const orc_env *e, const body_t *b, const body_t *prev,
                             const contacts_t *ct, v3 *DX, v3 *DA) {
  for (int k = 0; k < ct->count; ++k) {
    float pen = ct->pen[k];
    if (!(pen > 0.0f)) continue;
    int i = ct->body[k]; v3 n = ct->n[k]; float im = e->inv_mass[i];
    v3 pe = contact_point(e, b, ct, k);
    v3 cp = vfma(n, -ct->r[k], pe);
    v3 rr = vsub(cp, b->x[i]);
    v3 cn = vcross(rr, n);
    FL(2 + 8);
    float w = im + vdot(cn, cn);
    float lam = pen * (1.0f / w);
    v3 P = vscl(n, lam);
    DX[i] = vfma(P, im, DX[i]);
    DA[i] = vadd(DA[i], vcross(rr, P));
    /* static friction against the motion of the contact point over the substep */
    v3 cprev = qrot_add(qrot(rr, qinv(b->q[i])), prev->q[i], prev->x[i]);
    v3 dp = vsub(cp, cprev);
    v3 dpt = vfma(n, -vdot(dp, n), dp);
    float lt = sqrtf(vdot(dpt, dpt));
    FL(1);
    if (lt > 0.0f) {
      v3 t = vdivs(dpt, lt);
      v3 ctn = vcross(rr, t);
      float wt = im + vdot(ctn, ctn);
      float lamt = lt * (1.0f / wt);
      FL(3);
      if (lamt < e->friction * lam) {
        FL(8);
        v3 Pt = vscl(t, -lamt);
        DX[i] = vfma(Pt, im, DX[i]);
        DA[i] = vadd(DA[i], vcross(rr, Pt));
      }
    }
  }
}

/* velocity-level contact solve (dynamic friction + inelastic normal), Jacobi */
static void contact_velocity(const orc_env *e, const body_t *b, const contacts_t *ct, v3 *dV, v3 *dW) {
  for (int k = 0; k < ct->count; ++k) {
    float pen = ct->pen[k];
    if (!(pen > 0.0f)) continue;
    int i = ct->body[k]; v3 n = ct->n[k]; float im = e->inv_mass[i];
    v3 pe = contact_point(e, b, ct, k);
    v3 cp = vfma(n, -ct->r[k], pe);
    v3 rr = vsub(cp, b->x[i]);
    v3 vr = vadd(b->v[i], vcross(b->w[i], rr));
    float vn = vdot(vr, n);
    v3 vt = vfma(n, -vn, vr);
    float lt = sqrtf(vdot(vt, vt));
    FL(1);
    v3 dv = V(0.0f, 0.0f, 0.0f);
    if (lt > 0.0f) {
      FL(4);
      float fr = fminf(e->friction * pen * e->inv_h, lt);
      dv = vscl(vt, -(fr * (1.0f / lt)));
    }
    if (vn < 0.0f) dv = vfma(n, -vn, dv);
    float D = sqrtf(vdot(dv, dv));
    FL(1);
    if (D > 0.0f) {
      FL(1);
      v3 dh = vdivs(dv, D);
      v3 cd = vcross(rr, dh);
      float w = im + vdot(cd, cd);
      v3 P = vdivs(dv, w);
      dV[i] = vfma(P, im, dV[i]);
      dW[i] = vadd(dW[i], vcross(rr, P));
    }
  }
}

/* ------------------------------------------------------------------ the PBD step */
/* acc += sign * 0.5 * d as one fused multiply-add per component (sign * 0.5 exact) */
static void qadd_half(q4 *acc, q4 d, float sign) {
  FL(9);
  const float h = 0.5f * sign;
  acc->w = fmaf(h, d.w, acc->w); acc->x = fmaf(h, d.x, acc->x);
  acc->y = fmaf(h, d.y, acc->y); acc->z = fmaf(h, d.z, acc->z);
}

/* Jacobi joint projection.  Every angular correction of a body in one substep is applied
 * through the SAME quaternion (the body's pose at the start of the projection), so the
 * per-constraint rotation updates 0.5 [0, a_k] q are summed as vectors first
 * (sum_k 0.5 [0, a_k] q = 0.5 [0, sum_k a_k] q): per joint, s = Pa + Pl, parent
 * += (rp x P) + s, child -= (rc x P) + s; the quaternion product happens once per body. */
static void joints_position(const orc_env *e, const body_t *b, v3 *DX, v3 *DA) {
  for (int j = 0; j < NJ; ++j) {
    int p = jparent(j), c = jchild(j);
    float imp = e->inv_mass[p], imc = e->inv_mass[c];
    /* the joint's vectors in world frame through the bodies' rotation matrices */
    const m3 Rp = qmat(b->q[p]), Rc = qmat(b->q[c]);
    v3 rp = mrot(&Rp, e->off_p[j]), rc = mrot(&Rc, e->off_c[j]);
    v3 ap = mrot(&Rp, e->axis[j]), ac = mrot(&Rc, e->axis[j]);
    v3 fp = mrot(&Rp, e->ref[j]), fc = mrot(&Rc, e->ref[j]);
    /* point-to-point: the XPBD step along n = d / L with generalized inverse masses
     * w = im + |r x n|^2 and lambda = s_pos L / (w_p + w_c), written without the square
     * root: P = n lambda = d k and r x P = (r x d) k with
     * k = s_pos L^2 / (L^2 (im_p + im_c) + |rp x d|^2 + |rc x d|^2).
     * P = 0 when the anchors coincide; the (zero) corrections are accumulated anyway. */
    v3 d = vsub(vadd(b->x[c], rc), vadd(b->x[p], rp));
    const float L2 = vdot(d, d);
    v3 P = V(0.0f, 0.0f, 0.0f), xp = P, xc = P;
    if (L2 > 0.0f) {
      FL(1 + 2 + 1 + 1 + 1);
      const v3 ep = vcross(rp, d), ec = vcross(rc, d);
      const float den = fmaf(L2, imp + imc, vdot(ep, ep) + vdot(ec, ec));
      const float k = (L2 * e->s_pos) * (1.0f / den);
      P = vscl(d, k); xp = vscl(ep, k); xc = vscl(ec, k);
    }
    DX[p] = vfma(P, imp, DX[p]);
    DX[c] = vfma(P, -imc, DX[c]);
    /* hinge axis alignment (unit inverse inertia: w_p = w_c = 1) */
    v3 Pa = vscl(vcross(ap, ac), e->half_s_ang);
    /* angle limits (brax math.signed_angle about the parent's hinge axis) */
    float psi = orc_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
    float dl = 0.0f;
    if (psi < e->lim_lo[j]) { FL(1); dl = psi - e->lim_lo[j]; }
    else if (psi > e->lim_hi[j]) { FL(1); dl = psi - e->lim_hi[j]; }
    FL(1);
    v3 Pl = vscl(ap, dl * e->half_s_ang);
    v3 s = vadd(Pa, Pl);
    DA[p] = vadd(DA[p], vadd(xp, s));
    DA[c] = vsub(DA[c], vadd(xc, s));
  }
}

/* Torque actuator gate: brax applies NO actuator torque while the joint angle is outside its
 * limits (pinned in legacy mode by the notebook trajectory, oracle/legacy_np.py; the Torque
 * actuator [ext] is shared by both dynamics modes).  Here at the substep-start pose: the
 * angle's direction (gx, gy) = (ref . u, (ref x u) . axis), u = the child's reference
 * direction in the parent frame through M = R(q_p^-1 q_c); psi = atan2(gy, gx) lies in
 * [lo, hi] (both within (-pi/2, pi/2), checked at env creation) iff gx > 0 and
 * tan(lo) gx <= gy <= tan(hi) gx -- the same decision as the angle test up to rounding at the
 * limit itself, without the arctangent. */
static int actuator_inside(const orc_env *e, int j, q4 qp, q4 qc) {
  const q4 r = qmul(qinv(qp), qc);
  const m3 M = qmat(r);
  const v3 u = mrot(&M, e->ref[j]);
  const float gx = vdot(e->ref[j], u), gy = vdot(vcross(e->ref[j], u), e->axis[j]);
  FL(2);
  return gx > 0.0f && gy >= e->tan_lo[j] * gx && gy <= e->tan_hi[j] * gx;
}

static void pbd_substep(const orc_env *e, body_t *b, const float *act, int collide, v3 *cvel, v3 *cang) {
  body_t prev = *b;
  /* 1. acceleration level: torque actuators + joint angular damping, gravity */
  v3 dw[NDYN];
  for (int i = 0; i < NDYN; ++i) dw[i] = V(0, 0, 0);
  for (int j = 0; j < NJ; ++j) {
    int p = jparent(j), c = jchild(j);
    v3 a = qrot(e->axis[j], b->q[p]);
    FL(1);
    const float aj = actuator_inside(e, j, b->q[p], b->q[c]) ? act[j] : 0.0f;
    v3 t = vscl(a, aj * e->strength[j]);
    v3 d = vscl(vsub(b->w[p], b->w[c]), e->jdamp[j]);
    v3 tt = vadd(t, d);
    dw[p] = vsub(dw[p], tt);
    dw[c] = vadd(dw[c], tt);
  }
  for (int i = 0; i < NDYN; ++i) {
    FL(18);
    v3 v = b->v[i], w = b->w[i];
    b->v[i] = V(fmaf(e->lin_damp, v.x, e->g[0] * e->h), fmaf(e->lin_damp, v.y, e->g[1] * e->h),
                fmaf(e->lin_damp, v.z, e->g[2] * e->h));
    b->w[i] = V(fmaf(e->ang_damp, w.x, dw[i].x * e->h), fmaf(e->ang_damp, w.y, dw[i].y * e->h),
                fmaf(e->ang_damp, w.z, dw[i].z * e->h));
  }
  /* 2. kinetic */
  for (int i = 0; i < NDYN; ++i) {
    b->x[i] = vfma(b->v[i], e->h, b->x[i]);
    q4 dq = qmul_vq(b->w[i], b->q[i]);
    FL(8);
    q4 q = b->q[i];
    q.w = fmaf(e->half_h, dq.w, q.w); q.x = fmaf(e->half_h, dq.x, q.x);
    q.y = fmaf(e->half_h, dq.y, q.y); q.z = fmaf(e->half_h, dq.z, q.z);
    b->q[i] = qnormalize(q);
  }
  /* 3. position projection (Jacobi over joints + contacts) */
  v3 DX[NDYN], DA[NDYN];
  for (int i = 0; i < NDYN; ++i) { DX[i] = V(0, 0, 0); DA[i] = V(0, 0, 0); }
  joints_position(e, b, DX, DA);
  contacts_t ct; ct.count = 0;
  if (collide) {
    detect(e, b, &ct);
    contact_position(e, b, &prev, &ct, DX, DA);
  }
  for (int i = 0; i < NDYN; ++i) {
    b->x[i] = vadd(b->x[i], DX[i]);
    qadd_half(&b->q[i], qmul_vq(DA[i], b->q[i]), 1.0f);
  }
  /* 4. velocity projection */
  for (int i = 0; i < NDYN; ++i) {
    b->q[i] = qnormalize(b->q[i]);
    b->v[i] = vscl(vsub(b->x[i], prev.x[i]), e->inv_h);
    q4 dq = qmul(b->q[i], qinv(prev.q[i]));
    float sg = dq.w >= 0.0f ? 1.0f : -1.0f;
    FL(9);
    b->w[i] = V(sg * ((2.0f * dq.x) * e->inv_h), sg * ((2.0f * dq.y) * e->inv_h), sg * ((2.0f * dq.z) * e->inv_h));
  }
  /* 5. velocity-level contact solve */
  if (collide) {
    v3 dV[NDYN], dW[NDYN];
    for (int i = 0; i < NDYN; ++i) { dV[i] = V(0, 0, 0); dW[i] = V(0, 0, 0); }
    contact_velocity(e, b, &ct, dV, dW);
    for (int i = 0; i < NDYN; ++i) {
      b->v[i] = vadd(b->v[i], dV[i]); b->w[i] = vadd(b->w[i], dW[i]);
      cvel[i] = vadd(cvel[i], dV[i]); cang[i] = vadd(cang[i], dW[i]);
    }
  }
}

static void load_body(const orc_env *e, const float *pos, const float *rot, const float *vel,
                      const float *ang, body_t *b) {
  (void)e;
  for (int i = 0; i < NDYN; ++i) {
    b->x[i] = V(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]);
    b->q[i].w = rot[4 * i]; b->q[i].x = rot[4 * i + 1]; b->q[i].y = rot[4 * i + 2]; b->q[i].z = rot[4 * i + 3];
    b->v[i] = V(vel[3 * i], vel[3 * i + 1], vel[3 * i + 2]);
    b->w[i] = V(ang[3 * i], ang[3 * i + 1], ang[3 * i + 2]);
  }
}
static void store_body(const body_t *b, float *pos, float *rot, float *vel, float *ang) {
  for (int i = 0; i < NDYN; ++i) {
    pos[3 * i] = b->x[i].x; pos[3 * i + 1] = b->x[i].y; pos[3 * i + 2] = b->x[i].z;
    rot[4 * i] = b->q[i].w; rot[4 * i + 1] = b->q[i].x; rot[4 * i + 2] = b->q[i].y; rot[4 * i + 3] = b->q[i].z;
    vel[3 * i] = b->v[i].x; vel[3 * i + 1] = b->v[i].y; vel[3 * i + 2] = b->v[i].z;
    ang[3 * i] = b->w[i].x; ang[3 * i + 1] = b->w[i].y; ang[3 * i + 2] = b->w[i].z;
  }
}

/* ------------------------------------------------------- the legacy spring step */
/* One-way contact impulses of brax <= 0.0.12 (OneWayCollider [ext]; ground contacts pinned by
 * the notebook trajectory): Baumgarte-stabilised inelastic normal impulse and Coulomb drag
 * capped by friction * normal impulse, applied when penetrating, approaching and the impulse
 * is positive (the drag also needs a tangential speed above 0.01).  Velocity deltas per
 * body, summed in contact order (ground contacts, then each capsule's deepest wall contact). */
static void legacy_contacts(const orc_env *e, const body_t *b, v3 *dV, v3 *dW) {
  contacts_t ct; detect(e, b, &ct);
  for (int k = 0; k < ct.count; ++k) {
    const float pen = ct.pen[k];
    if (!(pen > 0.0f)) continue;
    const int i = ct.body[k]; const v3 n = ct.n[k];
    const v3 pe = contact_point(e, b, &ct, k);
    const v3 rel = vsub(vfma(n, -ct.r[k], pe), b->x[i]);
    const v3 cv = vadd(b->v[i], vcross(b->w[i], rel));
    const float nv = vdot(n, cv);
    const float ang = vdot(n, vcross(vcross(rel, n), rel));
    FL(6);
    const float rden = 1.0f / (e->inv_mass[i] + ang);
    const float imp = (e->erp * pen - nv) * rden;
    if (!(nv < 0.0f && imp > 0.0f)) continue;
    const v3 vd = vfma(n, -nv, cv);
    const float nd = sqrtf(vdot(vd, vd));
    v3 P = vscl(n, imp);
    if (nd > 0.01f) {
      FL(6);
      const float impd = fminf(nd * rden, e->friction * imp);
      P = vfma(vd, -(impd * (1.0f / (1e-6f + nd))), P);
    }
    dV[i] = vfma(P, e->inv_mass[i], dV[i]);
    dW[i] = vadd(dW[i], vcross(rel, P));
  }
}

/* revolute spring joints + torque actuators of brax <= 0.0.12 as accelerations [ext]: anchor
 * spring k (p_p - p_c) + c (v_p - v_c), axis alignment k ap x ac, limit spring -k ap dang,
 * damping -20 (w_p - w_c); actuator ap * act * 350, gated off outside the limits.  Body terms
 * summed in joint order. */
static void legacy_joints(const orc_env *e, const body_t *b, const float *act, v3 *dv, v3 *dw) {
  for (int j = 0; j < NJ; ++j) {
    const int p = jparent(j), c = jchild(j);
    const v3 rp = qrot(e->off_p[j], b->q[p]), rc = qrot(e->off_c[j], b->q[c]);
    const v3 dpos = vsub(vadd(b->x[p], rp), vadd(b->x[c], rc));
    const v3 dvel = vsub(vadd(b->v[p], vcross(b->w[p], rp)), vadd(b->v[c], vcross(b->w[c], rc)));
    const v3 imp = vfma(dpos, e->k_spring, vscl(dvel, e->c_spring));
    const v3 ap = qrot(e->axis[j], b->q[p]), ac = qrot(e->axis[j], b->q[c]);
    const v3 fp = qrot(e->ref[j], b->q[p]), fc = qrot(e->ref[j], b->q[c]);
    const float psi = orc_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
    float dang = 0.0f;
    if (psi < e->lim_lo[j]) { FL(1); dang = e->lim_lo[j] - psi; }
    else if (psi > e->lim_hi[j]) { FL(1); dang = e->lim_hi[j] - psi; }
    FL(2);
    v3 tq = vscl(vcross(ap, ac), e->k_spring);
    tq = vfma(ap, -(e->k_limit * dang), tq);
    tq = vfma(vsub(b->w[p], b->w[c]), -e->jdamp[j], tq);
    const v3 ta = vscl(ap, (dang != 0.0f ? 0.0f : act[j]) * e->strength[j]);
    const v3 tw = vsub(tq, ta);  /* parent: + tw, child: - tw */
    dv[p] = vfma(imp, -e->inv_mass[p], dv[p]);
    dv[c] = vfma(imp, e->inv_mass[c], dv[c]);
    dw[p] = vadd(dw[p], vadd(vcross(rp, vscl(imp, -1.0f)), tw));
    dw[c] = vadd(dw[c], vsub(vcross(rc, imp), tw));
  }
}

static void legacy_substep(const orc_env *e, body_t *b, const float *act, v3 *cvel, v3 *cang) {
  /* kinetic */
  for (int i = 0; i < NDYN; ++i) {
    b->x[i] = vfma(b->v[i], e->h, b->x[i]);
    q4 dq = qmul_vq(b->w[i], b->q[i]);
    FL(8);
    q4 q = b->q[i];
    q.w = fmaf(e->half_h, dq.w, q.w); q.x = fmaf(e->half_h, dq.x, q.x);
    q.y = fmaf(e->half_h, dq.y, q.y); q.z = fmaf(e->half_h, dq.z, q.z);
    b->q[i] = qnormalize(q);
  }
  /* joints + actuators -> potential update (gravity, damping) */
  v3 dv[NDYN], dw[NDYN];
  for (int i = 0; i < NDYN; ++i) { dv[i] = V(0, 0, 0); dw[i] = V(0, 0, 0); }
  legacy_joints(e, b, act, dv, dw);
  for (int i = 0; i < NDYN; ++i) {
    FL(24);
    const v3 v = b->v[i], w = b->w[i];
    b->v[i] = V(fmaf(e->lin_damp, v.x, (dv[i].x + e->g[0]) * e->h), fmaf(e->lin_damp, v.y, (dv[i].y + e->g[1]) * e->h),
                fmaf(e->lin_damp, v.z, (dv[i].z + e->g[2]) * e->h));
    b->w[i] = V(fmaf(e->ang_damp, w.x, dw[i].x * e->h), fmaf(e->ang_damp, w.y, dw[i].y * e->h),
                fmaf(e->ang_damp, w.z, dw[i].z * e->h));
  }
  /* collisions: velocity impulses */
  v3 dV[NDYN], dW[NDYN];
  for (int i = 0; i < NDYN; ++i) { dV[i] = V(0, 0, 0); dW[i] = V(0, 0, 0); }
  legacy_contacts(e, b, dV, dW);
  for (int i = 0; i < NDYN; ++i) {
    b->v[i] = vadd(b->v[i], dV[i]); b->w[i] = vadd(b->w[i], dW[i]);
    cvel[i] = vadd(cvel[i], dV[i]); cang[i] = vadd(cang[i], dW[i]);
  }
}

/* brax System.step: PBD = substeps/2 iterations of (plain substep, collide substep); legacy
 * spring = substeps of (kinetic, joints + actuators, collisions) */
static void physics_step(const orc_env *e, body_t *b, const float *act, v3 *cvel, v3 *cang) {
  for (int i = 0; i < NDYN; ++i) { cvel[i] = V(0, 0, 0); cang[i] = V(0, 0, 0); }
  if (e->legacy) {
    for (int it = 0; it < e->substeps; ++it) legacy_substep(e, b, act, cvel, cang);
    return;
  }
  for (int it = 0; it < e->substeps / 2; ++it) {
    pbd_substep(e, b, act, 0, cvel, cang);
    pbd_substep(e, b, act, 1, cvel, cang);
  }
}

/* sys.info(qp).contact (a2): contact passes evaluated at a static state */
static void info_contact(const orc_env *e, const body_t *b, v3 *cvel, v3 *cang) {
  for (int i = 0; i < NDYN; ++i) { cvel[i] = V(0, 0, 0); cang[i] = V(0, 0, 0); }
  if (e->legacy) { legacy_contacts(e, b, cvel, cang); return; }  /* the colliders' impulses */
  contacts_t ct; detect(e, b, &ct);
  contact_velocity(e, b, &ct, cvel, cang);
}
void orc_contact_info(const orc_env *e, const float *pos, const float *rot, const float *vel,
                      const float *ang, float *cvel, float *cang) {
  body_t b; load_body(e, pos, rot, vel, ang, &b);
  v3 cv[NDYN], ca[NDYN];
  info_contact(e, &b, cv, ca);
  for (int i = 0; i < e->N; ++i) {
    float *o = cvel + 3 * i, *a = cang + 3 * i;
    if (i < NDYN) { o[0] = cv[i].x; o[1] = cv[i].y; o[2] = cv[i].z; a[0] = ca[i].x; a[1] = ca[i].y; a[2] = ca[i].z; }
    else { o[0] = o[1] = o[2] = a[0] = a[1] = a[2] = 0.0f; }
  }
}

/* ------------------------------------------------------------------ observations */
static inline float clip1(float x) { return x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x); }

/* sys.joints[0].angle_vel (a3): signed angle about the parent's hinge axis; d/dt */
static void angle_vel(const orc_env *e, const body_t *b, float *angle, float *avel) {
  for (int j = 0; j < NJ; ++j) {
    int p = jparent(j), c = jchild(j);
    v3 ap = qrot(e->axis[j], b->q[p]);
    v3 fp = qrot(e->ref[j], b->q[p]), fc = qrot(e->ref[j], b->q[c]);
    angle[j] = orc_atan2f(vdot(vcross(fp, fc), ap), vdot(fp, fc));
    avel[j] = vdot(vsub(b->w[c], b->w[p]), ap);
  }
}

/* the 29 + 6N shared prefix (ant_*.py _get_obs).  With sh = -2 it is the stock ant's
 * 27 + 6N layout (brax envs/ant.py _get_obs: qp.pos[0, 2:] keeps only the torso z). */
static void obs_common(const orc_env *e, const body_t *b, const v3 *cvel, const v3 *cang, float *o0, int sh) {
  float ja[NJ], jv[NJ];
  angle_vel(e, b, ja, jv);
  float *o = o0 + sh;
  if (sh == 0) { o[0] = b->x[0].x; o[1] = b->x[0].y; }
  o[2] = b->x[0].z;
  o[3] = b->q[0].w; o[4] = b->q[0].x; o[5] = b->q[0].y; o[6] = b->q[0].z;
  for (int j = 0; j < NJ; ++j) o[7 + j] = ja[j];
  o[15] = b->v[0].x; o[16] = b->v[0].y; o[17] = b->v[0].z;
  o[18] = b->w[0].x; o[19] = b->w[0].y; o[20] = b->w[0].z;
  for (int j = 0; j < NJ; ++j) o[21 + j] = jv[j];
  int N = e->N;
  for (int i = 0; i < N; ++i) {
    v3 c = i < NDYN ? cvel[i] : V(0, 0, 0), a = i < NDYN ? cang[i] : V(0, 0, 0);
    o[29 + 3 * i] = clip1(c.x); o[29 + 3 * i + 1] = clip1(c.y); o[29 + 3 * i + 2] = clip1(c.z);
    o[29 + 3 * N + 3 * i] = clip1(a.x); o[29 + 3 * N + 3 * i + 1] = clip1(a.y); o[29 + 3 * N + 3 * i + 2] = clip1(a.z);
  }
}

static inline float dist2d(float ax, float ay, float bx, float by) {
  float dx = ax - bx, dy = ay - by;
  return sqrtf(dx * dx + dy * dy);
}

/* ant_gather.py:152-181 _get_readings (XLA-CPU scatter order: last writer wins,
 * out-of-range bin -1 wraps to the last slot) */
static void ga_readings(const orc_env *e, const float *pos, q4 rot0, const float *dists, float *rd) {
  int nb = e->p.ga_n_bins, na = e->p.ga_n_apples, no = e->n_obj;
  float half = e->p.ga_sensor_span * 0.5f; /* python float, f32 when used */
  float half_span = (float)((double)e->p.ga_sensor_span / 2.0);
  float bin_res = (float)((2.0 * ((double)e->p.ga_sensor_span / 2.0)) / nb);
  (void)half;
  for (int s = 0; s < 2 * nb; ++s) rd[s] = 0.0f;
  q4 o = {0.0f, 1.0f, 0.0f, 0.0f};
  q4 t = qmul(qmul(rot0, o), qinv(rot0));
  float ori = orc_atan2f(t.y, t.x);
  for (int k = 0; k < no; ++k) {
    float ox = pos[3 * (11 + k)], oy = pos[3 * (11 + k) + 1];
    float angle = orc_atan2f(ox, oy) - ori;
    int in_range = dists[k] <= e->p.ga_sensor_range;
    int bin = (fabsf(angle) <= half_span && in_range) ? (int)((angle + half_span) / bin_res) : -1;
    if (k >= na) bin = bin >= 0 ? bin + na : -1;
    float inten = bin >= 0 ? 1.0f - dists[k] / e->p.ga_sensor_range : 0.0f;
    int slot = bin < 0 ? bin + 2 * nb : bin;
    if (slot >= 0 && slot < 2 * nb) rd[slot] = inten;
  }
}

/* per-env observation for the current env kind */
static void env_obs(const orc_env *e, const body_t *b, const float *pos, const v3 *cvel, const v3 *cang,
                    float flag, const float *dists, float *o) {
  if (e->kind == ORC_ANT) { obs_common(e, b, cvel, cang, o, -2); return; }
  obs_common(e, b, cvel, cang, o, 0);
  int base = 29 + 6 * e->N;
  if (e->kind == ORC_HH) {
    float tx = pos[3 * 11];
    float sgn = tx > 0.0f ? 1.0f : (tx < 0.0f ? -1.0f : 0.0f);
    o[base] = flag > 0.0f ? sgn : 0.0f;
  } else if (e->kind == ORC_GA) {
    ga_readings(e, pos, b->q[0], dists, o + base);
  } else {
    float tx = pos[3 * 10], ty = pos[3 * 10 + 1];
    int vis = dist2d(tx, ty, b->x[0].x, b->x[0].y) <= e->p.tag_visible_radius;
    o[base] = vis ? tx : 0.0f; o[base + 1] = vis ? ty : 0.0f;
  }
}

/* ---------------------------------------------------------------------------- reset */
static void reset_one(const orc_env *e, const uint32_t key[2], float *pos, float *rot, float *vel,
                      float *ang, float *obs, uint32_t *rng_out) {
  const float lo1 = -0.1f, hi1 = 0.1f;
  uint32_t ks[10];
  int nsplit = e->kind == ORC_GA ? 4 : (e->kind == ORC_ANT ? 3 : 5); /* ant.py: split(rng, 3) */
  orc_split(key, nsplit, ks);
  float noise[NJ], qpos[NJ], qvel[NJ];
  orc_uniform(ks + 2, NJ, &lo1, &hi1, 1, noise);
  for (int j = 0; j < NJ; ++j) qpos[j] = e->default_angle[j] + noise[j];
  orc_uniform(ks + 4, NJ, &lo1, &hi1, 1, qvel);
  orc_default_qp(e, qpos, qvel, pos, rot, vel, ang);
  float dists[MAXOBJ];
  if (e->kind == ORC_HH) {
    float lo[2] = {-0.5f, 0.5f}, hi[2] = {0.5f, 1.5f}, axy[2];
    orc_uniform(ks + 6, 2, lo, hi, 2, axy);
    for (int i = 0; i <= 9; ++i) { pos[3 * i] += axy[0]; pos[3 * i + 1] += axy[1]; }
    int idx[2]; orc_choice_idx(ks + 6, 2, 2, idx); /* rng3 reused (ant_heavenhell.py:99) */
    for (int k = 0; k < 2; ++k) {
      int src = idx[k];
      pos[3 * (11 + k)] = e->p.hh_heaven_hell[src][0];
      pos[3 * (11 + k) + 1] = e->p.hh_heaven_hell[src][1];
      pos[3 * (11 + k) + 2] = 1.0f;
    }
    rng_out[0] = ks[0]; rng_out[1] = ks[1];
  } else if (e->kind == ORC_GA) {
    int no = e->n_obj, idx[MAXOBJ];
    orc_choice_idx(ks + 6, e->n_grid, no, idx);
    for (int k = 0; k < no; ++k) {
      pos[3 * (11 + k)] = e->grid[idx[k]][0];
      pos[3 * (11 + k) + 1] = e->grid[idx[k]][1];
      pos[3 * (11 + k) + 2] = k < e->p.ga_n_apples ? 1.0f : e->grid[idx[k]][2];
    }
    for (int k = 0; k < no; ++k)
      dists[k] = dist2d(pos[0], pos[1], pos[3 * (11 + k)], pos[3 * (11 + k) + 1]);
    rng_out[0] = key[0]; rng_out[1] = key[1]; /* ant_gather.py:106 keeps the input key */
  } else if (e->kind == ORC_ANT) {
    rng_out[0] = ks[0]; rng_out[1] = ks[1]; /* not part of the stock ant's State */
  } else {
    float lo[2] = {-e->p.tag_cage_xy[0], -e->p.tag_cage_xy[1]};
    float hi[2] = {e->p.tag_cage_xy[0], e->p.tag_cage_xy[1]}, axy[2], txy[2];
    orc_uniform(ks + 6, 2, lo, hi, 2, axy);
    for (int i = 0; i <= 9; ++i) { pos[3 * i] += axy[0]; pos[3 * i + 1] += axy[1]; }
    uint32_t r[2] = {ks[8], ks[9]};
    orc_uniform(r, 2, lo, hi, 2, txy);
    for (int it = 0; it < 100000 && dist2d(txy[0], txy[1], axy[0], axy[1]) <= e->p.tag_min_spawn_distance; ++it) {
      uint32_t s[4]; orc_split(r, 2, s);
      r[0] = s[2]; r[1] = s[3];
      orc_uniform(r, 2, lo, hi, 2, txy);
    }
    pos[3 * 10] = txy[0]; pos[3 * 10 + 1] = txy[1]; pos[3 * 10 + 2] = 0.5f;
    rng_out[0] = ks[0]; rng_out[1] = ks[1];
  }
  body_t b; load_body(e, pos, rot, vel, ang, &b);
  v3 cv[NDYN], ca[NDYN];
  info_contact(e, &b, cv, ca);
  env_obs(e, &b, pos, cv, ca, 0.0f, dists, obs);
}

void orc_reset(const orc_env *e, int B, const uint32_t *keys, orc_state *s, int nthreads) {
  int N = e->N, D = e->D;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
  for (int b = 0; b < B; ++b) {
    reset_one(e, keys + 2 * b, s->pos + (size_t)b * N * 3, s->rot + (size_t)b * N * 4,
              s->vel + (size_t)b * N * 3, s->ang + (size_t)b * N * 3, s->obs + (size_t)b * D,
              s->rng + 2 * b);
    s->reward[b] = 0.0f; s->done[b] = 0.0f;
    if (s->steps) s->steps[b] = 0.0f;
    if (s->truncation) s->truncation[b] = 0.0f;
    if (s->m0) s->m0[b] = 0.0f;
    if (s->m1) s->m1[b] = 0.0f;
    if (s->m2) s->m2[b] = 0.0f;
    if (s->first_pos) {
      memcpy(s->first_pos + (size_t)b * N * 3, s->pos + (size_t)b * N * 3, sizeof(float) * N * 3);
      memcpy(s->first_rot + (size_t)b * N * 4, s->rot + (size_t)b * N * 4, sizeof(float) * N * 4);
      memcpy(s->first_vel + (size_t)b * N * 3, s->vel + (size_t)b * N * 3, sizeof(float) * N * 3);
      memcpy(s->first_ang + (size_t)b * N * 3, s->ang + (size_t)b * N * 3, sizeof(float) * N * 3);
      memcpy(s->first_obs + (size_t)b * D, s->obs + (size_t)b * D, sizeof(float) * D);
    }
  }
}

/* ----------------------------------------------------------------------------- step */
static void step_one(const orc_env *e, int b, const orc_state *in, const float *act, orc_state *out,
                     int flags, int L) {
  int N = e->N, D = e->D;
  const float *pin = in->pos + (size_t)b * N * 3;
  float *pos = out->pos + (size_t)b * N * 3, *rot = out->rot + (size_t)b * N * 4;
  float *vel = out->vel + (size_t)b * N * 3, *ang = out->ang + (size_t)b * N * 3;
  float *obs = out->obs + (size_t)b * D;
  if (out->pos != in->pos) {
    memcpy(pos, pin, sizeof(float) * N * 3);
    memcpy(rot, in->rot + (size_t)b * N * 4, sizeof(float) * N * 4);
    memcpy(vel, in->vel + (size_t)b * N * 3, sizeof(float) * N * 3);
    memcpy(ang, in->ang + (size_t)b * N * 3, sizeof(float) * N * 3);
  }
  float prev_done = in->done[b];
  float steps = in->steps ? in->steps[b] : 0.0f;
  uint32_t rng[2] = {in->rng[2 * b], in->rng[2 * b + 1]};
  float m0 = in->m0 ? in->m0[b] : 0.0f, m1 = in->m1 ? in->m1[b] : 0.0f, m2 = in->m2 ? in->m2[b] : 0.0f;
  if (flags & ORC_F_AUTORESET) { if (prev_done != 0.0f) steps = 0.0f; }

  body_t bd; load_body(e, pos, rot, vel, ang, &bd);
#ifdef ORC_COUNT_FLOPS
  g_items_env = b; g_items_sub = 0;
#endif
  const float x_before = bd.x[0].x;
  v3 cv[NDYN], ca[NDYN];
  physics_step(e, &bd, act + (size_t)b * NJ, cv, ca);
  store_body(&bd, pos, rot, vel, ang);

  float tz = bd.x[0].z;
  float dead = tz < 0.2f ? 1.0f : 0.0f;
  dead = tz > 1.0f ? 1.0f : dead;
  float reward, done;
  if (e->kind == ORC_HH) {
    reward = dead > 0.0f ? e->p.hh_dying_cost : 0.0f;
    int inr[3];
    for (int k = 0; k < 3; ++k) {
      int idx = k == 0 ? 11 : (k == 1 ? 12 : 10);
      inr[k] = dist2d(pos[3 * idx], pos[3 * idx + 1], bd.x[0].x, bd.x[0].y) <= e->p.hh_visible_radius;
    }
    if (inr[0]) reward = 1.0f;
    if (inr[1]) reward = -1.0f;
    done = reward != 0.0f ? 1.0f : 0.0f;
    env_obs(e, &bd, pos, cv, ca, inr[2] ? 1.0f : 0.0f, NULL, obs);
    m2 = done; /* metrics['hits'] */
  } else if (e->kind == ORC_GA) {
    int no = e->n_obj, na = e->p.ga_n_apples;
    float d[MAXOBJ];
    for (int k = 0; k < no; ++k) d[k] = dist2d(bd.x[0].x, bd.x[0].y, pos[3 * (11 + k)], pos[3 * (11 + k) + 1]);
    env_obs(e, &bd, pos, cv, ca, 0.0f, d, obs);
    reward = dead > 0.0f ? e->p.ga_dying_cost : 0.0f;
    int any_a = 0, any_b = 0, na_hit = 0, nb_hit = 0, all_wait = 1;
    for (int k = 0; k < no; ++k) {
      int c = d[k] <= e->p.ga_catch_range;
      if (c) { pos[3 * (11 + k)] = e->waiting[0]; pos[3 * (11 + k) + 1] = e->waiting[1]; pos[3 * (11 + k) + 2] = e->waiting[2]; }
      if (k < na) { any_a |= c; na_hit += c; } else { any_b |= c; nb_hit += c; }
      all_wait &= (pos[3 * (11 + k)] == e->waiting[0]) & (pos[3 * (11 + k) + 1] == e->waiting[1]) &
                  (pos[3 * (11 + k) + 2] == e->waiting[2]);
    }
    if (any_a && dead == 0.0f) reward = 1.0f;
    if (any_b && dead == 0.0f) reward = -1.0f;
    done = all_wait ? 1.0f : dead;
    m0 = (float)na_hit; m1 = (float)nb_hit;
  } else if (e->kind == ORC_ANT) {
    /* brax envs/ant.py step (brax <= 0.0.12) [ext, recalled]: forward velocity reward,
     * .5 * sum(act^2) control cost, .5e-3 * sum(clip(contact.vel)^2), survive 1; done on
     * torso height.  Sums run in row-major element order (parity unpinned vs XLA). */
    const float *a = act + (size_t)b * NJ;
    float sa = 0.0f;
    for (int j = 0; j < NJ; ++j) sa = sa + a[j] * a[j];
    const float ctrl = 0.5f * sa;
    float sc = 0.0f;
    for (int i = 0; i < NDYN; ++i) {
      float cx = clip1(cv[i].x), cy = clip1(cv[i].y), cz = clip1(cv[i].z);
      sc = sc + cx * cx; sc = sc + cy * cy; sc = sc + cz * cz;
    }
    const float contact = 0.0005f * sc;
    const float forward = (bd.x[0].x - x_before) / e->ctrl_dt;
    reward = ((forward - ctrl) - contact) + 1.0f;
    done = dead;
    env_obs(e, &bd, pos, cv, ca, 0.0f, NULL, obs);
    m0 = ctrl; m1 = contact; m2 = forward;
  } else {
    reward = dead > 0.0f ? e->p.tag_dying_cost : 0.0f;
    /* _step_target (ant_tag.py:129-146) */
    uint32_t s[4]; orc_split(rng, 2, s);
    int ch = orc_randint(s + 2, 0, 4);
    float ax = bd.x[0].x, ay = bd.x[0].y, tx = pos[3 * 10], ty = pos[3 * 10 + 1];
    float vx = ax - tx, vy = ay - ty;
    float nrm = sqrtf(vx * vx + vy * vy);
    vx = vx / nrm; vy = vy / nrm;
    float cx, cy;
    if (ch == 0) { cx = vy * 1.0f; cy = vx * -1.0f; }
    else if (ch == 1) { cx = vy * -1.0f; cy = vx * 1.0f; }
    else if (ch == 2) { cx = -vx; cy = -vy; }
    else { cx = 0.0f; cy = 0.0f; }
    float nx = cx * e->p.tag_target_step + tx, ny = cy * e->p.tag_target_step + ty;
    if (fabsf(nx) > e->p.tag_cage_xy[0] || fabsf(ny) > e->p.tag_cage_xy[1]) { nx = tx; ny = ty; }
    pos[3 * 10] = nx; pos[3 * 10 + 1] = ny; pos[3 * 10 + 2] = 1.0f;
    rng[0] = s[0]; rng[1] = s[1];
    env_obs(e, &bd, pos, cv, ca, 0.0f, NULL, obs);
    float tag = dist2d(bd.x[0].x, bd.x[0].y, nx, ny) <= e->p.tag_tag_radius ? 1.0f : 0.0f;
    m0 = tag;
    if (tag > 0.0f) reward = 1.0f;
    done = (dead != 0.0f || tag != 0.0f) ? 1.0f : 0.0f;
  }
  float trunc = in->truncation ? in->truncation[b] : 0.0f;
  if (flags & ORC_F_EPISODE) {
    steps = steps + 1.0f;
    trunc = steps >= (float)L ? 1.0f - done : 0.0f;
    done = steps >= (float)L ? 1.0f : done;
  }
  if ((flags & ORC_F_AUTORESET) && done != 0.0f) {
    memcpy(pos, in->first_pos + (size_t)b * N * 3, sizeof(float) * N * 3);
    memcpy(rot, in->first_rot + (size_t)b * N * 4, sizeof(float) * N * 4);
    memcpy(vel, in->first_vel + (size_t)b * N * 3, sizeof(float) * N * 3);
    memcpy(ang, in->first_ang + (size_t)b * N * 3, sizeof(float) * N * 3);
    memcpy(obs, in->first_obs + (size_t)b * D, sizeof(float) * D);
  }
  if ((flags & ORC_F_AUTORESET) && out->first_pos != in->first_pos) {
    memcpy(out->first_pos + (size_t)b * N * 3, in->first_pos + (size_t)b * N * 3, sizeof(float) * N * 3);
    memcpy(out->first_rot + (size_t)b * N * 4, in->first_rot + (size_t)b * N * 4, sizeof(float) * N * 4);
    memcpy(out->first_vel + (size_t)b * N * 3, in->first_vel + (size_t)b * N * 3, sizeof(float) * N * 3);
    memcpy(out->first_ang + (size_t)b * N * 3, in->first_ang + (size_t)b * N * 3, sizeof(float) * N * 3);
    memcpy(out->first_obs + (size_t)b * D, in->first_obs + (size_t)b * D, sizeof(float) * D);
  }
  out->reward[b] = reward; out->done[b] = done;
  if (out->steps) out->steps[b] = steps;
  if (out->truncation) out->truncation[b] = trunc;
  if (out->m0) out->m0[b] = m0;
  if (out->m1) out->m1[b] = m1;
  if (out->m2) out->m2[b] = m2;
  out->rng[2 * b] = rng[0]; out->rng[2 * b + 1] = rng[1];
}

void orc_step(const orc_env *e, int B, const orc_state *in, const float *act, orc_state *out, int flags,
              int episode_length, int nthreads) {
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
  for (int b = 0; b < B; ++b) step_one(e, b, in, act, out, flags, episode_length);
}

/* AutoresetVmapGymWrapper.step (wrappers.py:245-262): when any env is done, split the
 * gym key into B+1, reset every env with keys[1:], take qp/obs where done, zero steps. */
void orc_gym_autoreset(const orc_env *e, int B, uint32_t gym_key[2], orc_state *s, int nthreads) {
  int any = 0;
  for (int b = 0; b < B; ++b) any |= s->done[b] != 0.0f;
  if (!any) return;
  int N = e->N, D = e->D;
  uint32_t k0[2];
  split_k(gym_key, B + 1, 0, k0);
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
  for (int b = 0; b < B; ++b) {
    if (s->done[b] == 0.0f) continue;
    uint32_t kb[2], rng_unused[2];
    split_k(gym_key, B + 1, b + 1, kb);
    reset_one(e, kb, s->pos + (size_t)b * N * 3, s->rot + (size_t)b * N * 4, s->vel + (size_t)b * N * 3,
              s->ang + (size_t)b * N * 3, s->obs + (size_t)b * D, rng_unused);
    if (s->steps) s->steps[b] = 0.0f;
  }
  gym_key[0] = k0[0]; gym_key[1] = k0[1];
}
