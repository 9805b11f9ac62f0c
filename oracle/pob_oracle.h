/* pob_oracle.h -- CPU restatement of the po-brax rollout hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product (po-brax_amd/, libpob.so) never links or calls it.
 *
 * It restates, in plain C99 with one env per loop iteration (OpenMP over envs):
 *   - jax.random threefry2x32 split/uniform/randint/choice   (more_jp.py:57-77)
 *   - System.default_angle/default_qp forward kinematics      (a4)
 *   - the PBD physics step (brax v1 dynamics_mode "pbd" as restated in DESIGN.md §3;
 *     brax is not vendored, so this part is PARITY UNPINNED against brax itself)
 *   - AntHeavenHell / AntGather / AntTag reset, step, obs      (ant_*.py)
 *   - EpisodeWrapper / AutoResetWrapper / gym autoreset semantics (wrappers.py)
 * Memory layout = the reference's batch-major pytree layout (B, N, 3) etc.
 */
#ifndef POB_ORACLE_H
#define POB_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_HH = 0, ORC_GA = 1, ORC_TAG = 2, ORC_ANT = 3 };

typedef struct orc_params {
  /* AntHeavenHell (ant_heavenhell.py:51-56) */
  float hh_heaven_hell[2][2];
  float hh_priest[2];
  float hh_visible_radius;
  float hh_dying_cost;
  /* AntGather (ant_gather.py:59-69) */
  int ga_n_apples, ga_n_bombs;
  float ga_cage_xy[2];
  float ga_robot_object_spacing, ga_catch_range;
  int ga_n_bins;
  float ga_sensor_range, ga_sensor_span, ga_dying_cost;
  /* AntTag (ant_tag.py:38-45) */
  float tag_tag_radius, tag_visible_radius, tag_target_step, tag_min_spawn_distance;
  float tag_cage_xy[2];
  float tag_dying_cost;
  /* physics */
  int action_repeat;
  float solver_scale_pos, solver_scale_ang;
  /* dynamics: 0 = PBD (brax 0.0.13-0.0.16 "pbd"), 1 = legacy spring (brax <= 0.0.12, the
   * physics of the notebook trajectory notebooks/ant_tag.ipynb:449) */
  int legacy_spring;
  /* Ant x Arena contact model: 0 = brax v1 capsule x TriangulatedBox (capsule_mesh: every
   * box a 12-triangle mesh, closest segment-triangle points, one contact per penetrating
   * triangle; the reference's algorithm), 1 = the round-1..3 restatement (the
   * deepest sphere-box contact over the capsule's end points, one per capsule) -- kept only to
   * measure the divergence between the two */
  int wall_contact;
} orc_params;

typedef struct orc_state {
  float *pos, *rot, *vel, *ang; /* (B,N,3) (B,N,4) (B,N,3) (B,N,3) */
  float *obs;                   /* (B,D) */
  float *reward, *done;         /* (B,) */
  float *steps, *truncation;    /* (B,) EpisodeWrapper info */
  float *m0, *m1, *m2;          /* metrics, env-specific */
  uint32_t *rng;                /* (B,2) info['rng'] */
  float *first_pos, *first_rot, *first_vel, *first_ang, *first_obs; /* AutoResetWrapper */
} orc_state;

enum {
  ORC_F_EPISODE = 1,    /* EpisodeWrapper: steps/truncation/time-limit done   */
  ORC_F_AUTORESET = 2,  /* brax AutoResetWrapper: first_qp/first_obs on done */
};

typedef struct orc_env orc_env;

orc_env *orc_env_create(int kind, const orc_params *p);
void orc_env_destroy(orc_env *e);
void orc_default_params(orc_params *p);
void orc_env_dims(const orc_env *e, int *n_bodies, int *obs_dim, int *act_dim);

/* algorithmic FLOP counter (only in the -DORC_COUNT_FLOPS build; else -1) */
long long orc_flops_read_and_reset(void);
/* counter mode: 0 every collider pair (reference algorithm), 1 the pairs the HIP kernel
 * evaluates (its exact culls); returns -1 when the counter is not built */
int orc_flops_set_mode(int mode);
/* contact statistics of the mesh contact model (single-threaded runs only; zeroed by the
 * read): out[0] capsule x wall pairs evaluated, [1] faces surviving the face cull, [2]
 * triangle contacts, [3] capsule-substeps with >= 1 wall contact, [4] the largest number of
 * wall contacts of one capsule in one detection, [5] contacts whose segment point lies inside
 * the box, [6] contacts with a zero distance (segment touching the triangle), [7] detections,
 * [8..15] histogram of wall contacts per capsule per detection (0..6, >= 7) */
void orc_contact_stats(long long out[16]);
void orc_contact_stats_enable(int on);
/* test hook: mesh contacts of one capsule (world end points a, b; seg 0 = sphere at a, radius r)
 * against one wall box (cx, cy, cz, cos, sin, hx, hy, hz): out (tau, nx, ny, nz, pen, cd) x count */
int orc_mesh_contacts(const float *wall, const float *a, const float *b, int seg, float r, float *out);
/* 0: evaluate every face of every wall (no face cull; the FLOP counter's reference mode does
 * this too) -- results must be identical to the default (1) */
void orc_set_face_cull(int on);
/* capsule x TriangulatedBox spelling: bit 1 eps-regularised normal, 2 safe_norm, 4 contact at the
 * triangle point, 8 brax's closest-point forms (pob_oracle.c MV_*) */
void orc_set_mesh_variant(int v);
int orc_get_mesh_variant(void);
/* test hook: op 0 atan2f(a, b); op 1 substep quaternion normalisation of a (n x 4) */
void orc_math_check(int op, int n, const float *a, const float *b, float *out);

/* RNG (jax threefry, pre-partitionable) */
void orc_threefry2x32(const uint32_t key[2], uint32_t x0, uint32_t x1, uint32_t out[2]);
void orc_split(const uint32_t key[2], int n, uint32_t *out /* (n,2) */);
void orc_uniform(const uint32_t key[2], int n, const float *lo, const float *hi, int lohi_n,
                 float *out);
int orc_randint(const uint32_t key[2], int lo, int hi);
void orc_choice_idx(const uint32_t key[2], int n, int k, int *out);

/* kinematics: qpos/qvel (8,) -> pos/rot/vel/ang (N, .) of the default qp */
void orc_default_qp(const orc_env *e, const float *qpos, const float *qvel, float *pos,
                    float *rot, float *vel, float *ang);

/* batched env API (B envs, OpenMP over envs when nthreads > 1) */
void orc_reset(const orc_env *e, int B, const uint32_t *keys, orc_state *s, int nthreads);
void orc_step(const orc_env *e, int B, const orc_state *in, const float *act, orc_state *out,
              int flags, int episode_length, int nthreads);
/* AutoresetVmapGymWrapper.step tail (wrappers.py:245-262), in place on s. */
void orc_gym_autoreset(const orc_env *e, int B, uint32_t gym_key[2], orc_state *s,
                       int nthreads);
/* sys.info(qp).contact at a static state (a2) */
void orc_contact_info(const orc_env *e, const float *pos, const float *rot, const float *vel,
                      const float *ang, float *cvel, float *cang);

#ifdef __cplusplus
}
#endif
#endif
