/* pob.h -- C ABI of the MI355X-native po-brax rollout engine (libpob.so).
 *
 * The reference (po_brax, pure Python over brax v1 / JAX) has no native FFI; its
 * drop-in surface for this path is the brax ``Env`` API.  Each entry point below
 * replaces one JAX sub-graph of that surface (file:line in /root/reference):
 *
 *   pob_env_create      AntHeavenHellEnv.__init__  po_brax/envs/ant_heavenhell.py:51-73
 *                       AntGatherEnv.__init__      po_brax/envs/ant_gather.py:59-91
 *                       AntTagEnv.__init__         po_brax/envs/ant_tag.py:38-61
 *                       stock brax Ant             po_brax/envs/__init__.py:30 ('ant' ->
 *                                                  brax.envs.ant.Ant, brax <= 0.0.12) [ext]
 *                       (+ brax.System(cfg) [ext], ActionRepeatWrapper wrappers.py:16-24)
 *   pob_reset           Env.reset: ant_heavenhell.py:75-103, ant_gather.py:93-123,
 *                       ant_tag.py:63-105 ; EpisodeWrapper.reset / AutoResetWrapper.reset
 *                       [ext]; VmapGymWrapper reset closure wrappers.py:160-164
 *   pob_step            Env.step: ant_heavenhell.py:106-158, ant_gather.py:125-213,
 *                       ant_tag.py:107-181, incl. brax System.step [ext] and the
 *                       Episode/AutoReset/RandomizedAutoReset wrappers (__init__.py:59-70,
 *                       wrappers.py:30-123)
 *   pob_step_mixed      several of the above Env.step calls (different env kinds, one
 *                       batch each) fused into ONE kernel launch (BASELINE.json config 5)
 *   pob_reset_where_done AutoresetVmapGymWrapper.step tail wrappers.py:245-262 and
 *                       RandomizedAutoResetWrapperNaive/OnTerminal wrappers.py:30-80
 *   pob_reset_where_done_shard  the same tail for one rank's shard of the gym batch
 *                       (global keys split(gym_key, B_total + 1), all-reduced any-done)
 *   pob_default_qp      System.default_qp(joint_angle, joint_velocity) [ext], called at
 *                       ant_heavenhell.py:95, ant_gather.py:116, ant_tag.py:72
 *   pob_random_*        brax.jumpy.random_split / random_uniform under jit ->
 *                       jax.random.split / uniform (threefry2x32) [ext]; more_jp.py:57-77;
 *                       pob_random_split_batch = the per-env split of
 *                       RandomizedAutoResetWrapperCached.step wrappers.py:103
 *   pob_obs_gather      obs[:, idx] with the index sets of
 *                       po_brax/standard_observability_masks.py:5-67
 *   pob_env_set_obs_mask  the same gather fused into pob_step (pob_state.obs_masked)
 *
 * Conventions: every pointer argument of a compute call is DEVICE memory owned by the
 * caller (the library allocates only its static tables at create time and never per
 * step).  Layouts are the reference's batch-major pytree layouts: pos (B,N,3),
 * rot (B,N,4) wxyz, vel/ang (B,N,3), obs (B,D), keys (B,2) uint32.  `stream` is a
 * hipStream_t (NULL = default stream); calls are stream-ordered and never synchronise
 * the host.  Return value 0 = success, else a negative status; pob_last_error() gives
 * a thread-local message.
 */
#ifndef POB_H
#define POB_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define POB_ABI_VERSION 8

enum pob_kind { POB_HEAVENHELL = 0, POB_GATHER = 1, POB_TAG = 2, POB_ANT = 3 };

/* storage type of the qp tensors (pos/rot/vel/ang and first_qp); compute is float32 */
enum pob_qp_storage { POB_QP_F32 = 0, POB_QP_F16 = 1 };

#define POB_MIX_MAX 4 /* envs per pob_step_mixed launch */

enum pob_status {
  POB_OK = 0,
  POB_EINVAL = -1,   /* bad argument (ValueError on the Python side) */
  POB_EHIP = -2,     /* HIP runtime error (RuntimeError) */
  POB_ENOMEM = -3,
};

/* step flags: the wrapper chain of po_brax.envs.create (__init__.py:59-70) */
enum pob_step_flags {
  POB_F_EPISODE = 1u,         /* brax EpisodeWrapper: steps += 1, time-limit done, truncation */
  POB_F_AUTORESET = 2u,       /* brax AutoResetWrapper: zero steps on prev done, first_qp/obs */
  POB_F_ZERO_STEPS_ON_DONE = 4u, /* RandomizedAutoResetWrapper*: zero steps on prev done only */
};

/* reset_where_done modes */
enum pob_reset_mode {
  POB_RESET_GYM = 0,  /* keys = split(gym_key, B+1)[1:], gym_key <- keys[0] if any done */
  POB_RESET_OWN = 1,  /* keys = state.rng (RandomizedAutoResetWrapperNaive) */
};

/* constructor kwargs of the three env classes (defaults: pob_default_params) */
typedef struct pob_params {
  float hh_heaven_hell[2][2]; /* ant_heavenhell.py:52 */
  float hh_priest[2];         /* :53 */
  float hh_visible_radius;    /* :54 */
  float hh_dying_cost;        /* :55 */
  int ga_n_apples, ga_n_bombs;        /* ant_gather.py:60-61 */
  float ga_cage_xy[2];                /* :62 */
  float ga_robot_object_spacing;      /* :63 */
  float ga_catch_range;               /* :64 */
  int ga_n_bins;                      /* :65 */
  float ga_sensor_range, ga_sensor_span, ga_dying_cost; /* :66-68 */
  float tag_tag_radius, tag_visible_radius, tag_target_step, tag_min_spawn_distance; /* ant_tag.py:39-42 */
  float tag_cage_xy[2];               /* :43 */
  float tag_dying_cost;               /* :44 */
  int action_repeat;                  /* ActionRepeatWrapper wrappers.py:16-24 */
  float solver_scale_pos, solver_scale_ang; /* PBD joint solver scales */
  int qp_storage;                     /* pob_qp_storage (engine extension; default F32) */
  int legacy_spring;                  /* 1: brax <= 0.0.12 spring dynamics (brax Ant(legacy_spring=True),
                                         the physics of notebooks/ant_tag.ipynb:449); 0: PBD */
} pob_params;

/* Env state: device pointers, batch-major.  Optional members may be NULL.  With
 * qp_storage == POB_QP_F16 the qp and first_qp pointers address IEEE binary16 arrays. */
typedef struct pob_state {
  float *pos, *rot, *vel, *ang; /* qp */
  float *obs;
  float *reward, *done;
  float *steps, *truncation;    /* EpisodeWrapper info (optional) */
  float *m0, *m1, *m2;          /* metrics: HH heavens/hells/hits, GA apples/bombs/objects, TAG hits */
  uint32_t *rng;                /* info['rng'] (B,2) */
  float *first_pos, *first_rot, *first_vel, *first_ang, *first_obs; /* AutoResetWrapper (optional) */
  uint32_t *any_done;           /* optional: step ORs 1 into *any_done when any env is done */
  /* Optional typed copies of step outputs, written by pob_step / pob_step_mixed next to the
   * float32 fields so that the caller needs no conversion kernels for the reference's dtypes
   * (ABI v5): AntTag's bool done (done != 0 as bytes 0/1, ant_tag.py:127) and int32 truncation
   * (EpisodeWrapper on a bool done [ext]); AntGather's int32 apples / bombs counts
   * (ant_gather.py:147-148) as (int32) m0 / m1.  The reset entry points ignore them. */
  uint8_t *done_u8;
  int32_t *trunc_i32;
  int32_t *m0_i32, *m1_i32;
  /* Optional (ABI v5): pob_reset_where_done[_shard] zeroes *any_done_clear, so that a caller
   * double-buffering the any-done word (step k ORs into word k % 2, its masked reset reads
   * that word and clears the other) needs no fill kernel per step. */
  uint32_t *any_done_clear;
  /* Optional (ABI v7): obs[:, idx] of the env's observation mask (pob_env_set_obs_mask), (B, K)
   * float32, written by pob_step / pob_step_mixed from the same observation rows in the same
   * launch (po_brax/standard_observability_masks.py:5-67 applied as obs[:, idx]).  Since ABI v8
   * pob_reset and pob_reset_where_done[_shard] write it too, for the rows they reset. */
  float *obs_masked;
  /* Optional (ABI v8): per-env scratch bytes (B of them, any contents on entry) for the
   * four-lane kernel's split launch: its fast launch records in ovf_mark[b] (b = the first env
   * of each 16-env wave) whether that wave's wall contacts overflowed its store, and the fix-up
   * launch right after it re-steps exactly the marked waves.  The marks live outside every
   * output, so no state the caller wrote (first_obs rows copied by AUTORESET, edited info
   * entries) can be taken for one.  NULL: the one-launch form runs instead (the same results,
   * slower at large batches).  pob_step / pob_step_mixed read it from `out`; two launches
   * that may run concurrently must not share it (slices of one buffer are fine). */
  uint8_t *ovf_mark;
} pob_state;

typedef struct pob_env pob_env;

int pob_abi_version(void);
const char *pob_last_error(void);
int pob_default_params(pob_params *p);
int pob_env_create(int kind, const pob_params *p, pob_env **out);
/* Never calls the HIP runtime (safe while a stream is being captured into a hipGraph): the
 * env's device tables (~4 KB) are KEPT until the next pob_env_create or
 * pob_release_deferred call.  The caller must not destroy an env whose launches are still
 * queued or captured in a graph it will replay. */
void pob_env_destroy(pob_env *env);
/* Free the device tables of every destroyed env now (ABI v6); returns how many buffers were
 * released.  Calls hipFree: never call it while a stream is being captured. */
int pob_release_deferred(void);
/* The env's observation mask (ABI v7): K column indices into its observation (0 <= idx < D,
 * K <= 256, host memory); K = 0 clears it.  A step whose pob_state.obs_masked is set stores
 * obs[:, idx] there.  Copies the env's device table (hipMemcpy): call it before stepping,
 * never while a stream is being captured or a launch of this env is queued. */
int pob_env_set_obs_mask(pob_env *env, const int32_t *idx, int K);
int pob_env_dims(const pob_env *env, int *n_bodies, int *obs_dim, int *act_dim);
/* host copy of default_angle() (8 floats, radians): System.default_angle [ext] */
int pob_env_default_angle(const pob_env *env, float *out8);

int pob_reset(pob_env *env, int B, const uint32_t *keys, const pob_state *out, void *stream);
int pob_step(pob_env *env, int B, const pob_state *in, const float *act, const pob_state *out,
             uint32_t flags, int episode_length, void *stream);
/* One launch stepping n (<= POB_MIX_MAX) envs, env k over its own batch B[k] with its own
 * state / action buffers; same semantics per env as pob_step.  All envs must live on the
 * same device and share qp_storage. */
int pob_step_mixed(int n, pob_env *const *envs, const int *B, const pob_state *in,
                   const float *const *act, const pob_state *out, uint32_t flags,
                   int episode_length, void *stream);
int pob_reset_where_done(pob_env *env, int B, int mode, const uint32_t *gym_key_in,
                         uint32_t *gym_key_out, const pob_state *s, void *stream);
/* gym_key_in / gym_key_out must be distinct words, and s->any_done_clear (if set) must not
 * be s->any_done (POB_EINVAL otherwise): the kernel's first block writes the outputs while
 * every block reads the inputs.
 * The same for a shard: this env batch holds rows [first, first + B) of a global batch of
 * `total` envs split over ranks (AutoresetVmapGymWrapper under index sharding).  Gym mode
 * keys are split(gym_key, total + 1)[1 + first + b]; s->any_done must then hold the GLOBAL
 * any-done flag (the caller all-reduces it, MAX, across ranks before this call). */
int pob_reset_where_done_shard(pob_env *env, int B, int total, int first, int mode,
                               const uint32_t *gym_key_in, uint32_t *gym_key_out, const pob_state *s,
                               void *stream);
int pob_default_qp(pob_env *env, int B, const float *qpos, const float *qvel, float *pos, float *rot,
                   float *vel, float *ang, void *stream);

/* jax.random on device: split(key, num) rows [first, first+count) -> out (count,2) */
int pob_random_split(const uint32_t *key, int num, int first, int count, uint32_t *out, void *stream);
/* vmap(split)(keys, num): keys (B,2) -> out (B,num,2)  (jax.vmap(jax.random.split)) */
int pob_random_split_batch(const uint32_t *keys, int B, int num, uint32_t *out, void *stream);
/* uniform(key, (n,), lo, hi) elements [first, first+count) */
int pob_random_uniform(const uint32_t *key, int n, int first, int count, float lo, float hi, float *out,
                       void *stream);
/* bench/rollout helper: key_io <- split(key_io)[0]; act = uniform(split(key_io)[1], (total,A), -1, 1)
 * rows [first, first+B) (a shard of a batch of `total` envs) */
int pob_random_actions(uint32_t *key_io, int total, int first, int B, int A, float *act, void *stream);
/* out[b, k] = obs[b, idx[k]] */
int pob_obs_gather(const float *obs, int B, int D, const int32_t *idx, int K, float *out, void *stream);

#ifdef __cplusplus
}
#endif
#endif
