/*
 * mgx.h -- C ABI of the MI355X-native vectorised MiniGrid engine (libmgx.so).
 *
 * Drop-in boundary.  The reference reaches this path through Python objects,
 * not an FFI; each entry point below replaces one of them:
 *
 *   mgx_create   <- make_vec_env(make_env, n_envs, seed, SubprocVecEnv)  src/ppo.py:118-122
 *                   + PlaygroundEnv.__init__                              src/custom_env.py:74-116
 *                   + VecTransposeImage / VecFrameStack(n_stack,'first')  src/ppo.py:124-126
 *   mgx_reset    <- VecEnv.reset() -> env_i.reset(seed=seed+i)
 *                   -> PlaygroundEnv._gen_grid                            src/custom_env.py:122-267
 *                   -> TokenizeVocabWrapper / Discrete2BoxWrapper         src/environment.py:69-149
 *   mgx_step     <- VecEnv.step(actions): PlaygroundEnv.step              src/custom_env.py:269-330
 *                   + SubprocVecEnv auto-reset, Monitor episode stats,
 *                   terminal_observation, TimeLimit.truncated (SB3, via ppo.py:159)
 *   mgx_gae      <- DictRolloutBuffer.compute_returns_and_advantage (SB3, via ppo.py:159)
 *   mgx_destroy  <- VecEnv.close()                                        src/ppo.py:169
 *
 * Conventions: plain C, no exceptions cross the ABI; every call returns an
 * mgx_status (0 = OK) and mgx_last_error() describes the last failure of the
 * calling thread.  All buffers named *_dev are caller-owned DEVICE pointers
 * (e.g. torch.Tensor.data_ptr()); `stream` is a hipStream_t (NULL = default).
 * mgx_reset / mgx_step / mgx_gae only enqueue work on `stream` (no host sync,
 * no allocation) and are therefore hipGraph-capturable.  A handle is not
 * thread-safe; use one handle per device (per rank).
 */
#ifndef MGX_H_
#define MGX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGX_ABI_VERSION 7

/* Live-lock cap (engine policy; the reference hangs): a
 * reset attempt may consume at most this many MT19937 words; the attempt that
 * would take one more is abandoned and the reset re-runs unseeded with both
 * RNG streams continuing. */
#define MGX_LIVELOCK_WORDS 4096

typedef enum {
    MGX_OK = 0,
    MGX_ERR_INVALID = 1,      /* bad argument / unsupported configuration */
    MGX_ERR_HIP = 2,          /* a HIP runtime call failed */
    MGX_ERR_DEVICE = 3,       /* the device reported an error (see mgx_poll_error) */
    MGX_ERR_OOM = 4
} mgx_status;

/* PlaygroundEnv problems (custom_env.py:134-152) */
typedef enum {
    MGX_PROBLEM_MULTI = 0, MGX_PROBLEM_FULL = 1, MGX_PROBLEM_GTO = 2, MGX_PROBLEM_GTG = 3,
    MGX_PROBLEM_OPN = 4, MGX_PROBLEM_PKP = 5, MGX_PROBLEM_DRP = 6, MGX_PROBLEM_MOV = 7
} mgx_problem;

/* which done envs get a stacked terminal observation written */
typedef enum { MGX_TERMINAL_NONE = 0, MGX_TERMINAL_TRUNCATED = 1, MGX_TERMINAL_ALL = 2 } mgx_terminal_mode;

/* Device error bits reported by mgx_poll_error */
#define MGX_DEVERR_MT_TABLE   1u   /* an env's MT19937 cursor left the window of the stream the device holds
                                      (live cursors spread over more than mt_table_words) */
#define MGX_DEVERR_BAD_ACTION 2u   /* action outside 0..6 (minigrid raises ValueError) */
#define MGX_DEVERR_PCG_LOOP   4u   /* a PCG64 rejection loop exceeded its safety bound */
#define MGX_DEVERR_OBJECTS    8u   /* generator ran out of objects (AssertionError / IndexError in the reference) */
#define MGX_DEVERR_RING_EMPTY 16u  /* an env found its episode ring empty (engine invariant broken) */

typedef struct mgx_config {
    int32_t problem;           /* mgx_problem; `env.problem` */
    int32_t mission;           /* `env.mission` (problem multi): 0 'go to', 1 'toggle', 2 'pick up',
                                  5 'go to goal'; -1 = None */
    int32_t size;              /* `env.size` (5..16); max_steps = size^2 (custom_env.py:114) */
    int32_t num_objects;       /* `env.num_objects` */
    int32_t see_through_walls; /* `env.see_through_walls`; 0 = minigrid Grid.process_vis occlusion */
    int32_t all_doors_open;    /* `env.all_doors_open` */
    int32_t obstacles;         /* `env.obstacles`: floor((size-2)^2 * percent_obstacles) lava (multi) or
                                  lava/wall (single room) cells (custom_env.py:154-172) */
    int32_t n_stack;           /* `algorithm.n_frames_stack` (1..8) */
    int64_t n_envs;            /* envs owned by this handle */
    int64_t base_seed;         /* `seed`; env i: PCG64(SeedSequence(base_seed + env_index_offset + i)), MT19937(base_seed) */
    int64_t env_index_offset;  /* global index of env 0 (rank * n_envs when sharding) */
    int32_t livelock_words;    /* 0 -> MGX_LIVELOCK_WORDS */
    int32_t terminal_mode;     /* mgx_terminal_mode */
    int32_t mission_int64;     /* 1: mission tokens int64 (TokenizeVocabWrapper dtype), 0: uint8 */
    int32_t refill_cap;        /* > 0 (0 -> max(2, round(0.19 * refill_every))): a refill epoch's production
                                  per env follows the consumption of its 64-env wave since the previous
                                  refill (the mean, rounded up), beyond what keeps the ring from running
                                  dry; < 0 -> fill the ring every epoch.  mgx_reset fills every ring */
    int64_t mt_table_words;    /* 0 -> default (2^26): MT19937 output words the device keeps (rounded up to a
                                  power of two of 10-word groups, >= 5,120).  The stream is extended on the
                                  device as cursors advance -- no lifetime limit; only the spread between
                                  the oldest live cursor and the newest must stay below it */
    int32_t ring_depth;        /* pre-generated episodes per env (0 -> 512 since ABI 7, 256 before; rounded up to a power of two
                                  <= 4096, ring positions are mod 2^16; -1 = no ring: every auto-reset
                                  generated inline) */
    int32_t refill_every;      /* steps per refill epoch K (0 -> min(ring_depth/4, 64); clamped to <= ring_depth/2:
                                  each epoch keeps >= K queued, and a step pops <= 1 episode) */
    double percent_obstacles;  /* `env.percent_obstacles` (single.yaml:28: 0.05); used when obstacles */
    int32_t manual;            /* PlaygroundEnv(manual=True) (make_env(manual=True), environment.py:10-20):
                                  a 'done' before the mission is complete is a no-op -- no termination,
                                  no reset (custom_env.py:319-328 `elif not self.manual`) */
    int32_t reserved0;         /* 0 */
} mgx_config;

/* Stacked observation in the layout SB3's VecFrameStack(VecTransposeImage(.))
 * hands the policy: image u8 [N][3*n_stack][7][7] ([c][vx][vy] per frame,
 * newest frame last), direction u8 [N][4*n_stack] (one-hot per frame),
 * mission [N][32*n_stack] (int64 or uint8 tokens per frame). */
typedef struct mgx_obs {
    void *image_dev;
    void *direction_dev;
    void *mission_dev;
} mgx_obs;

typedef struct mgx_step_out {
    mgx_obs obs;               /* updated in place (the stacks roll) */
    mgx_obs terminal;          /* stacked terminal obs, valid where written (terminal_mode) */
    float *reward_dev;         /* f32 [N] */
    double *reward64_dev;      /* f64 [N] (optional): the env's Python-float reward */
    uint8_t *terminated_dev;   /* u8 [N] */
    uint8_t *truncated_dev;    /* u8 [N] (gymnasium truncated; TimeLimit.truncated = trunc & !term) */
    uint8_t *done_dev;         /* u8 [N] = term | trunc (SB3 `dones`) */
    float *ep_return_dev;      /* f32 [N] Monitor 'r', valid where done (optional) */
    int32_t *ep_len_dev;       /* i32 [N] Monitor 'l', valid where done (optional) */
    int32_t *livelock_dev;     /* i32 [N] abandoned reset attempts where done (optional) */
} mgx_step_out;

typedef struct mgx_handle mgx_handle;

const char *mgx_last_error(void);
int mgx_abi_version(void);

mgx_status mgx_create(const mgx_config *cfg, int device, mgx_handle **out);
mgx_status mgx_destroy(mgx_handle *h);

/* VecEnv.reset() of every env; writes the stacked first observation (zeros +
 * newest frame).  The first call after mgx_create is the seeded reset of
 * make_vec_env (PCG64 <- base_seed + env_index_offset + i, MT cursor 0).  Later
 * calls follow SB3: seeded (PCG64 only) if mgx_set_seed was called since the
 * last reset, else unseeded; both streams continue from each env's current
 * episode, and mission_done / the stored reward persist.
 * It also pre-generates ring_depth episodes per env (on `stream`; ~26 ms at
 * 65,536 envs, S = 8, D = 512).  `livelock_dev` (optional i32 [N]). */
mgx_status mgx_reset(mgx_handle *h, const mgx_obs *obs, int32_t *livelock_dev, void *stream);

/* VecEnv.seed(seed) (SB3): the NEXT mgx_reset seeds env i's PCG64 with
 * seed + env_index_offset + i.  The MT19937 stream keeps cfg.base_seed: the
 * reference seeds CPython `random` once, in PlaygroundEnv.__init__
 * (custom_env.py:82), from the config, not from reset(seed). */
mgx_status mgx_set_seed(mgx_handle *h, int64_t seed);

/* One vectorised step.  actions_dev: [N] int32 (action_bytes = 4) or int64 (8).
 * Episode pre-generation runs CONCURRENTLY with the steps on a handle-owned
 * side stream, in epochs of K = refill_every calls: the first call of an epoch
 * joins the previous epoch's refill (and the slide that publishes its episodes) and
 * forks the next refill off `stream`.  Whatever the caller enqueues between two
 * epochs (GAE, the policy) overlaps the refill's tail.  The launch sequence
 * depends only on the call count; end a stream capture (hipGraph) with mgx_join
 * to make it self-contained. */
mgx_status mgx_step(mgx_handle *h, const void *actions_dev, int action_bytes,
                    const mgx_step_out *out, void *stream);

/* ---- Compact rollout layout ------------------------------
 * One observation = one 148-B ROW (byte 0: agent direction 0..3; bytes 1..147: the
 * [c][vx][vy] frame, VecTransposeImage order) + one mission-id byte (mgx_mission_text;
 * tokens = TokenizeVocabWrapper of that text).  A rollout buffer is [T][N] rows; the
 * SB3 stacked observation of any (t, env) is rebuilt by mgx_gather from rows t-n_stack+1..t
 * and the episode-start flags (VecFrameStack zero-fills before an episode's first obs).
 * 150 B per env-step instead of 588 + 16 + 32*n_stack*(1|8) B; no stack roll per step. */
typedef struct mgx_compact_out {
    uint8_t *row_dev;             /* u8 [N][148]: the observation after this step (the new
                                     episode's first one where done) */
    uint8_t *mission_id_dev;      /* u8 [N]: its mission id */
    uint8_t *terminal_row_dev;    /* u8 [N][148]: the final observation of each episode that ended
                                     (written where terminal_mode selects; its mission id is the
                                     previous row's) */
    float *reward_dev;            /* as mgx_step_out */
    double *reward64_dev;
    uint8_t *terminated_dev;
    uint8_t *truncated_dev;
    uint8_t *done_dev;            /* u8 [N]: done of this step = start flag of the row written */
    float *ep_return_dev;
    int32_t *ep_len_dev;
    int32_t *livelock_dev;
} mgx_compact_out;

/* mgx_step with compact outputs (same transition, RNG, auto-reset and refill epochs as
 * mgx_step; the two may not be mixed on one handle between resets).  Needs the ring. */
mgx_status mgx_step_compact(mgx_handle *h, const void *actions_dev, int action_bytes, const mgx_compact_out *out,
                            void *stream);

/* K consecutive mgx_step_compact calls fused into ONE launch, for a rollout whose actions are
 * known up front (random-action or scripted rollouts: BASELINE config 2's workload; a policy in the
 * loop needs mgx_step_compact per step).  actions_dev: int32 [K][N].  The outputs of step t go to
 * row t of the [K][N] arrays below; terminal rows, ep_return, ep_len and livelock are left as
 * after the last step.  Transitions, RNG streams, auto-resets, refill epochs and counters are
 * those of the K calls, bit for bit.  The K steps must lie within one refill epoch:
 * (mgx_step calls so far % refill_every) + K <= refill_every.  Needs the ring. */
typedef struct mgx_rollout_out {
    uint8_t *rows_dev;            /* u8 [K][N][148]: the observation after step t at row t */
    uint8_t *mission_ids_dev;     /* u8 [K][N] */
    uint8_t *terminal_row_dev;    /* u8 [N][148] (as mgx_compact_out) */
    float *rewards_dev;           /* f32 [K][N] */
    double *rewards64_dev;        /* f64 [K][N] (optional) */
    uint8_t *terminated_dev;      /* u8 [K][N] */
    uint8_t *truncated_dev;       /* u8 [K][N] */
    uint8_t *dones_dev;           /* u8 [K][N] */
    float *ep_return_dev;         /* f32 [N] (optional) */
    int32_t *ep_len_dev;          /* i32 [N] (optional) */
    int32_t *livelock_dev;        /* i32 [N] (optional) */
} mgx_rollout_out;
mgx_status mgx_rollout_compact(mgx_handle *h, const int32_t *actions_dev, int K, const mgx_rollout_out *out,
                               void *stream);

/* The current observation of every env as compact rows (e.g. row 0 after mgx_reset). */
mgx_status mgx_observe_compact(mgx_handle *h, uint8_t *row_dev, uint8_t *mission_id_dev, void *stream);

/* Stacked observations (VecFrameStack(n_stack) of the handle) of n_samples (t, env) pairs from
 * a compact buffer: rows_dev u8 [R][n_envs][148], mission_ids_dev / starts_dev u8 [R][n_envs]
 * (start = the row is an episode's first observation); index_dev i64 [n_samples] = t*n_envs +
 * env of the newest row, which must have n_stack-1 rows before it.  terminal_rows_dev (u8
 * [n_envs][148], optional): the newest frame is env's terminal row and the older ones start at
 * row index (SB3's stacked terminal_observation).  Outputs (device): image [n][3*n_stack][7][7]
 * u8 or f32 (= u8 / 255, SB3 preprocess_obs), direction [n][4*n_stack] u8 or f32 one-hot,
 * mission [n][32*n_stack] u8 tokens. */
mgx_status mgx_gather(const mgx_handle *h, const uint8_t *rows_dev, const uint8_t *mission_ids_dev,
                      const uint8_t *starts_dev, int64_t n_envs, const int64_t *index_dev, int64_t n_samples,
                      const uint8_t *terminal_rows_dev, void *image_dev, int image_f32, void *direction_dev,
                      int direction_f32, uint8_t *mission_dev, void *stream);

/* mgx_gather over a RING of ring_rows rows (ABI 6): walking back from a sample's newest row wraps
 * from row 0 to row ring_rows - 1, so a rollout that starts where the previous one ended reads its
 * n_stack - 1 history rows in place -- no per-rollout copy of them (mgx/compact.py ring mode).
 * ring_rows = 0 is mgx_gather; else ring_rows >= n_stack. */
mgx_status mgx_gather_ring(const mgx_handle *h, const uint8_t *rows_dev, const uint8_t *mission_ids_dev,
                           const uint8_t *starts_dev, int64_t n_envs, int64_t ring_rows, const int64_t *index_dev,
                           int64_t n_samples, const uint8_t *terminal_rows_dev, void *image_dev, int image_f32,
                           void *direction_dev, int direction_f32, uint8_t *mission_dev, void *stream);

/* Makes `stream` wait for the in-flight refill, if any (no host sync). */
mgx_status mgx_join(mgx_handle *h, void *stream);

/* The effective configuration (defaults resolved: ring_depth, refill_every, ...). */
mgx_status mgx_get_config(const mgx_handle *h, mgx_config *out);

/* GAE over a [T][N] f32 rollout (DictRolloutBuffer.compute_returns_and_advantage):
 * episode_starts_dev f32 [T][N], last_values f32 [N], last_dones u8 [N];
 * writes advantages/returns f32 [T][N].  adv_stats_dev (optional, f64 [3]):
 * accumulates (sum A, sum A^2, count) for RCCL advantage-stat reduction, through per-workgroup
 * partials in stats_scratch_dev (f64 [MGX_GAE_SCRATCH_WORDS], caller-owned, zeroed before its first
 * use; every call leaves it zeroed).  Calls that may overlap (two collectors on two streams) pass
 * scratches of their own; NULL = one device-global scratch (such calls must then not overlap). */
#define MGX_GAE_SCRATCH_WORDS 512
mgx_status mgx_gae(const float *rewards_dev, const float *values_dev, const float *episode_starts_dev,
                   const float *last_values_dev, const uint8_t *last_dones_dev, int64_t T, int64_t N,
                   float gamma, float gamma_lambda, float *advantages_dev, float *returns_dev,
                   double *adv_stats_dev, double *stats_scratch_dev, void *stream);

/* GAE over the compact rollout layout: dones_dev u8 [T][N] is the `done` output of
 * step t (what mgx_step writes to done_dev), so next_non_terminal(t) = 1 - dones[t]
 * -- SB3's episode_starts[t+1] for t < T-1 and its last_dones at T-1.  Same fp32
 * op order, outputs and adv_stats_dev as mgx_gae; 17 B of traffic per element. */
mgx_status mgx_gae_dones(const float *rewards_dev, const float *values_dev, const uint8_t *dones_dev,
                         const float *last_values_dev, int64_t T, int64_t N, float gamma, float gamma_lambda,
                         float *advantages_dev, float *returns_dev, double *adv_stats_dev,
                         double *stats_scratch_dev, void *stream);

/* mgx_rollout_compact followed by mgx_gae_dones over the K steps it runs (its rewards_dev and dones_dev,
 * T = K), the GAE fused into the launch: each workgroup runs the recurrence of its 64 envs as soon as its
 * own K steps are done, reading back the rewards and dones it wrote (no second kernel over the rollout).
 * Same fp32 op order and outputs as mgx_gae_dones (bit for bit); adv_stats_dev / stats_scratch_dev as
 * there (the fold of the per-workgroup partials is a second, one-workgroup launch).  Replaces the
 * reference's collect_rollouts + compute_returns_and_advantage pair for a rollout whose actions are
 * known up front and whose horizon is this launch (ppo.py:159; SB3 OnPolicyAlgorithm.collect_rollouts). */
typedef struct mgx_gae_args {
    const float *values_dev;       /* f32 [K][N] */
    const float *last_values_dev;  /* f32 [N]: V(observation after step K-1) */
    float gamma, gamma_lambda;     /* gamma_lambda = float(gamma * gae_lambda), as mgx_gae_dones */
    float *advantages_dev;         /* f32 [K][N] */
    float *returns_dev;            /* f32 [K][N] */
    double *adv_stats_dev;         /* f64 [3] (optional) */
    double *stats_scratch_dev;     /* f64 [MGX_GAE_SCRATCH_WORDS] (optional) */
} mgx_gae_args;
mgx_status mgx_rollout_compact_gae(mgx_handle *h, const int32_t *actions_dev, int K, const mgx_rollout_out *out,
                                   const mgx_gae_args *gae, void *stream);

/* Scene record of env `env`'s current episode, for PlaygroundEnv.llm_description /
 * LLMDescriptionWrapper (environment.py:152-195; manual mode, one env): the episode is
 * regenerated on the device from the RNG state its generation started from, which only the
 * inline reset mode keeps (ring_depth = -1).  record (HOST, MGX_SCENE_WORDS u32):
 *   [0] number of objs entries, [1] agent x | y<<8 | dir<<16, [2] mission id | tx<<8 | ty<<16 |
 *   target action<<24, [3] abandoned attempts, [4] error bits, [8 .. 8+32) objs entries in
 *   placement order (type | COLOR_NAMES index<<4 | x<<8 | y<<16 | 1<<24 for a door's key or key
 *   box), [40 ..) the generated grid, one cell code byte per cell (y*S + x; S <= 16).
 * Synchronises `stream`. */
#define MGX_SCENE_WORDS 104
mgx_status mgx_scene(mgx_handle *h, int64_t env, uint32_t *record, void *stream);

/* Kernel clocks (measurement; ABI 6).  With clock_dev set, every workgroup of every launch of the step
 * kernels (mgx_step, mgx_step_compact, mgx_rollout_compact[_gae]: class 0) and of the refill kernel
 * (class 1) and the MT slide after it (class 2) records its start and end on the device (wall-clock ticks; *tick_khz, optional, receives
 * their rate), so that a caller can time the kernels INSIDE a replayed hipGraph, beside whatever runs
 * concurrently (bench.py: the timed region's own launches); a launch's span is the min start to the
 * max end over its workgroups.  clock_dev: u64 [mgx_clock_words(h, slots)], caller-owned, zeroed;
 * per class c (G = mgx_clock_groups(h, c) workgroups per launch), in order: cnt u64 [G] (launches so
 * far, per workgroup), then rec u64 [slots][G][2] {start, end} of launches 0 .. slots-1 (later
 * launches are counted, not recorded).  Kernel parameters are captured at launch: set the clock
 * before capturing a graph.  NULL clock_dev: off (the default). */
#define MGX_CLOCK_CLASSES 4   /* 0 step kernels (64-env blocks), 1 refill, 2 MT slide (the kernel that follows each
                                 refill), 3 (ABI 7) the fused rollout's 32-env blocks at S = 16 (0 groups otherwise):
                                 every launch of a class has its class's grid */
int64_t mgx_clock_words(const mgx_handle *h, int slots);
int mgx_clock_groups(const mgx_handle *h, int cls);
mgx_status mgx_set_clock(mgx_handle *h, uint64_t *clock_dev, int slots, int *tick_khz);

/* Synchronises `stream`, returns the device error bits (MGX_DEVERR_*) and clears them. */
mgx_status mgx_poll_error(mgx_handle *h, void *stream, uint32_t *bits);

/* Counters since create: [0] env-steps, [1] resets (incl. first), [2] abandoned
 * (live-locked) reset attempts, [3] max MT cursor, [4] pre-generated episodes
 * queued in the rings now (between two mgx_reset calls, episodes produced by
 * the refill = resets consumed + change of [4]), [5] refill launches enqueued (incl. the
 * synchronous fills of mgx_reset), [6] mgx_step calls since the last mgx_reset,
 * [7] MT19937 words generated so far (the device ring holds the last mt_table_words of them).
 * Synchronises `stream` and the refill stream. */
mgx_status mgx_stats(mgx_handle *h, void *stream, uint64_t out[8]);

/* The fused rollout's own random policy (ABI 7): once set, mgx_rollout_compact[_gae] may be called with
 * actions_dev = NULL, and each launch then draws its K x N actions on the device, in the DMA wave that would have
 * loaded them -- exactly mgx_random_actions' draws (n_actions 7) over a [K][N] buffer at counter c = the number of
 * such launches since this call (no actions buffer, nothing read).  enable = 0 turns it off.  Synchronises. */
mgx_status mgx_set_random_policy(mgx_handle *h, int enable, uint64_t seed);

/* Synthetic random policy (ABI 7; env.action_space.sample() for a whole batch -- the benchmark's random-action
 * rollouts, a random agent's evaluation): out_dev i32 [count] = uniform draws on {0 .. n_actions-1}
 * (1 <= n_actions <= 65536) from a counter-based hash of (seed, counter, i): key = splitmix64(seed + c *
 * 0x9E3779B97F4A7C15), h = splitmix64(key ^ (i * 0xD1B54A32D192ED03)), out = ((h >> 32) * n_actions) >> 32
 * (mod 2^64; c = counter_dev[0]).  The launch then advances counter_dev[0] by one on the device, so the same launch
 * captured in a hipGraph draws fresh actions at every replay.  counter_dev: u64 [2], caller-owned, zeroed before
 * the first use (word 1 is the launch's own workgroup tally; launches sharing a counter must not overlap). */
mgx_status mgx_random_actions(int32_t *out_dev, int64_t count, int n_actions, uint64_t seed, uint64_t *counter_dev,
                              void *stream);

/* Diagnostics (ABI 7): the episodes queued in each env's ring now, (tail - head) mod 2^16, into a HOST
 * array levels[N] (what mgx_stats [4] sums).  Synchronises `stream` and the refill stream.  Measurement
 * only, no reference counterpart (tools/diag_ring_levels.py: the ring-level distribution over long runs). */
mgx_status mgx_ring_levels(mgx_handle *h, void *stream, uint16_t *levels);

/* Diagnostics: the first n (<= 32) raw device counters (phase / section clocks of
 * -DMGX_STAMPS / -DMGX_GEN_STAMPS builds; zero otherwise).  Synchronises. */
mgx_status mgx_debug_counters(mgx_handle *h, void *stream, uint64_t *out, int n);

/* Test/debug: copy env state to HOST buffers (any may be NULL); synchronises.
 * grid u8 [N][S][S][4] (x-major (type,colour,state,box-holds-key)), agent u8 [N][3],
 * carrying u8 [N][4], step_count i32 [N], mission_done u8 [N], stored_reward f64 [N]
 * (NaN = None), mt_words i64 [N], pcg u64 [N][6] (state hi/lo, inc hi/lo,
 * has_uint32, uinteger), target u8 [N][3], mission_id u8 [N]. */
mgx_status mgx_dump_state(mgx_handle *h, void *stream, uint8_t *grid, uint8_t *agent, uint8_t *carrying,
                          int32_t *step_count, uint8_t *mission_done, double *stored_reward,
                          int64_t *mt_words, uint64_t *pcg, uint8_t *target, uint8_t *mission_id);

/* Mission text / tokens for a mission_id (host side, no device access). */
mgx_status mgx_mission_text(int mission_id, char *buf, size_t buflen);

#ifdef __cplusplus
}
#endif
#endif /* MGX_H_ */
