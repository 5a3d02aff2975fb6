/*
 * lsm_rollout.h -- C ABI of the MI355X-native navigation_graph_safe rollout.
 *
 * One handle = one device-resident batch of `num_envs` environments (one GPU
 * process owns one handle; envs shard across GPUs by `env_offset`).  Every
 * entry point replaces one piece of the reference's vec-env surface:
 *
 *   lsm_create/destroy   GraphSubprocVecEnv.__init__/close
 *                        (onpolicy/envs/env_wrappers.py:951-969, 1014-1024) and the
 *                        per-env GraphMPEEnv(args) + env.seed(seed + 1000*rank)
 *                        (multiagent/MPE_env.py:56-84, scripts/train_mpe.py:23-45)
 *   lsm_set_value_table  HjDataHandle.__init__ (multiagent/safety_filter.py:154-168)
 *   lsm_set_ttr_table    SafeAamScenario.make_world TTR load (navigation_graph_safe.py:128-138)
 *   lsm_bind_output      the arrays returned by step/reset (env_wrappers.py:988-1005);
 *                        caller-owned device buffers (e.g. torch tensors)
 *   lsm_reset            GraphSubprocVecEnv.reset(num_current_episode) -> env.reset()
 *                        (env_wrappers.py:998-1005, multiagent/environment.py:1046-1074)
 *   lsm_step             GraphSubprocVecEnv.step(actions, num_current_episode)
 *                        (env_wrappers.py:103-110, 851-874, 983-996) ->
 *                        MultiAgentGraphEnv.step (environment.py:963-1042) incl. the
 *                        worker's auto-reset on np.all(done) (env_wrappers.py:866-871)
 *   lsm_last_error       exception text (Python wrapper raises RuntimeError)
 *   lsm_bind_output_ring / lsm_select_ring
 *                        outputs written in place into GraphReplayBuffer rows
 *                        (graph_mpe_runner.py:444-487, graph_buffer.py:223-249)
 *   lsm_edges_*          GNNBase.process_adj (onpolicy/algorithms/utils/gnn.py:376-407)
 *   lsm_buffer_insert    GMPERunner.insert's derived rows (graph_mpe_runner.py:449-484)
 *
 * Kernels: N <= 32 and N * (1 + L) <= 64 run one 64-lane wavefront per env; larger envs
 * (up to N = 64, E = 256: BASELINE config 5) one 256-thread workgroup per env.
 *
 * All pointers passed to lsm_step / lsm_bind_output are DEVICE pointers.
 * Calls are stream-ordered and asynchronous; a handle is not thread-safe.
 * Return value: 0 on success, nonzero error code (see lsm_last_error).
 */
#ifndef LSM_ROLLOUT_H
#define LSM_ROLLOUT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lsm_env lsm_env;

enum { LSM_DOUBLE_INTEGRATOR = 0, LSM_AIRTAXI = 1 };
enum { LSM_ACTIONS_INDEX_I32 = 0, LSM_ACTIONS_ONEHOT_F32 = 1, LSM_ACTIONS_ONEHOT_F64 = 2 };

/* Output slots (caller-owned device buffers; shapes in elements). */
enum {
  LSM_OUT_OBS = 0,        /* float32 [n][N][OBS]   OBS = 7 (DI) / 6 (airtaxi)       */
  LSM_OUT_NODE_OBS = 1,   /* float32 [n][N][E][F]  F = 10 (DI) / 11 (airtaxi)       */
  LSM_OUT_ADJ = 2,        /* float32 [n][N][E][E] (adj_layout 0) or [n][E][E] (1)    */
  LSM_OUT_REWARD = 3,     /* float32 [n][N]                                         */
  LSM_OUT_DONE = 4,       /* uint8   [n][N]                                         */
  LSM_OUT_RESET_FLAG = 5, /* uint8   [n]      env auto-reset during the last step   */
  LSM_OUT_EP_INFO = 6,    /* float64 [n][8]   episode summary returned by last reset */
  LSM_OUT_INFO = 7,       /* float64 [n][N][LSM_INFO_FIELDS] info_callback numbers   */
  LSM_OUT_EDGES = 8,      /* uint8   [n][E][E] update_graph() connectivity (optional)*/
  LSM_OUT_STATE = 9,      /* float64 [n][N][4] agent state after the last call      */
  LSM_OUT_DEBUG_STAMPS = 10, /* uint64 [n][16] per-phase clock stamps (diagnostic build only) */
  LSM_OUT_ADJ_MASK = 11,  /* uint64  [n][N][W] per-ego disconnect bits, W = ceil(E/64)
                             (adj_layout 1 only): bit r of ego e = entity r masked      */
  /* optional replay-buffer rows (GMPERunner.insert, graph_mpe_runner.py:457-481), written only
     when bound: */
  LSM_OUT_SHARE_OBS = 12, /* float32 [n][N][N*OBS] centralized share_obs (obs row per agent) */
  LSM_OUT_MASKS = 13,     /* float32 [n][N]   1 - done                                   */
  LSM_OUT_ACTIVE_MASKS = 14, /* float32 [n][N] done ? all(env dones) : 1                 */
  LSM_OUT_COLLISION_FORCE = 15, /* float64 [n][N][2] contact force per agent, written only with
                                   lsm_config.collision_forces (core.py:741-774; never applied) */
  LSM_OUT_DEPARTED = 16,  /* uint8   [n][N]   agent.departed after the call (info 'Departed',
                             navigation_graph_safe.py:446); written when bound                 */
  LSM_OUT_ADJ_NNZ = 17,   /* int64  [n][N]    nonzeros of each ego's adjacency as stored (either layout:
                             the per-graph count of GNNBase.process_adj's adj.nonzero(), gnn.py:376-407),
                             written when bound; lsm_edges_scan_emit takes it so the edge list needs
                             one adjacency pass. One-wave and team kernels (E <= 64) only */
  LSM_NUM_OUT = 18
};

/* Scenario sources (lsm_config.scenario).
 *  LSM_SCENARIO_TRAIN       the training Scenario.random_scenario drawn on the device at every
 *                           reset (navigation_graph_safe.py:1199-1367), auto-reset allowed.
 *  LSM_SCENARIO_LAYOUT      evaluation layouts (navigation_graph_safe_eval.py Scenario): the host
 *                           computes each reset's agent states / landmarks and passes them to
 *                           lsm_reset_layout; SafeAamScenario step semantics (departed = True).
 *  LSM_SCENARIO_DEPARTURES  RealisticScenario layouts (navigation_graph_safe_bayarea_*.py): as
 *                           LAYOUT plus per-agent departure timers and the RealisticScenario goal /
 *                           departure update (navigation_graph_safe.py:1153-1186); airtaxi only
 *                           (its reset_velocity(theta, speed) exists only for KinematicVehicleXY).
 * Layout scenarios are evaluation paths (scripts/eval_mpe.py forces n_rollout_threads = 1,
 * GraphDummyVecEnv): they need auto_reset = 0, N <= 32 and N * (1 + L) <= 64, and run the
 * generic one-wave kernel. */
enum { LSM_SCENARIO_TRAIN = 0, LSM_SCENARIO_LAYOUT = 1, LSM_SCENARIO_DEPARTURES = 2 };

/* Random streams of the device reset (lsm_config.rng, training scenario).
 *  LSM_RNG_MT19937  draw-exact replay of numpy's legacy MT19937 stream of env k
 *                   (np.random.seed(seed + 1000 k)): resets identical to the reference's.
 *  LSM_RNG_PHILOX   fast mode: Philox4x32-10 keyed by (seed + 1000 k), counter = (reset index,
 *                   draw index); the same scenario distribution, not the reference's draws. No
 *                   624-word state is read, twisted or written back at a reset. */
enum { LSM_RNG_MT19937 = 0, LSM_RNG_PHILOX = 1 };

/* Adjacency output layouts (lsm_config.adj_layout).
 *  0  reference: adj[e][r][c] per ego, what graph_observation returns
 *     (navigation_graph_safe.py:932-994) and the runner's buffer stores (graph_buffer.py:95-104).
 *  1  compact: the unmasked thresholded distance table A[r][c] (d if 0 < d < range, else 0)
 *     once per env plus per-ego disconnect masks M[e]; the reference array is
 *     adj[e][r][c] = (M[e] bit r | M[e] bit c) ? 0 : A[r][c]  (lossless; N x fewer bytes). */
enum { LSM_ADJ_REFERENCE = 0, LSM_ADJ_COMPACT = 1 };

/* Per-agent info fields (navigation_graph_safe.py:386-450 + environment.py:1025). */
enum {
  LSM_INFO_INDIVIDUAL_REWARD = 0, LSM_INFO_MIN_RELATIVE_DISTANCE, LSM_INFO_DIST_TO_GOAL,
  LSM_INFO_TIME_REQ_TO_GOAL, LSM_INFO_NUM_AGENT_COLLISIONS, LSM_INFO_DISTANCE_MEAN,
  LSM_INFO_DISTANCE_VARIANCE, LSM_INFO_DISTS_TRAVELED, LSM_INFO_TIME_MEAN, LSM_INFO_TIME_STDDEV,
  LSM_INFO_MIN_TIME_TO_GOAL, LSM_INFO_SAFETY_FILTERED, LSM_INFO_SAFETY_VIOLATED,
  LSM_INFO_DECONFLICTING_INDEX, LSM_INFO_ACTION_DIFF, LSM_INFO_REACHED_GOAL,
  LSM_INFO_POSITION_X, LSM_INFO_POSITION_Y, /* 'position' = agent.state.p_pos at info time */
  LSM_INFO_FIELDS
};

typedef struct lsm_config {
  int32_t dynamics;          /* LSM_DOUBLE_INTEGRATOR / LSM_AIRTAXI                    */
  int32_t num_envs;          /* envs in this handle (this GPU's shard)                */
  int32_t num_agents;        /* N                                                      */
  int32_t num_landmarks;     /* L (per agent)                                          */
  int32_t episode_length;    /* world_length                                           */
  int32_t use_safety_filter; /* args.use_safety_filter                                 */
  int32_t use_masking;       /* args.use_masking                                       */
  int32_t auto_reset;        /* 1: GraphSubprocVecEnv worker semantics, 0: Dummy       */
  int32_t emit_edges;        /* 1: fill LSM_OUT_EDGES at the start of each step        */
  int32_t adj_layout;        /* LSM_ADJ_REFERENCE / LSM_ADJ_COMPACT                    */
  double world_size;         /* args.world_size                                        */
  int64_t seed;              /* env k (global index env_offset + k) seeded seed+1000*k */
  int64_t env_offset;
  int32_t collision_forces;  /* 1: report World.get_entity_collision_force per agent each step
                                (LSM_OUT_COLLISION_FORCE). The reference has no caller for it
                                (core.py:741-836), so it never changes the dynamics. Default 0. */
  int32_t scenario;          /* LSM_SCENARIO_TRAIN (default) / _LAYOUT / _DEPARTURES            */
  int32_t rng;               /* LSM_RNG_MT19937 (default) / LSM_RNG_PHILOX                      */
  int32_t num_internal_step; /* args.num_internal_step (0 or 1 = one): World.step repeats filter ->
                                action_diff -> integrate this many times per env step, then the
                                distances and minimum relative distance (core.py:607-631)         */
  int32_t reward_terms;      /* LSM_REWARD_* bits: RewardBinaryConfig's optional reward terms
                                (multiagent/config.py:78-83, all off by default), added in
                                SafeAamScenario.reward (navigation_graph_safe.py:843-850). HJ_VALUE
                                needs the value table (lsm_set_value_table) even with the filter off:
                                the reference builds the HJ handle then (:195) and shifts it at every
                                reset like the filter's (core.py:483-486). Unknown bits are refused. */
  int32_t collaborative;     /* args.collaborative: MultiAgentGraphEnv.shared_reward
                                (environment.py:79-80) -- every agent's LSM_OUT_REWARD entry is the
                                numpy sum of the env's individual rewards (:1031-1037); info
                                'individual_reward' keeps each agent's own                        */
} lsm_config;

/* lsm_config.reward_terms bits (RewardBinaryConfig, multiagent/config.py:78-83) */
enum {
  LSM_REWARD_SAFETY_VIOLATION = 1,            /* reward_safety_violation, navigation_graph_safe.py:793-798 */
  LSM_REWARD_POTENTIAL_CONFLICT = 2,          /* reward_multiple_engagement, :800-823                    */
  LSM_REWARD_DIFF_FROM_FILTERED_ACTION = 4,   /* reward_diff_from_filtered_action, :825-828 (filter on)  */
  LSM_REWARD_HJ_VALUE = 8,                    /* reward_hj_value, :830-837 (World.get_hj_value..., core.py:459) */
  LSM_REWARD_ALL = 15
};

/* Curriculum block for one reset call (navigation_graph_safe.py:324-366), computed by the
 * host with the reference's own float64 expressions. */
typedef struct lsm_curriculum {
  double curriculum_ratio;   /* clip(ep / num_total_episode, 0, 1)                     */
  double sloped;             /* get_effective_curriculum_ratio_sloped()                */
  double stair;              /* get_effective_curriculum_ratio_stair()                 */
  double ratio_airtaxi;      /* sloped(0.25, 0.75), or 1 when use_safety_filter        */
  double ratio_scenario;     /* 1 when use_safety_filter else sloped (random_scenario) */
  double goal_heading_error_thresh;
  double goal_speed_error_thresh;
  double min_dist_thresh;
  double separation_distance;
  double engagement_distance;
  double world_use_safety_filter; /* 0/1 */
  double stair_is_int;       /* 1 when get_effective_curriculum_ratio_stair() returned the Python int
                                0 or 1 (ratio outside [start, end], :1115-1118), else 0: the scaled
                                reward weights (:340-345) are then Python ints, and an int times a
                                float32 HJ value stays float32 (reward_hj_value's sums)           */
} lsm_curriculum;

int lsm_create(const lsm_config* cfg, lsm_env** out);
void lsm_destroy(lsm_env* env);

/* Kernel selection for parity tests and A/B runs (no reference counterpart: the reference has one
 * Python implementation). lsm_create picks the kernel from the configuration alone; the library
 * reads no environment variables. Fields at their "default" value keep lsm_create's choice.
 *   workgroup_per_env  1: rollout_block_kernel even where a one-wave kernel fits (default 0)
 *   lanes_per_env      one-wave kernels: 64 (one env per wave, default; 0 = 64), 32 or 16 (2 / 4
 *                      envs per wave, needs num_agents <= lanes_per_env)
 *   team               -1 default (4 envs per workgroup for DI N = 8 and airtaxi N = 16), 0 the
 *                      plain one-wave kernel, 2 / 4 / 8 (team * num_agents <= 64)
 *   generic            1: never the compile-time-N instantiations (default 0)
 *   lean               -1 default (airtaxi team kernel: lean LDS layout), 0: the full table
 *   filter_search      -1 default (1: bound-pruned exact argmin in the workgroup kernel), 0: full search
 *   bounds_shift       0 default (2): log2 of the cells per dimension of a value-bounds block (1..4) */
typedef struct lsm_kernel_select {
  int32_t workgroup_per_env;
  int32_t lanes_per_env;
  int32_t team;
  int32_t generic;
  int32_t lean;
  int32_t filter_search;
  int32_t bounds_shift;
} lsm_kernel_select;
/* lsm_create with an explicit kernel selection (sel == NULL: lsm_create's defaults). */
int lsm_create_select(const lsm_config* cfg, const lsm_kernel_select* sel, lsm_env** out);
const char* lsm_last_error(const lsm_env* env);

/* values: float32 [prod(shape)] (values_hj, already negated/shifted); grads: float32
 * [prod(shape)][gwidth] with gwidth = 4 (ndim <= 4) or 8 (ndim == 5); periodic: 0/1 per dim.
 * separation_distance: the separation values_hj is calibrated for (HjDataHandle's
 * target_separation_distance, safety_filter.py:155-168). Each env then keeps its own table
 * history: every reset whose curriculum separation differs from the env's current one applies
 * `values_hj -= shift` (float32 <- float64, HjDataHandle.update_separation_distance,
 * safety_filter.py:170-174) to that env only, every shift rounded to float32 in turn as numpy does.
 * The chain has no length bound: its first 8 shifts live in the env's record, later ones in a
 * per-env HBM array that a call which can reset (lsm_reset, lsm_reset_layout, lsm_step with
 * auto_reset) grows before its launch when the number of separation changes since the upload needs
 * it (one stream synchronisation then). Needed with the filter on, or with LSM_REWARD_HJ_VALUE. */
int lsm_set_value_table(lsm_env* env, int32_t ndim, const double* lo, const double* hi,
                        const int32_t* shape, const int32_t* periodic,
                        const float* values_host, const float* grads_host, double separation_distance);
int lsm_set_ttr_table(lsm_env* env, int32_t ndim, const double* lo, const double* hi,
                      const int32_t* shape, const int32_t* periodic,
                      const float* values_host, double ttr_max);

int lsm_bind_output(lsm_env* env, int32_t slot, void* device_ptr, size_t bytes);
size_t lsm_output_bytes(const lsm_env* env, int32_t slot);

int lsm_reset(lsm_env* env, const lsm_curriculum* cur, void* hip_stream);
int lsm_step(lsm_env* env, const void* actions_device, int32_t action_kind,
             const lsm_curriculum* cur_for_auto_reset, void* hip_stream);

/* Reset of a layout scenario (LSM_SCENARIO_LAYOUT / _DEPARTURES): MultiAgentGraphEnv.reset
 * (environment.py:1046-1074) with random_scenario replaced by the host-computed layout of each
 * env -- an evaluation Scenario's random_scenario (navigation_graph_safe_eval.py:32-50,
 * navigation_graph_safe_bayarea_merge.py:63-69, navigation_graph_safe_bayarea_cross.py:59-65),
 * which draws from the env's numpy stream on the host. `layout` is a DEVICE pointer to float64
 * [n][lsm_layout_doubles(env)]: agent state [N][4] (x, y, v_x|theta, v_y|speed), landmarks
 * [N*L][4] (x, y, heading, speed; landmark k = order * N + agent), and with
 * LSM_SCENARIO_DEPARTURES departed [N] (0/1), departure_timer [N], init_theta [N]; last, one
 * keep-done word: 0 = the layout sets every agent.done = False (all layouts but one), nonzero =
 * agents done at the end of the previous episode stay done, unintegrated, with the layout's state
 * as their frozen state (scenario_circular_config, navigation_graph_safe_eval.py:100-121). Everything
 * else of the reset (episode summary, curriculum block, HJ separation shift, goal_min_time, the
 * observation outputs) is the device's, as in lsm_reset. */
int lsm_reset_layout(lsm_env* env, const lsm_curriculum* cur, const double* layout_device, void* hip_stream);
int32_t lsm_layout_doubles(const lsm_env* env);

/* Overwrite the agent states ([N][4], the LSM_OUT_STATE layout) and, if non-null,
 * reached_goal ([N]) of one env between calls -- what scripts do to `world.agents[i].state` /
 * `scenario.reached_goal` between env.step calls (e.g. tests/golden/make_golden.py's injection,
 * navigation_graph_safe.py:276-317 state fields). Synchronises `hip_stream` first. */
int lsm_set_agent_state(lsm_env* env, int32_t env_index, const double* agent_state,
                        const int32_t* reached, void* hip_stream);

/* Ring-bound outputs: write slot `slot` of ring index i at base + (i + index_offset) * stride_bytes
 * when 0 <= i + index_offset < count, else at the plain lsm_bind_output pointer. Binds the rows of
 * a caller's [T][...] replay buffer (GraphReplayBuffer, onpolicy/utils/graph_buffer.py:84-163) so
 * the step writes obs/node_obs/adj into buffer[t+1] and rewards into rewards[t] with no copy --
 * what GMPERunner.insert's `.copy()`s do (graph_mpe_runner.py:444-487, graph_buffer.py:223-249).
 * count <= 0 unbinds. lsm_select_ring(i) picks the index used by the following lsm_step /
 * lsm_reset calls (host-side only: no upload, no sync); -1 = plain bindings. */
int lsm_bind_output_ring(lsm_env* env, int32_t slot, void* base, size_t stride_bytes, int32_t count,
                         int32_t index_offset);
int lsm_select_ring(lsm_env* env, int32_t index);

/* 1 if a launch since the last call saw an index action outside [0, 25) (it was clamped to keep
 * the launch in bounds; the reference's one-hot decode, environment.py:386-410, has no such
 * input), else 0; -1 on error. Synchronises `hip_stream` and clears the flag. */
int32_t lsm_action_errors(lsm_env* env, void* hip_stream);

/* Name of the kernel instantiation lsm_step / lsm_reset launch for this handle (e.g.
 * "rollout_team_kernel<0, 8, 4>"), as rocprofv3 reports it without the namespace. Owned by the
 * library, valid until the next call on the same thread. */
const char* lsm_kernel_name(const lsm_env* env);

/* Identity of this library's build: the first 16 hex digits of the sha256 of the step kernel's
 * sources and compiler flags (lsm.build), baked in at compile time. Profiles under profiles/
 * record it, and bench.py reports PMC traffic only for the build that produced it. */
const char* lsm_build_id(void);

/* Test-only: the MT19937 words a team-kernel reset may draw from its staged blocks (default 2 MT_N
 * = 1248; values are clamped to [1, 1248]). A smaller stage makes every draw run out and take the
 * cooperative redraw (tests/test_gpu_parity.py). Applies from the next launch. */
int lsm_test_set_mt_stage(lsm_env* env, int32_t words);

/* Shape helpers. */
int32_t lsm_num_entities(const lsm_env* env);   /* E = N * (1 + L) */
int32_t lsm_node_features(const lsm_env* env);  /* F */
int32_t lsm_obs_dim(const lsm_env* env);        /* OBS */

/* Host-side entry points of the SAME scenario-generation / RNG code the reset kernel runs
 * (no GPU needed): used by CPU tests against numpy's legacy RandomState. */
int lsm_host_mt_uniforms(uint32_t seed, int32_t count, double lo, double hi, double* out);
/* The fast-mode (LSM_RNG_PHILOX) stream of reset `reset_index` of an env keyed `key`
 * (= seed + 1000 k): uniform(lo, hi) draws in order. */
int lsm_host_philox_uniforms(uint32_t key, uint32_t reset_index, int32_t count, double lo, double hi,
                             double* out);
/* The raw Philox4x32-10 block function (ctr [4], key [2] -> out [4]): Random123 known answers. */
int lsm_host_philox4x32(const uint32_t* ctr, const uint32_t* key, uint32_t* out);
/* The double integrator's step as the kernel computes it: scipy's solve_ivp(x' = v, v' = a,
 * [0, dt], y0, 'RK45').y[:, -1] restated operation for operation (core.py:199-210); returns the
 * number of RK45 steps. lsm_host_glibc_pow: the kernel's restatement of glibc's pow. */
int lsm_host_rk45_di(const double* y0 /* [4] */, double a0, double a1, double dt, double* y_out /* [4] */);
double lsm_host_glibc_pow(double x, double y);
/* random_scenario as the device draws it for the first reset of an env seeded `seed`
 * (cfg->rng: MT19937 replay, or the Philox stream of reset index 0). */
int lsm_host_scenario(const lsm_config* cfg, const lsm_curriculum* cur, uint32_t seed,
                      double* agent_state /* [N][4] */, double* landmarks /* [NL][4] */);

/* ---- Learner hand-off: GNNBase.process_adj on the device (lsm_edges.hip) ------------------
 * Replaces onpolicy/algorithms/utils/gnn.py:376-407 (GNNBase.process_adj): B adjacency matrices
 * [B][E][E] -> edge_index int64 [2][nnz] (b*E + r, b*E + c) and edge_attr float32 [nnz][1], in
 * nonzero() (row-major) order. `masks` == NULL: `adj` is the reference layout [B][E][E] (B = n*N
 * per-ego graphs, or any batch). `masks` != NULL: the compact layout, `adj` = A [B/N][E][E] and
 * `masks` = [B][ceil(E/64)] (LSM_OUT_ADJ / LSM_OUT_ADJ_MASK of an LSM_ADJ_COMPACT handle); the
 * per-ego matrix is expanded on the fly. Two calls, like torch.nonzero's count-then-fill:
 *   lsm_edges_count  offsets int64 [B+1] (offsets[B] = nnz), device; needs a device workspace of
 *                    lsm_edges_workspace_bytes(B) bytes (scratch, cleared by the call itself)
 *   lsm_edges_emit   fills edge_index / edge_attr given nnz (= offsets[B], read by the caller)
 *   lsm_edges_emit_dev  the same without the host round trip: nnz is read on the device from
 *                    offsets[B]; edge_index holds 2*cap int64 and edge_attr cap floats (cap >= nnz,
 *                    e.g. B*E*E), filled as [2][nnz] / [nnz][1] from their start; nothing is
 *                    written when nnz > cap (the caller checks offsets[B] afterwards)
 *   lsm_edges_scan_emit  one adjacency pass: `counts` int64 [B] = each graph's nonzeros as the step
 *                    kernel wrote them (LSM_OUT_ADJ_NNZ of the call that wrote `adj`), so there is
 *                    no count pass: scan into offsets (int64 [B + 2]: offsets[B] = nnz, offsets[B + 1]
 *                    = the number of graphs whose nonzeros differed from their count, 0 when the
 *                    counts belong to `adj`; such a graph's slot is zero-filled) and emit as
 *                    lsm_edges_emit_dev does (nothing written when nnz > cap); host_nnz_bad (host
 *                    int64 [2], nullable): the call then synchronises the stream and returns
 *                    offsets[B], offsets[B + 1] there (torch.nonzero's one sync, no extra host call)
 * Errors: nonzero return, text in lsm_edges_last_error() (per host thread). */
size_t lsm_edges_workspace_bytes(int64_t B);
int lsm_edges_count(const float* adj, const uint64_t* masks, int64_t B, int32_t E, int32_t N,
                    int64_t* offsets, void* workspace, size_t workspace_bytes, void* hip_stream);
int lsm_edges_emit(const float* adj, const uint64_t* masks, int64_t B, int32_t E, int32_t N,
                   const int64_t* offsets, int64_t nnz, int64_t* edge_index, float* edge_attr,
                   void* hip_stream);
int lsm_edges_emit_dev(const float* adj, const uint64_t* masks, int64_t B, int32_t E, int32_t N,
                       const int64_t* offsets, int64_t cap, int64_t* edge_index, float* edge_attr,
                       void* hip_stream);
int lsm_edges_scan_emit(const float* adj, const uint64_t* masks, int64_t B, int32_t E, int32_t N,
                        const int64_t* counts, int64_t* offsets, void* workspace, size_t workspace_bytes,
                        int64_t cap, int64_t* edge_index, float* edge_attr, int64_t* host_nnz_bad,
                        void* hip_stream);
const char* lsm_edges_last_error(void);

/* ---- Buffer insert: the derived rows of GMPERunner.insert / warmup (lsm_buffer.hip) ----------
 * Replaces graph_mpe_runner.py:444-487 (masks, active_masks, share_obs, share_agent_id) and the
 * agent_id rows, for one buffer index, from obs [n][N][OBS] f32 and dones [n][N] u8 (NULL at
 * warmup: masks untouched). centralized = args.use_centralized_V: share_obs [n][N][N*OBS] and
 * share_agent_id [n][N][N], else [n][N][OBS] / [n][N][1]. masks / active_masks f32 [n][N][1],
 * agent_id int32 [n][N][1]. */
int lsm_buffer_insert(const float* obs, const uint8_t* dones, int32_t n, int32_t N, int32_t OBS,
                      int32_t centralized, float* share_obs, int32_t* agent_id, int32_t* share_agent_id,
                      float* masks, float* active_masks, void* hip_stream);
const char* lsm_buffer_last_error(void);

/* ---- Episode summary for the runner's log (lsm_metrics.hip) ---------------------------------
 * Replaces the per-episode reduction of GMPERunner's ep-info parse (graph_mpe_runner.py:222-251:
 * the mean over threads of the 8-key summaries, the min of min_distance_min). From one rank's
 * ep_info [n][8] float64 (LSM_OUT_EP_INFO, 16-B aligned) it writes out[10] on the device, stream-
 * ordered, no host sync: out[0..7] column sums, out[8] = n, out[9] = min of column 6 (NaN
 * propagates). Across ranks out[0..8] is all_reduce(SUM)'d and out[9] all_reduce(MIN)'d (RCCL);
 * mean = sum / count. Fixed addition order (reproducible). Nonzero on bad arguments. */
int lsm_episode_summary(const double* ep_info, int32_t n, double* out /* [10] */, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif
