// lsm_rollout.hip -- MI355X (gfx950) kernels + C ABI for the navigation_graph_safe rollout.
//
// One 64-lane wavefront (one workgroup) per environment. Everything an env needs for a
// step -- agent states, landmarks, the E x E distance table, pairwise filter scratch and
// an output staging tile -- lives in that wave's LDS; state arrays in HBM are env-major
// SoA so a wave's loads/stores of its env are contiguous. One launch does the whole
// MultiAgentGraphEnv.step (multiagent/environment.py:963-1042) including the worker's
// auto-reset (onpolicy/envs/env_wrappers.py:866-871):
//
//   1. update_graph() edge mask from the state at step start    (navigation_graph_safe.py:996-1015)
//   2. decode Discrete(25) actions                               (environment.py:386-410)
//   3. pairwise HJ safety filter, lanes = (ego, other) pairs     (core.py:648-677, safety_filter.py)
//   4. integrate (closed form), speed clamp, travel distance     (core.py:118-131,199-210)
//   5. E x E distances in LDS, min relative distance             (core.py:514-543,696-709)
//   6. obs / reward / goal & done update per agent               (navigation_graph_safe.py:606-875)
//   7. per-ego node features + masked adjacency with the reference's sequential
//      snapshot rule (ego i sees agents j <= i after their reward update)  (:932-994)
//   8. episode statistics, info_callback numbers, done flags      (environment.py:1004-1029)
//   9. if all agents done: device reset with draw-exact numpy MT19937 replay (:264-366,1199-1367)
//
// Numerics: float64 state and decisions, -ffp-contract=off plus explicit fma() only where
// numpy/OpenBLAS fuses (lsm_numeric.h); HJ grid interpolation in float32 like the
// reference's JAX (oracle/hj_grid.py defines the semantics). No MFMA: nothing here is a
// dense contraction; the kernel is bound by HBM writes of the dense per-ego outputs.
#include <hip/hip_runtime.h>
#include <math.h>
#include <cmath>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/lsm_rollout.h"
#include "lsm_numeric.h"
#include "lsm_rk45.h"
#include "lsm_scenario.h"

// Diagnostic switches (bounds that compute wrong results on purpose, in-kernel stamps) exist only in
// variant builds (lsm.build.build_variants defines LSM_DIAGNOSTIC_BUILD); the product refuses them.
#if !defined(LSM_DIAGNOSTIC_BUILD) &&                                                              \
    (defined(LSM_STAMPS) || defined(LSM_XP_VALHOT) || defined(LSM_XP_GRADHOT) || defined(LSM_XP_NOFILT) || \
     defined(LSM_XP_NOOUT) || defined(LSM_XP_NORESETEMIT) || defined(LSM_XP_NORK) || defined(LSM_XP_NOSCEN) || \
     defined(LSM_XP_DELAY) || defined(LSM_XP_POISON))
#error "diagnostic switch in a product build: use lsm.build.build_variants (LSM_DIAGNOSTIC_BUILD)"
#endif

// Diagnostic builds: LSM_XP_POISON=pattern sets every 32-bit word of a workgroup's dynamic LDS to the
// pattern before the kernel's first LDS access. LDS is not cleared between workgroups, so a read of a
// word the kernel never wrote returns whatever the CU's previous workgroup left there; under the poison
// it returns the pattern instead. Outputs that stay equal to the oracle under two different patterns
// (tests run with LSM_LIB = the poisoned library) do not depend on unwritten LDS.
#ifdef LSM_XP_POISON
#define LDS_POISON(base, bytes, tid, nthr)                                                         \
  do {                                                                                             \
    for (uint32_t q_ = (uint32_t)(tid); q_ < (uint32_t)(bytes) / 4u; q_ += (uint32_t)(nthr))       \
      ((uint32_t*)(base))[q_] = (uint32_t)(LSM_XP_POISON);                                         \
  } while (0)
#else
#define LDS_POISON(base, bytes, tid, nthr) do { } while (0)
#endif

// LSM_PART (lsm.build): 0 = host code only, g > 0 = kernel group g only, undefined = everything
#if defined(LSM_PART) && LSM_PART != 0
#define LSM_HOST_PART 0
#else
#define LSM_HOST_PART 1
#endif

// stamps per env in LSM_OUT_DEBUG_STAMPS: 16 in the ABI; diagnostic builds stamp 40
#ifdef LSM_STAMPS
#define LSM_NSTAMP 40
#else
#define LSM_NSTAMP 16
#endif
#ifdef LSM_STAMPS
// diagnostic build only: per-phase s_memtime stamps of each env's wave (never in the product .so)
#define STAMP(k)                                                                             \
  do {                                                                                       \
    __syncthreads();                                                                         \
    if (lane == 0 && gptr(P.stamps)) gptr(P.stamps)[(size_t)env * LSM_NSTAMP + (k)] = __builtin_amdgcn_s_memtime(); \
    if (K.stop_after == (k)) return;  /* per-phase instruction counting (lsm.diag_stamps) */ \
  } while (0)
// slots 13/14: 100 MHz chip-wide clock at wave start / end (dispatch ramp and tail);
// slot 15: HW_ID (wave, simd, cu, se) | XCC_ID << 32
#define RTSTAMP(k)                                                                           \
  do {                                                                                       \
    if (lane == 0 && gptr(P.stamps)) gptr(P.stamps)[(size_t)env * LSM_NSTAMP + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define RTSTAMP(k) \
  do {             \
  } while (0)
#define STAMP(k) \
  do {           \
  } while (0)
#endif

namespace lsm {

constexpr int WAVE = 64;
constexpr int MAXN = 32;        // agents per env supported by the one-wave kernel
constexpr int MAXE = 64;        // entities per env (N * (1 + L))
constexpr int MT_WORDS = MT_N + 1;  // key[624] + pos
constexpr int NCUR = 12;
constexpr int NSTAT = 6;        // travel_length, travel_distance, done, conflict, min_distance, multiple
constexpr int NWINFO = 4;       // times_required, dists_to_goal, dist_left_to_goal, num_agent_collisions
// Per-env HJ separation history (record, after cur): HjDataHandle.update_separation_distance
// (safety_filter.py:170-174) runs `values_hj -= shift` on every reset of every env, so each env's
// table is the uploaded one minus its own chain of float64 shifts, each rounded to float32
// (numpy: float32 array -= float64 scalar). sep[0] = number of shifts, sep[1] = the env's current
// separation (sep[0] == 0: the uploaded table's, KParams::val_sep0), sep[2 + k] = shift k for
// k < KSEP; longer chains continue in StateDev::sepx (HBM, grown by the host as the number of
// separation changes since the upload grows), so no length is refused.
constexpr int KSEP = 8;
constexpr int NSEPW = 2 + KSEP;

// HJ / TTR table in "cell-corner" layout: every grid cell stores the 2^ndim corner values
// it interpolates (lexicographic corner order, dim 0 slowest) contiguously, so one query
// reads 64 B (4-D) / 128 B (5-D) of values and 2^ndim * 16 * gw B of gradients -- one or
// two cache lines instead of 2^ndim scattered nodes. 16x the node table (1.8 GB for the
// full DI table): sized for 288 GB HBM, expanded on the device at upload.
struct TableDev {
  const float* cells;    // [n_cells][2^ndim]
  const float4* gcells;  // [n_cells][2^ndim][gw]
  int ndim;
  int n[5];        // nodes per dim
  int cstride[5];  // cell strides (cells per dim: n (periodic) or n - 1)
  float lo[5];
  float sp[5];
  float rsp[5];    // 1 / sp (float32, correctly rounded)
  int mdiv[5];     // 1: (s - lo) / sp by the reciprocal + one FMA correction (grid_pos), checked at
                   // upload to equal the division bit for bit over every float32 the lookups can
                   // meet (mdiv_check_kernel); 0: the division
  int periodic[5];
  int gw;  // float4 per corner gradient (1 for <= 4 dims, 2 for 5 dims)
  // Value bounds per block of 2^bshift cells per dim: (min, max) of the block's nodes widened
  // by the fp32 interpolation error (bounds_kernel). Small enough to stay in L2; the
  // workgroup kernel uses them to skip exact lookups that cannot be the argmin. nullptr: none.
  const float2* bnd;
  int bshift;
  int bstride[5];   // blocks: stride per dim
};

// Persistent per-env state: ONE contiguous record per env (env-major, 128-B aligned
// stride) whose byte layout is exactly the head of the env's LDS block (lds_plan), so a
// step starts with a straight float4 copy HBM -> LDS and ends with the copy back. Fields
// (16-B aligned each), in record order:
//   [0, a1)   ps [4][N], pdist, adiff [N] f64, done, reached, sfilt, decon [N] i32, step i32
//   [a1, a2)  cur [NCUR] + the HJ shift chain                               (reset only)
//   [a2, a3)  stats [NSTAT][N], winfo [NWINFO][N], gmt, minrel [N] f64
//   [a3, rec) lm [6][NL] f64 (x, y, heading, speed, sin, cos), lmd            (reset only)
// A step rewrites [0, a1) and [a2, a3). Everything a step needs before its distances is in
// [0, a2) (state, done flags, curriculum, shifts): the team kernel loads that part first and
// the rest while its agent wave filters and integrates (lsm_team.h).
struct StateDev {
  float4* rec;          // [n][rec_stride16]
  uint32_t rec_stride16;
  uint32_t rec16;       // float4 per record
  uint32_t a1_16, a2_16, a3_16;   // the boundaries above, in float4
  double* prev;         // [n][8] previous episode summary
  uint32_t* mt;         // [n][MT_WORDS] (LSM_RNG_PHILOX: only word MT_N, the reset index + MT_N)
  double* dep;          // [n][DEPW(N)] departed [N], departure_timer [N], init_theta [N], and the
                        // final disconnect mask of the last call (u64 bits) (LSM_SCENARIO_DEPARTURES)
  double* sepx;         // [n][sepx_cap] HJ separation shifts KSEP, KSEP + 1, ... of each env's chain
  uint32_t sepx_cap;    // (nullptr / 0 until a chain can outgrow the record's KSEP slots)
};

struct OutDev {
  float* obs;
  float* node;
  float* adj;
  float* rew;
  uint8_t* dones;
  uint8_t* reset_flag;
  double* ep_info;
  double* info;
  uint8_t* edges;
  double* state;
  uint64_t* adjmask;   // LSM_OUT_ADJ_MASK (compact adjacency layout)
  float* share_obs;    // LSM_OUT_SHARE_OBS (optional)
  float* masks;        // LSM_OUT_MASKS (optional)
  float* active_masks; // LSM_OUT_ACTIVE_MASKS (optional)
  double* cforce;      // LSM_OUT_COLLISION_FORCE (lsm_config.collision_forces only)
  uint8_t* departed;   // LSM_OUT_DEPARTED (optional)
  int64_t* adjnnz;     // LSM_OUT_ADJ_NNZ (optional): nonzeros of each ego's adjacency as stored
};

struct KParams {
  int n_envs, N, L, NL, E, F, OBS, dyn, episode_length, use_masking, use_filter_arg, auto_reset;
  int adj_compact;   // LSM_ADJ_COMPACT: unmasked E x E table once per env + per-ego masks
  int lean;          // the team kernel carves the lean LDS layout (lds_plan)
  int filter_search; // workgroup kernel's HJ argmin: 1 bound-pruned (default), 0 every pair exact
  int scenario;      // LSM_SCENARIO_*
  int rng;           // LSM_RNG_*
  int nis;           // World.num_internal_step (>= 1): filter -> integrate repeats per step
  int rbin;          // lsm_config.reward_terms (LSM_REWARD_* bits)
  int collab;        // lsm_config.collaborative: shared reward
  int rext;          // rbin || collab: rewards finished after every agent's goal / done update
  int use_hj;        // the HJ handle exists (filter on, or LSM_REWARD_HJ_VALUE): resets shift it
  int mt_stage;      // team-kernel resets: MT19937 words one lane may draw from the staged blocks
                     // (2 MT_N; lsm_test_set_mt_stage lowers it so tests reach the cooperative redraw)
  int64_t seed, env_offset;   // Philox keys: seed + 1000 * (env_offset + env)
  uint32_t lds_dep_off;       // LSM_SCENARIO_DEPARTURES: LDS offset of the departure arrays
  double dt, world_size, coord_range, world_eng, sep_target, max_speed, min_speed, gs_min, gs_max;
  double coord_range_s;  // the largest double s with sqrt(s) <= coord_range (correctly rounded sqrt):
                         // sqrt(s) > coord_range <=> s > coord_range_s, for squared distances s >= 0
  double scen_d2lo, scen_d2hi;   // the scenario's separated-positions band (dmin, dmax) on squared
                                 // distances: sqrt(s) > dmin <=> s > d2lo, sqrt(s) < dmax <=> s < d2hi
  double act0[5], act1[5];
  double mag_c[50], mag_s[50];
  double cos_pi6, two_pi, pi;
  double di_thr_xmax, di_thr_xmin, di_thr_ymax, di_thr_ymin, di_axmax, di_axmin, di_aymax, di_aymin;
  double at_vmax, at_vmin, at_amax, at_amin, at_wmax, at_thr_amax, at_thr_amin;
  float at_box_w, at_box_amax, at_box_amin;  // float32 box corners (jnp)
  double ttr_max;
  double val_sep0;       // separation of the uploaded value table (HjDataHandle.separation_distance)
  uint32_t m_E, m_EE, m_EF, m_F, m_EF4, m_NL;  // ceil(2^32 / d) for exact small-numerator division
  unsigned long long* stamps;     // LSM_OUT_DEBUG_STAMPS (diagnostic builds only)
  int diag;                       // diagnostic builds: bit 0 skip adj/node stores, bit 1 skip filter (LSM_DIAG)
  uint32_t lds_env_bytes;         // LDS bytes per env (envs per wave > 1: consecutive blocks)
  const uint16_t* pairs;          // strict upper-triangle entity pairs (a | b << 8)
  int32_t* action_err;            // set to 1 by a launch that saw an action index outside [0, 25)
  TableDev val, ttr;
  StateDev s;
  OutDev o;
};

// Per-launch kernel arguments (the rest lives in a device-resident KParams per handle).
struct KStep {
  const void* actions;
  const double* layout;   // mode 2: [n][layout doubles] (lsm_reset_layout)
  int action_kind, mode, emit_edges, stop_after;   // mode 0 = step, 1 = reset all, 2 = reset from layout
  double cur_new[NCUR];
};

// ----------------------------------------------------------------------------------
// LDS layout (dynamic, 16-byte aligned carve). Two unions keep one env under ~9 KB at
// N = 8 so LDS does not cap residency below the VGPR limit (16 waves / CU):
//   U1 = {fval, aa, aa2} (step)         | {mt, scen, scratch} (reset) | {stage} (node output, last)
//   U2 = {dpair, vpair, inr} (filter)   | {feat, egooff} (DI node rows) | magnetic partial sums
// The lean layout (airtaxi team kernel at N = 16: 19.3 instead of 25.5 KB per env, so a CU's
// 160 KB holds 8 envs instead of 6, its VGPR limit) keeps the filter's pair matrices in U1
// (dead before the distances are computed), leaves U2 to the info rows and the node tables,
// and drops fval's landmark-landmark block (its values are the episode's lmd cache).
// ----------------------------------------------------------------------------------
__host__ __device__ inline size_t align16_(size_t x) { return (x + 15) & ~(size_t)15; }

struct Lds {
  // ---- persistent record (StateDev) ----
  double* ps;        // [4][N] agent state (after integration; velocities pre-freeze)
  double* stats;     // [NSTAT][N]
  double* winfo;     // [NWINFO][N]
  double* pdist;     // [N] travel distance (state.p_dist)
  double* gmt;       // [N] goal_min_time
  double* minrel;    // [N]
  double* adiff;     // [N]
  int32_t* dpost;    // [N] done after the reward update (record: done)
  int32_t* rpost;    // [N] reached_goal after (record: reached)
  int32_t* sfilt;    // [N]
  int32_t* decon;    // [N]
  int32_t* step;     // [2] env.current_step; 1 = cached distances unmasked (state edited)
  double* cur;       // [NCUR]
  double* sep;       // [NSEPW] HJ separation shift chain (= cur + NCUR)
  double* lm;        // [6][NL] x, y, heading, speed, sin, cos
  double* lmsc;      // = lm + 4 NL
  float* lmd;        // [NL(NL-1)/2] thresholded landmark-landmark distances (per episode)
  // ---- step scratch ----
  int32_t* dpre;     // [N] done before reward update
  int32_t* rpre;     // [N] reached_goal before
  double* raw;       // [2][N]
  double* safe;      // [2][N]
  double* wold;      // [2][N] dists_to_goal / times_required before this step's info
  double* wnew;      // [2][N] after
  uint64_t* emask;   // [N] bit r: entity r disconnected for ego e (snapshot rule)
  double* ecs;       // [2][N] cos / sin of the heading at step start (airtaxi filter frame)
  // U1
  float* fval;       // [E][E] d if 0 < d < range else 0 (float32, unmasked); lean: rows < N
                     // [N][E], then the landmark rows' agent columns [NL][N] (fv4; the
                     // landmark-landmark block is read from lmd)
  double* aa;        // [N][N] float64 agent-agent distances (episode stats)
  double* aa2;       // [N][N] np.linalg.norm agent-agent distances (min relative distance, collisions)
  uint32_t* mt;      // [MT_WORDS]
  uint32_t* mtn;     // [MT_N] the next MT19937 block (team kernel resets; U1 after scratch, or U2)
  double* scen;      // [SCEN_WS]
  double* scratch;   // [2][MAXN]
  // U2
  double* dpair;     // [N][N] [other j][ego i] (ego fastest)
  double* vpair;     // [N][N] [other j][ego i] float32 values held as float64: the team kernel's
                     // agent wave then reads 8-B words from G env blocks without bank conflicts
  uint8_t* inr;      // [N][N] [other j][ego i]
  double* feat;      // [2N + NL][F] DI entity rows: agents pre, agents post, landmarks
  double* egooff;    // [N][F] DI ego offsets
  float* stage;      // [64][F] airtaxi node staging
  double* info;      // [N][LSM_INFO_FIELDS] info rows staged for the coalesced copy-out (U2 base)
  bool lean;         // the lean one-wave layout (lds_plan): see fval and the U1 / U2 note
  // workgroup-per-env kernel only (lsm_block.h)
  double* ex;        // [E] entity x (agents after integration, then landmarks)
  double* ey;        // [E]
  int32_t* ccnt;     // [N] is_collision counts of this step
  uint64_t* mpre;    // [4] disconnect bits before the reward update (entity r = bit r)
  uint64_t* mpost;   // [4] after
  // LSM_SCENARIO_DEPARTURES only (generic airtaxi one-wave kernel; nullptr elsewhere, so every
  // departure test below folds away in the other kernels)
  int32_t* dep0;     // [N] departed before the reward update
  int32_t* dep1;     // [N] after
  int32_t* tmr;      // [N] departure_timer
  double* ith;       // [N] init_theta
  double* pth;       // [N] heading after the reward update (departure resets it)
  double* psp;       // [N] speed after the reward update (departure / freeze / done)
  double* trig1;     // [4][N] cos, sin, vx, vy of the post state (node features)
};

// doubles per env of StateDev::dep: departed, timer, init_theta [N], then the accumulated
// disconnect mask of the step's last ego (the next update_graph's), up to 4 words (E <= 256)
__host__ __device__ inline int depw(int N) { return 3 * N + 4; }

// LDS bytes of the departure arrays (appended after lds_plan's block)
__host__ __device__ inline size_t dep_lds_bytes(int N) {
  return 3 * align16_(4 * (size_t)N) + 3 * align16_(8 * (size_t)N) + align16_(32 * (size_t)N);
}

struct LdsPlan {
  size_t bytes;     // LDS per env
  size_t rec;       // persistent record bytes (LDS head == HBM record)
  size_t a1, a2, a3;   // record sections (StateDev)
  size_t off[40];
};

// Workgroup-per-env kernel (lsm_block.h): threads per env and its limits.
constexpr int BT = 256;
constexpr int BMAXN = 64;
constexpr int BMAXE = 256;   // masks: E <= BT so one ballot per wave gives a mask word

// q / d for q * d < 2^32 (all index math here): __umulhi(q, ceil(2^32 / d))
__device__ __forceinline__ int fdiv(int q, uint32_t m) { return (int)__umulhi((uint32_t)q, m); }

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// Kernels are specialised on the agent count NT (L = 2, the training setting) so every
// dimension, LDS offset and index division below folds to a constant; NT = 0 is the
// generic kernel reading the handle's runtime dimensions.
#define LSM_DIMS                        \
  const int N = NT ? NT : P.N;          \
  const int L = NT ? 2 : P.L;           \
  const int NL = N * L;                 \
  const int E = N + NL;                 \
  const int F = DYN ? 11 : 10;          \
  (void)L; (void)NL; (void)E; (void)F

// q / d for the small non-negative index math: a constant division when specialised
template <int NT>
__device__ __forceinline__ int qdiv(int q, int d, uint32_t m) {
  return NT ? (int)((uint32_t)q / (uint32_t)d) : fdiv(q, m);
}

// Pointers read from the device-resident KParams are generic; re-tagging them as global
// (address space 1) lets the compiler emit global_* instead of flat_* accesses (flat
// stores also count against lgkmcnt, so every later LDS wait would drain them).
#define GAS __attribute__((address_space(1)))
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <class T>
__device__ __forceinline__ GAS T* gptr(T* p) {
  return (GAS T*)p;
}

// One float4 of the per-step graph outputs. (Non-temporal stores were measured slower with
// the filter on: 37.9 vs 35.9 us per step at config 3.)
// Output stores. NTS = nontemporal (`nt`): measured on MI355X (profiles/r01_v9_nt_stores.txt)
// +5 % at config 4 (airtaxi N = 16) and +8.5 % at config 5 (workgroup kernel), within noise
// (-1 %) at config 3, so the N >= 16 one-wave kernels and the workgroup kernel use it. The N = 8
// team kernel with them: 34.82 vs 31.50 us at config 3 (profiles/r06_s07_ab_c3.txt).
template <bool NTS = false>
__device__ __forceinline__ void st_stream(GAS float* dst, float4 v) {
  const f32x4 x = {v.x, v.y, v.z, v.w};
  if (NTS) __builtin_nontemporal_store(x, (GAS f32x4*)dst);
  else *(GAS f32x4*)dst = x;
}

// Synchronise the lanes of one env. An env of <= 64 lanes lives in one wave (the one-wave
// kernels, and each wave of the team kernel, whose other waves hold other envs and must not be
// waited for): LDS accesses of a wave complete in order, so a compiler fence + wave barrier
// suffices. The workgroup-per-env kernel (LPE = BT) needs the workgroup barrier.
template <int LPE>
__device__ __forceinline__ void esync() {
  if (LPE > 64) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// all() over the LPE-lane group of the calling lane (one env)
template <int LPE>
__device__ __forceinline__ bool group_all(bool v) {
  if (LPE == 64) return __all(v);
  const uint64_t b = __ballot(v);
  const int g = (int)threadIdx.x / LPE;
  const uint64_t gm = (~0ull >> (64 - LPE)) << (g * LPE);
  return (b & gm) == gm;
}

// Offsets of every LDS array (shared by the host launch/record init and the device carve).
// The record prefix (fields 0..14) is common to both kernels; the workgroup kernel keeps no
// landmark-distance cache (lmd, 0 bytes), no E x E / N x N tables, and adds the entity
// position table, per-ego multi-word masks and a node staging area.
__host__ __device__ inline LdsPlan lds_plan(int N, int NL, int E, int F, bool block = false,
                                            bool lean = false) {
  LdsPlan p;
  size_t o = 0;
  int k = 0;
  auto put = [&](size_t bytes) { p.off[k++] = o; o += align16(bytes); };
  // record: fields 0..14 (carve order: ps stats winfo pdist gmt minrel adiff done reached sfilt
  // decon step cur lm lmd) placed in the section order of StateDev
  {
    const size_t fsz[15] = {(size_t)8 * 4 * N, (size_t)8 * NSTAT * N, (size_t)8 * NWINFO * N, (size_t)8 * N,
                            (size_t)8 * N, (size_t)8 * N, (size_t)8 * N, (size_t)4 * N, (size_t)4 * N,
                            (size_t)4 * N, (size_t)4 * N, 8, (size_t)8 * (NCUR + NSEPW), (size_t)8 * 6 * NL,
                            block ? 0 : (size_t)4 * (NL * (NL - 1) / 2)};
    const int order[15] = {0, 3, 6, 7, 8, 9, 10, 11, 12, 1, 2, 4, 5, 13, 14};
#pragma unroll
    for (int q = 0; q < 15; ++q) {
      const int f = order[q];
      p.off[f] = o;
      o += align16(fsz[f]);
      if (f == 11) p.a1 = o;
      if (f == 12) p.a2 = o;
      if (f == 5) p.a3 = o;
    }
    k = 15;
  }
  p.rec = o;
  const int MW = (E + 63) / 64;
  // scratch
  put(4 * N); put(4 * N); put(8 * 2 * N); put(8 * 2 * N); put(8 * 2 * N); put(8 * 2 * N);
  put(block ? 8 * N * MW : 8 * N);
  put(F == 10 ? 0 : 8 * 2 * N);
  if (block) {
    // fval aa aa2 -> none; U1 = {mt, scen, scratch} | {feat, egooff} | {pair partials, info rows}
    put(8 * E); put(8 * E); put(4 * N); put(8 * 8);   // ex, ey, ccnt, mpre[4] + mpost[4]
    const size_t u1 = o;
    size_t c = align16(4 * MT_WORDS), d = c + align16(8 * SCEN_WS), e = d + align16(8 * 2 * N);
    size_t g1 = F == 10 ? align16(8 * (2 * N + NL) * F) : align16(8 * 4 * N);
    size_t g2 = g1 + (F == 10 ? align16(8 * N * F) : 0);
    size_t m = 8 * 2 * BT;
    m = m > (size_t)(8 * LSM_INFO_FIELDS * N) ? m : (size_t)(8 * LSM_INFO_FIELDS * N);
    size_t u1sz = e > g2 ? e : g2;
    u1sz = u1sz > align16(m) ? u1sz : align16(m);
    // the filter's per-wave survivor queues (lsm_block.h): (i, j) u16 + value f32 per slot
    const int tpe = (64 * N <= BT) ? 64 : (32 * N <= BT) ? 32 : (16 * N <= BT) ? 16 : (8 * N <= BT) ? 8 : 4;
    const size_t qb = align16((size_t)(BT / WAVE) * WAVE * ((N + tpe - 1) / tpe) * 6);
    u1sz = u1sz > qb ? u1sz : qb;
    p.off[k++] = u1; p.off[k++] = u1 + c; p.off[k++] = u1 + d;   // mt, scen, scratch
    p.off[k++] = u1; p.off[k++] = u1 + g1;                         // feat, egooff
    p.off[k++] = u1;                                               // dpair: pair partials / info rows
    o = u1 + u1sz;
    // node staging (airtaxi, or DI with E * F % 4 != 0): live together with feat
    const bool stage = F != 10 || ((E * F) & 3) != 0;
    p.off[k++] = o;
    o += stage ? align16(4 * BT * F) : 0;
    p.bytes = o;
    return p;
  }
  // U1
  const size_t u1 = o;
  const size_t fvb = lean ? (size_t)4 * (N * E + NL * N) : (size_t)4 * E * E;
  size_t a = align16(fvb), a2 = a + align16(8 * N * N), b = a2 + align16(8 * N * N);
  size_t c = align16(4 * MT_WORDS), d = c + align16(8 * SCEN_WS), e = d + align16(8 * 2 * MAXN);
  p.off[k++] = u1; p.off[k++] = u1 + a; p.off[k++] = u1 + a2; p.off[k++] = u1; p.off[k++] = u1 + c;
  p.off[k++] = u1 + d;
  size_t u1sz = b > e ? b : e;
  const size_t h0 = align16(4 * WAVE * F);   // node staging for up to 64 pairs
  u1sz = u1sz > h0 ? u1sz : h0;
  // pair matrices dpair, vpair, inr, then the team kernel's per-ego filter slots (filter_slot)
  size_t f1 = align16(8 * N * N), f2 = f1 + align16(8 * N * N), f3 = f2 + align16(N * N) + align16(32 * N);
  if (lean) u1sz = u1sz > f3 ? u1sz : f3;   // the pair matrices at the head of U1
  o = u1 + u1sz;
  // U2
  const size_t u2 = o;
  const size_t pb = lean ? u1 : u2;   // pair matrices
  // DI entity rows + ego offsets; airtaxi: the [4][N] heading trig table (feat) only
  size_t g1 = F == 10 ? align16(8 * (2 * N + NL) * F) : align16(8 * 4 * N);
  size_t g2 = g1 + (F == 10 ? align16(8 * N * F) : 0);
  p.off[k++] = pb; p.off[k++] = pb + f1; p.off[k++] = pb + f2;
  p.off[k++] = u2; p.off[k++] = u2 + g1; p.off[k++] = u1;   // stage aliases U1 (adj emitted first)
  size_t m = lean ? g2 : (f3 > g2 ? f3 : g2);
  // magnetic partials + the segment constants (DI, filter off; team kernel: mag_table_store)
  if (F == 10) m = m > (size_t)(8 * (2 * 64 + 100)) ? m : (size_t)(8 * (2 * 64 + 100));
  m = m > (size_t)(8 * LSM_INFO_FIELDS * N) ? m : (size_t)(8 * LSM_INFO_FIELDS * N);   // info rows
  // the next MT19937 block of a team-kernel reset (live with mt / scen; U2 is free then): after
  // U1's scratch when it fits, else at the U2 base (the team kernels' layouts have room either way,
  // lsm_create checks)
  const size_t mtb = align16(4 * MT_N);
  const bool mtn_u1 = u1sz - e >= mtb;
  p.off[k++] = mtn_u1 ? u1 + e : u2;
  if (!mtn_u1 && m < mtb) m = mtb;
  o = u2 + m;
  p.bytes = o;
  return p;
}

__device__ __forceinline__ Lds carve(unsigned char* base, int N, int NL, int E, int F, bool lean = false) {
  const LdsPlan p = lds_plan(N, NL, E, F, false, lean);
  Lds L;
  int k = 0;
  L.ps = (double*)(base + p.off[k++]);
  L.stats = (double*)(base + p.off[k++]);
  L.winfo = (double*)(base + p.off[k++]);
  L.pdist = (double*)(base + p.off[k++]);
  L.gmt = (double*)(base + p.off[k++]);
  L.minrel = (double*)(base + p.off[k++]);
  L.adiff = (double*)(base + p.off[k++]);
  L.dpost = (int32_t*)(base + p.off[k++]);
  L.rpost = (int32_t*)(base + p.off[k++]);
  L.sfilt = (int32_t*)(base + p.off[k++]);
  L.decon = (int32_t*)(base + p.off[k++]);
  L.step = (int32_t*)(base + p.off[k++]);
  L.cur = (double*)(base + p.off[k++]);
  L.sep = L.cur + NCUR;
  L.lm = (double*)(base + p.off[k++]);
  L.lmsc = L.lm + 4 * NL;
  L.lmd = (float*)(base + p.off[k++]);
  L.dpre = (int32_t*)(base + p.off[k++]);
  L.rpre = (int32_t*)(base + p.off[k++]);
  L.raw = (double*)(base + p.off[k++]);
  L.safe = (double*)(base + p.off[k++]);
  L.wold = (double*)(base + p.off[k++]);
  L.wnew = (double*)(base + p.off[k++]);
  L.emask = (uint64_t*)(base + p.off[k++]);
  L.ecs = (double*)(base + p.off[k++]);
  L.fval = (float*)(base + p.off[k++]);
  L.aa = (double*)(base + p.off[k++]);
  L.aa2 = (double*)(base + p.off[k++]);
  L.mt = (uint32_t*)(base + p.off[k++]);
  L.scen = (double*)(base + p.off[k++]);
  L.scratch = (double*)(base + p.off[k++]);
  L.dpair = (double*)(base + p.off[k++]);
  L.vpair = (double*)(base + p.off[k++]);
  L.inr = (uint8_t*)(base + p.off[k++]);
  L.feat = (double*)(base + p.off[k++]);
  L.egooff = (double*)(base + p.off[k++]);
  L.stage = (float*)(base + p.off[k++]);
  L.mtn = (uint32_t*)(base + p.off[k++]);
  L.info = L.feat;   // U2 base (= dpair outside the lean layout)
  L.lean = lean;
  L.ex = L.ey = nullptr;
  L.ccnt = nullptr;
  L.mpre = L.mpost = nullptr;
  L.dep0 = L.dep1 = L.tmr = nullptr;
  L.ith = L.pth = L.psp = L.trig1 = nullptr;
  return L;
}

// The departure arrays of an env block (LSM_SCENARIO_DEPARTURES) at byte offset `off`.
__device__ __forceinline__ void carve_dep(Lds& L, unsigned char* base, size_t off, int N) {
  L.dep0 = (int32_t*)(base + off); off += align16_(4 * (size_t)N);
  L.dep1 = (int32_t*)(base + off); off += align16_(4 * (size_t)N);
  L.tmr = (int32_t*)(base + off); off += align16_(4 * (size_t)N);
  L.ith = (double*)(base + off); off += align16_(8 * (size_t)N);
  L.pth = (double*)(base + off); off += align16_(8 * (size_t)N);
  L.psp = (double*)(base + off); off += align16_(8 * (size_t)N);
  L.trig1 = (double*)(base + off);
}

// LDS carve of the workgroup-per-env kernel (lds_plan(..., block = true)).
__device__ __forceinline__ Lds carve_block(unsigned char* base, int N, int NL, int E, int F) {
  const LdsPlan p = lds_plan(N, NL, E, F, true);
  Lds L;
  int k = 0;
  L.ps = (double*)(base + p.off[k++]);
  L.stats = (double*)(base + p.off[k++]);
  L.winfo = (double*)(base + p.off[k++]);
  L.pdist = (double*)(base + p.off[k++]);
  L.gmt = (double*)(base + p.off[k++]);
  L.minrel = (double*)(base + p.off[k++]);
  L.adiff = (double*)(base + p.off[k++]);
  L.dpost = (int32_t*)(base + p.off[k++]);
  L.rpost = (int32_t*)(base + p.off[k++]);
  L.sfilt = (int32_t*)(base + p.off[k++]);
  L.decon = (int32_t*)(base + p.off[k++]);
  L.step = (int32_t*)(base + p.off[k++]);
  L.cur = (double*)(base + p.off[k++]);
  L.sep = L.cur + NCUR;
  L.lm = (double*)(base + p.off[k++]);
  L.lmsc = L.lm + 4 * NL;
  L.lmd = nullptr; k++;
  L.dpre = (int32_t*)(base + p.off[k++]);
  L.rpre = (int32_t*)(base + p.off[k++]);
  L.raw = (double*)(base + p.off[k++]);
  L.safe = (double*)(base + p.off[k++]);
  L.wold = (double*)(base + p.off[k++]);
  L.wnew = (double*)(base + p.off[k++]);
  L.emask = (uint64_t*)(base + p.off[k++]);
  L.ecs = (double*)(base + p.off[k++]);
  L.ex = (double*)(base + p.off[k++]);
  L.ey = (double*)(base + p.off[k++]);
  L.ccnt = (int32_t*)(base + p.off[k++]);
  L.mpre = (uint64_t*)(base + p.off[k++]);
  L.mpost = L.mpre + 4;
  L.mt = (uint32_t*)(base + p.off[k++]);
  L.scen = (double*)(base + p.off[k++]);
  L.scratch = (double*)(base + p.off[k++]);
  L.feat = (double*)(base + p.off[k++]);
  L.egooff = (double*)(base + p.off[k++]);
  L.dpair = (double*)(base + p.off[k++]);
  L.stage = (float*)(base + p.off[k++]);
  L.fval = nullptr; L.aa = nullptr; L.aa2 = nullptr; L.vpair = nullptr; L.inr = nullptr;
  L.mtn = nullptr;
  L.info = L.dpair;
  L.lean = false;
  L.dep0 = L.dep1 = L.tmr = nullptr;
  L.ith = L.pth = L.psp = L.trig1 = nullptr;
  return L;
}

enum { C_CR = 0, C_SLOPED, C_STAIR, C_RAT, C_RSC, C_GHE, C_GSE, C_MDT, C_SEP, C_ENG, C_FILT, C_SINT };

// ----------------------------------------------------------------------------------
// Wave-cooperative MT19937 (numpy legacy stream); all lanes run the same scalar sequence.
// ----------------------------------------------------------------------------------
// WSYNC: the generator is run by one wave of a larger workgroup (the workgroup-per-env
// kernel's reset): its refill synchronises that wave only.
template <int LPE, bool WSYNC = false>
struct WaveRng {
  uint32_t* key;
  int pos;
  __device__ __forceinline__ void sync() {
    esync<(WSYNC ? WAVE : LPE)>();
  }
  __device__ __forceinline__ void gen() {
    // chunks of C <= 64 lanes: phase B's element i reads the NEW key[i - 227], so a chunk
    // must not span more than 227 elements (the workgroup kernel's 256 lanes would)
    constexpr int C = LPE < 64 ? LPE : 64;
    const int lane = threadIdx.x & (LPE - 1);
    const bool act = lane < C;
    // phase A: i in [0, 227) reads old key[i], key[i+1], key[i+397]
    for (int base = 0; base < MT_N - MT_M; base += C) {
      int i = base + lane;
      uint32_t v = 0;
      if (act && i < MT_N - MT_M) v = mt_twist1(key[i], key[i + 1], key[i + MT_M]);
      sync();
      if (act && i < MT_N - MT_M) key[i] = v;
      sync();
    }
    // phases B, C: i in [227, 623) reads new key[i-227]
    for (int base = MT_N - MT_M; base < MT_N - 1; base += C) {
      int i = base + lane;
      uint32_t v = 0;
      if (act && i < MT_N - 1) v = mt_twist1(key[i], key[i + 1], key[i + (MT_M - MT_N)]);
      sync();
      if (act && i < MT_N - 1) key[i] = v;
      sync();
    }
    if (lane == 0) key[MT_N - 1] = mt_twist1(key[MT_N - 1], key[0], key[MT_M - 1]);
    sync();
    pos = 0;
  }
  __device__ __forceinline__ uint32_t next32() {
    if (pos >= MT_N) gen();
    uint32_t y = key[pos];
    pos++;
    return mt_temper(y);
  }
  __device__ __forceinline__ bool exhausted() const { return false; }
  __device__ __forceinline__ double next_double() {
    uint32_t a = next32() >> 5;
    uint32_t b = next32() >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
  __device__ __forceinline__ double uniform(double lo, double hi) {
    double range = hi - lo;
    return lo + range * next_double();
  }
};

// ----------------------------------------------------------------------------------
// HJ grid interpolation (float32; semantics of oracle/hj_grid.py)
// ----------------------------------------------------------------------------------
// Every dimension is computed without an early exit and the decision taken once at the end:
// the table's per-dimension constants then load together instead of one scalar round trip per
// dimension behind each exit (the latency-bound agent wave runs this in the filter).
// The grid coordinate y / sp (y = s - lo in float32): the IEEE division, or -- where the upload check
// found them equal for every float32 y the lookups can meet -- q = y r, q + (y - q sp) r with
// r = 1 / sp (Markstein's correction, two FMAs instead of the ~10-instruction division sequence).
__host__ __device__ __forceinline__ float grid_pos(float y, float sp, float rsp, int mdiv) {
  if (!mdiv) return y / sp;
  const float q = y * rsp;
  const float r = fmaf(-q, sp, y);
  return fmaf(r, rsp, q);
}

template <int ND>
__device__ __forceinline__ bool grid_cell(const TableDev& T, const double* s, int& cell, float* w) {
  float lo[ND], sp[ND], rs[ND];
  int nn[ND], per[ND], cs[ND], md[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    lo[d] = T.lo[d]; sp[d] = T.sp[d]; nn[d] = T.n[d]; per[d] = T.periodic[d]; cs[d] = T.cstride[d];
    rs[d] = T.rsp[d]; md[d] = T.mdiv[d];
  }
  float wl[ND], wh[ND];
  int il[ND];
  bool ok = true;
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    const float sd = (float)s[d];
    float p = grid_pos(sd - lo[d], sp[d], rs[d], md[d]);
    ok = ok && (p == p) && !(fabsf(p) > 1.0e9f);   // NaN / runaway coordinate: outside
    if (!ok) p = 0.0f;                              // keeps the index math finite (result unused)
    const int n = nn[d];
    const float fl = floorf(p);
    int f = (int)fl;
    if (per[d]) {
      wh[d] = p - (float)f;
      int a = f % n;
      if (a < 0) a += n;
      il[d] = a;
    } else {
      ok = ok && !(p < 0.0f || p > (float)(n - 1));
      if (f > n - 2) f = n - 2;
      wh[d] = p - (float)f;
      il[d] = f;
    }
    wl[d] = 1.0f - wh[d];
  }
  if (!ok) return false;
  int c0 = 0;
#pragma unroll
  for (int d = 0; d < ND; ++d) c0 += il[d] * cs[d];
  cell = c0;
#pragma unroll
  for (int c = 0; c < (1 << ND); ++c) {
    float ww = 0.0f;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      const int bit = (c >> (ND - 1 - d)) & 1;
      const float wd = bit ? wh[d] : wl[d];
      ww = (d == 0) ? wd : ww * wd;
    }
    w[c] = ww;
  }
  return true;
}

// One env's chain of separation shifts (Lds::sep): node values are the uploaded ones minus
// each shift in turn, float64 subtraction rounded to float32 (`values_hj -= shift`,
// safety_filter.py:173, a float32 array minus a numpy float64 scalar).
struct SepChain {
  const double* sh;   // shifts in application order: [0, KSEP) in the record (LDS) ...
  int n;
  const double* shx;  // ... the rest in the env's HBM overflow row (StateDev::sepx)
  __device__ __forceinline__ float apply(float v) const {
    const int n0 = n < KSEP ? n : KSEP;
    for (int k = 0; k < n0; ++k) v = (float)((double)v - sh[k]);
    for (int k = KSEP; k < n; ++k) v = (float)((double)v - ((const GAS double*)shx)[k - KSEP]);
    return v;
  }
};
__device__ __forceinline__ SepChain sep_chain(const double* sep, const StateDev& sd, int env) {
  SepChain c;
  c.n = (int)sep[0];
  c.sh = sep + 2;
  c.shx = sd.sepx ? sd.sepx + (size_t)env * sd.sepx_cap : nullptr;
  return c;
}

template <int ND>
__device__ __forceinline__ bool interp_value(const TableDev& T, const double* s, float& out,
                                             SepChain sc = SepChain{nullptr, 0, nullptr}) {
  int cell;
  float w[1 << ND];
  if (!grid_cell<ND>(T, s, cell, w)) return false;
#ifdef LSM_XP_VALHOT   // diagnostic bound only (wrong values): every lookup in a 256 KB hot region
  cell &= 4095;
#endif
  const GAS f32x4* c4 = (const GAS f32x4*)(gptr(T.cells) + (size_t)cell * (1 << ND));
  float v[1 << ND];
#pragma unroll
  for (int q = 0; q < (1 << ND) / 4; ++q) {
    const f32x4 x = c4[q];
    v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
  }
  if (sc.n > 0) {
#pragma unroll
    for (int c = 0; c < (1 << ND); ++c) v[c] = sc.apply(v[c]);
  }
  float acc = 0.0f;
#pragma unroll
  for (int c = 0; c < (1 << ND); ++c) acc = acc + w[c] * v[c];
  out = acc;
  return !(acc != acc);
}

template <int ND>
__device__ __forceinline__ void interp_grad(const TableDev& T, const double* s, float* g) {
  int cell;
  float w[1 << ND];
  for (int d = 0; d < ND; ++d) g[d] = 0.0f;
  if (!grid_cell<ND>(T, s, cell, w)) {
    for (int d = 0; d < ND; ++d) g[d] = __builtin_nanf("");
    return;
  }
#ifdef LSM_XP_GRADHOT   // diagnostic bound only (wrong values)
  cell &= 4095;
#endif
  const GAS f32x4* gc = (const GAS f32x4*)gptr(T.gcells) + (size_t)cell * (1 << ND) * T.gw;
#pragma unroll
  for (int c = 0; c < (1 << ND); ++c) {
    const f32x4 a = gc[c * T.gw];
    float gv[8] = {a.x, a.y, a.z, a.w, 0.f, 0.f, 0.f, 0.f};
    if (ND > 4) {
      const f32x4 b = gc[c * T.gw + 1];
      gv[4] = b.x; gv[5] = b.y; gv[6] = b.z; gv[7] = b.w;
    }
#pragma unroll
    for (int d = 0; d < ND; ++d) g[d] = g[d] + w[c] * gv[d];
  }
}

// Bounds of the interpolated value at s: the (widened) min / max of the block containing
// its cell. Same in-range decision and cell index as grid_cell(); false = out of the grid
// (the lookup is +inf, no load).
template <int ND>
__device__ __forceinline__ bool value_bounds(const TableDev& T, const double* s, float2& b,
                                             SepChain sc = SepChain{nullptr, 0, nullptr}) {
  int blk = 0;
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    float sd = (float)s[d];
    float p = grid_pos(sd - T.lo[d], T.sp[d], T.rsp[d], T.mdiv[d]);
    if (!(p == p) || fabsf(p) > 1.0e9f) return false;
    const int n = T.n[d];
    int f = (int)floorf(p);
    if (T.periodic[d]) {
      f = f % n;
      if (f < 0) f += n;
    } else {
      if (p < 0.0f || p > (float)(n - 1)) return false;
      if (f > n - 2) f = n - 2;
    }
    blk += (f >> T.bshift) * T.bstride[d];
  }
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const f32x2 x = *((const GAS f32x2*)gptr(T.bnd) + blk);
  b = make_float2(x.x, x.y);
  if (sc.n > 0) {
    // the shift chain is monotone, so the shifted corners stay within the shifted bounds;
    // widen again for the interpolation error at the shifted magnitude (bounds_kernel)
    const float lo = sc.apply(b.x), hi = sc.apply(b.y);
    const float m = 4.0e-6f * fmaxf(fabsf(lo), fabsf(hi));
    b = make_float2(lo - m, hi + m);
  }
  return true;
}

#if LSM_HOST_PART
// One thread per bounds block: min / max over the nodes its cells interpolate (cells
// [b B, (b + 1) B) per dim -> nodes [b B, (b + 1) B] clipped, wrapped on periodic dims),
// widened by 4e-6 max|v|: the fp32 sum of 2^d weighted corners stays within ~20 ulp of
// max|v| of the exact convex combination, so an interpolated value never leaves the bounds.
__global__ void bounds_kernel(const float* values, float2* bnd, TableDev T, int nblocks) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const int B = 1 << T.bshift;
  int lo[5], cnt[5];
  int rem = b;
  for (int d = T.ndim - 1; d >= 0; --d) {
    const int ncell = T.periodic[d] ? T.n[d] : T.n[d] - 1;
    const int nb = (ncell + B - 1) / B;
    const int bd = rem % nb;
    rem /= nb;
    lo[d] = bd * B;
    const int hi_cell = min(lo[d] + B, ncell);   // cells [lo, hi_cell)
    cnt[d] = hi_cell - lo[d] + 1;                // nodes lo .. hi_cell
  }
  float mn = INFINITY, mx = -INFINITY;
  int idx[5] = {0, 0, 0, 0, 0};
  for (;;) {
    int64_t node = 0;
    for (int d = 0; d < T.ndim; ++d) {
      int i = lo[d] + idx[d];
      if (T.periodic[d] && i >= T.n[d]) i -= T.n[d];
      node = node * T.n[d] + i;
    }
    const float v = values[node];
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
    int d = T.ndim - 1;
    while (d >= 0 && ++idx[d] == cnt[d]) idx[d--] = 0;
    if (d < 0) break;
  }
  const float m = 4.0e-6f * fmaxf(fabsf(mn), fabsf(mx));
  bnd[b] = make_float2(mn - m, mx + m);
}
#endif

#if LSM_HOST_PART
// grid_pos's reciprocal path against the division for every float32 y in [-neg, pos] (bit patterns
// 0 .. pos_bits and the sign-flipped 0 .. neg_bits): bad = 1 on any difference (NaN == NaN).
__global__ void mdiv_check_kernel(float sp, float rsp, uint32_t pos_bits, uint32_t neg_bits, int* bad) {
  const uint64_t n = (uint64_t)pos_bits + 1 + (uint64_t)neg_bits + 1;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t b = i <= pos_bits ? (uint32_t)i : 0x80000000u | (uint32_t)(i - pos_bits - 1);
    const float y = __uint_as_float(b);
    const float a = grid_pos(y, sp, rsp, 0), c = grid_pos(y, sp, rsp, 1);
    if (__float_as_uint(a) != __float_as_uint(c) && !(a != a && c != c)) *bad = 1;
  }
}
#endif

#if LSM_HOST_PART
// Expand a node table into the cell-corner layout (one thread per (cell, corner)).
__global__ void expand_cells_kernel(const float* values, const float4* grads, float* cells, float4* gcells,
                                    TableDev T, int64_t n_cells) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int nc = 1 << T.ndim;
  if (t >= n_cells * nc) return;
  const int64_t cell = t / nc;
  const int c = (int)(t - cell * nc);
  int64_t rem = cell, node = 0, nstride = 1;
  int idx[5];
  for (int d = T.ndim - 1; d >= 0; --d) {
    const int ncd = T.periodic[d] ? T.n[d] : T.n[d] - 1;
    idx[d] = (int)(rem % ncd);
    rem /= ncd;
  }
  for (int d = T.ndim - 1; d >= 0; --d) {
    const int bit = (c >> (T.ndim - 1 - d)) & 1;
    int i = idx[d] + bit;
    if (T.periodic[d] && i >= T.n[d]) i -= T.n[d];
    node += (int64_t)i * nstride;
    nstride *= T.n[d];
  }
  cells[t] = values[node];
  if (grads)
    for (int q = 0; q < T.gw; ++q) gcells[t * T.gw + q] = grads[node * T.gw + q];
}
#endif

// ----------------------------------------------------------------------------------
// per-agent helpers
// ----------------------------------------------------------------------------------
__device__ __forceinline__ int goal_index(int reached, int j, int N, int NL) {
  int order = reached * N + j;
  if (order >= NL) order = (reached - 1) * N + j;
  // the reference raises past the last landmark (use_masking=False only); clamp for safety
  int g = (int)(int8_t)order;
  return g < 0 ? 0 : (g >= NL ? NL - 1 : g);
}

// agent j velocity components for a given "post" choice.
// Agent j "inactive" in World.step before the reward update: done, or not departed yet
// (core.py:655, 669, 685, 700-705: `agent.done or not agent.departed`).
__device__ __forceinline__ bool inactive_pre(const Lds& S, int j) {
  return S.dpre[j] || (S.dep0 && !S.dep0[j]);
}

// freeze_agent (navigation_graph_safe.py:1091-1099) runs when an agent BECOMES done
// (update_reached_goal_and_done, :658-675): this step's transition. An agent done before the step
// already holds its frozen state in the record (zeroed velocity, or -- scenario_circular_config's
// kept-done agents -- the layout's state, which the reference never freezes again).
__device__ __forceinline__ bool froze_now(const Lds& S, int j) {
  return S.dpost[j] && !S.dpre[j];
}

template <int DYN>
__device__ __forceinline__ void agent_vel(const Lds& S, int N, int j, bool post, double& vx, double& vy) {
  const bool frozen = post && froze_now(S, j);
  if (DYN == 1 && post && S.psp) {   // departures: the post state carries departure / freezes
    const double th = S.pth[j], sp = S.psp[j];
    vx = sp * cos(th);
    vy = sp * sin(th);
    return;
  }
  if (DYN == 0) {
    vx = frozen ? 0.0 : S.ps[2 * N + j];
    vy = frozen ? 0.0 : S.ps[3 * N + j];
  } else {
    const double th = S.ps[2 * N + j];
    const double sp = frozen ? 0.0 : S.ps[3 * N + j];
    vx = sp * cos(th);
    vy = sp * sin(th);
  }
}

template <int DYN>
__device__ __forceinline__ double agent_speed(const Lds& S, int N, int j, bool post) {
  const bool frozen = post && froze_now(S, j);
  if (DYN == 1 && post && S.psp) return S.psp[j];
  if (DYN == 0) {
    const double vx = frozen ? 0.0 : S.ps[2 * N + j];
    const double vy = frozen ? 0.0 : S.ps[3 * N + j];
    return sqrt(vx * vx + vy * vy);
  }
  return frozen ? 0.0 : S.ps[3 * N + j];
}

// evaluate_agent_goal_reached (navigation_graph_safe.py:606-656) for goal gi, given the
// agent's heading th, speed spd and he = direction_alignment_error(th, goal heading).
template <int DYN>
__device__ __forceinline__ bool goal_reached_at(const Lds& S, int N, int NL, int i, int gi, double spd,
                                                double he) {
  const double gx = S.lm[gi], gy = S.lm[NL + gi], gs = S.lm[3 * NL + gi];
  const double px = S.ps[i], py = S.ps[N + i];
  const double dist = plain_norm2(px - gx, py - gy);
  const double verr = fabs(spd - gs);
  const double mdt = S.cur[C_MDT], ghe = S.cur[C_GHE], gse = S.cur[C_GSE];
  bool cond;
  if (DYN == 0) {
    const double d2 = blas_norm2(px - gx, py - gy);
    if (d2 > mdt) {
      cond = he < ghe;
    } else if (gs > 0.2) {
      cond = he < ghe;
    } else {
      const double sa = np_clip(1 - gs / 0.2, 0, 1);
      const double tc = 0.5 * sa + ghe * (1 - sa);
      const double da = np_clip(1 - d2 / mdt, 0, 1);
      const double tca = tc * da + ghe * (1 - da);
      cond = he < tca;
    }
  } else {
    cond = he < ghe;
  }
  return dist < mdt && cond && verr < gse;
}

// double_integrator_velocity_error_from_magnetic_field_reference (utils.py:276-349).
// The 50-segment Biot-Savart sum is split over G lanes per agent (segments g, g+G, ...);
// the G partial sums are combined in lane order (float64; ulp-level vs the reference's
// sequential sum, reward tolerance). Two halves: magnetic_partials_wave (all lanes of an env's
// wave: the segment sums into part[0, 2 LPE)) and magnetic_penalty_agent (one lane per agent:
// the sums combined, the reference heading, the penalty), so that the team kernel runs the
// second half once for its G envs in the agent wave.
template <int LPE>
__device__ __forceinline__ int mag_lanes_per_agent(int N) {
  int G = 1;
  while (G * 2 * N <= LPE) G *= 2;
  return G;
}

// The 50 segment constants (KParams::mag_c then mag_s, 100 contiguous doubles) into an env
// wave's LDS table: two 8-B loads per lane issued together, one memory round trip. The segment
// loop used to load mag_c[k] / mag_s[k] from KParams inside each iteration: 7 dependent round
// trips per lane at N = 8.
template <int LPE>
__device__ __forceinline__ void mag_table_issue(const KParams& P, double (&r)[2]) {
  const int lane = threadIdx.x & (LPE - 1);
  const GAS double* src = (const GAS double*)gptr(P.mag_c);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = lane + q * LPE;
    r[q] = src[k < 100 ? k : 0];
  }
}
template <int LPE>
__device__ __forceinline__ void mag_table_store(const double (&r)[2], double* tab) {
  const int lane = threadIdx.x & (LPE - 1);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = lane + q * LPE;
    if (k < 100) tab[k] = r[q];
  }
}

// tab: the env's staged constants (mag_table_store; cos at [k], sin at [50 + k]), or nullptr to
// read KParams directly (one-wave and workgroup kernels). The goal heading's cos / sin are the
// episode's cached ones (Lds::lmsc: the same functions of the same value, bit for bit).
template <int LPE, int NT>
__device__ __forceinline__ void magnetic_partials_wave(const KParams& P, const Lds& S, double* part,
                                                       const double* tab = nullptr) {
  const int lane = threadIdx.x & (LPE - 1);
  constexpr int DYN = 0;
  LSM_DIMS;
  const int G = mag_lanes_per_agent<LPE>(N);
  const int a = lane / G, g = lane - a * G;
  const bool act = a < N;
  const int ai = act ? a : 0;
  const int gi = goal_index(S.rpre[ai], ai, N, NL);
  const double gx = S.lm[gi], gy = S.lm[NL + gi];
  const double ch = S.lmsc[NL + gi], sh = S.lmsc[gi];
  const double px = S.ps[ai], py = S.ps[N + ai];
  double rpx, rpy;
  blas_rot(ch, sh, px - gx, py - gy, rpx, rpy);
  const double radius = 2 * S.cur[C_MDT];
  const double* mc = tab ? tab : P.mag_c;
  const double* ms = tab ? tab + 50 : P.mag_s;
  double m0 = 0.0, m1 = 0.0;
  if (act && !(fabs(rpx) < 1e-6)) {
    const double x = 0.5 * rpx, y = rpy;
    const double nr = -radius;
    // segments k and 50 - k (angles 2 pi k / 50 and 2 pi - 2 pi k / 50) contribute the same term:
    // with the segment at (0, -R cos, -R sin) and tangent (0, R sin, -R cos), c0 = R^2 sin^2 +
    // R cos (y + R cos), c1 = -R cos x and |r|^2 = x^2 + (y + R cos)^2 + R^2 sin^2 are even in sin.
    // So k = 1 .. 24 count twice and 0, 25 once: 26 terms instead of 50 (the mirrored cos / sin
    // values differ from these in the last bit only; ulp-level, like the rest of this sum).
    // 28.47 -> 27.95 us per step at config 2 (profiles/r05_s27_ab_c2.txt)
    for (int k = g; k <= 25; k += G) {
      const double wk = (k == 0 || k == 25) ? 1.0 : 2.0;
      const double Ly = nr * mc[k], Lz = nr * ms[k];
      const double dLy = radius * ms[k], dLz = nr * mc[k];
      const double r0 = x - 0.0, r1 = y - Ly, r2 = 0.0 - Lz;
      const double c0 = dLy * r2 - dLz * r1;
      const double c1 = dLz * r0 - 0.0 * r2;
      // 1 / |r|**3 from v_rsq_f64 (~2^-23 relative) and two Newton steps (~1 ulp), then two
      // multiplies: a few ulp per term, no division (|r| > 0: r0 = x != 0). Round 3 took sqrt, rn**3
      // and two float64 divisions: 33.08 vs 31.82 us per step at config 2 (r04_v2_ab_c2_mag.txt);
      // one Newton step measured no faster (r05_s27_ab_c2.txt)
      const double sq = fma(r2, r2, fma(r1, r1, r0 * r0));
      double ri = __builtin_amdgcn_rsq(sq);
      ri = fma(0.5 * ri, fma(-sq * ri, ri, 1.0), ri);
      ri = fma(0.5 * ri, fma(-sq * ri, ri, 1.0), ri);
      const double i3 = ri * ri * ri;
      m0 = fma(wk * c0, i3, m0);
      m1 = fma(wk * c1, i3, m1);
    }
  }
  part[lane] = m0;
  part[LPE + lane] = m1;
}

// agent i's penalty from the partial sums of its env's wave (LPE: that wave's width)
template <int LPE, int NT>
__device__ __forceinline__ double magnetic_penalty_agent(const KParams& P, const Lds& S, const double* part,
                                                         int i) {
  constexpr int DYN = 0;
  LSM_DIMS;
  const int G = mag_lanes_per_agent<LPE>(N);
  double pen = 0.0;
  {
    const int gj = goal_index(S.rpre[i], i, N, NL);
    const double gxx = S.lm[gj], gyy = S.lm[NL + gj], gs = S.lm[3 * NL + gj];
    const double c = S.lmsc[NL + gj], s = S.lmsc[gj];   // cos / sin of the goal heading (episode cache)
    double qx, qy, rvx, rvy;
    blas_rot(c, s, S.ps[i] - gxx, S.ps[N + i] - gyy, qx, qy);
    const double dist = blas_norm2(qx, qy);
    blas_rot(c, s, S.ps[2 * N + i] - 0.0, S.ps[3 * N + i] - 0.0, rvx, rvy);
    // cos / sin of atan2(y, x) as x / |(x, y)|, y / |(x, y)| (ulp-level vs the reference's
    // np.cos(np.arctan2(..)), inside the reward tolerance); the origin keeps atan2's signed zeros
    double ch = 1.0, sh = 0.0;
    if (!(fabs(qx) < 1e-6)) {
      double s0 = 0.0, s1 = 0.0;
      for (int q = 0; q < G; ++q) {
        s0 += part[i * G + q];
        s1 += part[LPE + i * G + q];
      }
      s0 = s0 / 0.5;
      const double hn = sqrt(s0 * s0 + s1 * s1);
      if (hn > 0.0 && hn < INFINITY) {
        ch = s0 / hn;
        sh = s1 / hn;
      } else {
        const double href = atan2(s1, s0);
        ch = cos(href);
        sh = sin(href);
      }
    }
    double ref_speed = py_max(gs, 0.1);
    const double dr = np_clip(dist / 1.5, 0, 1);
    ref_speed = ref_speed * (1 - dr) + 1.0 * dr;
    const double rfx = ref_speed * ch, rfy = ref_speed * sh;
    const double err = blas_norm2(rvx - rfx, rvy - rfy);
    const double cp = (dist > 0.0 && dist < INFINITY) ? qx / dist : cos(atan2(qy, qx));
    if (cp < P.cos_pi6) {
      pen = err;
    } else {
      const double ar = np_clip((cp - P.cos_pi6) / (1 - P.cos_pi6), 0, 1);
      pen = err * (1 - ar) + dist * ar;
    }
  }
  return pen;
}

// Called by ALL lanes; returns the penalty in lanes lane < N (agent = lane), 0 elsewhere.
template <int LPE, int NT>
__device__ __forceinline__ double magnetic_penalty_wave(const KParams& P, Lds& S, double* part) {
  const int lane = threadIdx.x & (LPE - 1);
  constexpr int DYN = 0;
  LSM_DIMS;
  magnetic_partials_wave<LPE, NT>(P, S, part);
  esync<LPE>();
  const double pen = lane < N ? magnetic_penalty_agent<LPE, NT>(P, S, part, lane) : 0.0;
  esync<LPE>();
  return pen;
}

__device__ __forceinline__ double seqdot4(const double* a, const double* b) {
  double acc = 0.0;
  for (int k = 0; k < 4; ++k) acc = acc + a[k] * b[k];
  return acc;
}

// ----------------------------------------------------------------------------------
// safety filter for one ego (lane), after pair scratch is filled
// ----------------------------------------------------------------------------------
template <int DYN>
__device__ __forceinline__ void rel_state(const Lds& S, int N, int e, int o, double* rel) {
  const double ex = S.ps[e], ey = S.ps[N + e], e2 = S.ps[2 * N + e], e3 = S.ps[3 * N + e];
  const double ox = S.ps[o], oy = S.ps[N + o], o2 = S.ps[2 * N + o], o3 = S.ps[3 * N + o];
  if (DYN == 0) {
    rel[0] = ex - ox; rel[1] = ey - oy; rel[2] = e2 - o2; rel[3] = e3 - o3;
  } else {
    // |d| cos / sin(atan2(dy, dx) - th_e) (safety_filter.py:277-284) as the rotation of d
    // into the ego frame (ulp-level in float64; the grid lookup rounds to float32)
    const double c = S.ecs[e], sn = S.ecs[N + e];
    const double dx = ox - ex, dy = oy - ey;
    rel[0] = dx * c + dy * sn;
    rel[1] = dy * c - dx * sn;
    rel[2] = o2 - e2;
    rel[3] = e3;
    rel[4] = o3;
  }
}

template <int DYN, int NT>
__device__ __forceinline__ void filter_apply(const KParams& P, const Lds& S, int i, int jv, float vmin,
                                             uint8_t& filtered, double& u0, double& u1);

// The deconflicting choice of ego i from its pair words (safety_filter.py:395-423): jv = argmin of
// the HJ value over the other active agents (dec), and whether the filter then applies (the
// nearest agent within the coordination range, the value lookup in range). Returns false when
// there is no other active agent.
template <int DYN, int NT>
__device__ __forceinline__ bool filter_select(const KParams& P, const Lds& S, int i, int& jv_out, float& vmin_out,
                                              bool& apply) {
  LSM_DIMS;
  int jd = -1, jv = -1;
  double dmin = 0.0;
  float vmin = 0.0f;
  bool in_jv = false;
  if (NT > 0) {
    // compile-time N: every pair word of this ego read up front (one LDS round trip for all),
    // then a branch-free argmin -- first occurrence on ties, np.argmin's rule
    constexpr int M = NT > 0 ? NT : 1;
    double dv[M];
    float vv[M];
    bool ac[M], in[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      ac[j] = S.dpre[j] == 0;
      dv[j] = S.dpair[j * N + i];   // pair matrices are [other][ego]: the lanes of an agent
      vv[j] = (float)S.vpair[j * N + i];   // wave read consecutive words
      in[j] = S.inr[j * N + i] != 0;
    }
    if (S.dep0) {   // RealisticScenario layouts only (uniform): not yet departed = inactive
#pragma unroll
      for (int j = 0; j < M; ++j) ac[j] = ac[j] && S.dep0[j] != 0;
    }
#pragma unroll
    for (int j = 0; j < M; ++j) {   // selects, no per-pair branches
      const bool a = ac[j] && j != i;
      const bool bd = a && (jd < 0 || dv[j] < dmin);
      const bool bv = a && (jv < 0 || vv[j] < vmin);
      jd = bd ? j : jd;
      dmin = bd ? dv[j] : dmin;
      jv = bv ? j : jv;
      vmin = bv ? vv[j] : vmin;
      in_jv = bv ? in[j] : in_jv;
    }
  } else {
    for (int j = 0; j < N; ++j) {
      if (j == i || inactive_pre(S, j)) continue;
      const double d = S.dpair[j * N + i];
      const float v = (float)S.vpair[j * N + i];
      if (jd < 0 || d < dmin) { jd = j; dmin = d; }
      if (jv < 0 || v < vmin) { jv = j; vmin = v; }
    }
    if (jv >= 0) in_jv = S.inr[jv * N + i] != 0;
  }
  jv_out = jv;
  vmin_out = vmin;
  apply = jd >= 0 && !(dmin > P.coord_range) && in_jv;
  (void)E; (void)F;
  return jd >= 0;
}

template <int DYN, int NT>
__device__ __forceinline__ void filter_ego(const KParams& P, Lds& S, int i, uint8_t& filtered, int& dec,
                                  double& u0, double& u1) {
  LSM_DIMS;
  u0 = S.raw[i];
  u1 = S.raw[N + i];
  filtered = 0;
  dec = -1;
  int jv;
  float vmin;
  bool apply;
  if (!filter_select<DYN, NT>(P, S, i, jv, vmin, apply)) return;   // no other active agent
  dec = jv;
  if (apply) filter_apply<DYN, NT>(P, S, i, jv, vmin, filtered, u0, u1);
  (void)E; (void)F;
}

// Team kernel: the filter split over its phases. Phase A (ego i's env wave, whose memory latency
// the other waves of the SIMD hide) selects the deconflicting agent and interpolates the HJ
// gradient there; phase B (the latency-bound agent wave) reads the slot and does the QP only.
// Slot of ego i: 8 words right after the pair matrices (U2, or U1 in the lean layout; free space
// there until phase D / E -- lds_plan): g[0..4], V, jv, status (0 ego inactive, 1 no other
// active agent, 2 unfiltered with dec = jv, 3 filter applies).
__device__ __forceinline__ float* filter_slot(const Lds& S, int N, int i) {
  return (float*)((uint8_t*)S.inr + align16_((size_t)N * N)) + 8 * i;
}

template <int DYN, int NT>
__device__ __forceinline__ void filter_qp(const KParams& P, const Lds& S, int i, int jv, float vmin,
                                          const double* rel, const float* g, uint8_t& filtered, double& u0,
                                          double& u1);

template <int DYN, int NT>
__device__ __forceinline__ void filter_prep(const KParams& P, Lds& S, int i) {
  LSM_DIMS;
  float* f = filter_slot(S, N, i);
  int st = 0, jv = -1;
  float vmin = 0.0f;
  float g[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  if (!inactive_pre(S, i)) {
    bool apply;
    if (!filter_select<DYN, NT>(P, S, i, jv, vmin, apply)) {
      st = 1;
    } else if (!apply) {
      st = 2;
    } else {
      st = 3;
      double rel[5];
      rel_state<DYN>(S, N, i, jv, rel);
      if (DYN == 0) interp_grad<4>(P.val, rel, g); else interp_grad<5>(P.val, rel, g);
    }
  }
  float4* f4 = (float4*)f;
  f4[0] = make_float4(g[0], g[1], g[2], g[3]);
  f4[1] = make_float4(g[4], vmin, __int_as_float(jv), __int_as_float(st));
}

// filter_prep of the double integrator's team kernel at N = 8 on all 64 lanes: lane 8 e + k is
// ego e's candidate k. The argmins are butterflies over the 8 lanes of an ego (the lower index wins
// ties, np.argmin's first occurrence, as filter_select); the gradient lookup of an applying ego runs
// one component per lane (lanes k < 4, 16 corner loads of 4 B each) with interp_grad's weights and
// summation order; lanes k write word k of the ego's slot. Same slots as filter_prep on 8 lanes,
// about a third fewer vector instructions for the wave.
template <int NT>
__device__ __forceinline__ void filter_prep_oct(const KParams& P, Lds& S, GAS unsigned long long* stp = nullptr) {
  constexpr int DYN = 0;
  static_assert(NT == 8, "8 egos x 8 candidate lanes");
  LSM_DIMS;
  const int lane = threadIdx.x & 63;
  const int e = lane >> 3, k = lane & 7;
  const bool eact = !inactive_pre(S, e);
  const bool kact = k != e && !inactive_pre(S, k);
  // candidate k of ego e ([other][ego] pair matrices; the team kernel's pair loop stores squared
  // distances: the nearest agent's only use is the coordination-range test, sqrt is monotone)
  double d = S.dpair[k * N + e];
  float v = (float)S.vpair[k * N + e];
  bool in = S.inr[k * N + e] != 0;
  int jd = kact ? k : 64, jv = kact ? k : 64;   // 64: no candidate
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) {
    const double od = __shfl_xor(d, m);
    const float ov = __shfl_xor(v, m);
    const int ojd = __shfl_xor(jd, m), ojv = __shfl_xor(jv, m);
    const bool oin = __shfl_xor((int)in, m) != 0;
    // take the other lane's candidate if it exists and is smaller, or equal with a lower index
    const bool td = ojd < 64 && (jd == 64 || od < d || (od == d && ojd < jd));
    const bool tv = ojv < 64 && (jv == 64 || ov < v || (ov == v && ojv < jv));
    d = td ? od : d;
    jd = td ? ojd : jd;
    v = tv ? ov : v;
    jv = tv ? ojv : jv;
    in = tv ? oin : in;
  }
  // every lane of the ego holds the same choice: the butterfly is order-independent for the values
  // it can meet (vpair is never NaN -- a NaN interpolation is stored as +inf, the reference's
  // np.isnan -> inf -- and ties go to the lower index as np.argmin's first occurrence); only NaN
  // positions could make lanes disagree, so lane 8 e's result is broadcast to its ego's lanes and
  // the slot words (written one per lane) always come from one choice
  {
    const int src = lane & ~7;
    d = __shfl(d, src);
    jd = __shfl(jd, src);
    v = __shfl(v, src);
    jv = __shfl(jv, src);
    in = __shfl((int)in, src) != 0;
  }
#ifdef LSM_STAMPS
  if (lane == 0 && stp) stp[32] = __builtin_amdgcn_s_memtime();
#endif
  int st = 0;
  if (eact) st = jd == 64 ? 1 : ((!(d > P.coord_range_s) && in) ? 3 : 2);
  if (st < 2) jv = -1;
  const float vmin = st >= 2 ? v : 0.0f;
  float gk = 0.0f;   // gradient component k (k < 4)
  if (st == 3) {
    double rel[5];
    rel_state<DYN>(S, N, e, jv, rel);
    int cell;
    float w[16];
    if (!grid_cell<4>(P.val, rel, cell, w)) {
      gk = __builtin_nanf("");
    } else if (k < 4) {
      const GAS float* gc = (const GAS float*)(gptr(P.val.gcells) + (size_t)cell * 16) + k;
      float gv[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) gv[c] = gc[4 * c];
#pragma unroll
      for (int c = 0; c < 16; ++c) gk = gk + w[c] * gv[c];
    }
  }
  float word = k < 4 ? gk : (k == 4 ? 0.0f : (k == 5 ? vmin : __int_as_float(k == 6 ? jv : st)));
  filter_slot(S, N, e)[k] = word;
}

// Phase B of the team kernel: filter_agent with the slot filter_prep filled.
template <int DYN, int NT>
__device__ __forceinline__ void filter_agent_slot(const KParams& P, Lds& S, int N, int i, bool filter_on) {
  double u0 = S.raw[i], u1 = S.raw[N + i];
  if (filter_on) {
    const float4* f4 = (const float4*)filter_slot(S, N, i);
    const float4 a = f4[0], b = f4[1];
    const int st = __float_as_int(b.w), jv = __float_as_int(b.z);
    uint8_t fl = 0;
    if (st == 3) {
      double rel[5];
      rel_state<DYN>(S, N, i, jv, rel);
      const float g[5] = {a.x, a.y, a.z, a.w, b.x};
      filter_qp<DYN, NT>(P, S, i, jv, b.y, rel, g, fl, u0, u1);
    }
    S.sfilt[i] = fl;
    S.decon[i] = st >= 2 ? jv : -1;
  }
  S.safe[i] = u0;
  S.safe[N + i] = u1;
  S.adiff[i] = blas_norm2(S.raw[i] - u0, S.raw[N + i] - u1);
}

// The filter for ego i once its deconflicting agent jv (argmin of the HJ value, V = vmin in
// range) is known and the nearest agent is within the coordination range: gradient lookup,
// optimal control (V < eps_hj) or the closed-form CBF-QP, clips (safety_filter.py:264-308,
// 395-433).
template <int DYN, int NT>
__device__ __forceinline__ void filter_qp(const KParams& P, const Lds& S, int i, int jv, float vmin,
                                          const double* rel, const float* g, uint8_t& filtered, double& u0,
                                          double& u1);

template <int DYN, int NT>
__device__ __forceinline__ void filter_apply(const KParams& P, const Lds& S, int i, int jv, float vmin,
                                             uint8_t& filtered, double& u0, double& u1) {
  LSM_DIMS;
  double rel[5];
  rel_state<DYN>(S, N, i, jv, rel);
  float g[5];
  if (DYN == 0) interp_grad<4>(P.val, rel, g); else interp_grad<5>(P.val, rel, g);
  filter_qp<DYN, NT>(P, S, i, jv, vmin, rel, g, filtered, u0, u1);
}

// The filter's control once the HJ gradient g at the relative state rel is known.
template <int DYN, int NT>
__device__ __forceinline__ void filter_qp(const KParams& P, const Lds& S, int i, int jv, float vmin,
                                          const double* rel, const float* g, uint8_t& filtered, double& u0,
                                          double& u1) {
  LSM_DIMS;
  const int ND = (DYN == 0) ? 4 : 5;
  double uref[4] = {S.raw[i], S.raw[N + i], S.raw[jv], S.raw[N + jv]};
  const float V = vmin;
  double u[4];
  bool alias = false;   // infeasible QP returns u_ref itself (safety_filter.py:304-305,373-375)
  if (DYN == 0) {
    if (V < 0.4f) {
      const float dirv[4] = {g[2], g[3], -g[2], -g[3]};
      for (int k = 0; k < 4; ++k) u[k] = (dirv[k] < 0.0f) ? -0.5 : 0.5;
    } else {
      const double a[4] = {(double)g[2], (double)g[3], -(double)g[2], -(double)g[3]};
      const double c0 = (double)(float)rel[2], c1 = (double)(float)rel[3];
      const double gg[4] = {(double)g[0], (double)g[1], (double)g[2], (double)g[3]};
      const double cc[4] = {c0, c1, 0.0, 0.0};
      const double b = seqdot4(gg, cc) + (double)(3.0f * V);
      const double s = seqdot4(a, uref) + b;
      if (s >= 0.0) {
        for (int k = 0; k < 4; ++k) u[k] = uref[k];
      } else {
        double den = 0.0;
        for (int k = 0; k < 4; ++k) den = den + a[k] * a[k] / 1.0;
        if (den == 0.0) {
          alias = true;
          for (int k = 0; k < 4; ++k) u[k] = uref[k];
        } else {
          const double lam = s / den;
          for (int k = 0; k < 4; ++k) u[k] = uref[k] - lam * (a[k] / 1.0);
        }
      }
    }
    const double axmax = (rel[2] < P.di_thr_xmax) ? P.di_axmax : 0.0;
    const double axmin = (rel[2] > P.di_thr_xmin) ? P.di_axmin : 0.0;
    u[0] = py_max(py_min(u[0], axmax), axmin);
    const double aymax = (rel[3] < P.di_thr_ymax) ? P.di_aymax : 0.0;
    const double aymin = (rel[3] > P.di_thr_ymin) ? P.di_aymin : 0.0;
    u[1] = py_max(py_min(u[1], aymax), aymin);
  } else {
    const float s0 = (float)rel[0], s1 = (float)rel[1];
    const float d0 = (g[0] * s1 + g[1] * (-s0)) + (-g[2]);
    const float dirv[4] = {d0, g[2], g[3], g[4]};
    bool f32u = false;
    if (V < 0.4f) {
      float lo[4] = {-P.at_box_w, -P.at_box_w, P.at_box_amin, P.at_box_amin};
      float hi[4] = {P.at_box_w, P.at_box_w, P.at_box_amax, P.at_box_amax};
      if (rel[4] >= P.at_vmax) hi[3] = 0.0f;
      else if (rel[4] <= P.at_vmin) lo[3] = 0.0f;
      else if (rel[3] >= P.at_vmax) hi[2] = 0.0f;
      else if (rel[3] <= P.at_vmin) lo[2] = 0.0f;
      for (int k = 0; k < 4; ++k) u[k] = (double)((dirv[k] < 0.0f) ? lo[k] : hi[k]);
      f32u = true;
    } else {
      const float th32 = (float)rel[2];
      const double ol0 = (double)(float)(-rel[3] + rel[4] * (double)cosf(th32));
      const double ol1 = (double)(float)(rel[4] * (double)sinf(th32));
      const double gg[5] = {(double)g[0], (double)g[1], (double)g[2], (double)g[3], (double)g[4]};
      double a[4];
      {
        double acc = 0.0;
        acc = acc + gg[0] * (double)s1;
        acc = acc + gg[1] * (-(double)s0);
        acc = acc + gg[2] * -1.0;
        acc = acc + gg[3] * 0.0;
        acc = acc + gg[4] * 0.0;
        a[0] = acc;
        for (int k = 1; k < 4; ++k) {
          double t = 0.0;
          for (int m = 0; m < 5; ++m) t = t + gg[m] * ((m == k + 1) ? 1.0 : 0.0);
          a[k] = t;
        }
      }
      double b = 0.0;
      b = b + gg[0] * ol0;
      b = b + gg[1] * ol1;
      b = b + gg[2] * 0.0;
      b = b + gg[3] * 0.0;
      b = b + gg[4] * 0.0;
      b = b + (double)(3.0f * V);
      const double W0[4] = {100.0, 10.0, 10.0, 1.0};
      const double W1[4] = {10.0, 1.0, 100.0, 10.0};
      const double* W = (rel[0] < 0) ? W0 : W1;
      const double s = seqdot4(a, uref) + b;
      if (s >= 0.0) {
        for (int k = 0; k < 4; ++k) u[k] = uref[k];
        u[0] = py_max(py_min(u[0], P.at_wmax), -P.at_wmax);
        u[2] = py_max(py_min(u[2], P.at_wmax), -P.at_wmax);
      } else {
        double den = 0.0;
        for (int k = 0; k < 4; ++k) den = den + a[k] * a[k] / W[k];
        if (den == 0.0) {
          alias = true;
          for (int k = 0; k < 4; ++k) u[k] = uref[k];
        } else {
          const double lam = s / den;
          for (int k = 0; k < 4; ++k) u[k] = uref[k] - lam * (a[k] / W[k]);
          u[0] = py_max(py_min(u[0], P.at_wmax), -P.at_wmax);
          u[2] = py_max(py_min(u[2], P.at_wmax), -P.at_wmax);
        }
      }
    }
    double amax = (rel[3] < P.at_thr_amax) ? P.at_amax : 0.0;
    double amin = (rel[3] > P.at_thr_amin) ? P.at_amin : 0.0;
    u[1] = py_max(py_min(u[1], amax), amin);
    if (f32u) u[1] = (double)(float)u[1];
    amax = (rel[4] < P.at_thr_amax) ? P.at_amax : 0.0;
    amin = (rel[4] > P.at_thr_amin) ? P.at_amin : 0.0;
    u[3] = py_max(py_min(u[3], amax), amin);
    if (f32u) u[3] = (double)(float)u[3];
  }
  if (alias) {
    filtered = 0;
  } else {
    filtered = blas_norm4(u[0] - uref[0], u[1] - uref[1], u[2] - uref[2], u[3] - uref[3]) > 1e-4;
  }
  u0 = u[0];
  u1 = u[1];
  (void)ND; (void)E; (void)F;
}

// ----------------------------------------------------------------------------------
// Outputs: per-ego node features + adjacency with the sequential snapshot rule.
// ego i sees agent j "post" (after its reward update) iff j <= i.
// ----------------------------------------------------------------------------------
// Airtaxi node features (utils.py:139-200, relative to the ego frame). Headings enter only
// through sin / cos, so the per-agent trig table built once per emission (trig_table_at:
// [0] cos th, [1] sin th, [2] vx, [3] vy unfrozen, per agent) and the cached landmark
// sin / cos replace the per-(ego, entity) sin / cos of differences by the angle-difference
// identities (fp32 outputs; ulp-level vs sin(a - b) in float64).
template <int DYN, int NT>
__device__ __forceinline__ void node_features(const KParams& P, const Lds& S, int e, int k, float* f) {
  LSM_DIMS;
  const double* tc = S.feat;            // cos th [N]
  const double* ts = S.feat + N;        // sin th [N]
  const double* tvx = S.feat + 2 * N;   // unfrozen velocity [N]
  const double* tvy = S.feat + 3 * N;
  // departures: post-update rows (heading / speed after a departure, waiting freeze or done
  // freeze) in trig1; otherwise the post state differs from the pre state only by the done freeze
  const bool dm = DYN == 1 && S.trig1 != nullptr;
  const double* tc1 = dm ? S.trig1 : tc;
  const double* ts1 = dm ? S.trig1 + N : ts;
  const double* tvx1 = dm ? S.trig1 + 2 * N : tvx;
  const double* tvy1 = dm ? S.trig1 + 3 * N : tvy;
  const double pex = S.ps[e], pey = S.ps[N + e];
  const double c = tc1[e], s = ts1[e];
  const bool efz = !dm && froze_now(S, e);     // the ego is seen after its own update
  const double vex = efz ? 0.0 : tvx1[e], vey = efz ? 0.0 : tvy1[e];
  if (k < N) {
    const bool post = k <= e;
    const bool kfz = !dm && post && froze_now(S, k);
    const double vkx = kfz ? 0.0 : (post ? tvx1 : tvx)[k], vky = kfz ? 0.0 : (post ? tvy1 : tvy)[k];
    const double ck = (post ? tc1 : tc)[k], sk = (post ? ts1 : ts)[k];
    const int gi = goal_index(post ? S.rpost[k] : S.rpre[k], k, N, NL);
    double rx, ry, gx, gy;
    blas_rot(c, s, S.ps[k] - pex, S.ps[N + k] - pey, rx, ry);
    const double rs = blas_norm2(vkx - vex, vky - vey);
    blas_rot(c, s, S.lm[gi] - pex, S.lm[NL + gi] - pey, gx, gy);
    const double sg = S.lmsc[gi], cg = S.lmsc[NL + gi];
    f[0] = (float)rx;
    f[1] = (float)ry;
    f[2] = (float)rs;
    f[3] = (float)(sk * c - ck * s);   // sin(th_k - th_e)
    f[4] = (float)(ck * c + sk * s);   // cos(th_k - th_e)
    f[5] = (float)gx;
    f[6] = (float)gy;
    f[7] = (float)(sg * c - cg * s);
    f[8] = (float)(cg * c + sg * s);
    f[9] = (float)S.lm[3 * NL + gi];
    f[10] = 0.0f;
  } else {
    const int l = k - N;
    double rx, ry;
    blas_rot(c, s, S.lm[l] - pex, S.lm[NL + l] - pey, rx, ry);
    const double sl = S.lmsc[l], cl = S.lmsc[NL + l];
    const float sn = (float)(sl * c - cl * s), cs = (float)(cl * c + sl * s);
    f[0] = (float)rx;
    f[1] = (float)ry;
    f[2] = (float)(dm ? S.psp[e] : (efz ? 0.0 : S.ps[3 * N + e]));
    f[3] = sn;
    f[4] = cs;
    f[5] = (float)rx;
    f[6] = (float)ry;
    f[7] = sn;
    f[8] = cs;
    f[9] = (float)S.lm[3 * NL + l];
    f[10] = 1.0f;
  }
}

// per-agent heading trig + unfrozen velocity for node_features<1> (in the DI row area of U2)
template <int LPE, int NT>
__device__ __forceinline__ void trig_table_at(const KParams& P, Lds& S) {
  const int lane = threadIdx.x & (LPE - 1);
  constexpr int DYN = 1;
  LSM_DIMS;
  for (int j = lane; j < N; j += LPE) {
    const double th = S.ps[2 * N + j], sp = S.ps[3 * N + j];
    const double c = cos(th), sn = sin(th);
    S.feat[j] = c;
    S.feat[N + j] = sn;
    S.feat[2 * N + j] = sp * c;
    S.feat[3 * N + j] = sp * sn;
    if (S.trig1) {
      const double th1 = S.pth[j], sp1 = S.psp[j];
      const double c1 = cos(th1), s1 = sin(th1);
      S.trig1[j] = c1;
      S.trig1[N + j] = s1;
      S.trig1[2 * N + j] = sp1 * c1;
      S.trig1[3 * N + j] = sp1 * s1;
    }
  }
}

// Disconnect mask of ego e (navigation_graph_safe.py:976-989) under the sequential snapshot
// rule: agent j is seen after its reward update iff j <= e. Bit r = entity r (agents first,
// landmark l = order * N + agent at N + l). e >= N - 1 gives the end-of-step mask.
__device__ __forceinline__ uint64_t ego_mask(const Lds& S, int N, int L, int e) {
  uint64_t m = 0;
  for (int j = 0; j < N; ++j) {
    const bool post = j <= e;
    if (post ? S.dpost[j] : S.dpre[j]) m |= 1ull << j;
    if (S.dep0 && !(post ? S.dep1[j] : S.dep0[j])) m |= 1ull << j;   // not departed (:979)
    const int rg = post ? S.rpost[j] : S.rpre[j];
    for (int o = 0; o < L; ++o)
      if (rg > o) m |= 1ull << (N + o * N + j);
  }
  return m;
}

// DI node features are (entity row) - (ego offset): rows for agents (pre, post update) and
// landmarks, offsets per ego, built once per step in LDS (utils.py:201-255).
template <int LPE, int NT>
__device__ __forceinline__ void build_rows_di(const KParams& P, Lds& S) {
  const int lane = threadIdx.x & (LPE - 1);
  constexpr int DYN = 0;
  LSM_DIMS;
  const int32_t* dpost = S.dpost;
  const int32_t* rpost = S.rpost;
  for (int t = lane; t < 2 * N + NL; t += LPE) {
    double* r = S.feat + (size_t)t * F;
    if (t < 2 * N) {
      const bool post = t >= N;
      const int k = post ? t - N : t;
      const bool frozen = post && dpost[k] && !S.dpre[k];
      const double vx = frozen ? 0.0 : S.ps[2 * N + k], vy = frozen ? 0.0 : S.ps[3 * N + k];
      const int gi = goal_index(post ? rpost[k] : S.rpre[k], k, N, NL);
      r[0] = S.ps[k]; r[1] = S.ps[N + k]; r[2] = vx; r[3] = vy;
      r[4] = S.lm[gi]; r[5] = S.lm[NL + gi];
      r[6] = S.lmsc[gi]; r[7] = S.lmsc[NL + gi]; r[8] = S.lm[3 * NL + gi]; r[9] = 0.0;
    } else {
      const int l = t - 2 * N;
      r[0] = S.lm[l]; r[1] = S.lm[NL + l]; r[2] = 0.0; r[3] = 0.0;
      r[4] = S.lm[l]; r[5] = S.lm[NL + l];
      r[6] = S.lmsc[l]; r[7] = S.lmsc[NL + l]; r[8] = S.lm[3 * NL + l]; r[9] = 1.0;
    }
  }
  if (lane < N) {
    const int e = lane;
    const bool frozen = froze_now(S, e);
    const double vx = frozen ? 0.0 : S.ps[2 * N + e], vy = frozen ? 0.0 : S.ps[3 * N + e];
    double* o = S.egooff + e * F;
    o[0] = S.ps[e]; o[1] = S.ps[N + e]; o[2] = vx; o[3] = vy; o[4] = S.ps[e]; o[5] = S.ps[N + e];
    o[6] = 0.0; o[7] = 0.0; o[8] = 0.0; o[9] = 0.0;
  }
}

// The thresholded distance table fval: entries (r, c) and float4 groups (c % 4 == 0) of either
// layout. Lean layout (N % 4 == 0, E % 4 == 0): agent rows [N][E], landmark rows' agent columns
// [NL][N], the landmark-landmark block from the episode cache lmd (diagonal 0).
__device__ __forceinline__ float fv_ll(const Lds& S, int NL, int la, int lb) {
  if (la == lb) return 0.0f;
  const int lo = la < lb ? la : lb, hi = la < lb ? lb : la;
  return S.lmd[lo * (2 * NL - lo - 1) / 2 + (hi - lo - 1)];
}
__device__ __forceinline__ float4 fv4(const Lds& S, int N, int NL, int E, int r, int c) {
  if (!S.lean || r < N) return *(const float4*)(S.fval + r * E + c);
  if (c < N) return *(const float4*)(S.fval + N * E + (r - N) * N + c);
  const int la = r - N, lb = c - N;
  return make_float4(fv_ll(S, NL, la, lb), fv_ll(S, NL, la, lb + 1), fv_ll(S, NL, la, lb + 2),
                     fv_ll(S, NL, la, lb + 3));
}
__device__ __forceinline__ float fv1(const Lds& S, int N, int NL, int E, int r, int c) {
  if (!S.lean || r < N) return S.fval[r * E + c];
  if (c < N) return S.fval[N * E + (r - N) * N + c];
  return fv_ll(S, NL, r - N, c - N);
}
// store entry (r, c); the lean layout keeps no landmark-landmark entries
__device__ __forceinline__ void fv_set(Lds& S, int N, int E, int r, int c, float v) {
  if (!S.lean || r < N) S.fval[r * E + c] = v;
  else if (c < N) S.fval[N * E + (r - N) * N + c] = v;
}

// node_obs [N][E][F] and adj [N][E][E] of one env. Node rows are computed per (ego, entity)
// pair by one lane, staged in LDS, and copied out as contiguous float4 when the env block is
// 16-byte aligned; the adjacency is a masked select over the thresholded distance table,
// one float4 (4 columns of one row) per lane-iteration when E % 4 == 0.
// Adjacency of egos [e0, e1) when every ego shares the disconnect mask m (E % 4 == 0): each
// lane owns fixed float4 column groups of the E x E table, masks them once and stores them
// for every ego of the range.
template <int LPE, int NT>
__device__ __forceinline__ void emit_adj_uniform(const KParams& P, const Lds& S, int env, uint64_t m, int e0,
                                                 int e1) {
  const int lane = threadIdx.x & (LPE - 1);
  constexpr int DYN = 0;
  LSM_DIMS;
  const int EE = E * E;
  GAS float* adj_out = gptr(P.o.adj) + (size_t)env * N * EE;
  const int Q = EE / 4, last = Q - 1;
  for (int t0 = lane; t0 < Q; t0 += 4 * LPE) {
    int u[4];
    float4 w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = t0 + j * LPE;
      u[j] = 4 * (t < last ? t : last);
      const int r = qdiv<NT>(u[j], E, P.m_E);
      const int c = u[j] - r * E;
      w[j] = fv4(S, N, NL, E, r, c);
      const uint32_t bits = ((m >> r) & 1ull) ? 0xfu : ((uint32_t)(m >> c) & 0xfu);
      if (bits & 1u) w[j].x = 0.f;
      if (bits & 2u) w[j].y = 0.f;
      if (bits & 4u) w[j].z = 0.f;
      if (bits & 8u) w[j].w = 0.f;
    }
#ifdef LSM_STAMPS
    if (P.diag & 1) continue;
#endif
    for (int e = e0; e < e1; ++e) {
      GAS float* dst = adj_out + (size_t)e * EE;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (t0 + j * LPE <= last) st_stream<(NT >= 16)>(dst + u[j], w[j]);
    }
  }
}

template <int DYN, int LPE, int NT>
__device__ __forceinline__ void emit_nodes(const KParams& P, Lds& S, int env, bool uni);

// LSM_OUT_ADJ_NNZ: the nonzeros of each ego's adjacency as emit_graph stores it (either layout: the
// thresholded table with ego e's disconnected rows and columns zeroed) -- the per-graph count of
// GNNBase.process_adj's adj.nonzero() (gnn.py:376-407), so the learner's edge list takes one pass
// over the adjacency (lsm_edges_scan_emit) instead of a count pass and an emit pass. Row r's nonzero
// columns as a ballot word (E <= 64), then lane e adds popcount(word & ~mask_e) over its unmasked
// rows. The test is on the stored float32 value, exactly what nonzero() sees.
template <int LPE, int NT>
__device__ __forceinline__ void emit_adj_nnz(const KParams& P, const Lds& S, int env) {
  const int lane = threadIdx.x & (LPE - 1);
  const int gsh = ((int)threadIdx.x & 63) & ~(LPE - 1);   // this env's first lane in the wave
  constexpr int DYN = 0;
  LSM_DIMS;
  const uint64_t me = lane < N ? S.emask[lane] : 0ull;
  int64_t cnt = 0;
  for (int r = 0; r < E; ++r) {
    uint64_t row = 0ull;
    for (int c0 = 0; c0 < E; c0 += LPE) {
      const int c = c0 + lane;
      const uint64_t b = __ballot(c < E && fv1(S, N, NL, E, r, c < E ? c : 0) != 0.0f);
      const uint64_t gb = LPE == 64 ? b : (b >> gsh) & ((1ull << LPE) - 1ull);
      row |= gb << c0;
    }
    if (lane < N && !((me >> r) & 1ull)) cnt += __popcll(row & ~me);
  }
  if (lane < N) gptr(P.o.adjnnz)[(size_t)env * N + lane] = cnt;
}

// `adj_done`: the uniform adjacency was already stored (speculatively, in phase D of the team
// kernel); it is rewritten here only if an agent changed status.
template <int DYN, int LPE, int NT>
__device__ __forceinline__ void emit_graph(const KParams& P, Lds& S, int env, bool adj_done = false) {
  const int lane = threadIdx.x & (LPE - 1);
  LSM_DIMS;
  // No agent changed done / reached status this step (the common case): every ego then has
  // the same disconnect mask and the same (pre == post) entity rows, so each lane computes
  // its output words once and stores them for all N egos.
  const bool uni = !S.dep0 &&
                   group_all<LPE>(lane >= N || (S.dpre[lane] == S.dpost[lane] && S.rpre[lane] == S.rpost[lane]));
  if (DYN == 0) build_rows_di<LPE, NT>(P, S); else trig_table_at<LPE, NT>(P, S);
  esync<LPE>();
  // ---- adjacency: ego e, row r, col c ------------------------------------------------------
  const int EE = E * E, atot = N * EE;
  GAS float* adj_out = gptr(P.o.adj) + (size_t)env * atot;
  if (P.adj_compact) {
    // LSM_ADJ_COMPACT: the unmasked table once + the per-ego masks (one word: E <= 64)
    GAS float* a = gptr(P.o.adj) + (size_t)env * EE;
    if ((E & 3) == 0) {
      for (int q = lane; q < EE / 4; q += LPE) {
        const int r = qdiv<NT>(4 * q, E, P.m_E);
        st_stream<(NT >= 16)>(a + 4 * q, fv4(S, N, NL, E, r, 4 * q - r * E));
      }
    } else {
      for (int q = lane; q < EE; q += LPE) {
        const int r = qdiv<NT>(q, E, P.m_E);
        a[q] = fv1(S, N, NL, E, r, q - r * E);
      }
    }
    if (lane < N) gptr(P.o.adjmask)[(size_t)env * N + lane] = S.emask[lane];
  } else if ((E & 3) == 0 && uni) {
    if (!adj_done) emit_adj_uniform<LPE, NT>(P, S, env, S.emask[0], 0, N);
  } else if ((E & 3) == 0) {
    // Each lane owns fixed float4 column groups u of the E x E table (loaded from LDS once)
    // and writes them for every ego: per ego only the mask word is read.
    const int Q = EE / 4;
    for (int t0 = lane; t0 < Q; t0 += 4 * LPE) {
      const int last = Q - 1;
      int u[4], rr[4];
      float4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int t = t0 + j * LPE;
        u[j] = 4 * (t < last ? t : last);
        rr[j] = qdiv<NT>(u[j], E, P.m_E);
        v[j] = fv4(S, N, NL, E, rr[j], u[j] - rr[j] * E);
      }
      for (int e = 0; e < N; ++e) {
        const uint64_t m = S.emask[e];
        GAS float* dst = adj_out + (size_t)e * EE;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (t0 + j * LPE > last) break;
          float4 w = v[j];
          const int c = u[j] - rr[j] * E;
          const uint32_t bits = ((m >> rr[j]) & 1ull) ? 0xfu : ((uint32_t)(m >> c) & 0xfu);
          if (bits & 1u) w.x = 0.f;
          if (bits & 2u) w.y = 0.f;
          if (bits & 4u) w.z = 0.f;
          if (bits & 8u) w.w = 0.f;
          st_stream<(NT >= 16)>(dst + u[j], w);
        }
      }
    }
  } else {
    for (int q = lane; q < atot; q += LPE) {
      const int e = qdiv<NT>(q, E * E, P.m_EE);
      const int u = q - e * EE;
      const int r = qdiv<NT>(u, E, P.m_E);
      const int c = u - r * E;
      const uint64_t m = S.emask[e];
      adj_out[q] = (((m >> r) | (m >> c)) & 1ull) ? 0.0f : fv1(S, N, NL, E, r, c);
    }
  }
  // the counts read the thresholded table, which the node staging of emit_nodes overwrites (U1)
  if (gptr(P.o.adjnnz)) emit_adj_nnz<LPE, NT>(P, S, env);
  emit_nodes<DYN, LPE, NT>(P, S, env, uni);
}

// node_obs [N][E][F] of one env (DI rows / airtaxi trig table already in LDS). `uni`: no
// agent changed status this step, so every ego sees the post rows.
// DI node_obs of egos [e0, e1) when no agent changed status (E * F % 4 == 0): lane owns float4 t
// of every ego block, entity rows read once, ego offset per ego.
template <int LPE, int NT>
__device__ __forceinline__ void emit_nodes_uniform_di(const KParams& P, const Lds& S, int env, int e0, int e1) {
  const int lane = threadIdx.x & (LPE - 1);
  constexpr int DYN = 0;
  LSM_DIMS;
  GAS float* node_out = gptr(P.o.node) + (size_t)env * N * E * F;
  const int EF4 = E * F / 4;
  for (int t = lane; t < EF4; t += LPE) {
    int k = qdiv<NT>(4 * t, F, P.m_F);
    int q = 4 * t - k * F;
    double fv[4];
    int qq[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      fv[c] = S.feat[(N + k) * F + q];   // post rows == pre rows here; landmarks at N + k
      qq[c] = q;
      if (++q == F) { q = 0; ++k; }
    }
#ifdef LSM_STAMPS
    if (P.diag & 1) continue;
#endif
    for (int e = e0; e < e1; ++e) {
      const double* o = S.egooff + e * F;
      st_stream<(NT >= 16)>(node_out + (size_t)e * E * F + 4 * t,
          make_float4((float)(fv[0] - o[qq[0]]), (float)(fv[1] - o[qq[1]]), (float)(fv[2] - o[qq[2]]),
                      (float)(fv[3] - o[qq[3]])));
    }
  }
}

template <int DYN, int LPE, int NT>
__device__ __forceinline__ void emit_nodes(const KParams& P, Lds& S, int env, bool uni) {
  const int lane = threadIdx.x & (LPE - 1);
  LSM_DIMS;
  const int npairs = N * E, ntot = npairs * F;
  GAS float* node_out = gptr(P.o.node) + (size_t)env * ntot;
  if (DYN == 0 && ((E * F) & 3) == 0 && uni) {
    emit_nodes_uniform_di<LPE, NT>(P, S, env, 0, N);
    return;
  }
  if (DYN == 0 && ((E * F) & 3) == 0) {
    // DI: node[e][k][q] = f32(row(e, k)[q] - off(e)[q]); written straight from the rows as
    // contiguous float4 (each ego block is E*F floats, a multiple of 4).
    const int q4 = ntot / 4, EF4 = E * F / 4;
    for (int t = lane; t < q4; t += LPE) {
      const int e = qdiv<NT>(t, E * F / 4, P.m_EF4);
      const int j0 = 4 * (t - e * EF4);
      int k = qdiv<NT>(j0, F, P.m_F);
      int q = j0 - k * F;
      const double* o = S.egooff + e * F;
      float f[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int row = (k < N) ? ((k > e) ? k : N + k) : N + k;
        f[c] = (float)(S.feat[row * F + q] - o[q]);
        if (++q == F) { q = 0; ++k; }
      }
      *(float4*)(node_out + 4 * (size_t)t) = make_float4(f[0], f[1], f[2], f[3]);
    }
    return;
  }
  esync<LPE>();   // fval dead from here: node staging reuses U1
  const bool nvec = (ntot & 3) == 0;
  for (int b0 = 0; b0 < npairs; b0 += LPE) {
    const int p = b0 + lane;
    if (p < npairs) {
      const int e = qdiv<NT>(p, E, P.m_E);
      const int k = p - e * E;
      float* st = S.stage + lane * F;
      if (DYN == 0) {
        const int row = (k < N) ? ((k > e) ? k : N + k) : N + k;
        const double* r = S.feat + row * F;
        const double* o = S.egooff + e * F;
#pragma unroll
        for (int q = 0; q < 10; ++q) st[q] = (float)(r[q] - o[q]);
      } else {
        float f[11];
        node_features<DYN, NT>(P, S, e, k, f);
#pragma unroll
        for (int q = 0; q < 11; ++q) st[q] = f[q];
      }
    }
    esync<LPE>();
    const int cnt = min(LPE, npairs - b0) * F;
    GAS float* dst = node_out + (size_t)b0 * F;
    if (nvec && (cnt & 3) == 0) {
      for (int q = lane; q < cnt / 4; q += LPE) ((GAS f32x4*)dst)[q] = ((const f32x4*)S.stage)[q];
    } else {
      for (int q = lane; q < cnt; q += LPE) dst[q] = S.stage[q];
    }
    esync<LPE>();
  }
}

// cached_dist_mag (core.py:514-543): float32 thresholded copy for the adjacency
// (adj = d * (d < range) * (d > 0), navigation_graph_safe.py:991-992) + float64 agent block.
// cached_dist_mag (core.py:514-543): float32 thresholded copy for the adjacency
// (adj = d * (d < range) * (d > 0), navigation_graph_safe.py:991-992) + float64 agent block.
// Landmarks do not move within an episode: their pairwise block is computed at the reset
// (`full`) into the record (lmd) and copied in afterwards.
template <int LPE, int NT>
__device__ __forceinline__ void compute_dist(const KParams& P, Lds& S, const uint32_t* prw = nullptr,
                                             bool full = false) {
  const int lane = threadIdx.x & (LPE - 1);
  constexpr int DYN = 0;
  LSM_DIMS;
  const int nmov = N * (N - 1) / 2 + N * NL;   // pairs with an agent (pair table classes 0, 1)
  const int npair = full ? E * (E - 1) / 2 : nmov;
#pragma unroll
  for (int t = lane; t < npair; t += LPE) {
    // specialised kernels preload this lane's pair words with the record (prw)
    const uint32_t pr = (NT && prw && t < nmov) ? prw[(t - lane) / LPE] : (uint32_t)gptr(P.pairs)[t];
    const int a = (int)(pr & 0xffu), b = (int)(pr >> 8);
    // a pair with an agent has it first (a < N): a step (not `full`) reads agent a directly
    const double xa = (!full || a < N) ? S.ps[a] : S.lm[a - N];
    const double ya = (!full || a < N) ? S.ps[N + a] : S.lm[NL + a - N];
    const double xb = b < N ? S.ps[b] : S.lm[b - N];
    const double yb = b < N ? S.ps[N + b] : S.lm[NL + b - N];
    const double dx = xa - xb, dy = ya - yb;
    const double d = sqrt(dx * dx + dy * dy);   // |p_a - p_b| == |p_b - p_a| bit for bit
    const float fv = (d < P.coord_range && d > 0) ? (float)d : 0.0f;
    fv_set(S, N, E, a, b, fv);
    fv_set(S, N, E, b, a, fv);
    if (t >= nmov) S.lmd[t - nmov] = fv;
    if (b < N) {
      const double d2 = blas_norm2(dx, dy);
      S.aa[a * N + b] = d;
      S.aa[b * N + a] = d;
      S.aa2[a * N + b] = d2;
      S.aa2[b * N + a] = d2;
    }
  }
  if (!full && !S.lean) {
    // landmark block from the episode cache: u = (la, lb) over NL x NL (diagonal -> 0 below)
    for (int u = lane; u < NL * NL; u += LPE) {
      const int la = qdiv<NT>(u, NL, P.m_NL), lb = u - la * NL;
      if (la == lb) continue;
      const int lo = la < lb ? la : lb, hi = la < lb ? lb : la;
      S.fval[(N + la) * E + N + lb] = S.lmd[lo * (2 * NL - lo - 1) / 2 + (hi - lo - 1)];
    }
  }
  for (int k = lane; k < E; k += LPE) {
    fv_set(S, N, E, k, k, 0.0f);
    if (k < N) { S.aa[k * N + k] = 0.0; S.aa2[k * N + k] = 0.0; }
  }
  esync<LPE>();
}

template <int DYN, int NT>
__device__ __forceinline__ void write_obs(const KParams& P, const Lds& S, int env, int i) {
  LSM_DIMS;
  const int gi = goal_index(S.rpre[i], i, N, NL);
  const double gx = S.lm[gi], gy = S.lm[NL + gi], gh = S.lm[2 * NL + gi], gs = S.lm[3 * NL + gi];
  constexpr int OB = DYN ? 6 : 7;
  GAS float* o = gptr(P.o.obs) + ((size_t)env * N + i) * OB;
  const double px = S.ps[i], py = S.ps[N + i];
  float v[OB];
  if (DYN == 0) {
    v[0] = (float)S.ps[2 * N + i];
    v[1] = (float)S.ps[3 * N + i];
    v[2] = (float)(gx - px);
    v[3] = (float)(gy - py);
    v[4] = (float)S.lmsc[gi];
    v[5] = (float)S.lmsc[NL + gi];
    v[DYN ? 5 : 6] = (float)gs;
  } else {
    const double th = S.ps[2 * N + i];
    double rx, ry;
    blas_rot(cos(th), sin(th), gx - px, gy - py, rx, ry);
    const double rh = gh - th;
    v[0] = (float)S.ps[3 * N + i];
    v[1] = (float)rx;
    v[2] = (float)ry;
    v[3] = (float)sin(rh);
    v[4] = (float)cos(rh);
    v[5] = (float)gs;
  }
#pragma unroll
  for (int f = 0; f < OB; ++f) o[f] = v[f];
  // LSM_OUT_SHARE_OBS (optional): GMPERunner.insert's centralized share_obs
  // (graph_mpe_runner.py:469-481): the env's obs row repeated for every agent k
  if (P.o.share_obs) {
    GAS float* so = gptr(P.o.share_obs) + (size_t)env * N * N * OB + (size_t)i * OB;
    for (int k = 0; k < N; ++k)
#pragma unroll
      for (int f = 0; f < OB; ++f) so[(size_t)k * N * OB + f] = v[f];
  }
}

// Workgroup -> env block. Workgroups are dispatched round-robin over the 8 XCDs (wg b on XCD b % 8).
// With LSM_XCD_REMAP each XCD takes one contiguous range of envs, so the output rows an XCD's L2
// writes back are contiguous (neighbouring envs' rows share cache lines: obs rows are 224 B).
__device__ __forceinline__ int xcd_block(int b, int nb) {
#ifdef LSM_XCD_REMAP
  if ((nb & 7) == 0) return (b & 7) * (nb >> 3) + (b >> 3);
#endif
  (void)nb;
  return b;
}

// LSM_OUT_MASKS / LSM_OUT_ACTIVE_MASKS (optional): GMPERunner.insert (graph_mpe_runner.py:457-467)
// masks = !done; active_masks = done ? all(dones of the env) : 1
__device__ __forceinline__ void write_masks(const KParams& P, int env, int N, int i, bool my_done, bool all_done) {
  if (i >= N) return;
  const size_t k = (size_t)env * N + i;
  if (P.o.masks) gptr(P.o.masks)[k] = my_done ? 0.0f : 1.0f;
  if (P.o.active_masks) gptr(P.o.active_masks)[k] = my_done ? (all_done ? 1.0f : 0.0f) : 1.0f;
}

// save_summary_of_episode (environment.py:895-911) from the LDS copy of the stats.
template <int NT>
__device__ __forceinline__ void summary(const KParams& P, const Lds& S, double* out) {
  constexpr int DYN = 0;
  LSM_DIMS;
  const double* tl = S.stats;
  const double* td = S.stats + N;
  const double* dn = S.stats + 2 * N;
  const double* cf = S.stats + 3 * N;
  const double* md = S.stats + 4 * N;
  const double* mu = S.stats + 5 * N;
  double* a = S.scratch;   // [2][N]
  double* b = S.scratch + N;
  out[0] = P.dt * np_mean(tl, N);
  out[1] = np_mean(td, N);
  out[2] = np_mean(dn, N);
  for (int i = 0; i < N; ++i) a[i] = (double)S.rpost[i];
  out[3] = np_mean(a, N);
  for (int i = 0; i < N; ++i) b[i] = (tl[i] == 0) ? 1.0 : tl[i];
  for (int i = 0; i < N; ++i) a[i] = cf[i] / b[i];
  out[4] = np_mean(a, N);
  out[5] = np_mean(md, N);
  for (int i = 0; i < N; ++i) a[i] = mu[i] / b[i];
  out[7] = np_mean(a, N);
  if (out[5] == INFINITY) out[5] = P.coord_range;
  double mn = md[0];
  for (int i = 1; i < N; ++i) mn = (md[i] < mn) ? md[i] : mn;
  out[6] = mn;
  if (out[6] == INFINITY) out[6] = P.coord_range;
}

// summary() with output k on lane k < 8: every lane runs the same pairwise sum over its own source
// (a per-lane LDS address; the two ratio outputs divide by travel time, the others by 1.0, which
// is exact), so the eight means cost one. Same sums, same order, same bits as summary().
struct SummaryLaneAcc {
  const double* src;     // this lane's stats row
  const int32_t* rp;     // S.rpost (lane 3)
  const double* tl;      // travel times (the ratio lanes' denominators)
  int k;
  __device__ __forceinline__ double operator()(int i) const {
    double x = k == 3 ? (double)rp[i] : src[i];
    if (k == 4 || k == 7) x = x / ((tl[i] == 0) ? 1.0 : tl[i]);
    return x;
  }
};
template <int NT>
__device__ __forceinline__ double summary_lane(const KParams& P, const Lds& S, int k) {
  constexpr int DYN = 0;
  LSM_DIMS;
  const int kk = k < 8 ? k : 0;
  // stats row of output kk: tl td dn (rpost) cf md (min) mu
  const int row = kk < 3 ? kk : (kk == 3 ? 0 : (kk <= 5 ? kk - 1 : kk - 2));
  SummaryLaneAcc a{S.stats + row * N, S.rpost, S.stats, kk};
  double out = np_sum_acc(a, N) / (double)N;
  if (kk == 0) out = P.dt * out;
  const double* md = S.stats + 4 * N;
  if (kk == 6) {
    out = md[0];
    for (int i = 1; i < N; ++i) out = (md[i] < out) ? md[i] : out;
  }
  if ((kk == 5 || kk == 6) && out == INFINITY) out = P.coord_range;
  return out;
}

// summary() with its loops kept rolled (workgroup kernel, N up to 64: unrolled, the scheduler
// hoists every LDS load of the five pairwise sums and the kernel spills). Same arithmetic.
template <int NT>
__device__ __forceinline__ void summary_rolled(const KParams& P, const Lds& S, double* out) {
  constexpr int DYN = 0;
  LSM_DIMS;
  const double* tl = S.stats;
  const double* td = S.stats + N;
  const double* dn = S.stats + 2 * N;
  const double* cf = S.stats + 3 * N;
  const double* md = S.stats + 4 * N;
  const double* mu = S.stats + 5 * N;
  double* a = S.scratch;   // [2][N]
  double* b = S.scratch + N;
  out[0] = P.dt * np_mean_rolled(tl, N);
  out[1] = np_mean_rolled(td, N);
  out[2] = np_mean_rolled(dn, N);
#pragma unroll 1
  for (int i = 0; i < N; ++i) a[i] = (double)S.rpost[i];
  out[3] = np_mean_rolled(a, N);
#pragma unroll 1
  for (int i = 0; i < N; ++i) b[i] = (tl[i] == 0) ? 1.0 : tl[i];
#pragma unroll 1
  for (int i = 0; i < N; ++i) a[i] = cf[i] / b[i];
  out[4] = np_mean_rolled(a, N);
  out[5] = np_mean_rolled(md, N);
#pragma unroll 1
  for (int i = 0; i < N; ++i) a[i] = mu[i] / b[i];
  out[7] = np_mean_rolled(a, N);
  if (out[5] == INFINITY) out[5] = P.coord_range;
  double mn = md[0];
#pragma unroll 1
  for (int i = 1; i < N; ++i) mn = (md[i] < mn) ? md[i] : mn;
  out[6] = mn;
  if (out[6] == INFINITY) out[6] = P.coord_range;
}

// Device reset of one env (MultiAgentGraphEnv.reset, environment.py:1046-1074). Expects the
// env's persistent per-agent arrays in LDS (S.stats, S.rpost = reached_goal before reset).
// Everything of the reset up to the outputs: summary, curriculum block, scenario draw,
// per-agent episode arrays. In three pieces (reset_head, the draw, reset_tail) so the team
// kernel can run the draws of its envs one lane per env (lsm_team.h).

// Summary of the ending episode, the new curriculum block and the HJ separation shift.
template <int DYN, int LPE, int NT>
__device__ __forceinline__ void reset_head(const KParams& P, Lds& S, int env, const double* cur_new) {
  const int lane = threadIdx.x & (LPE - 1);
  LSM_DIMS;
  GAS double* prev = gptr(P.s.prev) + (size_t)env * 8;
  if (LPE >= 8 && LPE <= WAVE) {
    const double o = summary_lane<NT>(P, S, lane);
    if (lane < 8) {
      prev[lane] = o;
      gptr(P.o.ep_info)[(size_t)env * 8 + lane] = o;
    }
  } else if (lane == 0) {
    double outv[8];
    if (LPE == BT) summary_rolled<NT>(P, S, outv); else summary<NT>(P, S, outv);
    for (int k = 0; k < 8; ++k) {
      prev[k] = outv[k];
      gptr(P.o.ep_info)[(size_t)env * 8 + k] = outv[k];
    }
  }
  esync<LPE>();
  for (int k = lane; k < NCUR; k += LPE) S.cur[k] = cur_new[k];
  if (lane == 0 && P.use_hj) {
    // update_curriculum -> world.update_safety_filter_separation_distance -> HjDataHandle.
    // update_separation_distance (navigation_graph_safe.py:363-364, core.py:483-486,
    // safety_filter.py:170-174): shift = target - previous in float64; a zero shift leaves the
    // table unchanged. Shifts past the record's KSEP slots go to the env's overflow row, which the
    // host has sized for every chain the launch can produce (sep_check).
    const int n = (int)S.sep[0];
    const double prev = n ? S.sep[1] : P.val_sep0;
    const double sh = cur_new[C_SEP] - prev;
    if (sh != 0.0) {
      if (n < KSEP) S.sep[2 + n] = sh;
      else gptr(P.s.sepx)[(size_t)env * P.s.sepx_cap + (n - KSEP)] = sh;
      S.sep[0] = (double)(n + 1);
      S.sep[1] = cur_new[C_SEP];
    }
  }
  esync<LPE>();
}

// random_scenario's parameters of an env (its curriculum block in S.cur)
template <int DYN, int NT>
__device__ __forceinline__ ScenarioParams scenario_params(const KParams& P, const Lds& S) {
  LSM_DIMS;
  ScenarioParams sp;
  sp.dyn = DYN; sp.N = N; sp.L = L; sp.world_size = P.world_size; sp.coordination_range = P.coord_range;
  sp.goal_speed_min = P.gs_min; sp.goal_speed_max = P.gs_max;
  sp.ratio_airtaxi = S.cur[C_RAT]; sp.ratio_scenario = S.cur[C_RSC]; sp.two_pi = P.two_pi; sp.pi = P.pi;
  sp.d2lo = P.scen_d2lo; sp.d2hi = P.scen_d2hi;
  return sp;
}

// The new episode's per-agent arrays once the scenario is in S.ps / S.lm.
template <int DYN, int LPE, int NT>
__device__ __forceinline__ void reset_tail(const KParams& P, Lds& S, bool keep_done) {
  const int lane = threadIdx.x & (LPE - 1);
  LSM_DIMS;
  for (int k = lane; k < NL; k += LPE) {
    S.lmsc[k] = sin(S.lm[2 * NL + k]);
    S.lmsc[NL + k] = cos(S.lm[2 * NL + k]);
  }
  for (int k = lane; k < N; k += LPE) {
    // every layout sets agent.done = False except scenario_circular_config (navigation_graph_safe_
    // eval.py:100-121): there a done agent stays done, with the layout's state as its frozen state
    const int32_t d = keep_done ? S.dpost[k] : 0;
    S.dpre[k] = d; S.dpost[k] = d; S.rpre[k] = 0; S.rpost[k] = 0;
    S.emask[k] = 0;
    S.winfo[k] = -1.0; S.winfo[N + k] = -1.0; S.winfo[2 * N + k] = -1.0; S.winfo[3 * N + k] = 0.0;
    for (int q = 0; q < NSTAT; ++q) S.stats[q * N + k] = (q == 4) ? INFINITY : 0.0;
    S.pdist[k] = 0.0;
    S.gmt[k] = plain_norm2(S.ps[k] - S.lm[k], S.ps[N + k] - S.lm[NL + k]) / P.max_speed;
  }
  if (lane == 0) { S.step[0] = 0; S.step[1] = 0; }
  esync<LPE>();   // MT words read out of U1 before compute_dist overwrites it
  if (S.dep0 || keep_done) {
    // departures: undeparted agents are disconnected from the reset's graph observation too;
    // kept-done agents are disconnected as done (the workgroup kernel builds its multi-word
    // masks itself, reset_block)
    for (int k = lane; k < N; k += LPE) {
      if (S.dep0) {
        S.pth[k] = S.ps[2 * N + k];
        S.psp[k] = S.ps[3 * N + k];
      }
      if (LPE != BT) S.emask[k] = ego_mask(S, N, L, k);
    }
    esync<LPE>();
  }
}

template <int DYN, int LPE, int NT>
__device__ __forceinline__ void reset_core(const KParams& P, Lds& S, int env, const double* cur_new,
                                           const double* layout = nullptr) {
  const int lane = threadIdx.x & (LPE - 1);
  LSM_DIMS;
  reset_head<DYN, LPE, NT>(P, S, env, cur_new);
  bool keep_done = false;   // scenario_circular_config leaves done agents done (see reset_tail)
  const ScenarioParams sp = scenario_params<DYN, NT>(P, S);
  if (layout) {
    // lsm_reset_layout: the host's evaluation layout replaces random_scenario (no device draws)
    const int LD = 4 * N + 4 * NL + (S.dep0 ? 3 * N : 0) + 1;   // last word: keep done
    const GAS double* g = gptr(layout) + (size_t)env * LD;
    keep_done = g[LD - 1] != 0.0;
    for (int k = lane; k < 4 * N; k += LPE) {
      const int i = k >> 2, c = k & 3;
      S.ps[c * N + i] = g[k];
    }
    for (int k = lane; k < 4 * NL; k += LPE) {
      const int l = k >> 2, c = k & 3;
      S.lm[c * NL + l] = g[4 * N + k];
    }
    if (S.dep0) {
      for (int k = lane; k < N; k += LPE) {
        S.dep0[k] = S.dep1[k] = g[4 * N + 4 * NL + k] != 0.0;
        S.tmr[k] = (int32_t)g[5 * N + 4 * NL + k];
        S.ith[k] = g[6 * N + 4 * NL + k];
      }
    }
    esync<LPE>();
  } else if (P.rng == LSM_RNG_PHILOX) {
    // fast mode: Philox keyed by the env's seed, counter = this env's reset index (kept in the
    // MT position word); no 624-word state is read, twisted or written back
    GAS uint32_t* rw = gptr(P.s.mt) + (size_t)env * MT_WORDS + MT_N;
    const uint32_t ridx = *rw - (uint32_t)MT_N;
    const uint32_t key = (uint32_t)(P.seed + 1000 * (P.env_offset + env));
    esync<LPE>();
    if (LPE <= WAVE || (int)threadIdx.x < WAVE) {   // workgroup kernel: one wave draws (see below)
      Philox rng;
      rng.init(key, ridx);
      random_scenario(rng, sp, S.ps, S.lm, S.scen);
    }
    esync<LPE>();
    if (lane == 0) *rw = ridx + 1 + (uint32_t)MT_N;
  } else {
  const GAS uint32_t* mtg = gptr(P.s.mt) + (size_t)env * MT_WORDS;
  for (int k = lane; k < MT_WORDS; k += LPE) S.mt[k] = mtg[k];
  esync<LPE>();
  if (LPE > WAVE) {
    // workgroup kernel: the scenario's read-modify-writes of its LDS workspace are only safe
    // when every writer runs in lockstep, so one wave draws it (the others wait below)
    if ((int)threadIdx.x < WAVE) {
      WaveRng<WAVE, true> rng;
      rng.key = S.mt;
      rng.pos = (int)S.mt[MT_N];
      random_scenario(rng, sp, S.ps, S.lm, S.scen);
      if (lane == 0) S.mt[MT_N] = (uint32_t)rng.pos;
    }
    esync<LPE>();
  } else {
    WaveRng<LPE> rng;
    rng.key = S.mt;
    rng.pos = (int)S.mt[MT_N];
    // every lane runs the identical draw sequence and stores the identical values
#ifndef LSM_XP_NOSCEN   // diagnostic bound only (the previous episode's layout is kept)
    random_scenario(rng, sp, S.ps, S.lm, S.scen);
#endif
    esync<LPE>();
    if (lane == 0) S.mt[MT_N] = (uint32_t)rng.pos;
    esync<LPE>();
  }
  GAS uint32_t* mtw = gptr(P.s.mt) + (size_t)env * MT_WORDS;
  for (int k = lane; k < MT_WORDS; k += LPE) mtw[k] = S.mt[k];
  }
  reset_tail<DYN, LPE, NT>(P, S, keep_done);
}

template <int DYN, int LPE, int NT>
__device__ __forceinline__ void reset_env(const KParams& P, Lds& S, int env, const double* cur_new,
                                          const double* layout = nullptr) {
  const int lane = threadIdx.x & (LPE - 1);
  LSM_DIMS;
  reset_core<DYN, LPE, NT>(P, S, env, cur_new, layout);
  compute_dist<LPE, NT>(P, S, nullptr, true);
  if (lane < N) write_obs<DYN, NT>(P, S, env, lane);
#ifndef LSM_XP_NORESETEMIT   // diagnostic bound only: no graph outputs after a reset
  emit_graph<DYN, LPE, NT>(P, S, env);
#endif
}

// Record copy between HBM and the head of the env's LDS block: up to 4 float4 per lane in
// flight before the first write, so a record of <= 4 KB costs one round trip.
template <int LPE, class SP, class DP>
__device__ __forceinline__ void rec_copy(SP src, DP dst, int n16) {
  const int lane = threadIdx.x & (LPE - 1);
  for (int k0 = lane; k0 < n16; k0 += 4 * LPE) {
    const int k1 = k0 + LPE, k2 = k0 + 2 * LPE, k3 = k0 + 3 * LPE;
    const int last = n16 - 1;   // clamped (always in-bounds) loads, predicated stores
    const f32x4 r0 = src[k0];
    const f32x4 r1 = src[k1 < last ? k1 : last];
    const f32x4 r2 = src[k2 < last ? k2 : last];
    const f32x4 r3 = src[k3 < last ? k3 : last];
    dst[k0] = r0;
    if (k1 < n16) dst[k1] = r1;
    if (k2 < n16) dst[k2] = r2;
    if (k3 < n16) dst[k3] = r3;
  }
}

// Persistent record: LDS -> HBM (done agents' velocity / speed stored as zero, core.py
// freezes them). `full` also writes cur + landmarks (after a reset).
template <int DYN, int LPE, int NT>
__device__ __forceinline__ void store_state(const KParams& P, Lds& S, const unsigned char* lbase, int env,
                                            bool full) {
  const int lane = threadIdx.x & (LPE - 1);
  LSM_DIMS;
  if (DYN == 1 && S.dep0) {
    // departures: the post-update heading / speed become the state; departure arrays persist
    GAS double* dg = gptr(P.s.dep) + (size_t)env * depw(N);
    // next step's update_graph mask: ego N - 1's words (one word per ego in the one-wave kernels,
    // ceil(E / 64) in the workgroup kernel)
    const int MW = LPE == BT ? (E + 63) >> 6 : 1;
    for (int w = lane; w < MW; w += LPE) ((GAS uint64_t*)(dg + 3 * N))[w] = S.emask[(N - 1) * MW + w];
    for (int j = lane; j < N; j += LPE) {
      S.ps[2 * N + j] = S.pth[j];
      S.ps[3 * N + j] = S.psp[j];
      dg[j] = (double)S.dep1[j];
      dg[N + j] = (double)S.tmr[j];
      dg[2 * N + j] = S.ith[j];
      if (P.o.departed) gptr(P.o.departed)[(size_t)env * N + j] = S.dep1[j] ? 1 : 0;
    }
    esync<LPE>();
  }
  for (int k = lane; k < 4 * N; k += LPE) {
    const int c = k / N, j = k - c * N;
    double v = S.ps[k];
    if (froze_now(S, j) && (DYN == 0 ? (c >= 2) : (c == 3))) v = 0.0;
    S.ps[k] = v;
    if (P.o.state) gptr(P.o.state)[((size_t)env * N + j) * 4 + c] = v;
  }
  esync<LPE>();
  GAS f32x4* rg = (GAS f32x4*)gptr(P.s.rec) + (size_t)env * P.s.rec_stride16;
  if (full) {
    rec_copy<LPE>((const f32x4*)lbase, rg, P.s.rec16);
  } else {   // the sections a step changes: [0, a1) and [a2, a3)
    rec_copy<LPE>((const f32x4*)lbase, rg, P.s.a1_16);
    rec_copy<LPE>((const f32x4*)lbase + P.s.a2_16, rg + P.s.a2_16, P.s.a3_16 - P.s.a2_16);
  }
}

// integration of agent i, speed clamp, travel distance (core.py:118-131,199-210,680-687):
// the double integrator replays scipy's RK45 call operation for operation (lsm_rk45.h), airtaxi
// uses a stable closed form (its RK45 right-hand side goes through numpy's SIMD cos / sin)
template <int DYN>
__device__ __forceinline__ void integrate_agent(const KParams& P, Lds& S, int N, int i) {
  const double dt = P.dt;
  const double a0 = S.safe[i], a1 = S.safe[N + i];
  double x = S.ps[i], y = S.ps[N + i], s2 = S.ps[2 * N + i], s3 = S.ps[3 * N + i];
  double spd;
  if (DYN == 0) {
#ifdef LSM_XP_NORK   // diagnostic bound only: closed form instead of the RK45 restatement
    x = x + s2 * dt + 0.5 * a0 * dt * dt; y = y + s3 * dt + 0.5 * a1 * dt * dt;
    s2 = s2 + a0 * dt; s3 = s3 + a1 * dt;
#else
    double yv[4] = {x, y, s2, s3};
    rk45_di(yv, a0, a1, dt);
    x = yv[0]; y = yv[1]; s2 = yv[2]; s3 = yv[3];
#endif
    spd = sqrt(s2 * s2 + s3 * s3);
    if (spd > P.max_speed) {
      s2 = P.max_speed * s2 / spd;
      s3 = P.max_speed * s3 / spd;
    }
    spd = sqrt(s2 * s2 + s3 * s3);
  } else {
    const double th0 = s2, v0 = s3, w = a0, ac = a1;
    const double th1 = th0 + w * dt;
    const double v1 = v0 + ac * dt;
    // stable closed form about the mid-heading (oracle/lsm_oracle.py closed_form_step)
    const double h = 0.5 * w * dt;
    const double m = th0 + h;
    const double cm = cos(m), sm = sin(m);
    double sc, q;
    if (fabs(h) < 0.1) {
      const double h2 = h * h;
      sc = 1.0 - h2 / 6.0 * (1.0 - h2 / 20.0 * (1.0 - h2 / 42.0 * (1.0 - h2 / 72.0)));
      q = -h / 3.0 * (1.0 - h2 / 10.0 * (1.0 - h2 / 28.0 * (1.0 - h2 / 54.0)));
    } else {
      sc = sin(h) / h;
      q = (cos(h) - sc) / h;
    }
    const double A = v0 * dt + 0.5 * ac * dt * dt;
    const double B = 0.5 * ac * dt * dt;
    x = x + (A * cm * sc + B * sm * q);
    y = y + (A * sm * sc - B * cm * q);
    s2 = th1;
    s3 = v1;
    if (s3 > P.max_speed) s3 = P.max_speed;
    if (s3 < P.min_speed) s3 = P.min_speed;
    spd = s3;
  }
  S.ps[i] = x; S.ps[N + i] = y; S.ps[2 * N + i] = s2; S.ps[3 * N + i] = s3;
  S.pdist[i] += spd * dt;
}

// ---- the double integrator's RK45 on a lane pair -------------------------------------------
// The team kernel's agent wave holds G * N = 32 agents on lanes 0..31 of 64. For the integration
// lane l runs agent l's x axis and lane l + 32 its y axis: per lane half the divisions and dot
// products of rk45_di, with the four-component norms (and the speed clamp) formed from both
// halves through one v_permlane32_swap per 32-bit word. The arithmetic per component and the
// order of the norm's fma chain (x pos, y pos, x vel, y vel) are rk45_di's, so the result is the
// same bits (tests/test_gpu_parity.py through the team kernel variants).
__device__ __forceinline__ double lane32_partner(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const bool up = (threadIdx.x & 63) >= 32;
  return __hiloint2double(up ? b[0] : b[1], up ? a[0] : a[1]);
}

// (x0, x1, x2, x3) = (x pos, y pos, x vel, y vel) of the pair's components -> rk_norm4
__device__ __forceinline__ double rk_norm4_pair(double mp, double mv, bool up) {
  const double qp = lane32_partner(mp), qv = lane32_partner(mv);
  const double x0 = up ? qp : mp, x1 = up ? mp : qp, x2 = up ? qv : mv, x3 = up ? mv : qv;
  double s = x0 * x0;
  s = fma(x1, x1, s);
  s = fma(x2, x2, s);
  s = fma(x3, x3, s);
  return sqrt(s) / 2.0;
}

// rk45_di for one axis (position p, velocity v, acceleration a) of a lane pair; `up` = y axis.
// Both lanes of a pair reach the same scalar decisions (same norms), so they stay in step.
#ifdef LSM_STAMPS
// diagnostic build: s_memtime of lane 0 inside the agent wave's integration (lsm.diag_stamps --team)
#define PSTAMP(k)                                                                                  \
  do {                                                                                             \
    if (stp && (threadIdx.x & 63) == 0) stp[k] = __builtin_amdgcn_s_memtime();                     \
  } while (0)
#else
#define PSTAMP(k) do { } while (0)
#endif
__device__ __forceinline__ void rk45_di_pair(double& p, double& v, double a, double tb, bool up,
                                             PowTabs pt = PowTabs(), GAS unsigned long long* stp = nullptr) {
  (void)stp;
  const double rtol = 1e-3, atol = 1e-6;
  // At rest with no acceleration on both axes (+0.0 velocity and acceleration, position not -0.0)
  // every stage is +-0 and every step leaves (p, v) as they are: the result without the ~6 steps
  // that select_initial_step's 1e-6 start takes to reach tb (its values feed nothing else).
  {
    const bool rest = __double_as_longlong(v) == 0 && __double_as_longlong(a) == 0 &&
                      __double_as_longlong(p) != (long long)0x8000000000000000ull;
    const bool prest = lane32_partner(rest ? 1.0 : 0.0) != 0.0;
    if (rest && prest) return;
  }

  const Rk45Tab& T = rk45_tab();
  double dv[6];
#pragma unroll
  for (int s = 1; s < 6; ++s) dv[s] = rk_gemv_const(a, T.A[s], s);
  const double gb = rk_gemv_const(a, T.B, 6), ge = rk_gemv_const(a, T.E, 7);
  const double scp = atol + fabs(p) * rtol, scv = atol + fabs(v) * rtol;
  const double d0 = rk_norm4_pair(p / scp, v / scv, up);
  const double d1 = rk_norm4_pair(v / scp, a / scv, up);
  double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
  h0 = (tb < h0) ? tb : h0;
  // (a - a) / scv is +0 for the finite accelerations here (scv >= atol > 0): no division
  const double d2 = rk_norm4_pair(((v + h0 * a) - v) / scp, (a - a) * 0.0, up) / h0;
  double h1;
  if (d1 <= 1e-15 && d2 <= 1e-15) {
    h1 = (h0 * 1e-3 > 1e-6) ? h0 * 1e-3 : 1e-6;
  } else {
    h1 = glibc_pow(0.01 / ((d2 > d1) ? d2 : d1), 1.0 / 5.0, pt);
  }
  double h_abs = 100 * h0;
  if (h1 < h_abs) h_abs = h1;
  if (tb < h_abs) h_abs = tb;
  double t = 0.0;
  double v0 = v;   // K[0] of the step: the step's starting velocity
  PSTAMP(27);
  while (t < tb) {
    bool rejected = false;
    for (;;) {
      double t_new = t + h_abs;
      if (t_new - tb > 0) t_new = tb;
      const double h = t_new - t;
      h_abs = fabs(h);
      double k[7];
      k[0] = v0;
#pragma unroll
      for (int s = 1; s < 6; ++s) k[s] = v + dv[s] * h;
      const double ynp = p + h * rk_gemv_col(k, T.B, 6);
      const double ynv = v + h * gb;
      k[6] = ynv;
      const double ep = rk_gemv_col(k, T.E, 7), ev = ge;
      // The error terms are rounding noise for this ODE (the stages are exact up to rounding):
      // when |e h| <= 1e-13 on all four components, each scaled term is <= 1e-7 (denominators
      // >= atol = 1e-6), so the computed norm is < 1e-6: the step is accepted with factor 10
      // (no pow), exactly the branch the full computation takes. Otherwise the full computation.
      const bool mine = fabs(ep * h) <= 1e-13 && fabs(ev * h) <= 1e-13;   // NaN: not small
      const bool small = mine && lane32_partner(mine ? 1.0 : 0.0) != 0.0;
      double en = 0.0;
      if (!small) {
        const double ap = fabs(p), anp = fabs(ynp), av = fabs(v), anv = fabs(ynv);
        const double rp = (ep * h) / (atol + ((ap >= anp) ? ap : anp) * rtol);
        const double rv = (ev * h) / (atol + ((av >= anv) ? av : anv) * rtol);
        en = rk_norm4_pair(rp, rv, up);
      }
      if (en < 1) {
        if (t_new < tb) {
          double fac = 10.0;
          if (en > 1e-6) {
            const double q = 0.9 * glibc_pow(en, -1.0 / 5.0, pt);
            if (q < fac) fac = q;
          }
          if (rejected && fac > 1) fac = 1;
          h_abs *= fac;
        }
        t = t_new;
        p = ynp;
        v = ynv;
        v0 = ynv;
        break;
      }
      const double q = 0.9 * glibc_pow(en, -1.0 / 5.0, pt);
      h_abs *= (q > 0.2) ? q : 0.2;
      rejected = true;
    }
  }
}

// integrate_agent<0> on a lane pair (axis `up` of agent i): RK45, speed clamp, travel distance
__device__ __forceinline__ void integrate_agent_di_pair(const KParams& P, Lds& S, int N, int i, bool up,
                                                        PowTabs pt = PowTabs(),
                                                        GAS unsigned long long* stp = nullptr) {
  const int c = up ? 1 : 0;
  double p = S.ps[c * N + i], v = S.ps[(2 + c) * N + i];
  const double a = S.safe[c * N + i];
  PSTAMP(29);
  rk45_di_pair(p, v, a, P.dt, up, pt, stp);
  PSTAMP(28);
  double q = lane32_partner(v);
  double sx = up ? q : v, sy = up ? v : q;
  double spd = sqrt(sx * sx + sy * sy);
  if (spd > P.max_speed) {   // unclamped, the second norm is the first (the same operands)
    v = P.max_speed * v / spd;
    q = lane32_partner(v);
    sx = up ? q : v;
    sy = up ? v : q;
    spd = sqrt(sx * sx + sy * sy);
  }
  S.ps[c * N + i] = p;
  S.ps[(2 + c) * N + i] = v;
  if (!up) S.pdist[i] += spd * P.dt;
}

// numpy's logaddexp(0, z) (npy_logaddexp: x + log1p(exp(y - x)) around the larger argument)
__device__ __forceinline__ double np_logaddexp0(double z) {
  if (z == 0.0) return 0.693147180559945309417232121458176568;   // NPY_LOGE2
  const double tmp = 0.0 - z;
  if (tmp > 0) return 0.0 + log1p(exp(-tmp));
  return z + log1p(exp(tmp));
}

// Optional (lsm_config.collision_forces, off by default): the contact force on agent i that the
// reference's World.get_entity_collision_force (core.py:741-774) returns for each agent pair,
// summed over the pairs in order as MPE's apply_environment_force accumulates it (p_force[a] =
// f_a + p_force[a]). The reference never calls it (no caller, SURVEY finding 1), so the rollout
// does not apply it; this reports it. Fresh post-integration distances (World.step's
// calculate_distances, core.py:626), done flags as World.step sees them (force_a is None for a
// done agent -> 0); landmarks do not collide (navigation_graph_safe.py:52). Masses are 1, so
// both members of a pair get +-130 (p_a - p_b) / d * penetration and every agent's terms are
// +130 (p_i - p_j) / d * penetration, j in increasing order. Transcendentals are the device's
// (ulp-level vs glibc exp / log1p); nothing downstream reads the result.
__device__ __forceinline__ void collision_force_agent(const Lds& S, int N, int i, double& fx, double& fy) {
  fx = 0.0;
  fy = 0.0;
  if (S.dpre[i]) return;
  const double k = 1.9e-3, dmin = 0.050 + 0.050;   // contact_margin, min_dists (core.py:400, 524-530)
  for (int j = 0; j < N; ++j) {
    if (j == i) continue;
    const double dx = S.ps[i] - S.ps[j], dy = S.ps[N + i] - S.ps[N + j];
    const double dist = sqrt(dx * dx + dy * dy);
    const double pen = np_logaddexp0(-(dist - dmin) / k) * k;
    fx = 1.3e+2 * dx / dist * pen + fx;
    fy = 1.3e+2 * dy / dist * pen + fy;
  }
}

// Python / numpy scalar kinds of the reward sums (PyNum, below)
enum { PY_INT = 0, NP_I64 = 1, NP_F32 = 2, NP_F64 = 3, PY_FLT = 4 };

// Per-agent values of the reward phase that the info phase reuses.
// `base`: reward_reach_goal's value before the clip and its scalar kind (base_kind);
// reward_finish adds the optional terms.
struct AgentTmp {
  double rew = 0.0, th_pre = 0.0, spd_pre = 0.0, ct_pre = 1.0, st_pre = 0.0, base = 0.0;
  bool reached_pre = false;
  int base_kind = PY_INT;   // PY_INT, PY_FLT or NP_F64
};

// obs (before the update), reward, goal / done update of agent i (navigation_graph_safe.py:
// 606-875): sequential per agent in the reference, independent per lane here (the snapshot
// rule is applied by the per-ego masks / rows afterwards).
template <int DYN, int NT>
__device__ __forceinline__ void reward_agent(const KParams& P, Lds& S, int env, int i, double mag, AgentTmp& t) {
  LSM_DIMS;
  write_obs<DYN, NT>(P, S, env, i);
  const int gi = goal_index(S.rpre[i], i, N, NL);
  const double gx = S.lm[gi], gy = S.lm[NL + gi], gh = S.lm[2 * NL + gi], gs = S.lm[3 * NL + gi];
  const double px = S.ps[i], py = S.ps[N + i];
  t.spd_pre = agent_speed<DYN>(S, N, i, false);
  const double spd = t.spd_pre;
  double he;
  if (DYN == 0) {
    // DI heading = atan2(vy, vx) (atan2(0, 0) = 0): its cos / sin are v / |v|, so
    // direction_alignment_error = 0.5 - 0.5 cos(th - gh) needs no atan2 / cos (ulp-level
    // vs the reference, like the integrator); goal sin / cos are cached per episode
    if (spd > 0.0) {
      const double inv = 1.0 / spd;
      t.ct_pre = S.ps[2 * N + i] * inv;
      t.st_pre = S.ps[3 * N + i] * inv;
    }
    he = 0.5 - 0.5 * (t.ct_pre * S.lmsc[NL + gi] + t.st_pre * S.lmsc[gi]);
  } else {
    t.th_pre = S.ps[2 * N + i];
    he = dae(t.th_pre, gh);
  }
  const double th = t.th_pre;
  const double hpr = 1 - np_clip(he / S.cur[C_GHE], 0, 1);
  const double se = fabs(spd - gs);
  const double sen = np_clip(se / S.cur[C_GSE], 0, 1);
  const double cra = P.use_filter_arg ? 1.0 : S.cur[C_RAT];
  const bool reached = goal_reached_at<DYN>(S, N, NL, i, gi, spd, he);
  t.reached_pre = reached;
  const bool done0 = S.dpre[i] != 0;
  double r = 0.0;
  if (reached) {
    const double spr = 1 - sen;
    const double ddx = gx - px, ddy = gy - py;
    double cte = (DYN == 0) ? ddx * t.st_pre - ddy * t.ct_pre : ddx * sin(th) - ddy * cos(th);
    cte = fabs(cte) / np_maximum(blas_norm2(ddx, ddy), 1e-6);
    const double ctp = 1 - np_clip(cte, 0, 1);
    const double perf = hpr * spr * ctp;
    const double grew = (DYN == 0) ? 50 * perf : 50 * (perf * cra + (1 - cra));
    if (!P.use_masking || !done0) r = r + grew;
  }
  if (!done0) {
    if (DYN == 0) {
      if (!P.use_filter_arg) {
        double pen = 3 * mag;
        pen = np_clip(1 - S.cur[C_SLOPED], 0, 1) * pen;
        r = r - pen;
      }
      r = P.use_filter_arg ? r - 1.0 : r - 1.0 * S.cur[C_SLOPED];
    } else {
      double rpx, rpy;
      blas_rot(S.lmsc[NL + gi], S.lmsc[gi], px - gx, py - gy, rpx, rpy);   // cached cos / sin(gh)
      const double rs[4] = {rpx, rpy, th - gh, spd};
      float ttr = 0.0f;
      if (interp_value<4>(P.ttr, rs, ttr)) {
        // reference: `rew -= 0.04 * ttr` with ttr a float32 (JAX) scalar: the product is
        // float32; a python-int `rew` (no goal reward added) stays float32
        const double ttrd = (double)(0.04f * ttr);
        r = (reached && (!P.use_masking || !done0)) ? r - ttrd : (double)(float)(r - ttrd);
      } else {
        r = r - 0.04 * P.ttr_max;
      }
      r = r - sen * cra;
    }
  }
  t.base = r;
  // the Python type of reward_reach_goal's `rew` (:692-791): the int 0, np.float64 once a goal reward
  // or a numpy penalty is added, a Python float after the double integrator's bare `rew -= 1.0`
  // (filter on, :780) on the int
  t.base_kind = (reached && (!P.use_masking || !done0)) ? NP_F64 : PY_INT;
  if (!done0) t.base_kind = (DYN == 0 && P.use_filter_arg) ? (t.base_kind == PY_INT ? PY_FLT : t.base_kind) : NP_F64;
  t.rew = np_clip(r, -40.0, 50.0);
  if (DYN == 1 && S.dep0) {
    // RealisticScenario.update_reached_goal_and_done (navigation_graph_safe.py:1153-1186): the
    // departure (heading / speed reset once the timer has run out) or the waiting freeze, then
    // the goal test on the updated state, recursing while goals keep being reached (a layout may
    // repeat a goal position); at most L + 1 rounds.
    int dep = S.dep0[i], tm = S.tmr[i], rp = S.rpre[i], dn = S.dpre[i];
    double th1 = S.ps[2 * N + i], v1 = S.ps[3 * N + i];
    for (int it = 0; it <= L + 1; ++it) {
      if (tm <= 0 && !dep) {
        if (S.minrel[i] > P.sep_target) {   // reset_velocity(theta=init_theta, speed=goal_speed_max)
          th1 = S.ith[i];
          v1 = P.gs_max;
          dep = 1;
        }
      } else if (!dep) {
        tm -= 1;
        v1 = 0.0;   // freeze_agent (:1091-1099)
      }
      const int g2 = goal_index(rp, i, N, NL);
      if (!goal_reached_at<DYN>(S, N, NL, i, g2, v1, dae(th1, S.lm[2 * NL + g2]))) break;
      if (!P.use_masking || !dn) rp += 1;
      if (rp >= L) {   // agent_reached_all_goals: done, frozen
        dn = 1;
        v1 = 0.0;
        break;
      }
    }
    S.dep1[i] = dep; S.tmr[i] = tm; S.pth[i] = th1; S.psp[i] = v1;
    S.rpost[i] = rp;
    S.dpost[i] = dn;
  } else {
    int rp = S.rpre[i];
    if (reached && (!P.use_masking || !done0)) rp += 1;
    S.rpost[i] = rp;
    S.dpost[i] = (rp >= L) ? 1 : S.dpre[i];
  }
  if (!P.rext) gptr(P.o.rew)[(size_t)env * N + i] = (float)t.rew;   // else reward_finish writes it
}

// ---- optional reward terms and the shared reward ---------------------------------------------
// SafeAamScenario.reward adds RewardBinaryConfig's terms (navigation_graph_safe.py:793-850) to
// reward_reach_goal before the clip, agent by agent: agent i's terms see agents a < i after their
// goal / done update of this step and agents a > i before it. Run once every agent's update is in
// LDS (reward_agent for all of the env's agents, then a sync), one lane per agent.
//
// The reference adds Python scalars of four kinds and numpy's promotion of them decides whether a
// sum is rounded to float32: reward_hj_value's terms are np.float32 (a Python-int weight -- the
// stair ratio is the int 0 or 1 outside its ramp -- times the JAX float32 value), np.int64 (np.abs
// of the int 0 that min() returns) or np.float64 (a float64 weight). PyNum restates those
// promotions (NumPy 2, NEP 50: Python int and float scalars are weak -- they take the other
// operand's numpy type; np.float32 + np.int64 and np.int64 + a Python float are float64).
struct PyNum {
  double v;
  int t;
};
__device__ __forceinline__ PyNum py_num(double v, int t) {
  PyNum r;
  r.v = v;
  r.t = t;
  return r;
}
__device__ __forceinline__ PyNum py_add(PyNum a, PyNum b) {
  int t;
  const bool i64 = a.t == NP_I64 || b.t == NP_I64, pyf = a.t == PY_FLT || b.t == PY_FLT;
  if (a.t == NP_F64 || b.t == NP_F64) t = NP_F64;
  else if (a.t == NP_F32 || b.t == NP_F32) t = i64 ? NP_F64 : NP_F32;
  else if (i64) t = pyf ? NP_F64 : NP_I64;
  else t = pyf ? PY_FLT : PY_INT;
  return py_num(t == NP_F32 ? (double)((float)a.v + (float)b.v) : a.v + b.v, t);
}

// agent j's state (x, y, v_x | theta, v_y | speed) as the reward of agent i sees it: `post` (j < i)
// after j's update -- a freeze, or a RealisticScenario departure / waiting freeze
template <int DYN>
__device__ __forceinline__ void agent_state_seen(const Lds& S, int N, int j, bool post, double* s) {
  s[0] = S.ps[j];
  s[1] = S.ps[N + j];
  if (DYN == 1 && post && S.psp) {
    s[2] = S.pth[j];
    s[3] = S.psp[j];
    return;
  }
  const bool fz = post && froze_now(S, j);
  s[2] = (DYN == 0 && fz) ? 0.0 : S.ps[2 * N + j];
  s[3] = fz ? 0.0 : S.ps[3 * N + j];
}

// state.p_vel (core.py:106-108, 184-185)
template <int DYN>
__device__ __forceinline__ void p_vel(const double* s, double& vx, double& vy) {
  if (DYN == 0) {
    vx = s[2];
    vy = s[3];
  } else {
    vx = s[3] * cos(s[2]);
    vy = s[3] * sin(s[2]);
  }
}

// reward_finish: agent i's optional terms, the clip, and its reward (individual, or kept in LDS for
// the shared sum: S.raw[i] value, S.safe[i] its scalar kind -- both dead after the integration).
template <int DYN, int NT>
__device__ __forceinline__ void reward_finish(const KParams& P, Lds& S, int env, int i, AgentTmp& t) {
  LSM_DIMS;
  const bool wint = S.cur[C_SINT] != 0.0;          // the scaled weights are Python ints
  const int wt = wint ? PY_INT : NP_F64;
  const double st = S.cur[C_STAIR], sep = S.cur[C_SEP], eng = S.cur[C_ENG];
  double si[4], vix, viy;
  agent_state_seen<DYN>(S, N, i, false, si);
  p_vel<DYN>(si, vix, viy);
  PyNum sv = py_num(0.0, PY_INT), hj = py_num(0.0, PY_INT);
  double me = 0.0;
  int me_cnt = 0;
  const SepChain sc = sep_chain(S.sep, P.s, env);
  for (int a = 0; a < N; ++a) {
    if (a == i) continue;
    const bool post = a < i;
    if ((post ? S.dpost[a] : S.dpre[a]) != 0) continue;   // every term skips done agents
    double sa[4];
    agent_state_seen<DYN>(S, N, a, post, sa);
    const double rx = sa[0] - si[0], ry = sa[1] - si[1];   // a.p_pos - agent.p_pos
    const double d = blas_norm2(rx, ry);                   // np.linalg.norm
    // reward_safety_violation / is_confliction (:503-506, :793-798)
    if ((P.rbin & LSM_REWARD_SAFETY_VIOLATION) && d < sep) sv = py_add(sv, py_num(-20.0 * st, wt));
    // reward_multiple_engagement / is_in_engagement (:508-511, :800-823)
    if ((P.rbin & LSM_REWARD_POTENTIAL_CONFLICT) && d < eng) {
      const double close = 1 - np_clip((d - sep) / (eng - sep), 0, 1);
      const double ang = atan2(ry, rx);
      const double dx = cos(ang), dy = sin(ang);
      double vax, vay;
      p_vel<DYN>(sa, vax, vay);
      const double ch = fma(dy, vay - viy, dx * (vax - vix));   // np.inner (BLAS ddot)
      me += (ch < 0 ? -ch : 0.0) * close;                       // np.abs(min(0, change)) * closeness
      ++me_cnt;
    }
    // reward_hj_value (:830-837): World.get_hj_value_between_two_agents(agent, a) (core.py:459-468)
    if (P.rbin & LSM_REWARD_HJ_VALUE) {
      double rel[5];
      if (DYN == 0) {
        for (int k = 0; k < 4; ++k) rel[k] = si[k] - sa[k];
      } else {   // KinematicVehicleSafetyHandle.get_relative_state (safety_filter.py:277-284)
        const double ox = sa[0] - si[0], oy = sa[1] - si[1];
        const double dd = sqrt(ox * ox + oy * oy);
        const double al = atan2(oy, ox);
        rel[0] = dd * cos(al - si[2]);
        rel[1] = dd * sin(al - si[2]);
        rel[2] = sa[2] - si[2];
        rel[3] = si[3];
        rel[4] = sa[3];
      }
      float v = 0.0f;
      const bool ok = DYN == 0 ? interp_value<4>(P.val, rel, v, sc) : interp_value<5>(P.val, rel, v, sc);
      // np.abs(min(value - eps_hj, 0)): the float32 |value - 0.4| when it is <= 0, else np.int64 0
      // (min returns its int 0; out of the grid the value is +inf)
      const float x = v - 0.4f;
      const PyNum pen = (ok && !(x > 0.0f)) ? py_num((double)fabsf(x), NP_F32) : py_num(0.0, NP_I64);
      const double w = -2.0 * st;
      PyNum term;   // conflict_value_rew_scaled * pen
      if (wint) term = py_num(pen.t == NP_F32 ? (double)((float)w * (float)pen.v) : w * pen.v, pen.t);
      else term = py_num(w * pen.v, NP_F64);
      hj = py_add(hj, term);
    }
  }
  PyNum rew = py_num(t.base, t.base_kind);
  if (P.rbin & LSM_REWARD_SAFETY_VIOLATION) rew = py_add(rew, sv);
  if (P.rbin & LSM_REWARD_POTENTIAL_CONFLICT)
    rew = py_add(rew, me_cnt > 1 ? py_num(-1.0 * st * me, NP_F64) : py_num(0.0, PY_INT));
  if ((P.rbin & LSM_REWARD_DIFF_FROM_FILTERED_ACTION) && P.use_filter_arg)   // reward_diff_from_filtered_action
    rew = py_add(rew, S.dpre[i] ? py_num(0.0, PY_INT) : py_num(-1.0 * st * S.adiff[i], NP_F64));
  if (P.rbin & LSM_REWARD_HJ_VALUE) rew = py_add(rew, hj);
  // np.clip(rew, -40, 50): a Python int becomes np.int64, a Python float np.float64; float32 stays
  // float32 (bounds exact)
  t.rew = np_clip(rew.v, -40.0, 50.0);
  const size_t k = (size_t)env * N + i;
  if (!P.collab) gptr(P.o.rew)[k] = (float)t.rew;
  S.raw[i] = t.rew;
  S.safe[i] = (double)(rew.t == PY_INT ? NP_I64 : rew.t == PY_FLT ? NP_F64 : rew.t);
}

// The shared reward (environment.py:1031-1037): np.sum(reward_n) -- the array's dtype is the
// promotion of the agents' scalars, summed pairwise in it -- for every agent. After reward_finish
// of all the env's agents.
template <int NT>
__device__ __forceinline__ void reward_shared(const KParams& P, const Lds& S, int env, int i) {
  constexpr int DYN = 0;
  LSM_DIMS;
  bool f64 = false, f32 = false, i64 = false;
  for (int j = 0; j < N; ++j) {
    const int ty = (int)S.safe[j];
    f64 |= ty == NP_F64;
    f32 |= ty == NP_F32;
    i64 |= ty == NP_I64;
  }
  double sum;
  if (f32 && !f64 && !i64) {   // float32 pairwise sum (FLOAT_pairwise_sum)
    if (N < 8) {
      float r = 0.0f;
      for (int j = 0; j < N; ++j) r += (float)S.raw[j];
      sum = r;
    } else {
      float r[8];
      for (int q = 0; q < 8; ++q) r[q] = (float)S.raw[q];
      int j = 8;
      for (; j < N - (N % 8); j += 8)
        for (int q = 0; q < 8; ++q) r[q] += (float)S.raw[j + q];
      float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
      for (; j < N; ++j) res += (float)S.raw[j];
      sum = res;
    }
  } else {   // float64 (int64 sums are exact in it)
    sum = np_sum_rolled(S.raw, N);
  }
  gptr(P.o.rew)[(size_t)env * N + i] = (float)sum;
}

// info_callback accumulators of agent i (navigation_graph_safe.py:386-450); `ncoll` = other
// agents within the collision distance (is_collision, :497-501).
template <int DYN, int NT>
__device__ __forceinline__ void info_agent(const KParams& P, Lds& S, int i, int cstep, const AgentTmp& t,
                                           int ncoll) {
  LSM_DIMS;
  const double tr_old = S.winfo[i], dg_old = S.winfo[N + i];
  S.wold[i] = dg_old; S.wold[N + i] = tr_old;
  double tr = tr_old, dg = dg_old, dl = S.winfo[2 * N + i];
  const int gi = goal_index(S.rpost[i], i, N, NL);
  const double dist = plain_norm2(S.ps[i] - S.lm[gi], S.ps[N + i] - S.lm[NL + gi]);
  const double pd = S.pdist[i];
  bool reached_post = t.reached_pre;   // same state and goal unless the goal advanced
  if (DYN == 1 && S.psp) {
    // departures: the update may have changed heading / speed (departure, freeze)
    reached_post = goal_reached_at<DYN>(S, N, NL, i, gi, S.psp[i], dae(S.pth[i], S.lm[2 * NL + gi]));
  } else if (S.rpost[i] != S.rpre[i]) {
    const bool frz = froze_now(S, i);
    const double spp = frz ? 0.0 : t.spd_pre;
    double hep;
    if (DYN == 0) {   // frozen: zero velocity, atan2(0, 0) = 0
      const double c = frz ? 1.0 : t.ct_pre, sn = frz ? 0.0 : t.st_pre;
      hep = 0.5 - 0.5 * (c * S.lmsc[NL + gi] + sn * S.lmsc[gi]);
    } else {
      hep = dae(t.th_pre, S.lm[2 * NL + gi]);
    }
    reached_post = goal_reached_at<DYN>(S, N, NL, i, gi, spp, hep);
  }
  if (reached_post && tr == -1) {
    tr = cstep * P.dt;
    dg = pd;
    dl = dist;
  }
  if (tr == -1) {
    dg = pd;
    dl = dist;
  }
  const double nc = S.winfo[3 * N + i] + (double)ncoll;   // is_collision count (:497-501)
  S.winfo[i] = tr; S.winfo[N + i] = dg; S.winfo[2 * N + i] = dl; S.winfo[3 * N + i] = nc;
  S.wnew[i] = dg; S.wnew[N + i] = tr;
}

// agent i's info row (LSM_INFO_FIELDS doubles at `inf`), after every agent's info_agent:
// Distance / Time mean and std over the agents under the sequential snapshot rule.
template <int NT, class DP>
__device__ __forceinline__ void info_row(const KParams& P, const Lds& S, int i, double rew, DP inf) {
  constexpr int DYN = 0;
  LSM_DIMS;
  struct Snap {
    const double* nw;
    const double* od;
    int i;
    __device__ double operator()(int j) const { return j <= i ? nw[j] : od[j]; }
  };
  double dm, ds, tm, ts;
  np_mean_std(Snap{S.wnew, S.wold, i}, N, dm, ds);
  np_mean_std(Snap{S.wnew + N, S.wold + N, i}, N, tm, ts);
  const double mr = S.minrel[i];
  inf[LSM_INFO_INDIVIDUAL_REWARD] = rew;
  inf[LSM_INFO_MIN_RELATIVE_DISTANCE] = mr;
  inf[LSM_INFO_DIST_TO_GOAL] = S.winfo[2 * N + i];
  inf[LSM_INFO_TIME_REQ_TO_GOAL] = S.winfo[i];
  inf[LSM_INFO_NUM_AGENT_COLLISIONS] = S.winfo[3 * N + i];
  inf[LSM_INFO_DISTANCE_MEAN] = dm;
  inf[LSM_INFO_DISTANCE_VARIANCE] = ds;
  inf[LSM_INFO_DISTS_TRAVELED] = S.winfo[N + i];
  inf[LSM_INFO_TIME_MEAN] = tm;
  inf[LSM_INFO_TIME_STDDEV] = ts;
  inf[LSM_INFO_MIN_TIME_TO_GOAL] = S.gmt[i];
  inf[LSM_INFO_SAFETY_FILTERED] = (double)S.sfilt[i];
  inf[LSM_INFO_SAFETY_VIOLATED] = (mr < S.cur[C_SEP]) ? 1.0 : 0.0;
  inf[LSM_INFO_DECONFLICTING_INDEX] = (double)S.decon[i];
  inf[LSM_INFO_ACTION_DIFF] = S.adiff[i];
  inf[LSM_INFO_REACHED_GOAL] = (double)S.rpost[i];
  inf[LSM_INFO_POSITION_X] = S.ps[i];
  inf[LSM_INFO_POSITION_Y] = S.ps[N + i];
}

// Episode statistics of an active agent i (environment.py:1004-1022) from its neighbour
// counts over the masked agent-agent distances: cnt in range, neng within the engagement
// distance, mn the minimum.
template <int DYN>
__device__ __forceinline__ void stats_agent(const KParams& P, Lds& S, int N, int i, int cnt, int neng, double mn) {
  S.stats[i] += 1;
  double vx, vy;
  agent_vel<DYN>(S, N, i, true, vx, vy);
  S.stats[N + i] += blas_norm2(vx, vy) * P.dt;
  if (cnt > 0) {
    if (neng > 1) S.stats[5 * N + i] += 1;
    if (mn < P.sep_target) S.stats[3 * N + i] += 1;
    if (mn < S.stats[4 * N + i]) S.stats[4 * N + i] = mn;
  }
}

// The end-of-step episode statistics of agent i (environment.py:1004-1022) over the agents its
// final disconnect mask S.emask[i] keeps; `departed` is always True in the training scenario.
template <int DYN>
__device__ __forceinline__ void episode_stats(const KParams& P, Lds& S, int N, int i) {
  if (!S.dpost[i] && (!S.dep1 || S.dep1[i])) {   // `agent.departed and not agent.done` (:1008)
    const uint64_t m = S.emask[i];
    int cnt = 0, neng = 0;
    double mn = INFINITY;
    for (int j = 0; j < N; ++j) {
      if (((m >> i) | (m >> j)) & 1ull) continue;
      const double d = S.aa[j * N + i];   // symmetric; column reads are conflict-free
      if (!(d < P.coord_range && d > 0)) continue;
      cnt++;
      if (d < P.world_eng) neng++;
      mn = (d < mn) ? d : mn;
    }
    stats_agent<DYN>(P, S, N, i, cnt, neng, mn);
  }
  if (S.dpost[i]) S.stats[2 * N + i] = 1;
}

// min relative distance of agent i over the other active agents (core.py:696-709)
__device__ __forceinline__ void min_relative(Lds& S, int N, int i) {
  double m = INFINITY;
  if (!inactive_pre(S, i)) {
    for (int j = 0; j < N; ++j) {
      if (j == i || inactive_pre(S, j)) continue;
      const double d = S.aa2[j * N + i];
      m = (d < m) ? d : m;
    }
  }
  S.minrel[i] = m;
}

// other agents within the collision distance of agent i (is_collision, navigation_graph_safe.py:497-501)
__device__ __forceinline__ int collision_count(const Lds& S, int N, int i) {
  int cc = 0;
  for (int a = 0; a < N; ++a)
    if (a != i && S.aa2[a * N + i] < 1.05 * (0.05 + 0.05)) cc++;
  return cc;
}

// This step's Discrete(25) action index of agent `i` of env `env` (index, or the argmax of a
// one-hot row as the reference's np.argmax decode, environment.py:386-410).
__device__ __forceinline__ int read_action(const KStep& K, int env, int N, int i) {
  const size_t base = (size_t)env * N + i;
  int ai = 0;
  if (K.action_kind == LSM_ACTIONS_INDEX_I32) {
    ai = ((const GAS int32_t*)gptr(K.actions))[base];
  } else if (K.action_kind == LSM_ACTIONS_ONEHOT_F32) {
    const GAS float* a = (const GAS float*)gptr(K.actions) + base * 25;
    float best = a[0];
    for (int q = 1; q < 25; ++q) if (a[q] > best) { best = a[q]; ai = q; }
  } else {
    const GAS double* a = (const GAS double*)gptr(K.actions) + base * 25;
    double best = a[0];
    for (int q = 1; q < 25; ++q) if (a[q] > best) { best = a[q]; ai = q; }
  }
  return ai;
}

// t[k] of a 5-entry KParams table for a lane-varying k in [0, 5): the five values are wave-uniform
// (scalar loads, issued with the launch's other parameter loads) and the lane picks by selects; a
// vector load t[k] was a memory round trip between the record load and the filter's pair lookups
__device__ __forceinline__ double sel5(const double* t, int k) {
  double v[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) v[q] = t[q];
  double r = v[0];
#pragma unroll
  for (int q = 1; q < 5; ++q) r = (k == q) ? v[q] : r;
  return r;
}

// decode into the env's raw action rows; an index outside Discrete(25) is an error of the
// caller (the reference's one-hot decode has no such input): flagged for lsm_action_errors(),
// and the launch kept in bounds
__device__ __forceinline__ void decode_action(const KParams& P, Lds& S, int N, int i, int ai) {
  if (ai < 0 || ai > 24) *gptr(P.action_err) = 1;
  const int a = ai < 0 ? 0 : (ai > 24 ? 24 : ai);
  const int xi = a / 5, yi = a - xi * 5;
  S.raw[i] = sel5(P.act0, xi);
  S.raw[N + i] = sel5(P.act1, yi);
}

// Safety filter of agent i once the pair scratch is filled (core.py:648-677): the filtered
// action, flag, deconflicting index and action difference.
template <int DYN, int NT>
__device__ __forceinline__ void filter_agent(const KParams& P, Lds& S, int N, int i, bool filter_on) {
  double u0 = S.raw[i], u1 = S.raw[N + i];
#ifdef LSM_XP_NOFILT   // diagnostic bound only: no filter
  filter_on = false;
#endif
  if (filter_on) {
    uint8_t fl = 0;
    int dec = -1;
    if (!inactive_pre(S, i)) filter_ego<DYN, NT>(P, S, i, fl, dec, u0, u1);
    S.sfilt[i] = fl;
    S.decon[i] = dec;
  }
  S.safe[i] = u0;
  S.safe[N + i] = u1;
  S.adiff[i] = blas_norm2(S.raw[i] - u0, S.raw[N + i] - u1);
}

// Double integrator: 4 waves per SIMD (<= 128 VGPRs): config 3 is exactly 4096 one-wave envs =
// 4 per SIMD, and at 134 VGPRs the 4th wave of every SIMD ran after the others (53 vs 41 us per
// step, measured). Airtaxi keeps 2 (~176 VGPRs; a 128 cap spills 200-350 B per lane).
#ifndef LSM_WAVES_PER_EU_AT
#define LSM_WAVES_PER_EU_AT 2
#endif
template <int DYN, int LPE, int NT>
__global__ __launch_bounds__(64, DYN == 0 ? (LPE == 64 ? 4 : 2) : LSM_WAVES_PER_EU_AT) void rollout_kernel(const KParams* __restrict__ Pp, const KStep K) {
  const KParams& P = *Pp;   // per-handle constants in device memory; per-launch fields in L
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int G = WAVE / LPE;   // envs per wave, one per LPE-lane group
  const int grp = (G == 1) ? 0 : (int)threadIdx.x / LPE;
  const int env = xcd_block(blockIdx.x, gridDim.x) * G + grp;
  const int lane = threadIdx.x & (LPE - 1);
  if (env >= P.n_envs) return;
  LSM_DIMS;
  unsigned char* lbase = smem + (size_t)grp * P.lds_env_bytes;
#ifdef LSM_XP_POISON
  LDS_POISON(lbase, P.lds_env_bytes, lane, LPE);
  __syncthreads();
#endif
  Lds S = carve(lbase, N, NL, E, F);
  // RealisticScenario departures run only here: the generic airtaxi kernel, one env per wave
  if (DYN == 1 && NT == 0 && LPE == 64 && P.scenario == LSM_SCENARIO_DEPARTURES) carve_dep(S, lbase, P.lds_dep_off, N);
  RTSTAMP(13);
#ifdef LSM_STAMPS
  if (lane == 0 && gptr(P.stamps))
    gptr(P.stamps)[(size_t)env * LSM_NSTAMP + 15] = (unsigned long long)__builtin_amdgcn_s_getreg(63492) |
                                      ((unsigned long long)__builtin_amdgcn_s_getreg(6164) << 32);
#endif
  STAMP(0);

  // ---- 0. the env's record HBM -> LDS (one round trip) + this step's actions ------------
  int ai = 0;
  if (K.mode == 0 && lane < N) ai = read_action(K, env, N, lane);
  // this lane's E x E pair words (compute_dist), loaded in the same round trip as the record
  constexpr bool PRE = NT != 0 && NT <= 8;   // <= 5 registers per lane
  constexpr int NPI = PRE ? ((NT * (NT - 1) / 2 + NT * 2 * NT) + LPE - 1) / LPE : 1;
  uint32_t prw[NPI];
  if (PRE) {
#pragma unroll
    for (int k = 0; k < NPI; ++k) {
      const int t = lane + k * LPE;
      prw[k] = gptr(P.pairs)[t < E * (E - 1) / 2 ? t : 0];   // classes 0, 1 come first
    }
  }
  rec_copy<LPE>((const GAS f32x4*)gptr(P.s.rec) + (size_t)env * P.s.rec_stride16, (f32x4*)lbase, P.s.rec16);
  __syncthreads();
  if (lane < N) {
    S.dpre[lane] = S.dpost[lane];
    S.rpre[lane] = S.rpost[lane];
    if (DYN == 1) {
      S.ecs[lane] = cos(S.ps[2 * N + lane]);
      S.ecs[N + lane] = sin(S.ps[2 * N + lane]);
    }
    if (S.dep0 && K.mode == 0) {
      const GAS double* dg = gptr(P.s.dep) + (size_t)env * depw(N);
      S.dep0[lane] = S.dep1[lane] = dg[lane] != 0.0;
      S.tmr[lane] = (int32_t)dg[N + lane];
      S.ith[lane] = dg[2 * N + lane];
      S.pth[lane] = S.ps[2 * N + lane];
      S.psp[lane] = S.ps[3 * N + lane];
    }
  }
  const int cstep = S.step[0] + 1;
  __syncthreads();
  STAMP(1);

  if (K.mode != 0) {   // 1: device scenario, 2: host layout (lsm_reset_layout)
    reset_env<DYN, LPE, NT>(P, S, env, K.cur_new, K.mode == 2 ? K.layout : nullptr);
    __syncthreads();
    store_state<DYN, LPE, NT>(P, S, lbase, env, true);
    return;
  }

  // ---- 1. update_graph() at step start (previous state, final masks) --------------
  if (K.emit_edges) {
    GAS uint8_t* eo = gptr(P.o.edges) + (size_t)env * E * E;
    // the previous step's observation masked cached_dist_mag in place; after an edit of the
    // state (lsm_set_agent_state = world.calculate_distances()) it is fresh
    uint64_t m0 = S.step[1] ? 0ull : ego_mask(S, N, L, N);
    if (S.dep0 && !S.step[1]) m0 = *(const GAS uint64_t*)(gptr(P.s.dep) + (size_t)env * depw(N) + 3 * N);
    for (int u = lane; u < E * E; u += LPE) {
      const int a = qdiv<NT>(u, E, P.m_E), b = u - a * E;
      double d = 0.0;
      if (a != b) {
        const int lo = a < b ? a : b, hi = a < b ? b : a;
        const double xa = lo < N ? S.ps[lo] : S.lm[lo - N];
        const double ya = lo < N ? S.ps[N + lo] : S.lm[NL + lo - N];
        const double xb = hi < N ? S.ps[hi] : S.lm[hi - N];
        const double yb = hi < N ? S.ps[N + hi] : S.lm[NL + hi - N];
        const double dx = xa - xb, dy = ya - yb;
        d = sqrt(dx * dx + dy * dy);
      }
      if (((m0 >> a) | (m0 >> b)) & 1ull) d = 0.0;
      eo[u] = (d <= P.coord_range && d > 0) ? 1 : 0;
    }
  }

  // ---- 2. decode actions ----------------------------------------------------------
  if (lane < N) decode_action(P, S, N, lane, ai);
  __syncthreads();
  STAMP(2);

  // ---- 3. safety filter ---------------------------------------------------------------
#ifdef LSM_STAMPS
  const bool filter_on = S.cur[C_FILT] != 0.0 && !(P.diag & 2);   // diag bit 1: filter skipped
#else
  const bool filter_on = S.cur[C_FILT] != 0.0;
#endif
  // World.step's inner loop (core.py:607-631): filter -> action_diff -> integrate, num_internal_step
  // times on the same raw actions; the distances and min relative distance of the final state follow
  for (int it = 0; it < P.nis; ++it) {
  if (filter_on) {
    const SepChain sc = sep_chain(S.sep, P.s, env);
    const int npairs = N * N;
    for (int p = lane; p < npairs; p += LPE) {
      const int j = p / N, i = p - j * N;   // [j][i]: ego i fastest (bank-conflict-free reads)
      if (i == j || inactive_pre(S, i) || inactive_pre(S, j)) continue;
      const double ex = S.ps[i], ey = S.ps[N + i], ox = S.ps[j], oy = S.ps[N + j];
      S.dpair[p] = sqrt((ox - ex) * (ox - ex) + (oy - ey) * (oy - ey));
      double rel[5];
      rel_state<DYN>(S, N, i, j, rel);
      float v = 0.0f;
      bool ok;
      if (DYN == 0) ok = interp_value<4>(P.val, rel, v, sc); else ok = interp_value<5>(P.val, rel, v, sc);
      S.vpair[p] = ok ? v : INFINITY;
      S.inr[p] = ok ? 1 : 0;
    }
    __syncthreads();
  }
  STAMP(3);
  if (lane < N) filter_agent<DYN, NT>(P, S, N, lane, filter_on);
  __syncthreads();
  STAMP(4);

  // ---- 4. integrate ----------------------------------------------------------------------
  if (lane < N && !inactive_pre(S, lane)) integrate_agent<DYN>(P, S, N, lane);
  __syncthreads();
  if (DYN == 1 && it + 1 < P.nis) {   // the next inner filter's ego frame: the new headings
    if (lane < N) {
      S.ecs[lane] = cos(S.ps[2 * N + lane]);
      S.ecs[N + lane] = sin(S.ps[2 * N + lane]);
    }
    __syncthreads();
  }
  }
  STAMP(5);

  // ---- 5. distances, min relative distance ---------------------------------------------
  compute_dist<LPE, NT>(P, S, PRE ? prw : nullptr);
  if (P.o.cforce && lane < N) {
    double fx, fy;
    collision_force_agent(S, N, lane, fx, fy);
    GAS double* cf = gptr(P.o.cforce) + ((size_t)env * N + lane) * 2;
    cf[0] = fx;
    cf[1] = fy;
  }
  if (lane < N) min_relative(S, N, lane);
  // Speculative adjacency: unless an agent changes done / reached status below (rare), every
  // ego's mask is the pre-update mask, so the adjacency can be stored now, in four chunks of
  // egos placed between the remaining phases: the stores drain while the wave computes
  // instead of queueing behind each other at the end. A status change rewrites it at the end.
  // (not for an env that auto-resets at the episode-length boundary: the reset emits its outputs)
  const bool chunked = (E & 3) == 0 && !P.adj_compact && !S.dep0 && !(P.auto_reset && cstep >= P.episode_length);
  const uint64_t m_pre = chunked ? ego_mask(S, N, L, -1) : 0;
  if (chunked) emit_adj_uniform<LPE, NT>(P, S, env, m_pre, 0, N / 4);
  STAMP(6);

  // ---- 6. obs, reward, goal/done update ---------------------------------------------------
  double mag = 0.0;
  if (DYN == 0 && !P.use_filter_arg) mag = magnetic_penalty_wave<LPE, NT>(P, S, S.dpair);
  AgentTmp at;
  if (lane < N) reward_agent<DYN, NT>(P, S, env, lane, mag, at);
  __syncthreads();
  if (P.rext) {   // optional reward terms / shared reward: after every agent's goal / done update
    if (lane < N) reward_finish<DYN, NT>(P, S, env, lane, at);
    __syncthreads();
    if (P.collab && lane < N) reward_shared<NT>(P, S, env, lane);
  }
  const double rew = at.rew;
  if (lane < N) S.emask[lane] = ego_mask(S, N, L, lane);
  if (S.dep0) {
    // graph_observation masks cached_dist_mag IN PLACE (navigation_graph_safe.py:986-987), so
    // masks accumulate over the egos of a step. Done / reached only ever disconnect, so for them
    // ego e's own mask is that union; a departure connects: agent j >= 1 undeparted before the
    // update was masked by ego 0 and stays masked for every later ego of this step.
    uint64_t acc = 0;
    for (int j = 1; j < N; ++j)
      if (!S.dep0[j]) acc |= 1ull << j;
    if (lane < N) S.emask[lane] |= acc;
  }
  if (chunked) emit_adj_uniform<LPE, NT>(P, S, env, m_pre, N / 4, N / 2);
  STAMP(7);

  // ---- 7/8. info_callback numbers -----------------------------------------------------
  if (lane < N) info_agent<DYN, NT>(P, S, lane, cstep, at, collision_count(S, N, lane));
  __syncthreads();
  if (lane < N) info_row<NT>(P, S, lane, rew, S.info + lane * LSM_INFO_FIELDS);   // staged in U2
  __syncthreads();
  rec_copy<LPE>((const f32x4*)S.info, (GAS f32x4*)(gptr(P.o.info) + (size_t)env * N * LSM_INFO_FIELDS),
                N * LSM_INFO_FIELDS / 2);
  if (chunked) emit_adj_uniform<LPE, NT>(P, S, env, m_pre, N / 2, 3 * N / 4);
  STAMP(8);

  // ---- episode stats (environment.py:1004-1022), dones ---------------------------------
  bool my_done = true;
  if (lane < N) {
    const int i = lane;
    episode_stats<DYN>(P, S, N, i);
    my_done = S.dpost[i] || cstep >= P.episode_length;
    gptr(P.o.dones)[(size_t)env * N + i] = my_done ? 1 : 0;
  }
  const bool all_done = group_all<LPE>(my_done);
  write_masks(P, env, N, lane, my_done, all_done);
  if (chunked && !(P.auto_reset && all_done)) emit_adj_uniform<LPE, NT>(P, S, env, m_pre, 3 * N / 4, N);
  __syncthreads();
  STAMP(9);

  // ---- 9. graph outputs, or the auto-reset (whose outputs replace them) ---------------------
  if (lane == 0) { S.step[0] = cstep; S.step[1] = 0; }
  if (P.auto_reset && all_done) {
    if (lane == 0) gptr(P.o.reset_flag)[env] = 1;
    reset_env<DYN, LPE, NT>(P, S, env, K.cur_new);
    __syncthreads();
    STAMP(12);
    store_state<DYN, LPE, NT>(P, S, lbase, env, true);
  } else {
    if (lane == 0) gptr(P.o.reset_flag)[env] = 0;
    emit_graph<DYN, LPE, NT>(P, S, env, chunked);
    __syncthreads();
    STAMP(10);
    store_state<DYN, LPE, NT>(P, S, lbase, env, false);
  }
  STAMP(11);
  RTSTAMP(14);
}

#include "lsm_block.h"
#include "lsm_team.h"

#if LSM_HOST_PART
// A new value table (a new HjDataHandle): every env's separation chain starts empty.
__global__ void sep_clear_kernel(float4* rec, uint32_t rec_stride16, int n_envs, uint32_t sep_off) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  double* sep = (double*)((unsigned char*)(rec + (size_t)env * rec_stride16) + sep_off);
  sep[0] = 0.0;
  sep[1] = 0.0;
}
#endif

#if LSM_HOST_PART
// env k's MT19937: np.random.seed(seed + 1000 * (env_offset + k))
__global__ void seed_kernel(uint32_t* mt, int n_envs, int64_t seed, int64_t env_offset) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  const uint32_t s = (uint32_t)(seed + 1000 * (env_offset + env));
  uint32_t* key = mt + (size_t)env * MT_WORDS;
  mt_seed(s, key, 1);
  key[MT_N] = MT_N;
}
#endif

}  // namespace lsm

// ====================================================================================
// C ABI
// ====================================================================================
using namespace lsm;

struct lsm_env {
  lsm_config cfg;
  int mt_stage = 2 * MT_N;   // KParams::mt_stage (lsm_test_set_mt_stage)
  uint16_t* pairs;
  int N, L, NL, E, F, OBS;
  StateDev s;
  std::vector<void*> allocs;
  void* out_ptr[LSM_NUM_OUT];
  size_t out_bytes[LSM_NUM_OUT];
  TableDev val, ttr;
  double ttr_max;
  double val_sep0;      // separation of the uploaded value table
  double sep_last;      // separation of the last reset / step call (chain-length bound)
  int sep_changes;      // changes of that separation since the table upload (>= any env's chain)
  std::string err;
  bool tables_ok;
  int device;
  KParams* dparams;   // device copy of the per-handle constants (re-uploaded when dirty)
  int32_t* action_err;   // device flag: an action index outside [0, 25) since the last check
  bool params_dirty;
  // ring-bound output slots (lsm_bind_output_ring): ring index i writes slot s at
  // ring_base[s] + (i + ring_off[s]) * ring_stride[s] when that lands in [0, ring_count[s]),
  // else at out_ptr[s]. One KParams copy per ring index lives in dring; selecting an index is a
  // host-side pointer choice (no upload, no sync per step).
  void* ring_base[LSM_NUM_OUT];
  size_t ring_stride[LSM_NUM_OUT];
  int32_t ring_count[LSM_NUM_OUT], ring_off[LSM_NUM_OUT];
  int32_t ring_len;    // number of ring indices (0: no ring slots)
  int32_t ring_cap;    // KParams copies allocated in dring
  int32_t ring_sel;    // -1: plain bindings
  KParams* dring;
  lsm_kernel_select sel;   // lsm_create_select's kernel choice (tests, A/B runs)
  int lpe;   // lanes per env: 64 (one env per wave), 32 or 16 (2 or 4 envs per wave)
  bool block;   // workgroup-per-env kernel (N > 32 or E > 64, or sel.workgroup_per_env)
  bool generic_only;   // sel.generic: never use the compile-time-N kernels (tests)
  int team;   // envs per workgroup of the team kernel (lsm_team.h); 0 = rollout_kernel
  bool lean;  // the team kernel's lean LDS layout (airtaxi, N % 4 == 0, E % 4 == 0)
};

static int fail(lsm_env* e, const std::string& msg) {
  if (e) e->err = msg;
  return 1;
}

// the reference builds an HjDataHandle (use_hj_handle, navigation_graph_safe.py:195)
static bool uses_hj(const lsm_env* e) {
  return e->cfg.use_safety_filter || (e->cfg.reward_terms & LSM_REWARD_HJ_VALUE);
}

#define HIPCHK(env, expr)                                                              \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess) return fail(env, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

template <class T>
static int dalloc(lsm_env* e, T** p, size_t count) {
  void* q = nullptr;
  hipError_t r = hipMalloc(&q, count * sizeof(T) + 16);
  if (r != hipSuccess) return fail(e, std::string("hipMalloc: ") + hipGetErrorString(r));
  e->allocs.push_back(q);
  *p = (T*)q;
  return 0;
}

static const KParams* active_params(const lsm_env* e) {
  return e->ring_sel >= 0 ? (const KParams*)(e->dring + e->ring_sel) : (const KParams*)e->dparams;
}

template <int DYN, int LPE, int NT>
void launch_t(lsm_env* e, const KStep& L, size_t env_lds, hipStream_t st) {
  constexpr int G = WAVE / LPE;
  const int blocks = (e->cfg.num_envs + G - 1) / G;
  hipLaunchKernelGGL((rollout_kernel<DYN, LPE, NT>), dim3(blocks), dim3(WAVE), env_lds * G, st,
                     active_params(e), L);
}

template <int DYN, int NT, int G, bool REXT>
int launch_team_t(lsm_env* e, const KStep& L, size_t env_bytes, hipStream_t st) {
  static bool attr = false;   // LDS above the 64 KB default needs an explicit opt-in
#ifndef LSM_AB_LDS_PAD   // A/B variant builds only: extra LDS per workgroup (fewer workgroups per CU)
#define LSM_AB_LDS_PAD 0
#endif
  const size_t lds = env_bytes * G + LSM_AB_LDS_PAD;
  if (!attr && lds > 65536) {
    HIPCHK(e, hipFuncSetAttribute((const void*)rollout_team_kernel<DYN, NT, G, REXT>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int blocks = (e->cfg.num_envs + G - 1) / G;
  hipLaunchKernelGGL((rollout_team_kernel<DYN, NT, G, REXT>), dim3(blocks), dim3(WAVE * G), lds, st,
                     active_params(e), L);
  return 0;
}

template <int DYN, int NT, bool NIS1, bool REXT>
int launch_block_nis(lsm_env* e, const KStep& L, size_t env_lds, hipStream_t st) {
  static bool attr = false;   // LDS above the 64 KB default needs an explicit opt-in
  if (!attr && env_lds > 65536) {
    HIPCHK(e, hipFuncSetAttribute((const void*)rollout_block_kernel<DYN, NT, NIS1, REXT>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)env_lds));
    attr = true;
  }
  hipLaunchKernelGGL((rollout_block_kernel<DYN, NT, NIS1, REXT>), dim3(e->cfg.num_envs), dim3(BT), env_lds, st,
                     active_params(e), L);
  return 0;
}

template <int DYN, int NT>
int launch_block_t(lsm_env* e, const KStep& L, size_t env_lds, hipStream_t st) {
  if (e->cfg.num_internal_step > 1) return launch_block_nis<DYN, NT, false, true>(e, L, env_lds, st);
  // fill_params' P.rext: reward_finish / reward_shared run only then
  const bool rext = e->cfg.reward_terms != 0 || e->cfg.collaborative;
  return rext ? launch_block_nis<DYN, NT, true, true>(e, L, env_lds, st)
              : launch_block_nis<DYN, NT, true, false>(e, L, env_lds, st);
}


// ---- kernel groups ------------------------------------------------------------------------
// lsm.build compiles this file once per group (-DLSM_PART=g, in parallel) plus once for the host
// code (-DLSM_PART=0, which declares every group's launchers extern); without LSM_PART everything
// is one translation unit (diagnostic builds).
#define LSM_G1(X) X(0, 64, 0) X(0, 32, 0) X(0, 16, 0) X(0, 32, 8) X(0, 64, 3) X(0, 64, 8)
#define LSM_G2(X) X(1, 64, 0) X(1, 32, 0) X(1, 16, 0) X(1, 32, 16) X(1, 64, 3) X(1, 64, 16)
#define LSM_G3(X) X(0, 8, 8, false) X(0, 8, 4, false) X(0, 8, 2, false)
#define LSM_G4(X) X(1, 16, 4, false) X(1, 16, 2, false)
#define LSM_G7(X) X(0, 8, 8, true) X(0, 8, 4, true) X(0, 8, 2, true)
#define LSM_G8(X) X(1, 16, 4, true) X(1, 16, 2, true)
#define LSM_G5(X) X(0, 64) X(0, 0)
#define LSM_G6(X) X(1, 64) X(1, 0)
#define LSM_RT(a, b, c) template void launch_t<a, b, c>(lsm_env*, const KStep&, size_t, hipStream_t);
#define LSM_TT(a, b, c, r) template int launch_team_t<a, b, c, r>(lsm_env*, const KStep&, size_t, hipStream_t);
#define LSM_BK(a, b) template int launch_block_t<a, b>(lsm_env*, const KStep&, size_t, hipStream_t);
#define LSM_RT_E(a, b, c) extern LSM_RT(a, b, c)
#define LSM_TT_E(a, b, c, r) extern LSM_TT(a, b, c, r)
#define LSM_BK_E(a, b) extern LSM_BK(a, b)
#if defined(LSM_PART) && LSM_PART == 0
LSM_G1(LSM_RT_E) LSM_G2(LSM_RT_E) LSM_G3(LSM_TT_E) LSM_G4(LSM_TT_E) LSM_G5(LSM_BK_E) LSM_G6(LSM_BK_E)
LSM_G7(LSM_TT_E) LSM_G8(LSM_TT_E)
#elif defined(LSM_PART) && LSM_PART == 1
LSM_G1(LSM_RT)
#elif defined(LSM_PART) && LSM_PART == 2
LSM_G2(LSM_RT)
#elif defined(LSM_PART) && LSM_PART == 3
LSM_G3(LSM_TT)
#elif defined(LSM_PART) && LSM_PART == 4
LSM_G4(LSM_TT)
#elif defined(LSM_PART) && LSM_PART == 5
LSM_G5(LSM_BK)
#elif defined(LSM_PART) && LSM_PART == 6
LSM_G6(LSM_BK)
#elif defined(LSM_PART) && LSM_PART == 7
LSM_G7(LSM_TT)
#elif defined(LSM_PART) && LSM_PART == 8
LSM_G8(LSM_TT)
#endif

#if LSM_HOST_PART

static void fill_params(const lsm_env* e, KParams& P) {
  memset(&P, 0, sizeof(P));
  const bool di = e->cfg.dynamics == LSM_DOUBLE_INTEGRATOR;
  P.n_envs = e->cfg.num_envs;
  P.N = e->N; P.L = e->L; P.NL = e->NL; P.E = e->E; P.F = e->F; P.OBS = e->OBS;
  P.dyn = di ? 0 : 1;
  P.episode_length = e->cfg.episode_length;
  P.use_masking = e->cfg.use_masking;
  P.use_filter_arg = e->cfg.use_safety_filter;
  P.auto_reset = e->cfg.auto_reset;
  P.adj_compact = e->cfg.adj_layout == LSM_ADJ_COMPACT;
  P.filter_search = e->sel.filter_search == 0 ? 0 : 1;
  P.scenario = e->cfg.scenario;
  P.rng = e->cfg.rng;
  P.nis = e->cfg.num_internal_step > 1 ? e->cfg.num_internal_step : 1;
  P.rbin = e->cfg.reward_terms;
  P.collab = e->cfg.collaborative ? 1 : 0;
  P.rext = (P.rbin != 0 || P.collab) ? 1 : 0;
  P.use_hj = (e->cfg.use_safety_filter || (e->cfg.reward_terms & LSM_REWARD_HJ_VALUE)) ? 1 : 0;
  P.mt_stage = e->mt_stage;
  P.seed = e->cfg.seed;
  P.env_offset = e->cfg.env_offset;
  P.lds_dep_off = (uint32_t)lds_plan(e->N, e->NL, e->E, e->F, e->block).bytes;
  P.lean = e->lean ? 1 : 0;
  P.world_size = e->cfg.world_size;
  const double pi = 3.141592653589793;
  P.pi = pi;
  P.two_pi = 2 * pi;
  if (di) {
    P.dt = 0.1; P.coord_range = 4; P.world_eng = 1.0; P.sep_target = 0.5;
    P.max_speed = 0.5; P.min_speed = 0.0; P.gs_min = 0.1; P.gs_max = 0.5;
    const double opts[5] = {-0.5, -0.25, 0.0, 0.25, 0.5};   // np.linspace(-0.5, 0.5, 5)
    for (int k = 0; k < 5; ++k) { P.act0[k] = opts[k]; P.act1[k] = opts[k]; }
  } else {
    P.dt = 1.0; P.coord_range = 3 * 1.60934; P.world_eng = 1.4; P.sep_target = 1500 * 0.0003048;
    P.max_speed = 175 * 0.514444 * 0.001; P.min_speed = 60 * 0.514444 * 0.001;
    P.gs_min = 60 * 0.514444 * 0.001; P.gs_max = 110 * 0.514444 * 0.001;
    // np.linspace(-0.1, 0.1, 5), np.linspace(-0.001, 0.002, 5)
    const double lo = -0.1, hi = 0.1, alo = -0.001, ahi = 0.002;
    for (int k = 0; k < 5; ++k) {
      P.act0[k] = (k == 4) ? hi : lo + k * ((hi - lo) / 4);
      P.act1[k] = (k == 4) ? ahi : alo + k * ((ahi - alo) / 4);
    }
  }
  {
    double t = P.coord_range * P.coord_range;
    while (std::sqrt(t) > P.coord_range) t = std::nextafter(t, 0.0);
    while (std::sqrt(std::nextafter(t, INFINITY)) <= P.coord_range) t = std::nextafter(t, INFINITY);
    P.coord_range_s = t;
  }
  {   // random_scenario_wave2's band, the device's products (lsm_team.h)
    const double dmin = di ? 0.25 * P.coord_range : 0.5 * P.coord_range;
    const double dmax = di ? 0.75 * P.coord_range : P.coord_range;
    double lo = dmin * dmin;
    while (std::sqrt(lo) > dmin) lo = std::nextafter(lo, 0.0);
    while (std::sqrt(std::nextafter(lo, INFINITY)) <= dmin) lo = std::nextafter(lo, INFINITY);
    double hi = dmax * dmax;
    while (std::sqrt(hi) < dmax) hi = std::nextafter(hi, INFINITY);
    while (std::sqrt(std::nextafter(hi, 0.0)) >= dmax) hi = std::nextafter(hi, 0.0);
    P.scen_d2lo = lo;
    P.scen_d2hi = hi;
  }
  P.cos_pi6 = cos(pi / 6);
  for (int k = 0; k < 50; ++k) {
    const double ph = k * ((2 * pi - 0) / 50);   // np.linspace(0, 2pi, 50, endpoint=False)
    P.mag_c[k] = cos(ph);
    P.mag_s[k] = sin(ph);
  }
  P.di_thr_xmax = 0.5 - 0.1 * 0.5; P.di_thr_xmin = -0.5 - 0.1 * -0.5;
  P.di_thr_ymax = 0.5 - 0.1 * 0.5; P.di_thr_ymin = -0.5 - 0.1 * -0.5;
  P.di_axmax = 0.5; P.di_axmin = -0.5; P.di_aymax = 0.5; P.di_aymin = -0.5;
  P.at_vmax = 175 * 0.514444 * 0.001; P.at_vmin = 60 * 0.514444 * 0.001;
  P.at_amax = 0.002; P.at_amin = -0.001; P.at_wmax = 0.1;
  P.at_thr_amax = P.at_vmax - 1.0 * 0.002; P.at_thr_amin = P.at_vmin - 1.0 * -0.001;
  P.at_box_w = (float)0.1; P.at_box_amax = (float)0.002; P.at_box_amin = (float)-0.001;
  auto magic = [](uint32_t d) { return (uint32_t)((((uint64_t)1 << 32) + d - 1) / d); };
  P.m_E = magic(e->E);
  P.m_EE = magic(e->E * e->E);
  P.m_EF = magic(e->E * e->F);
  P.m_F = magic(e->F);
  P.m_EF4 = magic(e->E * e->F / 4);
  P.m_NL = magic(e->NL);
  P.ttr_max = e->ttr_max;
  P.val_sep0 = e->val_sep0;
  P.val = e->val;
  P.ttr = e->ttr;
  P.s = e->s;
  P.o.obs = (float*)e->out_ptr[LSM_OUT_OBS];
  P.o.node = (float*)e->out_ptr[LSM_OUT_NODE_OBS];
  P.o.adj = (float*)e->out_ptr[LSM_OUT_ADJ];
  P.o.rew = (float*)e->out_ptr[LSM_OUT_REWARD];
  P.o.dones = (uint8_t*)e->out_ptr[LSM_OUT_DONE];
  P.o.reset_flag = (uint8_t*)e->out_ptr[LSM_OUT_RESET_FLAG];
  P.o.ep_info = (double*)e->out_ptr[LSM_OUT_EP_INFO];
  P.o.info = (double*)e->out_ptr[LSM_OUT_INFO];
  P.o.edges = (uint8_t*)e->out_ptr[LSM_OUT_EDGES];
  P.o.state = (double*)e->out_ptr[LSM_OUT_STATE];
  P.o.adjmask = (uint64_t*)e->out_ptr[LSM_OUT_ADJ_MASK];
  P.o.share_obs = (float*)e->out_ptr[LSM_OUT_SHARE_OBS];
  P.o.masks = (float*)e->out_ptr[LSM_OUT_MASKS];
  P.o.active_masks = (float*)e->out_ptr[LSM_OUT_ACTIVE_MASKS];
  P.o.cforce = e->cfg.collision_forces ? (double*)e->out_ptr[LSM_OUT_COLLISION_FORCE] : nullptr;
  P.o.departed = (uint8_t*)e->out_ptr[LSM_OUT_DEPARTED];
  P.o.adjnnz = (int64_t*)e->out_ptr[LSM_OUT_ADJ_NNZ];
  P.stamps = (unsigned long long*)e->out_ptr[LSM_OUT_DEBUG_STAMPS];
  P.diag = 0;
#ifdef LSM_STAMPS
  if (const char* v = getenv("LSM_DIAG")) P.diag = atoi(v);
#endif
  P.pairs = e->pairs;
  P.action_err = e->action_err;
}

extern "C" {

size_t lsm_output_bytes(const lsm_env* e, int32_t slot) {
  const size_t n = e->cfg.num_envs, N = e->N, E = e->E;
  switch (slot) {
    case LSM_OUT_OBS: return n * N * e->OBS * 4;
    case LSM_OUT_NODE_OBS: return n * N * E * e->F * 4;
    case LSM_OUT_ADJ: return (e->cfg.adj_layout == LSM_ADJ_COMPACT ? n : n * N) * E * E * 4;
    case LSM_OUT_ADJ_MASK: return n * N * ((E + 63) / 64) * 8;
    case LSM_OUT_REWARD: return n * N * 4;
    case LSM_OUT_DONE: return n * N;
    case LSM_OUT_RESET_FLAG: return n;
    case LSM_OUT_EP_INFO: return n * 8 * 8;
    case LSM_OUT_INFO: return n * N * LSM_INFO_FIELDS * 8;
    case LSM_OUT_EDGES: return n * E * E;
    case LSM_OUT_STATE: return n * N * 4 * 8;
    case LSM_OUT_DEBUG_STAMPS: return n * LSM_NSTAMP * 8;
    case LSM_OUT_SHARE_OBS: return n * N * N * e->OBS * 4;
    case LSM_OUT_MASKS: return n * N * 4;
    case LSM_OUT_ACTIVE_MASKS: return n * N * 4;
    case LSM_OUT_COLLISION_FORCE: return n * N * 2 * 8;
    case LSM_OUT_DEPARTED: return n * N;
    case LSM_OUT_ADJ_NNZ: return n * N * 8;
    default: return 0;
  }
}

int32_t lsm_num_entities(const lsm_env* e) { return e->E; }
int32_t lsm_layout_doubles(const lsm_env* e) {
  return e ? 4 * e->N + 4 * e->NL + (e->cfg.scenario == LSM_SCENARIO_DEPARTURES ? 3 * e->N : 0) + 1 : 0;
}
int32_t lsm_node_features(const lsm_env* e) { return e->F; }
int32_t lsm_obs_dim(const lsm_env* e) { return e->OBS; }
const char* lsm_last_error(const lsm_env* e) { return e ? e->err.c_str() : "null handle"; }

int lsm_create(const lsm_config* cfg, lsm_env** out) { return lsm_create_select(cfg, nullptr, out); }

int lsm_create_select(const lsm_config* cfg, const lsm_kernel_select* sel, lsm_env** out) {
  *out = nullptr;
  if (!cfg) return 1;
  lsm_env* e = new lsm_env();
  *out = e;
  e->cfg = *cfg;
  if (sel) {
    e->sel = *sel;
  } else {
    memset(&e->sel, 0, sizeof(e->sel));
    e->sel.team = -1;
    e->sel.lean = -1;
    e->sel.filter_search = -1;
  }
  {
    const lsm_kernel_select& s = e->sel;
    if (s.workgroup_per_env != 0 && s.workgroup_per_env != 1) return fail(e, "kernel select: workgroup_per_env must be 0 or 1");
    if (s.generic != 0 && s.generic != 1) return fail(e, "kernel select: generic must be 0 or 1");
    if (s.lanes_per_env != 0 && s.lanes_per_env != 16 && s.lanes_per_env != 32 && s.lanes_per_env != 64)
      return fail(e, "kernel select: lanes_per_env must be 0, 16, 32 or 64");
    if (s.team != -1 && s.team != 0 && s.team != 2 && s.team != 4 && s.team != 8)
      return fail(e, "kernel select: team must be -1, 0, 2, 4 or 8");
    if (s.lean < -1 || s.lean > 1) return fail(e, "kernel select: lean must be -1, 0 or 1");
    if (s.filter_search < -1 || s.filter_search > 1) return fail(e, "kernel select: filter_search must be -1, 0 or 1");
    if (s.bounds_shift < 0 || s.bounds_shift > 4) return fail(e, "kernel select: bounds_shift must be in [0, 4]");
  }
  e->tables_ok = false;
  e->dparams = nullptr;
  for (int k = 0; k < LSM_NUM_OUT; ++k) {
    e->ring_base[k] = nullptr; e->ring_stride[k] = 0; e->ring_count[k] = 0; e->ring_off[k] = 0;
  }
  e->ring_len = 0; e->ring_cap = 0; e->ring_sel = -1; e->dring = nullptr;
  e->params_dirty = true;
  e->ttr_max = 0.0;
  e->val_sep0 = e->sep_last = 0.0;
  e->sep_changes = 0;
  memset(&e->val, 0, sizeof(e->val));
  memset(&e->ttr, 0, sizeof(e->ttr));
  for (int k = 0; k < LSM_NUM_OUT; ++k) { e->out_ptr[k] = nullptr; e->out_bytes[k] = 0; }
  const int N = cfg->num_agents, L = cfg->num_landmarks;
  if (cfg->dynamics != LSM_DOUBLE_INTEGRATOR && cfg->dynamics != LSM_AIRTAXI)
    return fail(e, "dynamics must be LSM_DOUBLE_INTEGRATOR or LSM_AIRTAXI");
  if (N < 2 || N > BMAXN) return fail(e, "num_agents must be in [2, 64]");
  if (L < (cfg->scenario == LSM_SCENARIO_TRAIN ? 2 : 1) || L > MAX_L)
    return fail(e, "num_landmarks must be in [2, 8] (the training scenario asserts > 1, utils.py:31; "
                   "layout scenarios: [1, 8])");
  if (N * (1 + L) > BMAXE) return fail(e, "N * (1 + L) must be <= 256");
  if (N * L - 1 > 127) return fail(e, "landmark ids go through np.int8 (navigation_graph_safe.py:581)");
  if (cfg->adj_layout != LSM_ADJ_REFERENCE && cfg->adj_layout != LSM_ADJ_COMPACT)
    return fail(e, "adj_layout must be LSM_ADJ_REFERENCE or LSM_ADJ_COMPACT");
  if (cfg->scenario < LSM_SCENARIO_TRAIN || cfg->scenario > LSM_SCENARIO_DEPARTURES)
    return fail(e, "scenario must be LSM_SCENARIO_TRAIN, _LAYOUT or _DEPARTURES");
  if (cfg->rng != LSM_RNG_MT19937 && cfg->rng != LSM_RNG_PHILOX)
    return fail(e, "rng must be LSM_RNG_MT19937 or LSM_RNG_PHILOX");
  if (cfg->scenario != LSM_SCENARIO_TRAIN) {
    if (cfg->auto_reset)
      return fail(e, "layout scenarios are evaluation paths (GraphDummyVecEnv, scripts/eval_mpe.py): auto_reset must be 0");
    if (cfg->rng != LSM_RNG_MT19937) return fail(e, "layout scenarios draw on the host: rng must be LSM_RNG_MT19937");
  }
  if (cfg->scenario == LSM_SCENARIO_DEPARTURES && cfg->dynamics != LSM_AIRTAXI)
    return fail(e, "departure timers need airtaxi dynamics (RealisticScenario calls "
                   "reset_velocity(theta, speed), KinematicVehicleXYState only, core.py:137)");
  e->block = N > MAXN || N * (1 + L) > MAXE || e->sel.workgroup_per_env == 1;
  if (cfg->num_envs < 1) return fail(e, "num_envs must be >= 1");
  if (cfg->num_internal_step < 0 || cfg->num_internal_step > 64)
    return fail(e, "num_internal_step must be in [0, 64] (0 and 1: one inner step)");
  if (cfg->episode_length < 1) return fail(e, "episode_length must be >= 1");
  if (cfg->reward_terms & ~LSM_REWARD_ALL)
    return fail(e, "reward_terms: unknown LSM_REWARD_* bits (RewardBinaryConfig has four optional terms, "
                   "multiagent/config.py:78-83)");
  if (cfg->collaborative != 0 && cfg->collaborative != 1) return fail(e, "collaborative must be 0 or 1");
  e->N = N; e->L = L; e->NL = N * L; e->E = N * (1 + L);
  e->F = cfg->dynamics == LSM_DOUBLE_INTEGRATOR ? 10 : 11;
  e->OBS = cfg->dynamics == LSM_DOUBLE_INTEGRATOR ? 7 : 6;
  // Lanes per env: 64 = one env per wave (default; measured fastest at 4096 envs, where
  // 4 waves/SIMD hide LDS/HBM latency), 32/16 = 2/4 envs per wave sharing the per-agent
  // instruction stream (needs N <= lanes). sel.lanes_per_env overrides.
  e->lpe = e->sel.lanes_per_env ? e->sel.lanes_per_env : 64;
  e->generic_only = e->sel.generic == 1;
  if (e->block) e->lpe = 64;   // lanes_per_env applies to the one-wave kernel only
  if (cfg->scenario != LSM_SCENARIO_TRAIN) {   // layouts: the generic one-wave kernel (mode 2 resets)
    e->generic_only = true;
    e->lpe = 64;
  }
  // Team kernel (lsm_team.h) for the compile-time-N BASELINE agent counts: G envs per
  // workgroup share one wave for their per-agent phases. sel.team = 0 selects rollout_kernel,
  // sel.team = G another instantiated G.
  e->team = 0;
  // the team kernel runs World.step's inner loop once (num_internal_step = 1, the training
  // default, train.sh:35); more inner steps run in rollout_kernel / the workgroup kernel
  if (!e->block && e->lpe == 64 && L == 2 && !e->generic_only && cfg->num_internal_step <= 1) {
    if (cfg->dynamics == LSM_DOUBLE_INTEGRATOR && N == 8) e->team = 4;   // measured: 4 < 8 < 2 (us/step)
    if (cfg->dynamics == LSM_AIRTAXI && N == 16) e->team = 4;   // lean LDS: 4 < 2 < 0 (us/step)
    const int g = e->sel.team;
    if (g == 0) e->team = 0;
    else if (g > 0 && e->team && g * N <= 64) e->team = g;
    else if (g > 0 && e->team) return fail(e, "kernel select: team * num_agents must be <= 64");
  }
  // lean LDS layout for the airtaxi team kernel (6 -> 8 envs per CU at N = 16);
  // sel.lean = 0 keeps the full table (A/B)
  e->lean = e->team && cfg->dynamics == LSM_AIRTAXI && (N & 3) == 0 && (e->E & 3) == 0;
  if (e->sel.lean == 0) e->lean = false;
  if (!(e->lpe == 16 || e->lpe == 32 || e->lpe == 64) || e->lpe < (e->block ? 1 : N))
    return fail(e, "kernel select: lanes_per_env must be 16, 32 or 64 and >= num_agents");
  HIPCHK(e, hipGetDevice(&e->device));
  const size_t n = cfg->num_envs;
  int r = 0;
  const LdsPlan lp = lds_plan(N, e->NL, e->E, e->F, e->block);
  e->s.rec16 = (uint32_t)(lp.rec / 16);
  e->s.a1_16 = (uint32_t)(lp.a1 / 16);
  e->s.a2_16 = (uint32_t)(lp.a2 / 16);
  e->s.a3_16 = (uint32_t)(lp.a3 / 16);
  e->s.rec_stride16 = (uint32_t)(((lp.rec + 127) / 128) * 8);   // 128-B aligned records
  r |= dalloc(e, &e->s.rec, n * e->s.rec_stride16);
  r |= dalloc(e, &e->s.prev, n * 8);
  r |= dalloc(e, &e->dparams, 1);
  r |= dalloc(e, &e->s.mt, n * MT_WORDS);
  r |= dalloc(e, &e->pairs, (size_t)e->E * (e->E - 1) / 2 + 1);
  r |= dalloc(e, &e->action_err, 1);
  e->s.dep = nullptr;
  e->s.sepx = nullptr;
  e->s.sepx_cap = 0;
  if (cfg->scenario == LSM_SCENARIO_DEPARTURES) r |= dalloc(e, &e->s.dep, n * depw(N));
  if (r) return 1;
  if (e->s.dep) {   // Agent.departed defaults to True (core.py:343), timers 0
    std::vector<double> d(n * depw(N), 0.0);
    for (size_t k = 0; k < n; ++k)
      for (int i = 0; i < N; ++i) d[k * depw(N) + i] = 1.0;
    HIPCHK(e, hipMemcpy(e->s.dep, d.data(), d.size() * 8, hipMemcpyHostToDevice));
  }
  HIPCHK(e, hipMemset(e->action_err, 0, sizeof(int32_t)));
  {
    // agent-agent pairs first (the only ones needing the float64 blocks), then
    // agent-landmark, then landmark-landmark: the agent block stays in the first lane pass
    std::vector<uint16_t> pr;
    for (int cls = 0; cls < 3; ++cls)
      for (int a = 0; a < e->E; ++a)
        for (int b = a + 1; b < e->E; ++b) {
          const int c = (a < N ? 0 : 1) + (b < N ? 0 : 1);
          if (c == cls) pr.push_back((uint16_t)(a | (b << 8)));
        }
    pr.push_back(0);
    HIPCHK(e, hipMemcpy(e->pairs, pr.data(), pr.size() * 2, hipMemcpyHostToDevice));
  }
  {
    // reference initial values: prev summary (environment.py:873-881), stats and info
    // accumulators (init_episode_agent_info), decon -1, min distances inf
    const size_t stride = (size_t)e->s.rec_stride16 * 16;
    std::vector<unsigned char> rec(stride, 0);
    double* stats = (double*)(rec.data() + lp.off[1]);
    double* winfo = (double*)(rec.data() + lp.off[2]);
    double* gmt = (double*)(rec.data() + lp.off[4]);
    double* minrel = (double*)(rec.data() + lp.off[5]);
    int32_t* decon = (int32_t*)(rec.data() + lp.off[10]);
    for (int i = 0; i < N; ++i) {
      stats[4 * N + i] = INFINITY;
      for (int q = 0; q < 3; ++q) winfo[q * N + i] = -1.0;
      winfo[3 * N + i] = 0.0;
      gmt[i] = INFINITY;
      minrel[i] = INFINITY;
      decon[i] = -1;
    }
    std::vector<unsigned char> all(n * stride);
    for (size_t k = 0; k < n; ++k) memcpy(all.data() + k * stride, rec.data(), stride);
    HIPCHK(e, hipMemcpy(e->s.rec, all.data(), all.size(), hipMemcpyHostToDevice));
    std::vector<double> prev(n * 8, 0.0);
    for (size_t k = 0; k < n; ++k) prev[k * 8 + 0] = cfg->episode_length;
    HIPCHK(e, hipMemcpy(e->s.prev, prev.data(), prev.size() * 8, hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL(seed_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, e->s.mt, (int)n, cfg->seed,
                     cfg->env_offset);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipDeviceSynchronize());
  e->tables_ok = !uses_hj(e) && cfg->dynamics == LSM_DOUBLE_INTEGRATOR;
  return 0;
}

void lsm_destroy(lsm_env* e) {
  if (!e) return;
  for (void* p : e->allocs) (void)hipFree(p);
  delete e;
}

// Free one of the handle's allocations (a replaced table).
static void dfree(lsm_env* e, const void* p) {
  if (!p) return;
  for (size_t k = 0; k < e->allocs.size(); ++k)
    if (e->allocs[k] == p) {
      (void)hipFree(e->allocs[k]);
      e->allocs.erase(e->allocs.begin() + k);
      return;
    }
}

static int upload_table(lsm_env* e, TableDev& T, int32_t ndim, const double* lo, const double* hi,
                        const int32_t* shape, const int32_t* periodic, const float* values,
                        const float* grads) {
  if (ndim < 1 || ndim > 5) return fail(e, "table ndim must be in [1, 5]");
  HIPCHK(e, hipDeviceSynchronize());   // a replaced table may still be read by queued launches
  dfree(e, T.cells);
  dfree(e, T.gcells);
  dfree(e, T.bnd);
  memset(&T, 0, sizeof(T));
  T.ndim = ndim;
  size_t nodes = 1, cells = 1;
  for (int d = 0; d < ndim; ++d) {
    if (shape[d] < 2) return fail(e, "table dims must have >= 2 nodes");
    nodes *= (size_t)shape[d];
    cells *= (size_t)(periodic[d] ? shape[d] : shape[d] - 1);
  }
  size_t cst = 1;
  for (int d = ndim - 1; d >= 0; --d) {
    T.n[d] = shape[d];
    T.cstride[d] = (int)cst;
    cst *= (size_t)(periodic[d] ? shape[d] : shape[d] - 1);
    T.periodic[d] = periodic[d] ? 1 : 0;
    const double sp = T.periodic[d] ? (hi[d] - lo[d]) / shape[d] : (hi[d] - lo[d]) / (shape[d] - 1.0);
    T.lo[d] = (float)lo[d];
    T.sp[d] = (float)sp;
  }
  // grid_pos's reciprocal path, per dimension, where it equals the division for every y = s - lo
  // a lookup can meet: grid positions within [-4, n + 3] (non-periodic: outside, the lookup is out
  // of the grid either way -- a faithful quotient cannot cross those bounds) or within 1e9 in
  // magnitude (periodic: the wrap reads the position itself; beyond 1e9 grid_cell refuses it)
  {
    int* bad = nullptr;
    HIPCHK(e, hipMalloc((void**)&bad, sizeof(int)));
#ifdef LSM_DIAGNOSTIC_BUILD
    const bool no_mdiv = getenv("LSM_NO_MDIV") != nullptr;   // A/B of the division path (variant builds)
#else
    const bool no_mdiv = false;   // the product reads no environment knobs
#endif
    for (int d = 0; d < ndim; ++d) {
      T.rsp[d] = 1.0f / T.sp[d];
      T.mdiv[d] = 0;
      if (!(T.sp[d] > 0.0f) || no_mdiv) continue;
      const float plo = T.periodic[d] ? -1.0e9f : -4.0f;
      const float phi = T.periodic[d] ? 1.0e9f : (float)(T.n[d] + 3);
      const float ypos = phi * T.sp[d] * 1.0001f, yneg = -plo * T.sp[d] * 1.0001f;
      uint32_t pb, nb;
      memcpy(&pb, &ypos, 4);
      memcpy(&nb, &yneg, 4);
      HIPCHK(e, hipMemset(bad, 0, sizeof(int)));
      hipLaunchKernelGGL(mdiv_check_kernel, dim3(4096), dim3(256), 0, 0, T.sp[d], T.rsp[d], pb, nb, bad);
      HIPCHK(e, hipGetLastError());
      int h = 1;
      HIPCHK(e, hipMemcpy(&h, bad, sizeof(int), hipMemcpyDeviceToHost));
      T.mdiv[d] = h == 0 ? 1 : 0;
    }
    HIPCHK(e, hipFree(bad));
  }
  const size_t ncorner = (size_t)1 << ndim;
  if (cells * ncorner * 2 > (size_t)INT32_MAX) return fail(e, "table too large for 32-bit cell offsets");
  T.gw = ndim <= 4 ? 1 : 2;
  float* dv = nullptr;
  float4* dg = nullptr;
  HIPCHK(e, hipMalloc((void**)&dv, nodes * 4));
  HIPCHK(e, hipMemcpy(dv, values, nodes * 4, hipMemcpyHostToDevice));
  if (grads) {
    HIPCHK(e, hipMalloc((void**)&dg, nodes * T.gw * 16));
    HIPCHK(e, hipMemcpy(dg, grads, nodes * T.gw * 16, hipMemcpyHostToDevice));
  }
  float* cv = nullptr;
  float4* cg = nullptr;
  if (dalloc(e, &cv, cells * ncorner)) return 1;
  if (grads && dalloc(e, &cg, cells * ncorner * T.gw)) return 1;
  const int64_t work = (int64_t)(cells * ncorner);
  hipLaunchKernelGGL(expand_cells_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, 0, dv, dg, cv, cg,
                     T, (int64_t)cells);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipDeviceSynchronize());
  HIPCHK(e, hipFree(dv));
  if (dg) HIPCHK(e, hipFree(dg));
  T.cells = cv;
  T.gcells = cg;
  return 0;
}

// Value bounds per 4^ndim-cell block (TableDev::bnd), built from the node table.
static int upload_bounds(lsm_env* e, TableDev& T, const float* values) {
  // 4 cells per dim: 180 KB for the full DI table (L2-resident); sel.bounds_shift for tests
  T.bshift = e->sel.bounds_shift ? e->sel.bounds_shift : 2;
  const int B = 1 << T.bshift;
  int nblocks = 1;
  for (int d = T.ndim - 1; d >= 0; --d) {
    const int ncell = T.periodic[d] ? T.n[d] : T.n[d] - 1;
    T.bstride[d] = nblocks;
    nblocks *= (ncell + B - 1) / B;
  }
  size_t nodes = 1;
  for (int d = 0; d < T.ndim; ++d) nodes *= (size_t)T.n[d];
  float* dv = nullptr;
  HIPCHK(e, hipMalloc((void**)&dv, nodes * 4));
  HIPCHK(e, hipMemcpy(dv, values, nodes * 4, hipMemcpyHostToDevice));
  float2* bd = nullptr;
  if (dalloc(e, &bd, (size_t)nblocks)) return 1;
  hipLaunchKernelGGL(bounds_kernel, dim3((nblocks + 255) / 256), dim3(256), 0, 0, dv, bd, T, nblocks);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipDeviceSynchronize());
  HIPCHK(e, hipFree(dv));
  T.bnd = bd;
  return 0;
}

int lsm_set_value_table(lsm_env* e, int32_t ndim, const double* lo, const double* hi, const int32_t* shape,
                        const int32_t* periodic, const float* values, const float* grads,
                        double separation_distance) {
  const int want = e->cfg.dynamics == LSM_DOUBLE_INTEGRATOR ? 4 : 5;
  if (ndim != want) return fail(e, "value table must be 4-D (double integrator) or 5-D (airtaxi)");
  if (!grads) return fail(e, "value table needs its gradient table");
  if (upload_table(e, e->val, ndim, lo, hi, shape, periodic, values, grads)) return 1;
  if (upload_bounds(e, e->val, values)) return 1;
  e->val_sep0 = e->sep_last = separation_distance;
  e->sep_changes = 0;
  {
    const LdsPlan lp = lds_plan(e->N, e->NL, e->E, e->F, e->block);
    const int n = e->cfg.num_envs;
    hipLaunchKernelGGL(sep_clear_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, e->s.rec, e->s.rec_stride16, n,
                       (uint32_t)(lp.off[12] + 8 * NCUR));
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipDeviceSynchronize());
  }
  e->tables_ok = (e->cfg.dynamics == LSM_DOUBLE_INTEGRATOR) || e->ttr.cells != nullptr;
  e->params_dirty = true;
  return 0;
}

int lsm_set_ttr_table(lsm_env* e, int32_t ndim, const double* lo, const double* hi, const int32_t* shape,
                      const int32_t* periodic, const float* values, double ttr_max) {
  if (ndim != 4) return fail(e, "TTR table must be 4-D");
  if (upload_table(e, e->ttr, ndim, lo, hi, shape, periodic, values, nullptr)) return 1;
  e->ttr_max = ttr_max;
  e->tables_ok = !uses_hj(e) || e->val.cells != nullptr;
  e->params_dirty = true;
  return 0;
}

int lsm_bind_output(lsm_env* e, int32_t slot, void* ptr, size_t bytes) {
  if (slot < 0 || slot >= LSM_NUM_OUT) return fail(e, "bad output slot");
  const size_t need = lsm_output_bytes(e, slot);
  if (ptr && bytes < need) return fail(e, "output buffer too small for slot " + std::to_string(slot));
  e->out_ptr[slot] = ptr;
  e->params_dirty = true;
  e->out_bytes[slot] = bytes;
  return 0;
}

int lsm_bind_output_ring(lsm_env* e, int32_t slot, void* base, size_t stride_bytes, int32_t count,
                         int32_t index_offset) {
  if (!e) return 1;
  if (slot < 0 || slot >= LSM_NUM_OUT) return fail(e, "bad output slot");
  if (slot == LSM_OUT_RESET_FLAG || slot == LSM_OUT_EP_INFO || slot == LSM_OUT_EDGES ||
      slot == LSM_OUT_DEBUG_STAMPS || slot == LSM_OUT_DEPARTED || slot == LSM_OUT_ADJ_NNZ)
    return fail(e, "slot " + std::to_string(slot) + " cannot be ring-bound");
  if (count <= 0 || !base) {   // unbind
    e->ring_count[slot] = 0;
  } else {
    if (stride_bytes < lsm_output_bytes(e, slot))
      return fail(e, "ring stride smaller than slot " + std::to_string(slot) + "'s output");
    e->ring_base[slot] = base;
    e->ring_stride[slot] = stride_bytes;
    e->ring_count[slot] = count;
    e->ring_off[slot] = index_offset;
  }
  int len = 0;
  for (int s = 0; s < LSM_NUM_OUT; ++s)
    if (e->ring_count[s] > 0) len = std::max(len, e->ring_count[s] - e->ring_off[s]);
  e->ring_len = len;
  if (e->ring_sel >= len) e->ring_sel = -1;
  e->params_dirty = true;
  return 0;
}

int lsm_select_ring(lsm_env* e, int32_t index) {
  if (!e) return 1;
  if (index < -1 || index >= e->ring_len)
    return fail(e, "ring index " + std::to_string(index) + " outside [-1, " + std::to_string(e->ring_len) + ")");
  e->ring_sel = index;
  return 0;
}

static int check_ready(lsm_env* e, bool stepping) {
  if (!e->tables_ok) return fail(e, "HJ value table (filter on) / TTR table (airtaxi) not set");
  const int req[] = {LSM_OUT_OBS, LSM_OUT_NODE_OBS, LSM_OUT_ADJ, LSM_OUT_REWARD, LSM_OUT_DONE,
                     LSM_OUT_RESET_FLAG, LSM_OUT_EP_INFO, LSM_OUT_INFO};
  for (int s : req)
    if (!e->out_ptr[s]) return fail(e, "output slot " + std::to_string(s) + " not bound");
  if (e->cfg.adj_layout == LSM_ADJ_COMPACT && !e->out_ptr[LSM_OUT_ADJ_MASK])
    return fail(e, "compact adjacency layout needs LSM_OUT_ADJ_MASK bound");
  if (e->cfg.collision_forces && !e->out_ptr[LSM_OUT_COLLISION_FORCE])
    return fail(e, "collision_forces needs LSM_OUT_COLLISION_FORCE bound");
  if (e->block && e->out_ptr[LSM_OUT_ADJ_NNZ])
    return fail(e, "LSM_OUT_ADJ_NNZ is written by the one-wave and team kernels (E <= 64); the workgroup-per-env "
                   "kernel's edge lists take lsm_edges_count's pass");
  (void)stepping;
  return 0;
}

// An env's shift chain grows only at its resets, by one entry per change of the separation it
// resets with, so the changes across the calls' curriculum blocks since the table upload bound every
// chain. The record holds KSEP shifts; before a launch that could write shift k >= KSEP the per-env
// overflow rows (StateDev::sepx) are grown, stream-ordered, keeping the shifts already there. The
// reference has no bound (HjDataHandle.update_separation_distance shifts the table in place,
// safety_filter.py:170-174); neither has this.
static int sep_check(lsm_env* e, const lsm_curriculum* cur, hipStream_t st) {
  if (!uses_hj(e)) return 0;
  if (cur->separation_distance == e->sep_last) return 0;
  // the overflow rows are grown first; the change is recorded only once they can hold it, so a
  // failed allocation leaves the handle as it was (a retry grows them again)
  const int changes = e->sep_changes + 1;
  const uint32_t need = changes > KSEP ? (uint32_t)(changes - KSEP) : 0;
  if (need > e->s.sepx_cap) {
    const uint32_t cap = std::max<uint32_t>(std::max<uint32_t>(2 * e->s.sepx_cap, 16), need);
    const size_t n = (size_t)e->cfg.num_envs;
    double* nx = nullptr;
    if (dalloc(e, &nx, n * cap)) return 1;
    if (e->s.sepx) {
      if (hipMemcpy2DAsync(nx, (size_t)cap * 8, e->s.sepx, (size_t)e->s.sepx_cap * 8, (size_t)e->s.sepx_cap * 8, n,
                           hipMemcpyDeviceToDevice, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess) {
        dfree(e, nx);
        return fail(e, "growing the HJ separation shift rows failed");
      }
      dfree(e, e->s.sepx);
    }
    e->s.sepx = nx;
    e->s.sepx_cap = cap;
    e->params_dirty = true;
  }
  e->sep_changes = changes;
  e->sep_last = cur->separation_distance;
  return 0;
}

// output pointers of ring index i (see lsm_env::ring_*)
static void apply_ring(const lsm_env* e, int i, KParams& P) {
  auto at = [&](int slot, void* plain) -> void* {
    if (e->ring_count[slot] <= 0) return plain;
    const int j = i + e->ring_off[slot];
    if (j < 0 || j >= e->ring_count[slot]) return plain;
    return (char*)e->ring_base[slot] + (size_t)j * e->ring_stride[slot];
  };
  P.o.obs = (float*)at(LSM_OUT_OBS, P.o.obs);
  P.o.node = (float*)at(LSM_OUT_NODE_OBS, P.o.node);
  P.o.adj = (float*)at(LSM_OUT_ADJ, P.o.adj);
  P.o.rew = (float*)at(LSM_OUT_REWARD, P.o.rew);
  P.o.dones = (uint8_t*)at(LSM_OUT_DONE, P.o.dones);
  P.o.info = (double*)at(LSM_OUT_INFO, P.o.info);
  P.o.state = (double*)at(LSM_OUT_STATE, P.o.state);
  P.o.adjmask = (uint64_t*)at(LSM_OUT_ADJ_MASK, P.o.adjmask);
  P.o.share_obs = (float*)at(LSM_OUT_SHARE_OBS, P.o.share_obs);
  P.o.masks = (float*)at(LSM_OUT_MASKS, P.o.masks);
  P.o.active_masks = (float*)at(LSM_OUT_ACTIVE_MASKS, P.o.active_masks);
  P.o.cforce = (double*)at(LSM_OUT_COLLISION_FORCE, P.o.cforce);
}

static int launch(lsm_env* e, KStep& L, hipStream_t st) {
  size_t env_lds = lds_plan(e->N, e->NL, e->E, e->F, e->block, e->lean).bytes;
  if (e->team) env_lds = team_env_bytes(env_lds, e->N);
  if (e->cfg.scenario == LSM_SCENARIO_DEPARTURES) env_lds += dep_lds_bytes(e->N);
  if (e->block ? env_lds > 160 * 1024
               : (e->team ? env_lds * e->team > 160 * 1024 : env_lds * (WAVE / e->lpe) > 65536))
    return fail(e, "LDS footprint too large");
  if (e->params_dirty) {   // outputs / tables changed: refresh the device copy (stream-ordered)
    KParams P;
    fill_params(e, P);
    P.lds_env_bytes = (uint32_t)env_lds;
    HIPCHK(e, hipMemcpyAsync(e->dparams, &P, sizeof(P), hipMemcpyHostToDevice, st));
    if (e->ring_len > 0) {
      if (e->ring_cap < e->ring_len) {
        if (dalloc(e, &e->dring, (size_t)e->ring_len)) return 1;
        e->ring_cap = e->ring_len;
      }
      std::vector<KParams> ring((size_t)e->ring_len);
      for (int i = 0; i < e->ring_len; ++i) {
        ring[i] = P;
        apply_ring(e, i, ring[i]);
      }
      HIPCHK(e, hipMemcpyAsync(e->dring, ring.data(), sizeof(KParams) * ring.size(), hipMemcpyHostToDevice, st));
    }
    HIPCHK(e, hipStreamSynchronize(st));
    e->params_dirty = false;
  }
  L.stop_after = -1;
#ifdef LSM_STAMPS
  if (const char* v = getenv("LSM_STOP_AFTER")) L.stop_after = atoi(v);
#endif
  const bool di = e->cfg.dynamics == LSM_DOUBLE_INTEGRATOR;
  if (e->block) {
    // workgroup per env; compile-time N = 64 (config 5) or the generic kernel
    const bool spec64 = e->N == 64 && e->L == 2 && !e->generic_only;
    int rc;
    if (di) rc = spec64 ? launch_block_t<0, 64>(e, L, env_lds, st) : launch_block_t<0, 0>(e, L, env_lds, st);
    else rc = spec64 ? launch_block_t<1, 64>(e, L, env_lds, st) : launch_block_t<1, 0>(e, L, env_lds, st);
    if (rc) return rc;
    HIPCHK(e, hipGetLastError());
    return 0;
  }
  if (e->team) {
    int rc = 1;
    // fill_params' P.rext: the kernel without the optional-reward block unless it can run
    const bool rext = e->cfg.reward_terms != 0 || e->cfg.collaborative;
    if (di) {
      if (e->team == 8) rc = rext ? launch_team_t<0, 8, 8, true>(e, L, env_lds, st) : launch_team_t<0, 8, 8, false>(e, L, env_lds, st);
      else if (e->team == 4) rc = rext ? launch_team_t<0, 8, 4, true>(e, L, env_lds, st) : launch_team_t<0, 8, 4, false>(e, L, env_lds, st);
      else rc = rext ? launch_team_t<0, 8, 2, true>(e, L, env_lds, st) : launch_team_t<0, 8, 2, false>(e, L, env_lds, st);
    } else {
      if (e->team == 4) rc = rext ? launch_team_t<1, 16, 4, true>(e, L, env_lds, st) : launch_team_t<1, 16, 4, false>(e, L, env_lds, st);
      else rc = rext ? launch_team_t<1, 16, 2, true>(e, L, env_lds, st) : launch_team_t<1, 16, 2, false>(e, L, env_lds, st);
    }
    if (rc) return rc;
    HIPCHK(e, hipGetLastError());
    return 0;
  }
  // specialised kernels (compile-time N, L = 2, one env per wave) for the BASELINE agent
  // counts; everything else runs the generic kernel (runtime dims, LPE 64/32/16)
  const bool spec = e->lpe == 64 && e->L == 2 && !e->generic_only;
  const bool spec32 = e->lpe == 32 && e->L == 2 && !e->generic_only;
  if (spec32 && di && e->N == 8) launch_t<0, 32, 8>(e, L, env_lds, st);
  else if (spec32 && !di && e->N == 16) launch_t<1, 32, 16>(e, L, env_lds, st);
  else if (spec && di && e->N == 3) launch_t<0, 64, 3>(e, L, env_lds, st);
  else if (spec && di && e->N == 8) launch_t<0, 64, 8>(e, L, env_lds, st);
  else if (spec && !di && e->N == 3) launch_t<1, 64, 3>(e, L, env_lds, st);
  else if (spec && !di && e->N == 16) launch_t<1, 64, 16>(e, L, env_lds, st);
  else {
    const int k = (di ? 0 : 4) + (e->lpe == 64 ? 0 : e->lpe == 32 ? 1 : e->lpe == 16 ? 2 : 3);
    switch (k) {
      case 0: launch_t<0, 64, 0>(e, L, env_lds, st); break;
      case 1: launch_t<0, 32, 0>(e, L, env_lds, st); break;
      case 2: launch_t<0, 16, 0>(e, L, env_lds, st); break;
      case 4: launch_t<1, 64, 0>(e, L, env_lds, st); break;
      case 5: launch_t<1, 32, 0>(e, L, env_lds, st); break;
      case 6: launch_t<1, 16, 0>(e, L, env_lds, st); break;
      default: return fail(e, "unsupported lanes-per-env");
    }
  }
  HIPCHK(e, hipGetLastError());
  return 0;
}

#ifndef LSM_BUILD_ID
#define LSM_BUILD_ID "unknown"
#endif
const char* lsm_build_id(void) { return LSM_BUILD_ID; }

int lsm_test_set_mt_stage(lsm_env* e, int32_t words) {
  if (!e) return 1;
  e->mt_stage = std::max(1, std::min(2 * MT_N, (int)words));
  e->params_dirty = true;
  return 0;
}

// The kernel launch() dispatches to for this handle (same selection as launch()).
const char* lsm_kernel_name(const lsm_env* e) {
  static thread_local std::string name;
  if (!e) return "";
  const bool di = e->cfg.dynamics == LSM_DOUBLE_INTEGRATOR;
  const int D = di ? 0 : 1;
  const char* rext = (e->cfg.reward_terms != 0 || e->cfg.collaborative) ? "true" : "false";
  if (e->block) {
    const bool spec64 = e->N == 64 && e->L == 2 && !e->generic_only;
    const bool nis1 = e->cfg.num_internal_step <= 1;
    name = "rollout_block_kernel<" + std::to_string(D) + ", " + std::to_string(spec64 ? 64 : 0) + ", " +
           (nis1 ? "true" : "false") + ", " + (nis1 ? rext : "true") + ">";
  } else if (e->team) {
    name = "rollout_team_kernel<" + std::to_string(D) + ", " + std::to_string(e->N) + ", " + std::to_string(e->team) +
           ", " + rext + ">";
  } else {
    const bool specN = e->L == 2 && !e->generic_only &&
                       ((e->lpe == 64 && ((di && (e->N == 3 || e->N == 8)) || (!di && (e->N == 3 || e->N == 16)))) ||
                        (e->lpe == 32 && ((di && e->N == 8) || (!di && e->N == 16))));
    name = "rollout_kernel<" + std::to_string(D) + ", " + std::to_string(e->lpe) + ", " +
           std::to_string(specN ? e->N : 0) + ">";
  }
  return name.c_str();
}

int lsm_set_agent_state(lsm_env* e, int32_t env_index, const double* state, const int32_t* reached,
                        void* stream) {
  if (!e || !state) return 1;
  if (env_index < 0 || env_index >= e->cfg.num_envs) return fail(e, "env_index out of range");
  HIPCHK(e, hipStreamSynchronize((hipStream_t)stream));
  const LdsPlan lp = lds_plan(e->N, e->NL, e->E, e->F, e->block);
  std::vector<unsigned char> rec(lp.rec);
  float4* dev = e->s.rec + (size_t)env_index * e->s.rec_stride16;
  HIPCHK(e, hipMemcpy(rec.data(), dev, lp.rec, hipMemcpyDeviceToHost));
  double* ps = (double*)(rec.data() + lp.off[0]);   // record field 0: agent state [4][N]
  for (int i = 0; i < e->N; ++i)
    for (int c = 0; c < 4; ++c) ps[c * e->N + i] = state[i * 4 + c];
  if (reached) {
    int32_t* rp = (int32_t*)(rec.data() + lp.off[8]);   // record field 8: reached_goal
    for (int i = 0; i < e->N; ++i) rp[i] = reached[i];
  }
  ((int32_t*)(rec.data() + lp.off[11]))[1] = 1;   // step slot: distances recomputed, unmasked
  HIPCHK(e, hipMemcpy(dev, rec.data(), lp.rec, hipMemcpyHostToDevice));
  return 0;
}

int lsm_reset(lsm_env* e, const lsm_curriculum* cur, void* stream) {
  if (!e || !cur) return 1;
  if (e->cfg.scenario != LSM_SCENARIO_TRAIN) return fail(e, "layout scenario: reset with lsm_reset_layout");
  if (check_ready(e, false)) return 1;
  if (sep_check(e, cur, (hipStream_t)stream)) return 1;
  KStep L;
  memset(&L, 0, sizeof(L));
  memcpy(L.cur_new, cur, sizeof(double) * NCUR);
  L.mode = 1;
  L.emit_edges = 0;
  return launch(e, L, (hipStream_t)stream);
}

int lsm_reset_layout(lsm_env* e, const lsm_curriculum* cur, const double* layout, void* stream) {
  if (!e || !cur) return 1;
  if (e->cfg.scenario == LSM_SCENARIO_TRAIN) return fail(e, "lsm_reset_layout needs a layout scenario");
  if (!layout) return fail(e, "null layout");
  if (check_ready(e, false)) return 1;
  if (sep_check(e, cur, (hipStream_t)stream)) return 1;
  KStep L;
  memset(&L, 0, sizeof(L));
  memcpy(L.cur_new, cur, sizeof(double) * NCUR);
  L.mode = 2;
  L.layout = layout;
  return launch(e, L, (hipStream_t)stream);
}

int lsm_step(lsm_env* e, const void* actions, int32_t kind, const lsm_curriculum* cur, void* stream) {
  if (!e || !actions || !cur) return fail(e, "null argument");
  if (kind < 0 || kind > 2) return fail(e, "bad action kind");
  if (check_ready(e, true)) return 1;
  // a step's curriculum block is used only by its auto-resets: without them no chain can grow
  if (e->cfg.auto_reset && sep_check(e, cur, (hipStream_t)stream)) return 1;
  KStep L;
  memset(&L, 0, sizeof(L));
  memcpy(L.cur_new, cur, sizeof(double) * NCUR);
  L.mode = 0;
  L.action_kind = kind;
  L.actions = actions;
  L.emit_edges = e->cfg.emit_edges && e->out_ptr[LSM_OUT_EDGES] != nullptr;
  return launch(e, L, (hipStream_t)stream);
}

int32_t lsm_action_errors(lsm_env* e, void* stream) {
  if (!e) return -1;
  int32_t v = 0;
  if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return -1;
  if (hipMemcpy(&v, e->action_err, sizeof v, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (v && hipMemset(e->action_err, 0, sizeof(int32_t)) != hipSuccess) return -1;
  return v;
}

int lsm_host_rk45_di(const double* y0, double a0, double a1, double dt, double* y_out) {
  double y[4] = {y0[0], y0[1], y0[2], y0[3]};
  const int n = rk45_di(y, a0, a1, dt);
  for (int i = 0; i < 4; ++i) y_out[i] = y[i];
  return n;
}

double lsm_host_glibc_pow(double x, double y) { return glibc_pow(x, y); }

int lsm_host_philox4x32(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
  philox4x32_10(ctr, key, out);
  return 0;
}

int lsm_host_philox_uniforms(uint32_t key, uint32_t reset_index, int32_t count, double lo, double hi,
                             double* out) {
  Philox m;
  m.init(key, reset_index);
  for (int k = 0; k < count; ++k) out[k] = m.uniform(lo, hi);
  return 0;
}

int lsm_host_mt_uniforms(uint32_t seed, int32_t count, double lo, double hi, double* out) {
  HostMT m;
  m.seed(seed);
  for (int k = 0; k < count; ++k) out[k] = m.uniform(lo, hi);
  return 0;
}

int lsm_host_scenario(const lsm_config* cfg, const lsm_curriculum* cur, uint32_t seed, double* agent_state,
                      double* landmarks) {
  const int N = cfg->num_agents, L = cfg->num_landmarks, NL = N * L;
  if (N < 2 || N > BMAXN || L < 2 || L > MAX_L) return 1;
  ScenarioParams sp;
  const bool di = cfg->dynamics == LSM_DOUBLE_INTEGRATOR;
  sp.dyn = di ? 0 : 1; sp.N = N; sp.L = L; sp.world_size = cfg->world_size;
  sp.coordination_range = di ? 4.0 : 3 * 1.60934;
  sp.goal_speed_min = di ? 0.1 : 60 * 0.514444 * 0.001;
  sp.goal_speed_max = di ? 0.5 : 110 * 0.514444 * 0.001;
  sp.ratio_airtaxi = cur->ratio_airtaxi; sp.ratio_scenario = cur->ratio_scenario;
  sp.pi = 3.141592653589793; sp.two_pi = 2 * sp.pi;
  sp.d2lo = sp.d2hi = 0.0;   // (the device draw's squared band; random_scenario tests d itself)
  std::vector<double> st(4 * N), lm(4 * NL), ws(SCEN_WS);
  if (cfg->rng == LSM_RNG_PHILOX) {   // the device's first reset (reset index 0) of this seed
    Philox m;
    m.init(seed, 0);
    random_scenario(m, sp, st.data(), lm.data(), ws.data());
  } else {
    HostMT m;
    m.seed(seed);
    random_scenario(m, sp, st.data(), lm.data(), ws.data());
  }
  for (int i = 0; i < N; ++i)
    for (int c = 0; c < 4; ++c) agent_state[i * 4 + c] = st[c * N + i];
  for (int k = 0; k < NL; ++k)
    for (int c = 0; c < 4; ++c) landmarks[k * 4 + c] = lm[c * NL + k];
  return 0;
}

}  // extern "C"

#endif  // LSM_HOST_PART
