// lsm_team.h -- the "team" one-wave kernel: G envs per workgroup, one wave per env for the
// env-wide phases, ONE wave for the per-agent phases of all G envs.
//
// Included by lsm_rollout.hip after rollout_kernel (same helpers, same arithmetic, same
// outputs). Why: in rollout_kernel the per-agent float64 phases -- the filter's argmin and QP,
// RK45, obs / reward / goal update, info, episode statistics -- run on N of a wave's 64 lanes
// (8 of 64 at config 3), yet every one of those instructions costs a full wave issue slot. At
// 4096 envs the SIMDs are issue-bound (4 waves each, measured), so the idle lanes are the cost.
// Here the G = 64 / N envs of a workgroup put their agents side by side in one wave -- lane
// g * N + i is agent i of env g -- so that work is issued once for G envs, while the pair,
// distance and output phases keep one 64-lane wave per env. The other waves wait at the
// workgroup barrier (no issue) or, during the reward / info phase, store their adjacency.
//
// Phases (W = workgroup barrier; every wave reaches each W the same number of times):
//   A  (each env's wave)   record HBM -> LDS, actions, update_graph edges, decode, HJ pair lookups
//   W  B (agent wave 0)    filter per agent, integrate                  (core.py:648-687)
//   W  C (each env's wave) E x E distances, contact forces, magnetic field segment sums (filter off)
//   W  D (agent wave 1%G)  min relative distance, obs / reward / goal update, disconnect masks,
//                          info, episode stats;   other waves: speculative adjacency stores
//   W  E (each env's wave) info rows out, dones / masks, then the auto-reset or the graph outputs
//
// LDS: the workgroup holds G env blocks of `lds_env_bytes`, padded (team_env_bytes) so that the
// agent wave's lanes of different envs fall on different banks.
#pragma once
// (included inside namespace lsm)

// Env block stride for the team kernel: a multiple of 8 NT bytes with an odd quotient, so the
// 8-B per-agent fields of envs g = 0, 1, ... of one 32-lane ds_read_b64 group (256-B bank row)
// start on distinct bank offsets.
__host__ __device__ inline size_t team_env_bytes(size_t bytes, int N) {
  const size_t u = 8 * (size_t)N;
  size_t q = (bytes + u - 1) / u;
  if ((q & 1) == 0) ++q;
  return q * u;
}

// Team kernels target 4 waves / SIMD for the double integrator (<= 128 VGPRs, as rollout_kernel)
// and 2 for airtaxi.
// Diagnostic builds (-DLSM_STAMPS, lsm.diag_stamps --team): s_memtime of each env's wave at the
// phase boundaries: 0 start, 12 record in LDS, 6/7/8 own work of phases A / C / D done, 1-4 after
// barriers 1-4, 5 end; 9 / 10 / 11 inside the agent phases B / D; 13/14 realtime start / end;
// 15 HW_ID | XCC_ID << 32. Never in the product library.
#ifdef LSM_STAMPS
#define TSTAMP(k)                                                                                  \
  do {                                                                                             \
    if (lane == 0 && live && gptr(P.stamps)) gptr(P.stamps)[(size_t)env * LSM_NSTAMP + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define TRTSTAMP(k)                                                                                \
  do {                                                                                             \
    if (lane == 0 && live && gptr(P.stamps)) gptr(P.stamps)[(size_t)env * LSM_NSTAMP + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// per-phase dynamic instruction counts (lsm.diag_phasecount --team): the launch ends at stop k
// (launch-uniform; inside A every wave of a workgroup must be live, as at the bench's env counts)
#define TSTOP(k)                                                                                   \
  do {                                                                                             \
    if (K.stop_after == (k)) return;                                                               \
  } while (0)
#else
#define TSTOP(k) do { } while (0)
#define TSTAMP(k) do { } while (0)
#define TRTSTAMP(k) do { } while (0)
#endif
// Diagnostic builds: LSM_XP_DELAY=p sleeps ~3000 cycles in phase p (1 A's env waves, 2 B's agent
// wave, 3 C's env waves, 4 D's agent wave, 5 E's waves) -- how much of each phase lies on the path
// to the end of the launch (same results, slower). Never in the product library.
#if defined(LSM_XP_DELAY)
#define XDELAY(p)                                                                                  \
  do {                                                                                             \
    if (LSM_XP_DELAY == (p)) __builtin_amdgcn_s_sleep(47);                                         \
  } while (0)
#else
#define XDELAY(p) do { } while (0)
#endif

// ---- resets: the scenario draws ------------------------------------------------------------
// random_scenario is a long scalar sequence (rejection loops, atan2, ~120 MT19937 doubles at N =
// 8) that every lane of an env's wave used to run identically; with all G waves of the 4
// workgroups of a CU doing so at once, an auto-reset step cost ~2.5 plain steps. Here each env's
// wave prepares its stream (the rest of the current MT19937 block in LDS plus the next block,
// generated out of place), then draws its scenario with the draws spread over its lanes
// (random_scenario_wave2, below), and finishes its own reset. (Round 3's shape, one wave drawing
// every resetting env of the workgroup on lane g for env g, measured slower and was removed.)

// The next MT19937 block (HostMT::gen's arithmetic) into nxt, leaving key intact. Cooperative over
// the env's 64 lanes: element i >= 227 reads nxt[i - 227], so chunks of 64 run in order.
// Element i >= 227 reads nxt[i - 227], so three rounds: [0, 227) from the key, [227, 454) from the
// first, [454, 624) from the second (the last element also reads nxt[0]).
__device__ __forceinline__ void mt_next_block(const uint32_t* key, uint32_t* nxt) {
  const int lane = threadIdx.x & 63;
  constexpr int D = MT_N - MT_M;   // 227
  for (int i = lane; i < D; i += 64) nxt[i] = mt_twist1(key[i], key[i + 1], key[i + MT_M]);
  esync<64>();
  for (int i = D + lane; i < 2 * D; i += 64) nxt[i] = mt_twist1(key[i], key[i + 1], nxt[i - D]);
  esync<64>();
  for (int i = 2 * D + lane; i < MT_N; i += 64)
    nxt[i] = i < MT_N - 1 ? mt_twist1(key[i], key[i + 1], nxt[i - D]) : mt_twist1(key[MT_N - 1], nxt[0], nxt[MT_M - 1]);
  esync<64>();
}

// S.mt[MT_N] after a draw that ran past the staged stream (the env's wave then redraws it with the
// cooperative stream, team_reset_finish)
constexpr uint32_t MT_OVER = 0xffffffffu;

// ---- the scenario draw on a whole wave (one env per wave) -----------------------------------
// random_scenario (lsm_scenario.h) consumes its stream strictly in order, but only its rejection
// loops (randomly_generate_separated_positions, utils.py:39-68) make the consumption data-dependent,
// and every draw's words are known once the loops before it are resolved. So the wave computes
// every fixed-count draw of a stretch on separate lanes, and each rejection loop as 64 tries at once
// (try j on lane j, words c + 4 j): the first accepted try (a ballot) is the one the sequential
// loop stops at. Same words, same float64 operations, same values as the one-lane replay.
//
// Stream views: word k (k >= 0) of the env's stream from the reset's start position.
struct MtView {   // the staged MT19937 blocks (team_reset_prep): current from p0, then the next
  const uint32_t* key;
  const uint32_t* nxt;
  int p0, avail;   // words available from p0 (lane draws beyond avail are flagged by the caller)
  // one unconditional LDS read from a selected address (a branch per word made every read wait
  // for the previous one: 3.7 k cycles per agent of the draw instead of ~1 k)
  __device__ __forceinline__ uint32_t raw(int k) const {
    const int a = p0 + k;
    const bool in = a < 2 * MT_N;
    const uint32_t* q = a < MT_N ? key + a : nxt + (a - MT_N);
    const uint32_t y = *(in ? q : key);
    return in ? y : 0u;
  }
  __device__ __forceinline__ uint32_t word(int k) const { return mt_temper(raw(k)); }
  static __device__ __forceinline__ uint32_t tw(uint32_t y) { return mt_temper(y); }
};
struct PhiloxView {   // LSM_RNG_PHILOX: word k = element k % 4 of counter block k / 4
  uint32_t key, ridx;
  int avail;
  __device__ __forceinline__ uint32_t raw(int k) const { return word(k); }
  static __device__ __forceinline__ uint32_t tw(uint32_t y) { return y; }
  __device__ __forceinline__ uint32_t word(int k) const {
    const uint32_t ctr[4] = {(uint32_t)k >> 2, ridx, 0u, 0u}, kk[2] = {key, 0x4c534d31u};
    uint32_t o[4];
    philox4x32_10(ctr, kk, o);
    const int e = k & 3;
    return e == 0 ? o[0] : e == 1 ? o[1] : e == 2 ? o[2] : o[3];
  }
};
__device__ __forceinline__ double readlane_f64(double x, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
  return __hiloint2double(hi, lo);
}

// RandomState.uniform(lo, hi) from words k, k + 1 (numpy's random_sample)
template <class V>
__device__ __forceinline__ double view_uniform(const V& v, int k, double lo, double hi) {
  const uint32_t a = v.word(k) >> 5, b = v.word(k + 1) >> 6;
  const double range = hi - lo;
  return lo + range * ((a * 67108864.0 + b) / 9007199254740992.0);
}
// the same from raw (untempered) words already read
template <class V>
__device__ __forceinline__ double raw_uniform(uint32_t r0, uint32_t r1, double lo, double hi) {
  const uint32_t a = V::tw(r0) >> 5, b = V::tw(r1) >> 6;
  const double range = hi - lo;
  return lo + range * ((a * 67108864.0 + b) / 9007199254740992.0);
}

// random_scenario (lsm_scenario.h) on the 64 lanes of one wave, for two landmarks per agent (the
// team kernels run only with L = 2: lsm_create; every configuration the bench and the reference's
// training runs use). Returns the words consumed (> v.avail: the staged stream ran out and the caller
// redraws sequentially). Only the rejection loop's length decides where the next agent's
// words start, so the agent-by-agent pass resolves just that (64 tries per ballot) and everything
// else runs for all agents at once, agent i on lane i; no LDS writes, no wave barriers. Same words,
// same operations, same values as random_scenario.
#ifdef LSM_STAMPS
#define DSTAMP(k)                                                                                  \
  do {                                                                                             \
    if (stp && lane == 0) stp[k] = __builtin_amdgcn_s_memtime();                                   \
  } while (0)
#else
#define DSTAMP(k) do { } while (0)
#endif
template <class V>
__device__ int random_scenario_wave2(const V& v, const ScenarioParams& p, double* st, double* lm,
                                     GAS unsigned long long* stp = nullptr) {
  const int lane = threadIdx.x & 63;
  (void)stp;
  const int N = p.N, NL = 2 * N;
  const double wsz = p.world_size, cra = p.ratio_airtaxi, cr = p.ratio_scenario;
  int c = 0;
  const int per = p.dyn == 0 ? 4 : 8;
  for (int i = lane; i < N; i += 64) {
    const int k = c + per * i;
    if (p.dyn == 0) {
      const double x = view_uniform(v, k, -0.8 * wsz, 0.8 * wsz);
      const double y = view_uniform(v, k + 2, -0.8 * wsz, 0.8 * wsz);
      st[0 * N + i] = x; st[1 * N + i] = y; st[2 * N + i] = 0.0; st[3 * N + i] = 0.0;
    } else {
      const double xmin = -0.5 * wsz;
      const double xmax = 0.25 * wsz * cra + 0.0 * (1 - cra) * wsz;
      const double y = view_uniform(v, k, -0.5 * wsz, 0.5 * wsz);
      const double x = view_uniform(v, k + 2, xmin, xmax);
      const double spd = view_uniform(v, k + 4, p.goal_speed_min, p.goal_speed_max);
      const double th = view_uniform(v, k + 6, 0.0, p.two_pi);
      st[0 * N + i] = x; st[1 * N + i] = y; st[2 * N + i] = th; st[3 * N + i] = spd;
    }
  }
  c += per * N;
  DSTAMP(23);
  // the separation band (dmin, dmax) = (0.25, 0.75) x coordination_range (DI), (0.5, 1) x (airtaxi),
  // as squared-distance thresholds p.d2lo / p.d2hi (fill_params)
  double x0, x1, y0, y1;
  if (p.dyn == 0) {
    x0 = -0.5 * wsz; x1 = 0.5 * wsz; y0 = -0.5 * wsz; y1 = 0.5 * wsz;
  } else {
    const double yw = 0.1 * (1 - cra) + 0.5 * cra;
    x0 = 0.0; x1 = 0.75 * wsz; y0 = -yw * wsz; y1 = yw * wsz;
  }
  // Agent blocks in stream order: [point 0: 4][tries: 4 (acc + 1)][keep: 4, agents i > 0]
  // [speeds: 6, DI][noise: 2]; only acc varies. (1) The chain of block starts: per agent, point 0
  // and 64 tries at once (try j on lane j), the first accepted try by ballot -- nothing else on the
  // chain; (2) agent i's draws on lane i; (3) the keep-previous / airtaxi-swap chain in agent order
  // (readlane, uniform); (4) headings, speeds, noise on lane i.
  const int after = 4 + (p.dyn == 0 ? 6 : 0) + 2;
  // try j (>= 0) of the agent whose block starts at word cs: accepted? (point 0 = words cs..cs+3)
  auto accept = [&](int cs, int j) -> bool {
    uint32_t r[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = v.raw(cs + q);
#pragma unroll
    for (int q = 0; q < 4; ++q) r[4 + q] = v.raw(cs + 4 + 4 * j + q);
    const double ax = raw_uniform<V>(r[0], r[1], x0, x1), ay = raw_uniform<V>(r[2], r[3], y0, y1);
    const double x = raw_uniform<V>(r[4], r[5], x0, x1), y = raw_uniform<V>(r[6], r[7], y0, y1);
    const double dx = ax - x, dy = ay - y;
    // d = sqrt(dx * dx + dy * dy) in (dmin, dmax), tested on the square (exact: the band's ends are
    // the squared-distance thresholds of the correctly rounded sqrt, fill_params)
    const double d2 = dx * dx + dy * dy;
    return (d2 > p.d2lo && d2 < p.d2hi) || j == 999;   // the 1000th try is kept whatever it is
  };
  // the first accepted try >= j0 of the agent at cs, 64 tries per ballot (the rare long loops)
  auto first_from = [&](int cs, int j0) -> int {
    for (int base = j0; base < 1000; base += 64) {
      const int j = base + lane;
      const uint64_t m = __ballot(j < 1000 && accept(cs, j));
      if (m) return base + __ffsll((unsigned long long)m) - 1;
    }
    return 999;   // not reached: try 999 is always accepted
  };
  // Two agents per ballot: lanes 0-7 try 0-7 of agent i (block start c); lanes 8 + 8 g + t try t of
  // agent i + 1 as if agent i accepted its try g (its block then starts after g + 1 tries), g < 7.
  // One ballot gives acc_i (lowest set bit of lanes 0-7) and then, from group acc_i, acc_{i+1} --
  // the chain of block starts resolves in half the rounds. A try beyond those (< 1 % at these
  // acceptance rates) takes first_from. Same words, same arithmetic: the same acc as the sequential loop.
  int my_s = 0, my_acc = 0;
  for (int i = 0; i < N;) {
    const int after_i = after - (i == 0 ? 4 : 0);
    const bool two = i + 1 < N;
    const int g = (lane - 8) >> 3;
    const int cs = lane < 8 ? c : c + 4 + 4 * (g + 1) + after_i;
    const int j = lane < 8 ? lane : (lane & 7);
    const uint64_t m = __ballot((lane < 8 || two) && accept(cs, j));
    int acc = (m & 0xffull) ? __ffsll((unsigned long long)(m & 0xffull)) - 1 : first_from(c, 8);
    if (lane == i) { my_s = c; my_acc = acc; }
    c += 4 + 4 * (acc + 1) + after_i;
    ++i;
    if (two && acc < 7) {
      const uint64_t mg = (m >> (8 + 8 * acc)) & 0xffull;
      const int acc1 = mg ? __ffsll((unsigned long long)mg) - 1 : first_from(c, 8);
      if (lane == i) { my_s = c; my_acc = acc1; }
      c += 4 + 4 * (acc1 + 1) + after;
      ++i;
    }
  }
  DSTAMP(24);
  double dax = 0.0, day = 0.0, dbx = 0.0, dby = 0.0;
  int kp0 = 0, kp1 = 0, mcs = 0;
  if (lane < N) {
    const int t = my_s + 4 + 4 * my_acc;
    uint32_t r[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = v.raw(my_s + q);
#pragma unroll
    for (int q = 0; q < 4; ++q) r[4 + q] = v.raw(t + q);
    dax = raw_uniform<V>(r[0], r[1], x0, x1); day = raw_uniform<V>(r[2], r[3], y0, y1);
    dbx = raw_uniform<V>(r[4], r[5], x0, x1); dby = raw_uniform<V>(r[6], r[7], y0, y1);
    int k = t + 4;
    if (lane > 0) {   // the previous agent's goals, each kept with probability 1/2 (a draw each)
      kp0 = view_uniform(v, k, 0.0, 1.0) < 0.5;
      kp1 = view_uniform(v, k + 2, 0.0, 1.0) < 0.5;
      k += 4;
    }
    mcs = k;
  }
  double pax = 0.0, pay = 0.0, pbx = 0.0, pby = 0.0;   // the previous agent's goals
  double max_ = 0.0, may = 0.0, mbx = 0.0, mby = 0.0;  // lane i: agent i's goals
  for (int a = 0; a < N; ++a) {
    double ax = readlane_f64(dax, a), ay = readlane_f64(day, a);
    double bx = readlane_f64(dbx, a), by = readlane_f64(dby, a);
    if (a > 0) {
      if (__builtin_amdgcn_readlane(kp0, a)) { ax = pax; ay = pay; }
      if (__builtin_amdgcn_readlane(kp1, a)) { bx = pbx; by = pby; }
    }
    if (p.dyn != 0 && ax > bx) {
      const double tx = ax, ty = ay;
      ax = bx; ay = by;
      bx = tx; by = ty;
    }
    if (lane == a) { max_ = ax; may = ay; mbx = bx; mby = by; }
    pax = ax; pay = ay; pbx = bx; pby = by;
  }
  DSTAMP(25);
  if (lane < N) {
    const int i = lane;
    const double h = atan2(mby - may, mbx - max_);
    double s0, s1;
    if (p.dyn != 0) {
      s0 = s1 = p.goal_speed_max * 1.0;
    } else {
      const double var = view_uniform(v, mcs + 4, 0.0, 1.0);
      const bool use_rnd = var < py_min(cr, 1 - 0.2);
      const double r0 = view_uniform(v, mcs, p.goal_speed_min, p.goal_speed_max);
      const double r1 = view_uniform(v, mcs + 2, p.goal_speed_min, p.goal_speed_max);
      s0 = use_rnd ? r0 : p.goal_speed_max * 1.0;
      s1 = use_rnd ? r1 : p.goal_speed_min;
    }
    const double pr = (p.dyn == 0) ? cr * 0.25 * p.pi : cra * 0.1 * p.pi;
    const double h0 = h + view_uniform(v, mcs + (p.dyn == 0 ? 6 : 0), -pr, pr);
    lm[0 * NL + i] = max_;     lm[0 * NL + N + i] = mbx;
    lm[1 * NL + i] = may;      lm[1 * NL + N + i] = mby;
    lm[2 * NL + i] = h0;       lm[2 * NL + N + i] = h;
    lm[3 * NL + i] = s0;       lm[3 * NL + N + i] = s1;
  }
  DSTAMP(26);
  return c;
}
#undef DSTAMP

// env wave: summary, curriculum, shift; the MT19937 stream staged in LDS (start pos kept)
template <int DYN, int NT>
__device__ __forceinline__ int team_reset_prep(const KParams& P, Lds& S, int env, const double* cur_new) {
  const int lane = threadIdx.x & 63;
  // the env's MT19937 state loads are issued first, so their latency overlaps the summary
  constexpr int MQ = (MT_WORDS + 63) / 64;
  uint32_t mr[MQ];
  const bool mt = P.rng != LSM_RNG_PHILOX;
  const GAS uint32_t* mtg = gptr(P.s.mt) + (size_t)env * MT_WORDS;
  if (mt) {
#pragma unroll
    for (int q = 0; q < MQ; ++q) {
      const int k = lane + 64 * q;
      mr[q] = mtg[k < MT_WORDS ? k : 0];
    }
  }
  reset_head<DYN, 64, NT>(P, S, env, cur_new);
  if (!mt) return 0;
#pragma unroll
  for (int q = 0; q < MQ; ++q) {
    const int k = lane + 64 * q;
    if (k < MT_WORDS) S.mt[k] = mr[q];
  }
  esync<64>();
  const int p0 = (int)S.mt[MT_N];
  mt_next_block(S.mt, S.mtn);
  return p0;
}

// env wave: its own env's scenario on the whole wave (random_scenario_wave2), from the staged
// MT19937 blocks (or the Philox stream); S.mt[MT_N] = the new position, MT_OVER if it ran out.
// L = 2 only (the team kernels' scenario draw, random_scenario_wave2)
template <int DYN, int NT>
__device__ __forceinline__ void team_scenario_wave(const KParams& P, Lds& S, int env, int p0) {
  const int lane = threadIdx.x & 63;
  const ScenarioParams sp = scenario_params<DYN, NT>(P, S);
  if (P.rng == LSM_RNG_PHILOX) {
    GAS uint32_t* rw = gptr(P.s.mt) + (size_t)env * MT_WORDS + MT_N;
    const uint32_t ridx = *rw - (uint32_t)MT_N;
    PhiloxView v;
    v.key = (uint32_t)(P.seed + 1000 * (P.env_offset + env));
    v.ridx = ridx;
    v.avail = 1 << 30;
    random_scenario_wave2(v, sp, S.ps, S.lm);
    esync<64>();
    if (lane == 0) *rw = ridx + 1 + (uint32_t)MT_N;
    return;
  }
  MtView v;
  v.key = S.mt;
  v.nxt = S.mtn;
  v.p0 = p0;
  v.avail = min(2 * MT_N - p0, P.mt_stage);
#ifdef LSM_STAMPS
  GAS unsigned long long* stp = gptr(P.stamps) ? gptr(P.stamps) + (size_t)env * LSM_NSTAMP : nullptr;
#else
  GAS unsigned long long* stp = nullptr;
#endif
  const int used = random_scenario_wave2(v, sp, S.ps, S.lm, stp);
  esync<64>();
  if (lane == 0) S.mt[MT_N] = used > v.avail ? MT_OVER : (uint32_t)(p0 + used);
  esync<64>();
}

// env wave: the stream's new state to HBM (a redraw if the lane ran out), then reset_tail
template <int DYN, int NT>
__device__ __forceinline__ void team_reset_finish(const KParams& P, Lds& S, int env, int p0) {
  const int lane = threadIdx.x & 63;
  if (P.rng != LSM_RNG_PHILOX) {
    GAS uint32_t* mtw = gptr(P.s.mt) + (size_t)env * MT_WORDS;
    const uint32_t p = S.mt[MT_N];
    esync<64>();
    if (p == MT_OVER) {
      // rare: more draws than the two staged blocks -- the cooperative stream from the start
      WaveRng<64> rng;
      rng.key = S.mt;
      rng.pos = p0;
      const ScenarioParams sp = scenario_params<DYN, NT>(P, S);
      random_scenario(rng, sp, S.ps, S.lm, S.scen);
      esync<64>();
      if (lane == 0) S.mt[MT_N] = (uint32_t)rng.pos;
      esync<64>();
      for (int k = lane; k < MT_WORDS; k += 64) mtw[k] = S.mt[k];
    } else if (p <= (uint32_t)MT_N) {
      if (lane == 0) mtw[MT_N] = p;   // the block itself is unchanged
    } else {
      for (int k = lane; k < MT_N; k += 64) mtw[k] = S.mtn[k];   // the next block became current
      if (lane == 0) mtw[MT_N] = p - (uint32_t)MT_N;
    }
  }
  reset_tail<DYN, 64, NT>(P, S, false);
}

// The airtaxi kernel is held to 2 waves per SIMD both ways: its LDS allows no more (2 workgroups
// of 4 x 19.3 KB per CU), and with the upper bound open the compiler scheduled for 3 (135 VGPRs):
// 396.3 us per step at config 4 against 387.5 capped at 2 (224 VGPRs; profiles/r06_s08_ab_c4.txt).
// A/B variant builds may move either bound (LSM_AB_AT_WPE, LSM_AB_AT_WPE_MAX).
#ifndef LSM_AB_AT_WPE
#define LSM_AB_AT_WPE 2
#endif
#ifndef LSM_AB_AT_WPE_MAX
#define LSM_AB_AT_WPE_MAX 2
#endif
// REXT: the optional reward terms / shared reward may be on (P.rext); the host launches REXT = false
// when neither is configured. Compiled in, that block cost <0, 8, 4> 92 B of scratch per lane (spills
// across the whole kernel, 0 B without it; profiles/r06_s07_ab_c3.txt).
template <int DYN, int NT, int G, bool REXT>
__global__ __launch_bounds__(64 * G) __attribute__((amdgpu_waves_per_eu(DYN == 0 ? 4 : LSM_AB_AT_WPE, DYN == 0 ? 8 : LSM_AB_AT_WPE_MAX)))
void rollout_team_kernel(const KParams* __restrict__ Pp, const KStep K) {
  static_assert(NT > 0 && G >= 2 && G * NT <= 64, "team: G envs x NT agents in one wave");
  constexpr int LPE = 64;
  const KParams& P = *Pp;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int w = (int)threadIdx.x >> 6;        // this wave's env slot
  const int lane = (int)threadIdx.x & 63;
  const int env0 = (int)blockIdx.x * G;
  const int env = env0 + w;
  const bool live = env < P.n_envs;           // wave-uniform
  LSM_DIMS;
  const uint32_t B = P.lds_env_bytes;
  unsigned char* lbase = smem + (size_t)w * B;
#ifdef LSM_XP_POISON
  LDS_POISON(lbase, B, lane, 64);
  __syncthreads();
#endif
  Lds S = carve(lbase, N, NL, E, F, DYN == 1 && P.lean != 0);   // folds away for the DI kernels
  // agent view: lane = g * NT + i
  const int ag = lane / NT;
  const int ai = lane - ag * NT;
  const bool alane = ag < G && env0 + ag < P.n_envs;
  const int aslot = ag < G ? ag : 0;
  const int aenv = env0 + aslot;
  Lds A = carve(smem + (size_t)aslot * B, N, NL, E, F, DYN == 1 && P.lean != 0);
  constexpr int WB = 0, WD = 1 % G;           // agent-phase waves (different SIMDs)
  TRTSTAMP(13);
  TSTAMP(0);
#ifdef LSM_STAMPS
  if (lane == 0 && live && gptr(P.stamps))
    gptr(P.stamps)[(size_t)env * LSM_NSTAMP + 15] = (unsigned long long)__builtin_amdgcn_s_getreg(63492) |
                                          ((unsigned long long)__builtin_amdgcn_s_getreg(6164) << 32);
#endif

  // ---- A. record HBM -> LDS, actions, edges, decode, pair lookups --------------------------
  // launch-uniform. The double integrator only: the airtaxi agent wave's phase B (closed-form
  // integration) is too short to hide the second half (config 4: 400.7 -> 415.2 us split).
  const bool split = DYN == 0 && K.mode == 0 && !K.emit_edges;
  constexpr bool PRE = NT <= 8;
  constexpr int NPI = PRE ? ((NT * (NT - 1) / 2 + NT * 2 * NT) + LPE - 1) / LPE : 1;
  uint32_t prw[NPI];
  int act = 0;
  int cstep = 0;
  bool filter_on = false;
  // the agent wave's pow tables (lsm_rk45.h PowTabs) for its lane-pair RK45: 192 float4 of log rows
  // into env 0's U1 and 128 float4 of exp pairs into env 1's U1 (both free until the distances), a
  // slice per wave, issued with the record. The table loads inside pow were L2 round trips on the
  // latency-bound phase B: 32.40 -> 31.75 us per step at config 3 (profiles/r05_v3_ab_c3_powlds.txt)
  constexpr int NPQ = (320 + 64 * G - 1) / (64 * G);
  f32x4 ptq[NPQ];
  if (DYN == 0 && G * NT <= 32 && K.mode == 0) {
#pragma unroll
    for (int r = 0; r < NPQ; ++r) {
      const int q = lane + 64 * (w + G * r);
      const GAS f32x4* src = q < 192 ? (const GAS f32x4*)powl_tab(0) + q : (const GAS f32x4*)expd_tab_ptr() + (q - 192);
      ptq[r] = *(q < 320 ? src : (const GAS f32x4*)powl_tab(0));
    }
  }
  if (live) {
    if (K.mode == 0 && lane < N) act = read_action(K, env, N, lane);
    if (PRE) {
#pragma unroll
      for (int k = 0; k < NPI; ++k) {
        const int t = lane + k * LPE;
        prw[k] = gptr(P.pairs)[t < E * (E - 1) / 2 ? t : 0];
      }
    }
    // a plain step needs [0, a2) of the record before its distances; the rest (statistics,
    // landmarks) comes in phase B (cold_loads). Resets and the edge output read it all here.
    rec_copy<LPE>((const GAS f32x4*)gptr(P.s.rec) + (size_t)env * P.s.rec_stride16, (f32x4*)lbase,
                  split ? P.s.a2_16 : P.s.rec16);
    esync<LPE>();
    TSTAMP(12);
    TSTOP(1);
    if (lane < N) {
      S.dpre[lane] = S.dpost[lane];
      S.rpre[lane] = S.rpost[lane];
      if (DYN == 1) {
        S.ecs[lane] = cos(S.ps[2 * N + lane]);
        S.ecs[N + lane] = sin(S.ps[2 * N + lane]);
      }
    }
    cstep = S.step[0] + 1;
    esync<LPE>();
    if (K.mode == 1) {
      reset_env<DYN, LPE, NT>(P, S, env, K.cur_new);
      esync<LPE>();
      store_state<DYN, LPE, NT>(P, S, lbase, env, true);
    }
  }
  if (K.mode == 1) return;   // launch-uniform: no workgroup barrier is skipped by some waves only
  if (live) {
    if (K.emit_edges) {
      GAS uint8_t* eo = gptr(P.o.edges) + (size_t)env * E * E;
      const uint64_t m0 = S.step[1] ? 0ull : ego_mask(S, N, L, N);
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
    if (lane < N) decode_action(P, S, N, lane, act);
    filter_on = S.cur[C_FILT] != 0.0;
    if (filter_on) {
      const SepChain sc = sep_chain(S.sep, P.s, env);
      TSTAMP(30);
      for (int p = lane; p < N * N; p += LPE) {
        const int j = p / N, i = p - j * N;   // [j][i]: ego i fastest (bank-conflict-free reads)
        if (i == j || S.dpre[i] || S.dpre[j]) continue;
        const double ex = S.ps[i], ey = S.ps[N + i], ox = S.ps[j], oy = S.ps[N + j];
        const double sq = (ox - ex) * (ox - ex) + (oy - ey) * (oy - ey);
        // filter_prep_oct (DI, N = 8) works on squared distances (KParams::coord_range_s)
        S.dpair[p] = (DYN == 0 && NT == 8) ? sq : sqrt(sq);
        double rel[5];
        rel_state<DYN>(S, N, i, j, rel);
        float v = 0.0f;
        bool ok;
        if (DYN == 0) ok = interp_value<4>(P.val, rel, v, sc); else ok = interp_value<5>(P.val, rel, v, sc);
        S.vpair[p] = ok ? v : INFINITY;
        S.inr[p] = ok ? 1 : 0;
      }
      TSTAMP(16);
      TSTOP(2);
      // the deconflicting choice and the HJ gradient lookup of every ego, here where the other
      // waves of the SIMD hide the gather; the agent wave does the QP in B (filter_agent_slot)
      esync<LPE>();
#ifdef LSM_STAMPS
      GAS unsigned long long* ostp = gptr(P.stamps) && live ? gptr(P.stamps) + (size_t)env * LSM_NSTAMP : nullptr;
#else
      GAS unsigned long long* ostp = nullptr;
#endif
      // (the gradient at the previous step's deconflicting agent, gathered speculatively with the pair
      // values, served 98.65 % of the egos but lengthened the pair loop: 31.22 -> 32.47 us,
      // profiles/r06_s03_ab_c3_gspec.txt)
      if (DYN == 0 && NT == 8) filter_prep_oct<8>(P, S, ostp);   // 32.66 -> 32.28 us (profiles/r05_v5_ab_c3_oct.txt)
      else if (lane < N) filter_prep<DYN, NT>(P, S, lane);
      TSTAMP(17);
    }
  }
  if (DYN == 0 && G * NT <= 32 && K.mode == 0) {
#pragma unroll
    for (int r = 0; r < NPQ; ++r) {
      const int q = lane + 64 * (w + G * r);
      if (q < 192) ((f32x4*)carve(smem, N, NL, E, F, false).fval)[q] = ptq[r];
      else if (q < 320) ((f32x4*)carve(smem + B, N, NL, E, F, false).fval)[q - 192] = ptq[r];
    }
  }
  XDELAY(1);
  TSTAMP(6);
  TSTOP(3);
  __syncthreads();
  TSTAMP(1);

  // ---- B. filter + integration, one lane per (env, agent) ------------------------------------
  if (w != WB && split) {
    // the record's [a2, rec) of every env of the workgroup, while HBM and these waves would
    // otherwise idle; phase C is the first reader (landmarks), after the barrier below
    const int c16 = (int)(P.s.rec16 - P.s.a2_16);
    const int wi = w < WB ? w : w - 1;   // 0 .. G - 2 over the loading waves
    for (int t = wi * 64 + lane; t < G * c16; t += (G - 1) * 64) {
      const int g = t / c16, k = t - g * c16;
      if (env0 + g < P.n_envs)
        ((f32x4*)(smem + (size_t)g * B))[P.s.a2_16 + k] =
            ((const GAS f32x4*)gptr(P.s.rec) + (size_t)(env0 + g) * P.s.rec_stride16)[P.s.a2_16 + k];
    }
  }
  if (w == WB) {
    XDELAY(2);
    if (alane) filter_agent_slot<DYN, NT>(P, A, N, ai, A.cur[C_FILT] != 0.0);
    esync<LPE>();   // every filter of the env has read the pre-step state
    TSTAMP(9);
    if (DYN == 0 && G * NT <= 32) {
      // the double integrator's RK45 on lane pairs: lane l the x axis of agent l, lane l + 32
      // its y axis (integrate_agent_di_pair); both lanes of a pair have the same activity
      const int hl = lane & 31;
      const int g2 = hl / NT, i2 = hl - g2 * NT;
      if (g2 < G && env0 + g2 < P.n_envs) {
        Lds A2 = carve(smem + (size_t)g2 * B, N, NL, E, F, false);
        PowTabs pt;
        pt.log = (const double*)carve(smem, N, NL, E, F, false).fval;
        pt.exp = (const uint64_t*)carve(smem + B, N, NL, E, F, false).fval;
#ifdef LSM_STAMPS
        GAS unsigned long long* stp = gptr(P.stamps) ? gptr(P.stamps) + (size_t)env * LSM_NSTAMP : nullptr;
#else
        GAS unsigned long long* stp = nullptr;
#endif
        if (!A2.dpre[i2]) integrate_agent_di_pair(P, A2, N, i2, lane >= 32, pt, stp);
      }
    } else if (alane && !A.dpre[ai]) {
      integrate_agent<DYN>(P, A, N, ai);
    }
  }
  __syncthreads();
  TSTAMP(2);
  TSTOP(4);

  // ---- C. distances; contact forces and magnetic-field sums when asked ------------------------
  // the speculative adjacency stores of phase D are skipped for an env that auto-resets at the
  // episode-length boundary (known from the step count): the reset emits its outputs instead
  const bool chunked = (E & 3) == 0 && !P.adj_compact && !(P.auto_reset && cstep >= P.episode_length);
  uint64_t m_pre = 0;
  if (live) {
    // filter off: the magnetic field's segment constants, loaded while the distances are computed
    // and staged in U2 behind the partial sums (U2 holds no pair matrices without the filter)
    const bool mag = DYN == 0 && !P.use_filter_arg;
    double mr[2] = {0.0, 0.0};
    if (mag) mag_table_issue<LPE>(P, mr);
    compute_dist<LPE, NT>(P, S, PRE ? prw : nullptr);
    if (P.o.cforce && lane < N) {
      double fx, fy;
      collision_force_agent(S, N, lane, fx, fy);
      GAS double* cf = gptr(P.o.cforce) + ((size_t)env * N + lane) * 2;
      cf[0] = fx;
      cf[1] = fy;
    }
    // the magnetic-field segment sums (partials in U2, read by the agent wave in D, before the
    // info rows reuse U2)
    if (mag) {
      double* tab = S.dpair + 2 * LPE;
      mag_table_store<LPE>(mr, tab);
      esync<LPE>();
      magnetic_partials_wave<LPE, NT>(P, S, S.dpair, tab);
    }
  }
  XDELAY(3);
  TSTAMP(7);
  __syncthreads();
  TSTAMP(3);
  TSTOP(5);

  // ---- D. per-agent reward / info / stats (agent wave WD) while the other waves store their
  // env's adjacency speculatively (valid unless an agent changes done / reached status this step:
  // phase E then rewrites it). WD stores its own in E. (Splitting WD's env's egos over the other
  // waves in D was measured slower: 36.6 vs 34.5 us at config 3, G = 4.)
  if (w == WD) {
    XDELAY(4);
    AgentTmp at;
    if (alane) {
      min_relative(A, N, ai);
      // the per-agent half of the magnetic penalty, once for the G envs (was 4 env waves in C)
      const double mag = (DYN == 0 && !P.use_filter_arg) ? magnetic_penalty_agent<LPE, NT>(P, A, A.dpair, ai) : 0.0;
      reward_agent<DYN, NT>(P, A, aenv, ai, mag, at);
    }
    esync<LPE>();   // every agent's goal / done update before the snapshot masks
    if (REXT && P.rext) {   // optional reward terms / shared reward (reward_finish)
      if (alane) reward_finish<DYN, NT>(P, A, aenv, ai, at);
      esync<LPE>();
      if (P.collab && alane) reward_shared<NT>(P, A, aenv, ai);
    }
    TSTAMP(10);
    const int acstep = A.step[0] + 1;
    if (alane) {
      A.emask[ai] = ego_mask(A, N, L, ai);
      info_agent<DYN, NT>(P, A, ai, acstep, at, collision_count(A, N, ai));
    }
    esync<LPE>();
    TSTAMP(11);
    if (alane) {
      info_row<NT>(P, A, ai, at.rew, A.info + ai * LSM_INFO_FIELDS);   // staged in U2
      episode_stats<DYN>(P, A, N, ai);
    }
  } else if (live && chunked) {
    // the disconnect mask before this step's updates, here rather than at the end of C (phase C
    // is on the path to the first stores; these waves wait for the agent wave in D)
    m_pre = ego_mask(S, N, L, -1);
#ifndef LSM_XP_NOOUT   // diagnostic bound only: no graph outputs
    emit_adj_uniform<LPE, NT>(P, S, env, m_pre, 0, N);
#endif
  }
  TSTAMP(8);
  __syncthreads();
  TSTAMP(4);
  TSTOP(6);

  // ---- E. info rows, dones, then what the speculation did not cover, or the auto-reset --------
  __shared__ int team_rs[G];   // this step's auto-resets of the workgroup's envs
  bool rs = false;
  XDELAY(5);
  if (live) {
    rec_copy<LPE>((const f32x4*)S.info, (GAS f32x4*)(gptr(P.o.info) + (size_t)env * N * LSM_INFO_FIELDS),
                  N * LSM_INFO_FIELDS / 2);
    bool my_done = true;
    if (lane < N) {
      my_done = S.dpost[lane] || cstep >= P.episode_length;
      gptr(P.o.dones)[(size_t)env * N + lane] = my_done ? 1 : 0;
    }
    const bool all_done = __all(my_done);
    write_masks(P, env, N, lane, my_done, all_done);
    esync<LPE>();   // info rows read out of U2 before the node rows / a reset overwrite it
    TSTAMP(18);
    if (lane == 0) { S.step[0] = cstep; S.step[1] = 0; }
    rs = P.auto_reset && all_done;
    if (lane == 0) gptr(P.o.reset_flag)[env] = rs ? 1 : 0;
    if (!rs) {
      // adjacency already stored in D except WD's (emit_graph rewrites it if a status changed)
#ifndef LSM_XP_NOOUT
      emit_graph<DYN, LPE, NT>(P, S, env, chunked && w != WD);
#endif
      esync<LPE>();
      store_state<DYN, LPE, NT>(P, S, lbase, env, false);
    }
  }
  if (lane == 0) team_rs[w] = rs ? 1 : 0;
  __syncthreads();
  int nrs = 0;
#pragma unroll
  for (int g = 0; g < G; ++g) nrs += team_rs[g];
  if (nrs != 0) {   // workgroup-uniform
    int p0 = 0;
    if (rs) p0 = team_reset_prep<DYN, NT>(P, S, env, K.cur_new);
    TSTAMP(19);
    // each resetting env's wave draws its own scenario on all 64 lanes (random_scenario_wave2):
    // reset steps 70.0-73.6 us vs 86.4-90.2 with round 3's one wave drawing lane g for env g
    // (profiles/r04_v1_reset_wdraw.json, r04_v2_reset_lanedraw.json, config 3)
    if (rs) team_scenario_wave<DYN, NT>(P, S, env, p0);
    TSTAMP(20);
    if (rs) {
      team_reset_finish<DYN, NT>(P, S, env, p0);
      compute_dist<LPE, NT>(P, S, nullptr, true);
      TSTAMP(21);
      if (lane < N) write_obs<DYN, NT>(P, S, env, lane);
      emit_graph<DYN, LPE, NT>(P, S, env);
      TSTAMP(22);
      esync<LPE>();
      store_state<DYN, LPE, NT>(P, S, lbase, env, true);
    }
  }
  TSTAMP(5);
  TRTSTAMP(14);
}

