// lsm_block.h -- the workgroup-per-env rollout kernel (included by lsm_rollout.hip inside
// namespace lsm, after the one-wave kernel whose per-agent functions it reuses).
//
// The one-wave kernel keeps an env's E x E distance table, its N x N pair tables and one
// 64-bit disconnect mask per ego in one wave's LDS, so it stops at N <= 32, E <= 64.
// BASELINE config 5 (64 double-integrator agents, E = 192, 8192 envs per GPU) needs more;
// here one 256-thread workgroup (4 waves, one per SIMD) runs one env:
//   * pair work (the filter's HJ value lookups, the distance reductions of
//     update_agent_min_relative_distance / is_collision / the episode statistics) runs T =
//     256 / N threads per ego (a power of two <= 64, so an ego's threads sit in one wave):
//     each takes every T-th other agent and the partial argmin / min / counts are combined by
//     a butterfly over the T lanes -- no N x N table in LDS. Ties go to the lower agent
//     index, i.e. np.argmin's first occurrence (safety_filter.py:395-405);
//   * no E x E table: the adjacency is computed from an entity-position table in LDS as it
//     is stored (reference layout: masked for every ego; compact layout: once, plus the
//     per-ego disconnect masks);
//   * disconnect masks are ceil(E / 64) words per ego, built from two ballots (entity
//     flags before / after the reward update) and the snapshot-rule selector.
// Per-agent phases (integration, obs / reward, info) are the one-wave kernel's functions
// run by threads 0..N-1; the reset is the same reset_core.

// threads per ego in the pair passes: the largest power of two T <= 64 with T * N <= BT
__host__ __device__ constexpr int block_tpe(int N) {
  return (64 * N <= BT) ? 64 : (32 * N <= BT) ? 32 : (16 * N <= BT) ? 16 : (8 * N <= BT) ? 8 : (4 * N <= BT) ? 4 : (2 * N <= BT) ? 2 : 1;
}

__device__ __forceinline__ bool mbit(const uint64_t* m, int k) { return (m[k >> 6] >> (k & 63)) & 1ull; }

// entity k disconnected (navigation_graph_safe.py:976-989): a done or (RealisticScenario) not
// yet departed agent, or landmark l = o * N + j already reached by its agent j (reached_goal[j] > o)
template <bool POST>
__device__ __forceinline__ bool entity_disc(const Lds& S, int N, int E, int k) {
  if (k >= E) return false;
  if (k < N)
    return (POST ? S.dpost[k] : S.dpre[k]) != 0 || (S.dep0 && !(POST ? S.dep1[k] : S.dep0[k]));
  const int l = k - N, o = l / N, j = l - o * N;
  return (POST ? S.rpost[j] : S.rpre[j]) > o;
}

// S.mpre / S.mpost: entity k = thread k, word w = wave w (E <= BT). All threads call.
__device__ __forceinline__ void mask_words(const Lds& S, int N, int E) {
  const int tid = threadIdx.x;
  const uint64_t bpre = __ballot(entity_disc<false>(S, N, E, tid));
  const uint64_t bpost = __ballot(entity_disc<true>(S, N, E, tid));
  if ((tid & 63) == 0) {
    S.mpre[tid >> 6] = bpre;
    S.mpost[tid >> 6] = bpost;
  }
}

// bits [lo, hi) that fall in word w
__device__ __forceinline__ uint64_t range_bits(int lo, int hi, int w) {
  const int a = lo > 64 * w ? lo : 64 * w;
  const int b = hi < 64 * w + 64 ? hi : 64 * w + 64;
  if (a >= b) return 0ull;
  const int n = b - a;
  return (n == 64 ? ~0ull : ((1ull << n) - 1ull)) << (a - 64 * w);
}

// entities whose agent j <= e (agents, then landmark orders: N + o N + j): the ones ego e
// sees after their reward update (sequential snapshot rule)
__device__ __forceinline__ uint64_t post_sel(int N, int L, int e, int w) {
  uint64_t m = 0ull;
  for (int s = 0; s <= L; ++s) m |= range_bits(s * N, s * N + e + 1, w);
  return m;
}

// Discrete(25) action of agent `lane` (environment.py:386-410): argmax of a one-hot row or
// an index
__device__ __forceinline__ int load_action(const KStep& K, int env, int N, int lane) {
  int ai = 0;
  const size_t base = (size_t)env * N + lane;
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

// entity positions (agents at their current state, then landmarks)
template <int NT>
__device__ __forceinline__ void entity_table(const KParams& P, Lds& S) {
  constexpr int DYN = 0;
  LSM_DIMS;
  for (int k = threadIdx.x; k < E; k += BT) {
    S.ex[k] = k < N ? S.ps[k] : S.lm[k - N];
    S.ey[k] = k < N ? S.ps[N + k] : S.lm[NL + k - N];
  }
}

// thresholded distance of entities r, c (adj = d * (d < range) * (d > 0),
// navigation_graph_safe.py:991-992; |p_r - p_c| == |p_c - p_r| bit for bit)
__device__ __forceinline__ float adj_value(const KParams& P, const Lds& S, int r, int c) {
  const double dx = S.ex[r] - S.ex[c], dy = S.ey[r] - S.ey[c];
  const double d = sqrt(dx * dx + dy * dy);
  return (d < P.coord_range && d > 0) ? (float)d : 0.0f;
}

// node_obs + adjacency of one env (emission at a step end or after a reset). Expects the
// entity table, S.emask (per ego) and the pre / post flags.
template <int DYN, int NT>
__device__ __forceinline__ void emit_graph_block(const KParams& P, Lds& S, int env) {
  const int tid = threadIdx.x;
  LSM_DIMS;
  const int MW = (E + 63) >> 6;
  if (DYN == 0) build_rows_di<BT, NT>(P, S); else trig_table_at<BT, NT>(P, S);
  // departures: per-ego masks and post rows differ by the accumulation rule even without a status
  // change (the one-wave kernel's emit_graph does the same)
  const bool uni = __syncthreads_and(tid >= N || (S.dpre[tid] == S.dpost[tid] && S.rpre[tid] == S.rpost[tid])) &&
                   !S.dep0;
  const int EE = E * E;
  if (P.adj_compact) {
    GAS float* a = gptr(P.o.adj) + (size_t)env * EE;
    if ((E & 3) == 0) {
      for (int t = tid; t < EE / 4; t += BT) {
        const int u = 4 * t;
        const int r = qdiv<NT>(u, E, P.m_E), c = u - r * E;
        st_stream<true>(a + u, make_float4(adj_value(P, S, r, c), adj_value(P, S, r, c + 1), adj_value(P, S, r, c + 2),
                                     adj_value(P, S, r, c + 3)));
      }
    } else {
      for (int u = tid; u < EE; u += BT) {
        const int r = qdiv<NT>(u, E, P.m_E), c = u - r * E;
        a[u] = adj_value(P, S, r, c);
      }
    }
    GAS uint64_t* mo = gptr(P.o.adjmask) + (size_t)env * N * MW;
    for (int k = tid; k < N * MW; k += BT) mo[k] = S.emask[k];
  } else {
    GAS float* adj_out = gptr(P.o.adj) + (size_t)env * N * EE;
    if ((E & 3) == 0) {
      // each thread owns float4 column groups of the E x E table: values computed once,
      // masked per ego (once when every ego shares the mask) and stored for every ego
      for (int t = tid; t < EE / 4; t += BT) {
        const int u = 4 * t;
        const int r = qdiv<NT>(u, E, P.m_E), c = u - r * E;
        const float4 v = make_float4(adj_value(P, S, r, c), adj_value(P, S, r, c + 1), adj_value(P, S, r, c + 2),
                                     adj_value(P, S, r, c + 3));
#pragma unroll 1
        for (int e = 0; e < N; ++e) {
          const uint64_t* m = S.emask + (uni ? 0 : e * MW);
          const uint32_t bits = mbit(m, r) ? 0xfu : (uint32_t)((m[c >> 6] >> (c & 63)) & 0xfull);
          float4 w = v;
          if (bits & 1u) w.x = 0.f;
          if (bits & 2u) w.y = 0.f;
          if (bits & 4u) w.z = 0.f;
          if (bits & 8u) w.w = 0.f;
          st_stream<true>(adj_out + (size_t)e * EE + u, w);
        }
      }
    } else {
      for (int q = tid; q < N * EE; q += BT) {
        const int e = qdiv<NT>(q, EE, P.m_EE);
        const int u = q - e * EE;
        const int r = qdiv<NT>(u, E, P.m_E), c = u - r * E;
        const uint64_t* m = S.emask + e * MW;
        adj_out[q] = (mbit(m, r) || mbit(m, c)) ? 0.0f : adj_value(P, S, r, c);
      }
    }
  }
  emit_nodes<DYN, BT, NT>(P, S, env, uni);
}

template <int DYN, int NT>
__device__ __forceinline__ void reset_block(const KParams& P, Lds& S, int env, const double* cur_new,
                                            const double* layout = nullptr) {
  const int tid = threadIdx.x;
  LSM_DIMS;
  reset_core<DYN, BT, NT>(P, S, env, cur_new, layout);   // ends with a barrier
  const int MW = (E + 63) >> 6;
  // the reset's disconnect masks: nothing in the training scenario; undeparted agents
  // (RealisticScenario) and circular_config's kept-done agents in a layout (pre == post here)
  mask_words(S, N, E);
  __syncthreads();
  for (int k = tid; k < N * MW; k += BT) S.emask[k] = S.mpost[k % MW];
  entity_table<NT>(P, S);
  if (tid < N) write_obs<DYN, NT>(P, S, env, tid);
  __syncthreads();
  emit_graph_block<DYN, NT>(P, S, env);
}

// NIS1: num_internal_step == 1 (the training default), compiled without the inner loop. Config 5
// went from 1240 to 1490 us per step (same-session A/B, profiles/r03_v14_bisect_c5.txt) when the
// loop came in: 172 VGPRs instead of 165, so 2 waves per SIMD instead of 3. waves_per_eu(3) holds
// the kernel to the 168 VGPRs of 3 waves.
// REXT: the optional reward terms / shared reward may be on (P.rext). Config 5 (training default,
// rext off) ran 1232 us with the rext block compiled in and 1206 us without it (same-session A/B,
// profiles/r06_s05_ab_c5_bisect.txt: the round 3 -> 4 regression), so the host launches a REXT=false
// instance when neither is configured.
template <int DYN, int NT, bool NIS1, bool REXT>
__global__ __launch_bounds__(BT) __attribute__((amdgpu_waves_per_eu(DYN == 0 ? 3 : 1)))
void rollout_block_kernel(const KParams* __restrict__ Pp, const KStep K) {
  const KParams& P = *Pp;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int env = xcd_block(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int lane = tid;   // (STAMP macros)
  if (env >= P.n_envs) return;   // uniform over the workgroup
  LSM_DIMS;
  const int MW = (E + 63) >> 6;
  constexpr int T = NT ? block_tpe(NT) : 64;      // butterfly bound (generic: up to 64 lanes)
  const int TE = NT ? T : block_tpe(N);           // threads per ego actually used
#ifdef LSM_XP_POISON
  LDS_POISON(smem, P.lds_env_bytes, tid, BT);
  __syncthreads();
#endif
  Lds S = carve_block(smem, N, NL, E, F);
  // RealisticScenario departure arrays (airtaxi layouts; the Bay Area intersection at 16 agents)
  if (DYN == 1 && NT == 0 && P.scenario == LSM_SCENARIO_DEPARTURES) carve_dep(S, smem, P.lds_dep_off, N);
  RTSTAMP(13);
#ifdef LSM_STAMPS
  if (tid == 0 && gptr(P.stamps))
    gptr(P.stamps)[(size_t)env * LSM_NSTAMP + 15] = (unsigned long long)__builtin_amdgcn_s_getreg(63492) |
                                      ((unsigned long long)__builtin_amdgcn_s_getreg(6164) << 32);
#endif
  STAMP(0);

  // ---- 0. the env's record HBM -> LDS + this step's actions ------------------------------
  const int ai = (K.mode == 0 && tid < N) ? load_action(K, env, N, tid) : 0;
  rec_copy<BT>((const GAS f32x4*)gptr(P.s.rec) + (size_t)env * P.s.rec_stride16, (f32x4*)smem, P.s.rec16);
  __syncthreads();
  if (tid < N) {
    S.dpre[tid] = S.dpost[tid];
    S.rpre[tid] = S.rpost[tid];
    if (DYN == 1) {
      S.ecs[tid] = cos(S.ps[2 * N + tid]);
      S.ecs[N + tid] = sin(S.ps[2 * N + tid]);
    }
    if (S.dep0 && K.mode == 0) {
      const GAS double* dg = gptr(P.s.dep) + (size_t)env * depw(N);
      S.dep0[tid] = S.dep1[tid] = dg[tid] != 0.0;
      S.tmr[tid] = (int32_t)dg[N + tid];
      S.ith[tid] = dg[2 * N + tid];
      S.pth[tid] = S.ps[2 * N + tid];
      S.psp[tid] = S.ps[3 * N + tid];
    }
  }
  const int cstep = S.step[0] + 1;
  __syncthreads();
  STAMP(1);

  if (K.mode != 0) {   // 1: device scenario, 2: host layout (lsm_reset_layout)
    reset_block<DYN, NT>(P, S, env, K.cur_new, K.mode == 2 ? K.layout : nullptr);
    __syncthreads();
    store_state<DYN, BT, NT>(P, S, smem, env, true);
    return;
  }

  // ---- 1. update_graph() at step start (previous state, final masks) ----------------------
  if (K.emit_edges) {
    entity_table<NT>(P, S);
    mask_words(S, N, E);
    __syncthreads();
    const bool fresh = S.step[1] != 0;   // lsm_set_agent_state: calculate_distances() unmasked
    if (S.dep0 && !fresh) {
      // departures: the last ego's accumulated mask of the previous step, as stored
      if (tid < MW) S.mpost[tid] = ((const GAS uint64_t*)(gptr(P.s.dep) + (size_t)env * depw(N) + 3 * N))[tid];
      __syncthreads();
    }
    GAS uint8_t* eo = gptr(P.o.edges) + (size_t)env * E * E;
    for (int u = tid; u < E * E; u += BT) {
      const int a = qdiv<NT>(u, E, P.m_E), b = u - a * E;
      const double dx = S.ex[a] - S.ex[b], dy = S.ey[a] - S.ey[b];
      double d = sqrt(dx * dx + dy * dy);
      if (!fresh && (mbit(S.mpost, a) || mbit(S.mpost, b))) d = 0.0;
      eo[u] = (d <= P.coord_range && d > 0) ? 1 : 0;
    }
  }

  // ---- 2. decode actions ----------------------------------------------------------------
  if (tid < N) {
    if (ai < 0 || ai > 24) *gptr(P.action_err) = 1;   // lsm_action_errors() reports it
    const int a = ai < 0 ? 0 : (ai > 24 ? 24 : ai);
    const int xi = a / 5, yi = a - xi * 5;
    S.raw[tid] = P.act0[xi];
    S.raw[N + tid] = P.act1[yi];
  }
  __syncthreads();
  STAMP(2);

  // ---- 3. safety filter: T threads per ego, butterfly argmins --------------------------------
  // The argmin of the HJ value over the other active agents needs exact values only where it
  // can be decided: pass 1 bounds every in-range pair by its block's (min, max) (an L2-resident
  // table) and takes the smallest upper bound U over the ego's pairs; pass 2 looks up the exact
  // value only where the lower bound is <= U. A skipped pair's value exceeds U >= the minimum,
  // so the argmin (first occurrence on ties) and its value are exactly the full search's.
  const bool filter_on = S.cur[C_FILT] != 0.0;
  // World.step's inner loop (core.py:607-631): filter -> action_diff -> integrate, num_internal_step
  // times on the same raw actions
  const int nis = NIS1 ? 1 : P.nis;
  for (int it = 0; it < nis; ++it) {
  if (filter_on) {
    const SepChain sc = sep_chain(S.sep, P.s, env);
    const int i = tid / TE, q = tid - (tid / TE) * TE;
    int jd = -1, jv = -1, okv = 0;
    double dmin = 0.0;
    float vmin = 0.0f;
    const bool ego = i < N && !inactive_pre(S, i);
    constexpr int JN = NT ? (NT + T - 1) / T : 0;   // pairs per thread (compile-time N)
    if (JN > 0 && P.filter_search == 1) {
      // pass 1: bounds of every pair, loads issued together (slots unrolled)
      float lbk[JN > 0 ? JN : 1];   // +inf: no candidate; -inf: candidate outside the grid
      float ub = INFINITY;
#pragma unroll
      for (int k = 0; k < JN; ++k) {
        const int j = q + k * TE;
        lbk[k] = INFINITY;
        if (ego && j < N && j != i && !inactive_pre(S, j)) {
          const double ex = S.ps[i], ey = S.ps[N + i], ox = S.ps[j], oy = S.ps[N + j];
          const double d = sqrt((ox - ex) * (ox - ex) + (oy - ey) * (oy - ey));
          if (jd < 0 || d < dmin) { jd = j; dmin = d; }
          double rel[5];
          rel_state<DYN>(S, N, i, j, rel);
          float2 b;
          if (DYN == 0 ? value_bounds<4>(P.val, rel, b, sc) : value_bounds<5>(P.val, rel, b, sc)) {
            lbk[k] = b.x;
            ub = fminf(ub, b.y);
          } else {
            lbk[k] = -INFINITY;
          }
        }
      }
#pragma unroll
      for (int off = 1; off < T; off <<= 1) ub = fminf(ub, __shfl_xor(ub, off));
      // pass 2: exact values where the lower bound can still win. The survivors of the wave's
      // 64 lanes are compacted into a per-wave LDS queue (in U1, free during the filter) and
      // looked up 64 at a time, so the gathers of different slots overlap instead of running
      // one slot after another; each lane then walks its slots in order for the argmin.
      uint32_t smask = 0;
#pragma unroll
      for (int k = 0; k < JN; ++k)
        if (lbk[k] != INFINITY && lbk[k] != -INFINITY && !(lbk[k] > ub)) smask |= 1u << k;
      const int wl = tid & (WAVE - 1);
      const int cnt = __popc(smask);
      int incl = cnt;
#pragma unroll
      for (int o = 1; o < WAVE; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (wl >= o) incl += y;
      }
      const int total = __shfl(incl, WAVE - 1);
      const int base = incl - cnt;
      uint16_t* qij = (uint16_t*)S.feat + (tid / WAVE) * (WAVE * JN);
      float* qv = (float*)((uint16_t*)S.feat + (BT / WAVE) * (WAVE * JN)) + (tid / WAVE) * (WAVE * JN);
      {
        int p = base;
        uint32_t m = smask;
        while (m) {
          const int k = __ffs(m) - 1;
          m &= m - 1;
          qij[p++] = (uint16_t)(i | ((q + k * TE) << 8));
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int x = wl; x < total; x += WAVE) {
        const int ii = qij[x] & 0xff, jj = qij[x] >> 8;
        double rel[5];
        rel_state<DYN>(S, N, ii, jj, rel);
        float v = 0.0f;
        const bool ok = DYN == 0 ? interp_value<4>(P.val, rel, v, sc) : interp_value<5>(P.val, rel, v, sc);
        qv[x] = ok ? v : __builtin_nanf("");
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      int p = base;
#pragma unroll
      for (int k = 0; k < JN; ++k) {
        const float lb = lbk[k];
        if (lb == INFINITY) continue;   // no candidate
        float v = INFINITY;
        bool ok = false;
        if (lb != -INFINITY) {
          if (lb > ub) continue;        // cannot be the argmin
          const float r = qv[p++];
          ok = !(r != r);
          v = ok ? r : INFINITY;
        }
        const int j = q + k * TE;
        if (jv < 0 || v < vmin) { jv = j; vmin = v; okv = ok ? 1 : 0; }
      }
    } else {
      // full search: every pair's exact value (UNR lookups in flight per thread)
      if (ego) {
#pragma unroll 4
        for (int j = q; j < N; j += TE) {
          if (j == i || inactive_pre(S, j)) continue;
          const double ex = S.ps[i], ey = S.ps[N + i], ox = S.ps[j], oy = S.ps[N + j];
          const double d = sqrt((ox - ex) * (ox - ex) + (oy - ey) * (oy - ey));
          double rel[5];
          rel_state<DYN>(S, N, i, j, rel);
          float v = 0.0f;
          bool ok;
          if (DYN == 0) ok = interp_value<4>(P.val, rel, v, sc); else ok = interp_value<5>(P.val, rel, v, sc);
          if (!ok) v = INFINITY;
          if (jd < 0 || d < dmin) { jd = j; dmin = d; }
          if (jv < 0 || v < vmin) { jv = j; vmin = v; okv = ok ? 1 : 0; }
        }
      }
    }
#pragma unroll
    for (int off = 1; off < T; off <<= 1) {
      if (off >= TE) break;
      const int jd2 = __shfl_xor(jd, off), jv2 = __shfl_xor(jv, off), ok2 = __shfl_xor(okv, off);
      const double d2 = __shfl_xor(dmin, off);
      const float v2 = __shfl_xor(vmin, off);
      if (jd2 >= 0 && (jd < 0 || d2 < dmin || (d2 == dmin && jd2 < jd))) { jd = jd2; dmin = d2; }
      if (jv2 >= 0 && (jv < 0 || v2 < vmin || (v2 == vmin && jv2 < jv))) { jv = jv2; vmin = v2; okv = ok2; }
    }
    STAMP(3);
    if (q == 0 && i < N) {
      double u0 = S.raw[i], u1 = S.raw[N + i];
      uint8_t fl = 0;
      int dec = -1;
      if (ego && jd >= 0) {   // else: no other active agent
        dec = jv;
        if (!(dmin > P.coord_range) && okv) filter_apply<DYN, NT>(P, S, i, jv, vmin, fl, u0, u1);
      }
      S.sfilt[i] = fl;
      S.decon[i] = dec;
      S.safe[i] = u0;
      S.safe[N + i] = u1;
      S.adiff[i] = blas_norm2(S.raw[i] - u0, S.raw[N + i] - u1);
    }
  } else if (tid < N) {
    const double u0 = S.raw[tid], u1 = S.raw[N + tid];
    S.safe[tid] = u0;
    S.safe[N + tid] = u1;
    S.adiff[tid] = blas_norm2(S.raw[tid] - u0, S.raw[N + tid] - u1);
  }
  __syncthreads();
  STAMP(4);

  // ---- 4. integrate ------------------------------------------------------------------------
  if (tid < N && !inactive_pre(S, tid)) integrate_agent<DYN>(P, S, N, tid);
  __syncthreads();
  if (DYN == 1 && it + 1 < nis) {   // the next inner filter's ego frame: the new headings
    if (tid < N) {
      S.ecs[tid] = cos(S.ps[2 * N + tid]);
      S.ecs[N + tid] = sin(S.ps[2 * N + tid]);
    }
    __syncthreads();
  }
  }
  STAMP(5);
  if (P.o.cforce && tid < N) {   // optional contact forces (collision_force_agent)
    double fx, fy;
    collision_force_agent(S, N, tid, fx, fy);
    GAS double* cf = gptr(P.o.cforce) + ((size_t)env * N + tid) * 2;
    cf[0] = fx;
    cf[1] = fy;
  }
  entity_table<NT>(P, S);

  // ---- 5. min relative distance (active agents) and is_collision counts (all agents) ------
  {
    const int i = tid / TE, q = tid - (tid / TE) * TE;
    double m = INFINITY;
    int cc = 0;
    if (i < N) {
      const bool iact = !inactive_pre(S, i);
#pragma unroll 4
      for (int j = q; j < N; j += TE) {
        if (j == i) continue;
        const double d2 = blas_norm2(S.ps[i] - S.ps[j], S.ps[N + i] - S.ps[N + j]);
        if (iact && !inactive_pre(S, j)) m = (d2 < m) ? d2 : m;
        if (d2 < 1.05 * (0.05 + 0.05)) cc++;
      }
    }
#pragma unroll
    for (int off = 1; off < T; off <<= 1) {
      if (off >= TE) break;
      const double o = __shfl_xor(m, off);
      m = (o < m) ? o : m;
      cc += __shfl_xor(cc, off);
    }
    if (q == 0 && i < N) {
      S.minrel[i] = m;
      S.ccnt[i] = cc;
    }
  }
  STAMP(6);

  // ---- 6. obs, reward, goal/done update ---------------------------------------------------
  double mag = 0.0;
  if (DYN == 0 && !P.use_filter_arg) mag = magnetic_penalty_wave<BT, NT>(P, S, S.dpair);   // has barriers
  AgentTmp at;
  if (tid < N) reward_agent<DYN, NT>(P, S, env, tid, mag, at);
  __syncthreads();
  if (REXT && P.rext) {   // optional reward terms / shared reward (reward_finish)
    if (tid < N) reward_finish<DYN, NT>(P, S, env, tid, at);
    __syncthreads();
    if (P.collab && tid < N) reward_shared<NT>(P, S, env, tid);
    __syncthreads();
  }
  mask_words(S, N, E);
  __syncthreads();
  for (int k = tid; k < N * MW; k += BT) {
    const int e = k / MW, w = k - e * MW;
    const uint64_t sel = post_sel(N, L, e, w);
    uint64_t m = (S.mpost[w] & sel) | (S.mpre[w] & ~sel);
    if (S.dep0 && w == 0) {
      // graph_observation masks cached_dist_mag IN PLACE (navigation_graph_safe.py:986-987): a
      // departure connects, so agent j >= 1 undeparted before the update was masked by ego 0 and
      // stays masked for every later ego of this step (agents are entities 0..N-1 <= 63: word 0)
      for (int j = 1; j < N; ++j)
        if (!S.dep0[j]) m |= 1ull << j;
    }
    S.emask[k] = m;
  }
  STAMP(7);

  // ---- 7/8. info_callback numbers -----------------------------------------------------------
  if (tid < N) info_agent<DYN, NT>(P, S, tid, cstep, at, S.ccnt[tid]);
  __syncthreads();
  if (tid < N) info_row<NT>(P, S, tid, at.rew, S.dpair + tid * LSM_INFO_FIELDS);
  __syncthreads();
  rec_copy<BT>((const f32x4*)S.dpair, (GAS f32x4*)(gptr(P.o.info) + (size_t)env * N * LSM_INFO_FIELDS),
               N * LSM_INFO_FIELDS / 2);
  STAMP(8);

  // ---- episode stats (environment.py:1004-1022), dones -------------------------------------
  {
    const int i = tid / TE, q = tid - (tid / TE) * TE;
    int cnt = 0, neng = 0;
    double mn = INFINITY;
    // `agent.departed and not agent.done` (environment.py:1008); departed is always True in the
    // training scenario
    const bool act = i < N && !S.dpost[i] && (!S.dep1 || S.dep1[i]);
    if (act) {
      const uint64_t* m = S.emask + i * MW;
      const bool mi = mbit(m, i);
#pragma unroll 4
      for (int j = q; j < N; j += TE) {
        if (mi || mbit(m, j)) continue;
        const double dx = S.ps[i] - S.ps[j], dy = S.ps[N + i] - S.ps[N + j];
        const double d = sqrt(dx * dx + dy * dy);
        if (!(d < P.coord_range && d > 0)) continue;
        cnt++;
        if (d < P.world_eng) neng++;
        mn = (d < mn) ? d : mn;
      }
    }
#pragma unroll
    for (int off = 1; off < T; off <<= 1) {
      if (off >= TE) break;
      const double o = __shfl_xor(mn, off);
      mn = (o < mn) ? o : mn;
      cnt += __shfl_xor(cnt, off);
      neng += __shfl_xor(neng, off);
    }
    if (q == 0 && act) stats_agent<DYN>(P, S, N, i, cnt, neng, mn);
  }
  bool my_done = true;
  if (tid < N) {
    if (S.dpost[tid]) S.stats[2 * N + tid] = 1;
    my_done = S.dpost[tid] || cstep >= P.episode_length;
    gptr(P.o.dones)[(size_t)env * N + tid] = my_done ? 1 : 0;
  }
  const bool all_done = __syncthreads_and(my_done);
  write_masks(P, env, N, tid, my_done, all_done);
  STAMP(9);

  // ---- 9. graph outputs, or the auto-reset (whose outputs replace them) ---------------------
  if (tid == 0) { S.step[0] = cstep; S.step[1] = 0; }
  if (P.auto_reset && all_done) {
    if (tid == 0) gptr(P.o.reset_flag)[env] = 1;
    reset_block<DYN, NT>(P, S, env, K.cur_new);
    __syncthreads();
    store_state<DYN, BT, NT>(P, S, smem, env, true);
  } else {
    if (tid == 0) gptr(P.o.reset_flag)[env] = 0;
    emit_graph_block<DYN, NT>(P, S, env);
    __syncthreads();
    STAMP(10);
    store_state<DYN, BT, NT>(P, S, smem, env, false);
  }
  STAMP(11);
  RTSTAMP(14);
}
