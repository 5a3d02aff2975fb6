// lsm_scenario.h -- Scenario.random_scenario (navigation_graph_safe.py:1199-1367) and
// randomly_generate_separated_positions (custom_scenarios/utils.py:39-68), replayed
// draw-for-draw on numpy's legacy MT19937 stream of env k (seed + 1000 k).
//
// Written once for both targets: the reset kernel instantiates it with the
// wave-cooperative RNG (all 64 lanes execute the identical scalar sequence, the
// MT19937 twist is split across lanes), the host test entry point with HostMT.
// Output layout is the device's SoA: st[c * N + i] (c = x, y, v_x|theta, v_y|v),
// lm[c * NL + k] (c = x, y, heading, speed), landmark k = order * N + agent.
#pragma once
#include "lsm_numeric.h"

namespace lsm {

constexpr int MAX_L = 8;
constexpr int SCEN_WS = 7 * MAX_L;   // workspace doubles (LDS on the device)

struct ScenarioParams {
  int dyn;          // 0 DI, 1 airtaxi
  int N, L;
  double world_size;
  double coordination_range;
  double goal_speed_min, goal_speed_max;
  double ratio_airtaxi;     // curriculum_ratio_airtaxi in random_scenario
  double ratio_scenario;    // curriculum_ratio (1 with the filter, else sloped)
  double two_pi, pi;
  double d2lo, d2hi;        // the device draw's band on squared distances (KParams::scen_d2lo / hi)
};

template <class Rng>
LSM_HD void separated_positions(Rng& rng, int n, double x0, double x1, double y0, double y1,
                                double dmin, double dmax, double* pos /* [n][2] */) {
  for (int i = 0; i < n; ++i) {
    double x, y;
    if (i > 0) {
      for (int j = 0; j < 1000; ++j) {
        x = rng.uniform(x0, x1);
        y = rng.uniform(y0, y1);
        double d = 0.0;
        for (int k = 0; k < i; ++k) {
          double dx = pos[2 * k] - x, dy = pos[2 * k + 1] - y;
          double dk = sqrt(dx * dx + dy * dy);
          if (k == 0 || dk < d) d = dk;
        }
        if (d > dmin && d < dmax) break;
        if (rng.exhausted()) break;   // a lane stream ran out: the scenario is redrawn (lsm_team.h)
      }
    } else {
      x = rng.uniform(x0, x1);
      y = rng.uniform(y0, y1);
    }
    pos[2 * i] = x;
    pos[2 * i + 1] = y;
  }
}

template <class Rng>
LSM_HD void random_scenario(Rng& rng, const ScenarioParams& p, double* st, double* lm, double* ws) {
  const int N = p.N, L = p.L, NL = N * L;
  const double wsz = p.world_size;
  const double cra = p.ratio_airtaxi;
  double* gp = ws;                  // [L][2]
  double* prev = ws + 2 * MAX_L;    // [L][2]
  double* heads = ws + 4 * MAX_L;   // [L]
  double* speeds = ws + 5 * MAX_L;  // [L]
  double* rnd = ws + 6 * MAX_L;     // [L]
  for (int i = 0; i < N; ++i) {
    if (p.dyn == 0) {
      double x = rng.uniform(-0.8 * wsz, 0.8 * wsz);
      double y = rng.uniform(-0.8 * wsz, 0.8 * wsz);
      st[0 * N + i] = x; st[1 * N + i] = y; st[2 * N + i] = 0.0; st[3 * N + i] = 0.0;
    } else {
      double xmin = -0.5 * wsz;
      double xmax = 0.25 * wsz * cra + 0.0 * (1 - cra) * wsz;
      double y = rng.uniform(-0.5 * wsz, 0.5 * wsz);
      double x = rng.uniform(xmin, xmax);
      double spd = rng.uniform(p.goal_speed_min, p.goal_speed_max);
      double th = rng.uniform(0.0, p.two_pi);
      st[0 * N + i] = x; st[1 * N + i] = y; st[2 * N + i] = th; st[3 * N + i] = spd;
    }
  }
  bool have_prev = false;
  for (int i = 0; i < N; ++i) {
    if (p.dyn == 0) {
      separated_positions(rng, L, -0.5 * wsz, 0.5 * wsz, -0.5 * wsz, 0.5 * wsz,
                          0.25 * p.coordination_range, 0.75 * p.coordination_range, gp);
      if (have_prev)
        for (int k = 0; k < L; ++k)
          if (rng.uniform(0.0, 1.0) < 0.5) { gp[2 * k] = prev[2 * k]; gp[2 * k + 1] = prev[2 * k + 1]; }
    } else {
      double yw = 0.1 * (1 - cra) + 0.5 * cra;
      separated_positions(rng, L, 0.0, 0.75 * wsz, -yw * wsz, yw * wsz,
                          0.5 * p.coordination_range, p.coordination_range, gp);
      if (have_prev)
        for (int k = 0; k < L; ++k)
          if (rng.uniform(0.0, 1.0) < 0.5) { gp[2 * k] = prev[2 * k]; gp[2 * k + 1] = prev[2 * k + 1]; }
      if (gp[0] > gp[2]) {
        double tx = gp[0], ty = gp[1];
        gp[0] = gp[2]; gp[1] = gp[3];
        gp[2] = tx; gp[3] = ty;
      }
    }
    for (int k = 0; k < L - 1; ++k) heads[k] = atan2(gp[2 * k + 3] - gp[2 * k + 1], gp[2 * k + 2] - gp[2 * k]);
    const double last = heads[L - 2];
    const double cr = p.ratio_scenario;
    if (p.dyn != 0) {
      for (int k = 0; k < L; ++k) speeds[k] = p.goal_speed_max * 1.0;
    } else {
      for (int k = 0; k < L; ++k) rnd[k] = rng.uniform(p.goal_speed_min, p.goal_speed_max);
      double var = rng.uniform(0.0, 1.0);
      bool use_rnd = var < py_min(cr, 1 - 0.2);
      for (int k = 0; k < L; ++k) speeds[k] = use_rnd ? rnd[k] : p.goal_speed_max * 1.0;
      if (!use_rnd) speeds[L - 1] = p.goal_speed_min;
    }
    for (int k = 0; k < L - 1; ++k) {
      double pr = (p.dyn == 0) ? cr * 0.25 * p.pi : cra * 0.1 * p.pi;
      heads[k] += rng.uniform(-pr, pr);
    }
    heads[L - 1] = last;
    for (int k = 0; k < L; ++k) {
      int idx = k * N + i;
      lm[0 * NL + idx] = gp[2 * k];
      lm[1 * NL + idx] = gp[2 * k + 1];
      lm[2 * NL + idx] = heads[k];
      lm[3 * NL + idx] = speeds[k];
    }
    for (int k = 0; k < 2 * L; ++k) prev[k] = gp[k];
    have_prev = true;
  }
}

}  // namespace lsm
