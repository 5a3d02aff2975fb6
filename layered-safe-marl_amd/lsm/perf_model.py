"""Algorithmic HBM bytes of one ``rollout_kernel`` launch (the bench's roofline numerator).

Counts the bytes that MUST cross HBM for one env-step of the reference-layout
path, per env:

* the env's persistent record (lsm_rollout.hip StateDev / lds_plan), read whole and
  written back up to the curriculum block: agent state 4N f64, episode stats 6N f64,
  info accumulators 4N f64, travel distance / goal_min_time / min relative distance /
  action diff N f64 each, done / reached / safety flag / deconflicting index N i32
  each, step counter i32 (every field 16-B aligned) | curriculum block 12 f64 + the HJ
  separation shift chain 10 f64, landmarks 6NL f64 and the landmark-pair distance cache
  NL(NL-1)/2 f32 (read only; written back only at a reset);
* actions: N i32 read;
* outputs written: obs N*OBS f32, node_obs N*E*F f32, adj N*E*E f32, reward N f32,
  done N u8, reset flag 1 u8, info N*18 f64, state copy 4N f64.

* filter on, the HJ-table gathers SURVEY §8(d) counts: one value query per ordered pair of
  agents (2^d corners x 4 B: 64 B for the 4-D DI table, 128 B for the 5-D airtaxi table) and
  one gradient query per ego (2^d corners x 16 B / 32 B). The device table is the
  cell-corner-replicated layout (16x / 32x the node table, ~1.8 GB for the full DI table), far
  larger than L2 + Infinity Cache, and rocprofv3 FETCH_SIZE per launch exceeds the record reads
  by about these bytes (profiles/), so they are HBM bytes. Also reported alone as
  ``gather_bytes``.
"""
from __future__ import annotations


def step_bytes(N: int, L: int = 2, dynamics: str = "double_integrator", filter_on: bool = True,
               adj_layout: str = "reference") -> dict:
    """`adj_layout` "compact": one unmasked E x E f32 table per env + N * ceil(E/64) u64
    masks instead of N * E * E f32. Envs with N > 32 or E > 64 run the workgroup kernel,
    whose record has no landmark-pair cache."""
    NL = N * L
    E = N + NL
    block = N > 32 or E > 64
    di = dynamics == "double_integrator"
    F = 10 if di else 11
    OBS = 7 if di else 6
    a16 = lambda x: (x + 15) // 16 * 16
    hot = (a16(8 * 4 * N) + a16(8 * 6 * N) + a16(8 * 4 * N) + 4 * a16(8 * N) + 4 * a16(4 * N) + 16)
    rec = hot + a16(8 * (12 + 10)) + a16(8 * 6 * NL) + (0 if block else a16(4 * (NL * (NL - 1) // 2)))
    state_r = rec + N * 4
    state_w = hot
    adj = E * E * 4 + N * ((E + 63) // 64) * 8 if adj_layout == "compact" else N * E * E * 4
    outputs = N * OBS * 4 + N * E * F * 4 + adj + N * 4 + N + 1 + N * 18 * 8 + 4 * N * 8
    corners = 16 if di else 32
    gw = 16 if di else 32
    gathers = (corners * 4 * N * (N - 1) + corners * gw * N) if filter_on else 0
    hbm = state_r + state_w + outputs + gathers
    return dict(hbm_bytes=hbm, outputs=outputs, state=state_r + state_w, gather_bytes=gathers,
                E=E, F=F, OBS=OBS, block=block)
