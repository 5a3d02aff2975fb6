// lsm_buffer.hip -- the env-side half of GMPERunner.insert / warmup on the device.
//
// Reference: onpolicy/runner/shared/graph_mpe_runner.py:444-487 (insert) and :253-283 (warmup).
// From one step's obs [n][N][OBS] f32 and dones [n][N] it writes the GraphReplayBuffer rows
// (onpolicy/utils/graph_buffer.py:84-163, 223-249) for buffer index t + 1:
//   masks[n][N][1]        = dones ? 0 : 1                               (:457-462)
//   active_masks[n][N][1] = dones ? (all(dones[env]) ? 1 : 0) : 1       (:463-467)
//   share_obs             = centralized ? obs[env].reshape(-1) repeated per agent [n][N][N*OBS]
//                                       : obs                          (:469-484)
//   agent_id[n][N][1]     = agent index (int32, the buffer's dtype)
//   share_agent_id        = centralized ? [n][N][N] (all agent ids per row) : agent_id
// obs / node_obs / adj / rewards themselves are written by the rollout kernel straight into the
// buffer rows (lsm_bind_output_ring), so this launch only adds the derived rows. dones == NULL
// (warmup) writes share_obs / agent_id / share_agent_id only.
//
// One 64-lane wave per env: the N done flags are one ballot; share_obs is N copies of the env's
// N*OBS floats, stored as consecutive 4-B lanes (coalesced, the env's obs row read once into
// registers).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

namespace {

constexpr int WAVE = 64;
constexpr int ENVS_PER_BLOCK = 4;

struct InsertArgs {
  const float* obs;
  const uint8_t* dones;
  float* share_obs;
  int32_t* agent_id;
  int32_t* share_agent_id;
  float* masks;
  float* active_masks;
  int32_t n, N, OBS, centralized;
};

__global__ __launch_bounds__(256) void insert_kernel(InsertArgs a) {
  const int env = blockIdx.x * ENVS_PER_BLOCK + (threadIdx.x >> 6);
  if (env >= a.n) return;
  const int lane = threadIdx.x & (WAVE - 1);
  const int N = a.N, OBS = a.OBS;
  const size_t e0 = (size_t)env * N;
  if (a.dones) {
    bool all = true;   // np.all(dones, axis=1) over the env's agents
    for (int j0 = 0; j0 < N; j0 += WAVE) {
      const int j = j0 + lane;
      const bool d = j < N ? a.dones[e0 + j] != 0 : true;
      all = all && __all(d);
    }
    for (int j = lane; j < N; j += WAVE) {
      const bool d = a.dones[e0 + j] != 0;
      a.masks[e0 + j] = d ? 0.0f : 1.0f;
      a.active_masks[e0 + j] = d ? (all ? 1.0f : 0.0f) : 1.0f;
    }
  }
  for (int j = lane; j < N; j += WAVE) a.agent_id[e0 + j] = j;
  const float* o = a.obs + e0 * OBS;
  if (a.centralized) {
    const int row = N * OBS;
    float* so = a.share_obs + e0 * row;
    if ((row & 3) == 0) {   // 16-B rows (N * OBS % 4 == 0, e.g. 8 x 7): float4 copies
      const int row4 = row >> 2;
      const float4* o4 = (const float4*)o;
      float4* so4 = (float4*)so;
      for (int q = lane; q < N * row4; q += WAVE) so4[q] = o4[q % row4];
    } else {
      for (int q = lane; q < N * row; q += WAVE) so[q] = o[q % row];
    }
    int32_t* sa = a.share_agent_id + e0 * N;
    for (int q = lane; q < N * N; q += WAVE) sa[q] = q % N;
  } else {
    float* so = a.share_obs + e0 * OBS;
    for (int q = lane; q < N * OBS; q += WAVE) so[q] = o[q];
    for (int j = lane; j < N; j += WAVE) a.share_agent_id[e0 + j] = j;
  }
}

thread_local char g_err[256];

int fail(const char* m) {
  snprintf(g_err, sizeof g_err, "%s", m);
  return 1;
}

}  // namespace

extern "C" {

const char* lsm_buffer_last_error(void) { return g_err; }

int lsm_buffer_insert(const float* obs, const uint8_t* dones, int32_t n, int32_t N, int32_t OBS,
                      int32_t centralized, float* share_obs, int32_t* agent_id, int32_t* share_agent_id,
                      float* masks, float* active_masks, void* stream) {
  if (n < 0 || N <= 0 || OBS <= 0) return fail("bad shape");
  if (!obs || !share_obs || !agent_id || !share_agent_id) return fail("null obs / share_obs / agent_id pointer");
  if (dones && (!masks || !active_masks)) return fail("dones given without masks / active_masks");
  if (n == 0) return 0;
  InsertArgs a{obs, dones, share_obs, agent_id, share_agent_id, masks, active_masks, n, N, OBS, centralized != 0};
  const int blocks = (n + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK;
  insert_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(a);
  return hipGetLastError() == hipSuccess ? 0 : fail("insert_kernel launch failed");
}

}  // extern "C"
