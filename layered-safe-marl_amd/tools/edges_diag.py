"""DIAGNOSTIC: lsm_edges_count at config-3 size (compact layout) run repeatedly on static inputs,
with this tree's library and with the round-4 one (LSM_DIAG_OLDLIB, hipcub scan): per-graph counts vs
numpy's; for a miscounted graph, the values and mask bits of its row elements."""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    import torch
    from lsm import capi, hj_tables
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    libs = [("new", capi.load_library())]
    old = os.path.join(os.path.dirname(HERE), "csrc", "liblsm_rollout_head.so")
    if os.path.exists(old):
        lo = C.CDLL(old)
        for f, (res, args) in {"lsm_edges_count": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32,
                                                                C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
                               "lsm_edges_workspace_bytes": (C.c_size_t, [C.c_int64])}.items():
            getattr(lo, f).restype = res
            getattr(lo, f).argtypes = args
        libs.append(("old", lo))
    args = EnvArgs(num_agents=8, num_env_steps=250 * 4, use_safety_filter=True, seed=0)
    vt, _ = hj_tables.default_tables("double_integrator", small=True)
    env = GpuGraphVecEnv(args, num_envs=4096, device="cuda:0", value_table=vt, return_numpy=False,
                         build_infos=False, adj_layout="compact")
    env.reset(4)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    env.step(torch.randint(0, 25, (4096, 8), generator=g, device="cuda:0", dtype=torch.int32), 4)
    torch.cuda.synchronize()
    E, N = env.E, env.N
    ref = env.reference_adj().reshape(-1, E, E).contiguous()
    torch.cuda.synchronize()
    refn = ref.cpu().numpy()
    want = (refn != 0).reshape(ref.shape[0], -1).sum(axis=1)
    A = env.t_adj.cpu().numpy()
    M = env.t_adj_mask.cpu().numpy()
    print("t_adj", env.t_adj.shape, env.t_adj.stride(), "mask", env.t_adj_mask.shape, env.t_adj_mask.stride(),
          env.t_adj_mask.dtype)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    adj, masks, B = env.t_adj, env.t_adj_mask, ref.shape[0]
    seen = set()
    for name, lib in libs:
        ws_bytes = int(lib.lsm_edges_workspace_bytes(B))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device="cuda:0")
        off = torch.empty(B + 1, dtype=torch.int64, device="cuda:0")
        nbad = 0
        for rep in range(24):
            lib.lsm_edges_count(C.c_void_p(adj.data_ptr()), C.c_void_p(masks.data_ptr()), B, E, N,
                                C.c_void_p(off.data_ptr()), C.c_void_p(ws.data_ptr()), ws_bytes, st)
            torch.cuda.synchronize()
            cnt = np.diff(off.cpu().numpy())
            badg = np.nonzero(cnt != want)[0]
            nbad += len(badg)
            for b in badg[:2]:
                if b in seen:
                    continue
                seen.add(b)
                e, ego = divmod(int(b), N)
                nz = np.argwhere(refn[b] != 0)
                print(name, rep, "graph", b, "env", e, "ego", ego, "got", int(cnt[b]), "want", int(want[b]),
                      "mask word", hex(int(M[e, ego, 0]) & 0xffffffffffffffff))
                vals = refn[b][refn[b] != 0]
                tiny = vals[np.abs(vals) < 1e-30]
                print("   nonzero values: min |v|", float(np.min(np.abs(vals))), "tiny", tiny[:5].tolist(),
                      "nan", int(np.isnan(vals).sum()), "A nonzero (unmasked table)", int((A[e] != 0).sum()))
        print(name, "miscounted graphs over 24 calls:", nbad, flush=True)
    env.close()


if __name__ == "__main__":
    main()
