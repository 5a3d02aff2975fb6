"""DIAGNOSTIC: lsm_edges_count / lsm_edges_emit on a random compact-layout input (the failing case
of tests/test_edges.py::test_gpu_process_adj_compact_layout) -- per-graph counts against numpy, and
per graph the emitted edges against the oracle: which graphs and elements differ, with their mask
words. Optional argv[1:]: other libraries whose lsm_edges_* are compared too."""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def bind(lib):
    P, I32, I64, SZ = C.c_void_p, C.c_int32, C.c_int64, C.c_size_t
    for f, (res, args) in {"lsm_edges_count": (I32, [P, P, I64, I32, I32, P, P, SZ, P]),
                           "lsm_edges_emit": (I32, [P, P, I64, I32, I32, P, I64, P, P, P]),
                           "lsm_edges_workspace_bytes": (SZ, [I64])}.items():
        getattr(lib, f).restype = res
        getattr(lib, f).argtypes = args
    return lib


def main():
    import torch
    from lsm import capi
    from oracle.process_adj import expand_compact, process_adj as ora
    from test_edges import _random_adj, _random_masks
    libs = [("cur", bind(capi.load_library()))]
    for path in sys.argv[1:]:   # other builds' lsm_edges_* (e.g. round 5's, a failing variant's)
        libs.append((os.path.basename(path), bind(C.CDLL(path))))
    for (n, N, E) in [(64, 8, 24), (3, 3, 9), (9, 16, 48)]:
        rng = np.random.default_rng(n * N)
        A = _random_adj(rng, n, E)
        M = _random_masks(rng, n, N, E)
        ref = expand_compact(A, M).reshape(-1, E, E)
        want_cnt = (ref != 0).reshape(ref.shape[0], -1).sum(axis=1)
        wei, wea = ora(ref)
        B = n * N
        dA = torch.as_tensor(A).cuda()
        dM = torch.as_tensor(M).cuda()
        dR = torch.as_tensor(np.ascontiguousarray(ref)).cuda()
        st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        for name, lib in libs:
            for src, (a, m, NN) in (("compact", (dA, dM, N)), ("reference", (dR, None, 1))):
                wsb = int(lib.lsm_edges_workspace_bytes(B))
                ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
                off = torch.zeros(B + 2, dtype=torch.int64, device="cuda")
                mp = C.c_void_p(m.data_ptr()) if m is not None else None
                assert lib.lsm_edges_count(C.c_void_p(a.data_ptr()), mp, B, E, NN, C.c_void_p(off.data_ptr()),
                                           C.c_void_p(ws.data_ptr()), wsb, st) == 0
                o = off.cpu().numpy()[:B + 1]
                cnt = np.diff(o)
                badc = np.nonzero(cnt != want_cnt)[0]
                nnz = int(o[B])
                ei = torch.zeros((2, max(nnz, 1)), dtype=torch.int64, device="cuda")
                ea = torch.zeros((max(nnz, 1), 1), dtype=torch.float32, device="cuda")
                assert lib.lsm_edges_emit(C.c_void_p(a.data_ptr()), mp, B, E, NN, C.c_void_p(off.data_ptr()), nnz,
                                          C.c_void_p(ei.data_ptr()), C.c_void_p(ea.data_ptr()), st) == 0
                gei = ei.cpu().numpy()[:, :nnz]
                bad_g = []
                if len(badc) == 0 and gei.shape == wei.shape:
                    diff = np.nonzero((gei != wei).any(axis=0))[0]
                    bad_g = sorted(set((wei[0, diff] // E).tolist()))
                print("%s E=%d %s: nnz %d want %d, count-bad graphs %d %s, emit-bad graphs %d %s" %
                      (name, E, src, nnz, int(want_cnt.sum()), len(badc), badc[:5].tolist(), len(bad_g), bad_g[:5]))
                for b in bad_g[:2]:
                    e, ego = divmod(b, N)
                    sel = wei[0] // E == b
                    gw = wei[:, sel] - b * E
                    gg = gei[:, sel] - b * E
                    d = np.nonzero((gw != gg).any(axis=0))[0]
                    print("   graph %d (env %d ego %d) mask %s: first differing edge #%d want %s got %s" %
                          (b, e, ego, [hex(int(x) & (2 ** 64 - 1)) for x in M[e, ego]], int(d[0]),
                           gw[:, d[0]].tolist(), gg[:, d[0]].tolist()))
                    print("     want", gw[:, d[0]:d[0] + 6].T.tolist())
                    print("     got ", gg[:, d[0]:d[0] + 6].T.tolist())


def config3_compact(libs):
    """BASELINE config 3's compact adjacency after 40 steps (disconnect bits in many graphs): per-graph
    counts and the emitted edges of each library against the oracle (test_gpu_env_edge_list_full_size)."""
    import torch
    from lsm import hj_tables
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    from oracle.process_adj import process_adj as ora
    args = EnvArgs(num_agents=8, num_env_steps=250 * 4, use_safety_filter=True, seed=0)
    vt, _ = hj_tables.default_tables("double_integrator", small=True)
    env = GpuGraphVecEnv(args, num_envs=4096, device="cuda:0", value_table=vt, return_numpy=False,
                         build_infos=False, adj_layout="compact")
    env.reset(4)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    for _ in range(40):
        env.step(torch.randint(0, 25, (4096, 8), generator=g, device="cuda:0", dtype=torch.int32), 4)
    E, N, B = env.E, env.N, 4096 * 8
    ref = env.reference_adj().reshape(-1, E, E).cpu().numpy()
    want_cnt = (ref != 0).reshape(B, -1).sum(axis=1)
    wei, _ = ora(ref)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, lib in libs:
        for rep in range(3):
            wsb = int(lib.lsm_edges_workspace_bytes(B))
            ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
            off = torch.zeros(B + 2, dtype=torch.int64, device="cuda")
            assert lib.lsm_edges_count(C.c_void_p(env.t_adj.data_ptr()), C.c_void_p(env.t_adj_mask.data_ptr()), B, E, N,
                                       C.c_void_p(off.data_ptr()), C.c_void_p(ws.data_ptr()), wsb, st) == 0
            o = off.cpu().numpy()[:B + 1]
            badc = np.nonzero(np.diff(o) != want_cnt)[0]
            nnz = int(o[B])
            ei = torch.zeros((2, nnz), dtype=torch.int64, device="cuda")
            ea = torch.zeros((nnz, 1), dtype=torch.float32, device="cuda")
            assert lib.lsm_edges_emit(C.c_void_p(env.t_adj.data_ptr()), C.c_void_p(env.t_adj_mask.data_ptr()), B, E, N,
                                      C.c_void_p(off.data_ptr()), nnz, C.c_void_p(ei.data_ptr()),
                                      C.c_void_p(ea.data_ptr()), st) == 0
            gei = ei.cpu().numpy()
            bad_e = int((gei != wei).any(axis=0).sum()) if gei.shape == wei.shape else -1
            print("%s config-3 compact call %d: count-bad graphs %d, emit-bad edges %d" % (name, rep, len(badc), bad_e),
                  flush=True)
    env.close()


if __name__ == "__main__":
    main()
    import ctypes as _C
    from lsm import capi as _capi
    libs = [("cur", bind(_capi.load_library()))] + [(os.path.basename(p), bind(_C.CDLL(p))) for p in sys.argv[1:]]
    config3_compact(libs)
