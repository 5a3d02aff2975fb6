"""GNNBase.process_adj (gnn.py:376-407) on the device: lsm_edges.hip through the C ABI vs the numpy
oracle (oracle/process_adj.py), which is itself pinned here against torch.nonzero -- the call the
reference makes -- on CPU tensors. Bit-exact: edge_index equal, edge_attr equal (a copy of the
adjacency values, no arithmetic)."""
import numpy as np
import pytest

from golden_replay import fixture_names, load
from oracle.process_adj import expand_compact, process_adj as ora_process_adj


def _torch_process_adj(adj):
    """The reference's own expressions (gnn.py:392-406), run with torch on the CPU."""
    import torch
    adj = torch.as_tensor(adj)
    if adj.dim() == 3:
        E = adj.shape[1]
        ei = adj.nonzero(as_tuple=False)
        attr = adj[ei[:, 0], ei[:, 1], ei[:, 2]]
        batch = ei[:, 0] * E
        ei = torch.stack([batch + ei[:, 1], batch + ei[:, 2]], dim=0)
    else:
        ei = adj.nonzero(as_tuple=False).t().contiguous()
        attr = adj[ei[0], ei[1]]
    return ei.numpy(), attr.unsqueeze(1).numpy()


def _random_adj(rng, B, E, density=0.3, specials=True):
    a = rng.uniform(0.01, 2.0, (B, E, E)).astype(np.float32)
    a[rng.random((B, E, E)) > density] = 0.0
    if specials and B * E * E > 8:
        flat = a.reshape(-1)
        idx = rng.choice(flat.size, 4, replace=False)
        flat[idx[0]] = -0.0            # not an edge (torch: -0.0 == 0)
        flat[idx[1]] = np.nan          # an edge (NaN != 0)
        flat[idx[2]] = -1.5            # negative values are edges too
        flat[idx[3]] = np.float32(1e-38)
    if B > 2:
        a[1] = 0.0                     # an empty graph inside the batch
    return a


def _random_masks(rng, n, N, E):
    W = (E + 63) // 64
    m = rng.integers(0, 2 ** 63, (n, N, W), dtype=np.int64)
    sparse = rng.random((n, N, W)) < 0.7   # mostly connected, like the common step
    m[sparse] &= rng.integers(0, 2 ** 63, (int(sparse.sum()),), dtype=np.int64) & \
        rng.integers(0, 2 ** 63, (int(sparse.sum()),), dtype=np.int64) & 0x0F0F0F0F0F0F0F0F
    tail = E - 64 * (W - 1)
    if tail < 64:
        m[:, :, W - 1] &= (1 << tail) - 1
    return m


def _assert_same(got, want):
    ge, ga = got
    we, wa = want
    assert ge.dtype == np.int64 and ge.shape == we.shape
    np.testing.assert_array_equal(ge, we)
    assert ga.shape == wa.shape and ga.dtype == np.float32
    np.testing.assert_array_equal(ga, wa)   # NaN == NaN positions via assert_array_equal


# ---------------- CPU: pin the oracle ----------------

@pytest.mark.parametrize("B,E", [(1, 9), (5, 24), (3, 48), (2, 192), (4, 1)])
def test_oracle_matches_torch_nonzero(B, E):
    rng = np.random.default_rng(B * 1000 + E)
    a = _random_adj(rng, B, E)
    _assert_same(ora_process_adj(a), _torch_process_adj(a))
    _assert_same(ora_process_adj(a[0]), _torch_process_adj(a[0]))


def test_oracle_on_golden_adjacency():
    for name in fixture_names():
        z, meta = load(name)
        for k in [k for k in z.files if k.endswith("_adj")][:3]:
            adj = np.asarray(z[k], dtype=np.float32)
            E = adj.shape[-1]
            flat = adj.reshape(-1, E, E)
            _assert_same(ora_process_adj(flat), _torch_process_adj(flat))


def test_oracle_expand_compact_matches_host_expansion():
    import torch
    from lsm.vec_env import expand_compact_adj
    rng = np.random.default_rng(5)
    for (n, N, E) in [(3, 8, 24), (2, 64, 192), (2, 3, 9)]:
        A = _random_adj(rng, n, E, specials=False)
        M = _random_masks(rng, n, N, E)
        want = expand_compact_adj(torch.as_tensor(A), torch.as_tensor(M), E).numpy()
        np.testing.assert_array_equal(expand_compact(A, M), want)


def test_wrapper_rejects_host_tensors_and_bad_shapes():
    import torch
    from lsm import edges
    with pytest.raises(edges.EdgeError):
        edges.process_adj(torch.zeros(2, 3, 4))
    with pytest.raises(edges.EdgeError):
        edges.process_adj(torch.zeros(2, 3, 3, dtype=torch.float64))
    with pytest.raises(edges.EdgeError):
        edges.process_adj(torch.zeros(2, 3, 3))   # CPU tensor: no fallback


# ---------------- GPU: the HIP path ----------------

def _gpu(x):
    import torch
    return torch.as_tensor(x).to("cuda:0")


def _run_ref(a):
    from lsm import edges
    ei, ea = edges.process_adj(_gpu(a))
    return ei.cpu().numpy(), ea.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("B,E", [(1, 1), (7, 9), (1000, 24), (257, 48), (33, 192), (3, 256), (5, 65)])
def test_gpu_process_adj_reference_layout(B, E):
    rng = np.random.default_rng(B + 7 * E)
    a = _random_adj(rng, B, E)
    _assert_same(_run_ref(a), ora_process_adj(a))


@pytest.mark.gpu
@pytest.mark.parametrize("B,E", [(1023, 3), (1025, 3), (8193, 3), (32769, 2), (65536, 2), (65537, 2)])
def test_gpu_process_adj_scan_sizes(B, E):
    """Graph counts around 1024 / 8192 / 32 768 / 65 536 for the offsets scan (a one-workgroup scan
    kernel was measured at these sizes against hipcub's and dropped, profiles/r05_s3{8,9}_*)."""
    rng = np.random.default_rng(B)
    a = _random_adj(rng, B, E)
    _assert_same(_run_ref(a), ora_process_adj(a))


@pytest.mark.gpu
def test_gpu_process_adj_2d_empty_and_dense():
    rng = np.random.default_rng(1)
    a = _random_adj(rng, 1, 24)[0]
    _assert_same(_run_ref(a), ora_process_adj(a))
    z = np.zeros((4, 24, 24), np.float32)
    ei, ea = _run_ref(z)
    assert ei.shape == (2, 0) and ea.shape == (0, 1)
    d = rng.uniform(0.5, 1.0, (6, 48, 48)).astype(np.float32)   # every entry an edge
    _assert_same(_run_ref(d), ora_process_adj(d))


@pytest.mark.gpu
@pytest.mark.parametrize("n,N,E", [(3, 3, 9), (64, 8, 24), (9, 16, 48), (5, 64, 192)])
def test_gpu_process_adj_compact_layout(n, N, E):
    from lsm import edges
    rng = np.random.default_rng(n * N)
    A = _random_adj(rng, n, E)
    M = _random_masks(rng, n, N, E)
    ei, ea = edges.process_adj_compact(_gpu(A), _gpu(M), N)
    want = ora_process_adj(expand_compact(A, M).reshape(-1, E, E))
    _assert_same((ei.cpu().numpy(), ea.cpu().numpy()), want)


@pytest.mark.gpu
def test_gpu_process_adj_golden_adjacency():
    for name in fixture_names():
        z, meta = load(name)
        for k in [k for k in z.files if k.endswith("_adj")]:
            adj = np.asarray(z[k], dtype=np.float32)
            E = adj.shape[-1]
            flat = np.ascontiguousarray(adj.reshape(-1, E, E))
            _assert_same(_run_ref(flat), ora_process_adj(flat))


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["reference", "compact"])
def test_gpu_env_edge_list_full_size(layout):
    """Config 3 size (8 agents x 4096 envs): the env's own edge list vs the oracle on its adjacency,
    over a few steps with auto-resets; both layouts give the same edges."""
    import torch
    from lsm import hj_tables
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    args = EnvArgs(num_agents=8, num_env_steps=250 * 4, use_safety_filter=True, seed=0)
    vt, _ = hj_tables.default_tables("double_integrator", small=True)
    env = GpuGraphVecEnv(args, num_envs=4096, device="cuda:0", value_table=vt, return_numpy=False,
                         build_infos=False, adj_layout=layout)
    env.reset(4)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    for t in range(3):
        env.step(torch.randint(0, 25, (4096, 8), generator=g, device="cuda:0", dtype=torch.int32), 4)
        ei, ea = env.edge_list()
        ref = env.reference_adj().reshape(-1, env.E, env.E).cpu().numpy()
        _assert_same((ei.cpu().numpy(), ea.cpu().numpy()), ora_process_adj(ref))
    env.close()


@pytest.mark.gpu
@pytest.mark.parametrize("B,E", [(1000, 24), (33, 192), (7, 9)])
def test_gpu_process_adj_bounded_and_exact_paths_agree(B, E):
    """The one-sync path (outputs sized by B*E*E, nnz read on the device by the emit kernel) and the
    count-first path (outputs sized exactly) give the same tensors, both equal to the oracle; the
    bounded results are contiguous [2, nnz] / [nnz, 1] views."""
    from lsm import edges
    rng = np.random.default_rng(B * 3 + E)
    a = _random_adj(rng, B, E)
    want = ora_process_adj(a)
    saved = edges.BOUNDED_OUTPUT_BYTES
    try:
        edges.BOUNDED_OUTPUT_BYTES = 4 << 30
        ei, ea = edges.process_adj(_gpu(a))
        assert ei.is_contiguous() and ea.is_contiguous()
        _assert_same((ei.cpu().numpy(), ea.cpu().numpy()), want)
        edges.BOUNDED_OUTPUT_BYTES = 0
        _assert_same(_run_ref(a), want)
    finally:
        edges.BOUNDED_OUTPUT_BYTES = saved


@pytest.mark.gpu
def test_gpu_edges_emit_dev_writes_nothing_past_cap():
    """lsm_edges_emit_dev with cap < nnz (offsets[B] read on the device) leaves the outputs untouched."""
    import ctypes as C
    import torch
    from lsm import capi
    lib = capi.load_library()
    rng = np.random.default_rng(5)
    a = _gpu(_random_adj(rng, 16, 24, density=0.8))
    B, E = 16, 24
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    off = torch.empty(B + 2, dtype=torch.int64, device="cuda:0")
    wsb = int(lib.lsm_edges_workspace_bytes(B))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device="cuda:0")
    assert lib.lsm_edges_count(C.c_void_p(a.data_ptr()), None, B, E, 1, C.c_void_p(off.data_ptr()),
                               C.c_void_p(ws.data_ptr()), wsb, st) == 0
    nnz = int(off[B].item())
    cap = nnz // 2
    ei = torch.full((2 * cap,), -7, dtype=torch.int64, device="cuda:0")
    ea = torch.full((cap,), -7.0, dtype=torch.float32, device="cuda:0")
    assert lib.lsm_edges_emit_dev(C.c_void_p(a.data_ptr()), None, B, E, 1, C.c_void_p(off.data_ptr()), cap,
                                  C.c_void_p(ei.data_ptr()), C.c_void_p(ea.data_ptr()), st) == 0
    torch.cuda.synchronize()
    assert bool((ei == -7).all()) and bool((ea == -7.0).all())


@pytest.mark.gpu
def test_gpu_bounded_result_storage_is_o_nnz():
    """a bounded-path result must not pin the B*E*E*20-byte buffers when it holds far
    fewer edges -- it is copied to exact size (storage <= SHRINK_RATIO x the exact bytes)."""
    from lsm import edges
    rng = np.random.default_rng(17)
    B, E = 2000, 24
    a = _random_adj(rng, B, E, density=0.02, specials=False)
    want = ora_process_adj(a)
    ei, ea = edges.process_adj(_gpu(a))
    _assert_same((ei.cpu().numpy(), ea.cpu().numpy()), want)
    nnz = want[0].shape[1]
    assert nnz * edges.SHRINK_RATIO < B * E * E
    assert ei.untyped_storage().nbytes() <= edges.SHRINK_RATIO * 16 * nnz
    assert ea.untyped_storage().nbytes() <= edges.SHRINK_RATIO * 4 * nnz


@pytest.mark.gpu
def test_gpu_process_adj_compact_repeatable_config3():
    """Round 5's intermittent undercount (profiles/r05_s21_edges_diag.txt: a variant reading the mask
    word of every element from global memory lost one edge in a few graphs of some calls): the
    shipped count, on a config-3 compact adjacency with disconnect bits, 24 times on unchanged
    inputs, every per-graph count equal to numpy's."""
    import torch
    from lsm import hj_tables
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    args = EnvArgs(num_agents=8, num_env_steps=250 * 4, use_safety_filter=True, seed=0)
    vt, _ = hj_tables.default_tables("double_integrator", small=True)
    env = GpuGraphVecEnv(args, num_envs=4096, device="cuda:0", value_table=vt, return_numpy=False,
                         build_infos=False, adj_layout="compact")
    env.reset(4)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    for _ in range(40):   # agents reach goals: disconnect bits set in many graphs
        env.step(torch.randint(0, 25, (4096, 8), generator=g, device="cuda:0", dtype=torch.int32), 4)
    assert int((env.t_adj_mask != 0).sum()) > 0
    want = (env.reference_adj().reshape(-1, env.E, env.E) != 0).sum(dim=(1, 2)).cpu().numpy()
    from lsm import capi, edges
    import ctypes as C
    lib = capi.load_library()
    B = 4096 * 8
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    off = torch.empty(B + 2, dtype=torch.int64, device="cuda:0")
    wsb = int(lib.lsm_edges_workspace_bytes(B))
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda:0")
    for rep in range(24):
        assert lib.lsm_edges_count(C.c_void_p(env.t_adj.data_ptr()), C.c_void_p(env.t_adj_mask.data_ptr()), B,
                                   env.E, 8, C.c_void_p(off.data_ptr()), C.c_void_p(ws.data_ptr()), wsb, st) == 0
        got = np.diff(off[:B + 1].cpu().numpy())
        np.testing.assert_array_equal(got, want, err_msg="call %d" % rep)
    env.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["di8_team", "di8_team_compact", "di8_wave", "di3_lpe16", "di5_lpe32",
                                  "at16_team_lean", "at4_generic"])
def test_gpu_step_edge_counts_one_pass(case):
    """LSM_OUT_ADJ_NNZ: the step kernel's per-ego nonzero counts equal the stored adjacency's (numpy
    count of the reference-layout adj, either output layout, across auto-resets and goal / done
    status changes), and edge_list()'s one-pass path (lsm_edges_scan_emit) equals the oracle's
    process_adj bit for bit; counts of another adjacency are refused."""
    import torch
    from lsm import edges, hj_tables
    from lsm.config import EnvArgs
    from lsm.vec_env import GpuGraphVecEnv
    spec = dict(di8_team=("double_integrator", 8, "reference", None),
                di8_team_compact=("double_integrator", 8, "compact", None),
                di8_wave=("double_integrator", 8, "reference", {"team": 0}),
                di3_lpe16=("double_integrator", 3, "reference", {"lanes_per_env": 16}),
                di5_lpe32=("double_integrator", 5, "reference", {"lanes_per_env": 32}),
                at16_team_lean=("airtaxi", 16, "reference", None),
                at4_generic=("airtaxi", 4, "compact", {"generic": 1}))[case]
    dyn, N, layout, ksel = spec
    ws = 4 if dyn == "double_integrator" else 6
    args = EnvArgs(dynamics_type=dyn, num_agents=N, world_size=ws, episode_length=12, num_env_steps=12 * 4,
                   use_safety_filter=True, seed=4)
    n = 37
    env = GpuGraphVecEnv(args, num_envs=n, device="cuda:0", small_tables=True, return_numpy=False,
                         build_infos=False, adj_layout=layout, kernel_select=ksel, emit_edge_counts=True)
    if ksel is None:
        assert env.kernel_name.startswith("rollout_team_kernel<")
    env.reset(4)
    E = env.E
    rng = np.random.default_rng(N)
    for t in range(30):   # resets at steps 11 and 23
        env.step(rng.integers(0, 25, (n, N)), 4)
        ref = env.reference_adj().reshape(-1, E, E)
        want = (ref != 0).sum(dim=(1, 2)).cpu().numpy()
        np.testing.assert_array_equal(env.t_adj_nnz.reshape(-1).cpu().numpy(), want, err_msg="step %d" % t)
        ei, ea = env.edge_list()
        _assert_same((ei.cpu().numpy(), ea.cpu().numpy()), ora_process_adj(ref.cpu().numpy()))
    bad = env.t_adj_nnz.clone()
    bad[3, 1] += 1
    with pytest.raises(edges.EdgeError, match="differ"):
        if layout == "compact":
            edges.process_adj_compact(env.t_adj, env.t_adj_mask, N, counts=bad)
        else:
            edges.process_adj(env.t_adj.view(-1, E, E), counts=bad)
    env.close()


def test_scratch_reuse_keys_and_bound():
    """lsm.edges reuses the offsets / scan workspace per (device, stream, B) and keeps at most 8 keys
    (host logic only: a stand-in for the workspace query, CPU tensors)."""
    import torch
    from lsm import edges

    class _Lib:
        calls = 0

        def lsm_edges_workspace_bytes(self, B):
            _Lib.calls += 1
            return 64 * B + 256

    lib, dev = _Lib(), torch.device("cpu")
    edges._SCRATCH.clear()
    o1, w1, n1 = edges._scratch(lib, dev, 0, 10)
    o2, w2, n2 = edges._scratch(lib, dev, 0, 10)
    assert o1 is o2 and w1 is w2 and n1 == n2 == 64 * 10 + 256 and _Lib.calls == 1
    assert o1.shape == (12,) and o1.dtype == torch.int64 and w1.numel() == n1   # [B + 2]: + error word
    assert edges._scratch(lib, dev, 1, 10)[0] is not o1      # another stream: its own buffers
    assert edges._scratch(lib, dev, 0, 11)[0].shape == (13,)  # another graph count
    for b in range(20, 40):
        edges._scratch(lib, dev, 0, b)
    assert len(edges._SCRATCH) <= 8
    edges._SCRATCH.clear()
