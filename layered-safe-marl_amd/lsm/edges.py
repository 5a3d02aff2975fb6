"""Device-side ``GNNBase.process_adj`` (``onpolicy/algorithms/utils/gnn.py:376-407``).

``process_adj(adj)`` takes the rollout's adjacency (a CUDA float32 tensor ``(B, E, E)`` or
``(E, E)``, e.g. ``GpuGraphVecEnv.t_adj`` viewed as ``(n*N, E, E)``) and returns
``(edge_index int64 [2, nnz], edge_attr float32 [nnz, 1])`` in ``nonzero()`` order, the pair the
reference's GNN consumes. ``process_adj_compact(A, masks, N)`` does the same for the compact layout
(``LSM_ADJ_COMPACT``: one ``[n, E, E]`` table + per-ego disconnect masks), expanding each ego's
matrix on the fly instead of materialising ``(n, N, E, E)``.

Like ``torch.nonzero`` the call synchronises once (the edge count sizes the outputs): after both
kernels when the upper bound B*E*E of the outputs fits BOUNDED_OUTPUT_BYTES (the results are then
contiguous views of those buffers, copied to exact size when they would hold more than twice the
edges), else between them. ``counts`` (int64 [B], the step kernel's LSM_OUT_ADJ_NNZ for this
adjacency) skips the count pass: the call is then a scan and one emit pass over the adjacency
(``lsm_edges_scan_emit``), and a count that does not match its graph raises. All work runs in
``lsm_edges.hip`` through the C ABI; there is no torch/CPU fallback.
"""
from __future__ import annotations

import ctypes as C

from . import capi


class EdgeError(RuntimeError):
    pass


def _torch():
    import torch
    return torch


def _check(rc, lib):
    if rc != 0:
        raise EdgeError(lib.lsm_edges_last_error().decode())


# outputs sized by the edge-count upper bound B*E*E up to this many bytes: count and emit then run back
# to back and the call synchronises once, after both (the returned tensors are views of the
# bounded buffers); above it the count is read first and the outputs are sized exactly
BOUNDED_OUTPUT_BYTES = 1 << 30
# a bounded result holding fewer than cap / SHRINK_RATIO edges is copied to exact size, so what the
# caller keeps is O(nnz) (at most SHRINK_RATIO x the exact storage), not O(B*E*E)
SHRINK_RATIO = 2


# offsets + scan workspace of the last few (device, stream, B): reused by the next call with the same
# key (stream-ordered: that call's count kernel runs after this call's emit kernel has read them), so a
# call's host prologue before its first launch -- GPU idle time after the previous call's sync -- is
# two ctypes launches instead of two allocations and a workspace query more
_SCRATCH = {}


def _scratch(lib, dev, stream_handle, B):
    torch = _torch()
    key = (dev.index, stream_handle, B)
    hit = _SCRATCH.get(key)
    if hit is None:
        ws_bytes = int(lib.lsm_edges_workspace_bytes(B))
        hit = (torch.empty(B + 2, dtype=torch.int64, device=dev),   # offsets[B + 1]: counts-path error word
               torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev), ws_bytes)
        if len(_SCRATCH) >= 8:
            _SCRATCH.clear()
        _SCRATCH[key] = hit
    return hit


def _bounded(ebuf, abuf, nnz, cap):
    """The [2, nnz] / [nnz, 1] results as views of the bounded buffers, or exact-size copies when the
    buffers are more than SHRINK_RATIO x what they hold (a kept view pins B*E*E*20 B)."""
    ei, ea = ebuf[:2 * nnz].view(2, nnz), abuf[:nnz].view(nnz, 1)
    if nnz * SHRINK_RATIO < cap:
        ei, ea = ei.clone(), ea.clone()
    return ei, ea


def _run(adj, masks, B, E, N, counts=None):
    torch = _torch()
    lib = capi.load_library()
    dev = adj.device
    if dev.type != "cuda":
        raise EdgeError("process_adj needs a CUDA (HIP) tensor; the edge list is built on the GPU")
    sh = torch.cuda.current_stream(dev).cuda_stream
    stream = C.c_void_p(sh)
    offsets, ws, ws_bytes = _scratch(lib, dev, sh, B)
    mp = C.c_void_p(masks.data_ptr()) if masks is not None else None
    ap = C.c_void_p(adj.data_ptr())
    cap = B * E * E
    if counts is not None:
        # one adjacency pass: the step kernel's per-graph counts -> scan -> emit (one ctypes call)
        if counts.dtype != torch.int64 or counts.numel() != B or counts.device != dev:
            raise EdgeError("counts must be int64 [B] on the adjacency's device (LSM_OUT_ADJ_NNZ)")
        counts = counts.contiguous()
        ebuf = torch.empty(2 * max(cap, 1), dtype=torch.int64, device=dev)
        abuf = torch.empty(max(cap, 1), dtype=torch.float32, device=dev)
        host = (C.c_int64 * 2)()   # nnz, mismatched graphs: read back by the call itself (the one sync)
        _check(lib.lsm_edges_scan_emit(ap, mp, B, E, N, C.c_void_p(counts.data_ptr()),
                                       C.c_void_p(offsets.data_ptr()), C.c_void_p(ws.data_ptr()), ws_bytes, cap,
                                       C.c_void_p(ebuf.data_ptr()), C.c_void_p(abuf.data_ptr()), host, stream), lib)
        nnz, bad = int(host[0]), int(host[1])
        if nnz > cap:
            raise EdgeError("edge count %d exceeds B*E*E = %d" % (nnz, cap))
        if bad:
            raise EdgeError("%d graphs' nonzeros differ from the given counts (counts of another adjacency?)" % bad)
        return _bounded(ebuf, abuf, nnz, cap)
    _check(lib.lsm_edges_count(ap, mp, B, E, N, C.c_void_p(offsets.data_ptr()), C.c_void_p(ws.data_ptr()),
                               ws_bytes, stream), lib)
    if 0 < cap * 20 <= BOUNDED_OUTPUT_BYTES:
        ebuf = torch.empty(2 * cap, dtype=torch.int64, device=dev)
        abuf = torch.empty(cap, dtype=torch.float32, device=dev)
        _check(lib.lsm_edges_emit_dev(ap, mp, B, E, N, C.c_void_p(offsets.data_ptr()), cap,
                                      C.c_void_p(ebuf.data_ptr()), C.c_void_p(abuf.data_ptr()), stream), lib)
        nnz = int(offsets[B].item())   # the one sync, as in torch.nonzero (after both kernels)
        if nnz > cap:
            raise EdgeError("edge count %d exceeds B*E*E = %d" % (nnz, cap))
        return _bounded(ebuf, abuf, nnz, cap)
    nnz = int(offsets[B].item())   # the one sync, as in torch.nonzero
    edge_index = torch.empty((2, nnz), dtype=torch.int64, device=dev)
    edge_attr = torch.empty((nnz, 1), dtype=torch.float32, device=dev)
    if nnz:
        _check(lib.lsm_edges_emit(ap, mp, B, E, N, C.c_void_p(offsets.data_ptr()), nnz,
                                  C.c_void_p(edge_index.data_ptr()), C.c_void_p(edge_attr.data_ptr()), stream), lib)
    return edge_index, edge_attr


def process_adj(adj, counts=None):
    """gnn.py:376-407 on a (B, E, E) or (E, E) float32 CUDA tensor; counts: optional int64 [B]
    per-graph nonzeros (LSM_OUT_ADJ_NNZ of the step that wrote adj)."""
    torch = _torch()
    if not (2 <= adj.dim() <= 3) or adj.size(-1) != adj.size(-2):
        raise EdgeError("adj must be (B, E, E) or (E, E)")   # the reference asserts the same
    if adj.dtype != torch.float32:
        raise EdgeError("adj must be float32 (the runner's buffer dtype, graph_buffer.py:95-104)")
    a = adj.contiguous()
    E = a.size(-1)
    B = a.size(0) if a.dim() == 3 else 1
    return _run(a, None, B, E, 1, None if counts is None else counts.reshape(-1))


def process_adj_compact(table, masks, num_agents: int, counts=None):
    """Edges of the per-ego graphs of a compact-layout adjacency: ``table`` [n, E, E] float32,
    ``masks`` [n, N, ceil(E/64)] int64 (bit r of ego e = entity r disconnected). Graph b = env*N +
    ego, so the result equals ``process_adj(expand_compact_adj(table, masks, E).view(-1, E, E))``."""
    torch = _torch()
    n, E = table.size(0), table.size(-1)
    W = (E + 63) // 64
    if table.dtype != torch.float32 or tuple(table.shape) != (n, E, E):
        raise EdgeError("table must be float32 [n, E, E]")
    if tuple(masks.shape) != (n, num_agents, W) or masks.dtype != torch.int64:
        raise EdgeError("masks must be int64 [n, N, ceil(E/64)]")
    return _run(table.contiguous(), masks.contiguous(), n * num_agents, E, num_agents,
                None if counts is None else counts.reshape(-1))
