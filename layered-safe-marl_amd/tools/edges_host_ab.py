"""process_adj per-call time with the scratch buffers reused (lsm.edges._SCRATCH) vs allocated per
call (the cache cleared before each call, as the wrapper did before), alternated in one process.

    python layered-safe-marl_amd/tools/edges_host_ab.py [--graphs 32768] [--E 24] [--reps 50] [--rounds 3]

Synthetic adjacency with config 3's edge density (14.95 M of 32768 x 24 x 24 entries nonzero). Times
are HIP-event spans over `reps` back-to-back calls (each call synchronises once on its edge count).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from lsm import edges
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", type=int, default=32768)
    ap.add_argument("--E", type=int, default=24)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    adj = torch.rand((a.graphs, a.E, a.E), generator=g, device=dev)
    adj = torch.where(adj < 0.79, adj + 0.01, torch.zeros_like(adj))

    def span(reuse):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        edges.process_adj(adj)   # warm (allocator, kernels, cache entry)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            if not reuse:
                edges._SCRATCH.clear()
            edges.process_adj(adj)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps * 1e3

    ref = edges.process_adj(adj)
    nnz = ref[0].shape[1]
    res = {"reuse_us": [], "alloc_us": []}
    for _ in range(a.rounds):
        res["alloc_us"].append(round(span(False), 2))
        res["reuse_us"].append(round(span(True), 2))
    res.update({"graphs": a.graphs, "E": a.E, "nnz": nnz, "reps": a.reps})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
