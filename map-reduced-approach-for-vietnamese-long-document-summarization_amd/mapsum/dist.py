"""Chunk data-parallelism for the map phase.

Each map call depends only on its chunk (runners/run_summarization_ollama_mapreduce.py:103-106)
and summaries meet only at collect/reduce (:114-164), so the map phase shards with no
data-path communication: one process per GPU, each with a full weight replica, owns a
subset of the (doc, chunk) units.  The only collective is one gather of the per-chunk
summary ids to the reduce rank -- over RCCL (torch.distributed backend "nccl") on GPUs,
gloo in the CPU tests.  The payload is tiny (int32 [n_local, 3 + max_tokens]) and
latency-bound, so it is a single fixed-size all_gather, not a ring of buckets.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True, order=True)
class Unit:
    doc: int
    chunk: int
    n_tokens: int


def shard_static(units: list, rank: int, world: int) -> list:
    """Uniform chunks (configs 1-3): unit i goes to rank i mod world (order kept)."""
    return [u for i, u in enumerate(units) if i % world == rank]


def shard_lpt(units: list, rank: int, world: int) -> list:
    """Ragged chunks (config 4): longest-processing-time greedy on prompt length, so every
    rank gets about the same prefill work; ties broken by (doc, chunk) for determinism."""
    loads = [0] * world
    mine = []
    for u in sorted(units, key=lambda u: (-u.n_tokens, u.doc, u.chunk)):
        r = min(range(world), key=lambda k: (loads[k], k))
        loads[r] += u.n_tokens
        if r == rank:
            mine.append(u)
    return sorted(mine, key=lambda u: (u.doc, u.chunk))


def pack_results(units: list, token_lists: list, max_tokens: int) -> np.ndarray:
    """[n, 3 + max_tokens] int32 rows: doc, chunk, n, ids (zero padded)."""
    out = np.zeros((len(units), 3 + max_tokens), np.int32)
    for i, (u, t) in enumerate(zip(units, token_lists)):
        t = list(t)[:max_tokens]
        out[i, 0], out[i, 1], out[i, 2] = u.doc, u.chunk, len(t)
        out[i, 3:3 + len(t)] = t
    return out


def unpack_results(rows: np.ndarray) -> dict:
    """{(doc, chunk): ids} from gathered rows (padding rows have n == -1)."""
    res = {}
    for r in rows:
        if r[2] < 0:
            continue
        res[(int(r[0]), int(r[1]))] = r[3:3 + int(r[2])].tolist()
    return res


def gather_summaries(packed: np.ndarray, max_rows: int, device=None, group=None) -> np.ndarray | None:
    """all_gather the ranks' packed rows (padded to ``max_rows``); returns every rank's
    rows on rank 0 (and on the others, which the reduce step may ignore).  With one
    process it is the identity."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return packed
    width = packed.shape[1]
    buf = np.full((max_rows, width), -1, np.int32)
    buf[:len(packed)] = packed
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    from ._lib import trace
    with trace("mapsum.gather"):
        dist.all_gather(outs, t, group=group)
        return torch.cat(outs).cpu().numpy()


def env_rank() -> tuple[int, int, int]:
    """(rank, local_rank, world) from torchrun's environment (1 process if unset)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


# ---------------------------------------------------------------- weight broadcast
class _DeviceBytes:
    """A zero-copy torch view of engine-owned device memory (__cuda_array_interface__)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3}


def broadcast_tensors(tensors: list, src: int = 0, group=None) -> None:
    """Broadcast each tensor from ``src`` in place (RCCL over xGMI for CUDA tensors; gloo
    for the CPU tests)."""
    import torch.distributed as dist
    for t in tensors:
        dist.broadcast(t, src=src, group=group)


def broadcast_engine_weights(engine, src: int = 0, group=None) -> int:
    """SURVEY.md §5 "distributed communication backend": rank ``src`` has loaded the weights
    (bf16, or a K-quant model); every other rank receives them over RCCL instead of reading
    the checkpoint itself.  The K-quant layout travels first (a manifest of (tensor, layer,
    type) the receivers declare), then every device weight buffer, in the engine's fixed
    region order.  Returns the bytes broadcast."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    box = [engine.quant_manifest() if rank == src else None]
    dist.broadcast_object_list(box, src=src, group=group)
    if rank != src:
        for tensor, layer, ty in box[0]:
            engine.declare_weight_q(tensor, layer, ty)
    views = region_views(engine)
    if views and views[0].is_cuda:
        torch.cuda.synchronize(views[0].device)
    broadcast_tensors(views, src=src, group=group)
    if views and views[0].is_cuda:
        torch.cuda.synchronize(views[0].device)
    return sum(v.numel() for v in views)


def region_views(engine) -> list:
    """uint8 tensors aliasing the engine's weight regions (engines that are not libmapsum --
    the CPU test double -- provide ``region_views`` themselves)."""
    import torch
    if hasattr(engine, "region_views"):
        return engine.region_views()
    dev = torch.device("cuda", engine.device)
    return [torch.as_tensor(_DeviceBytes(p, n), device=dev) for p, n in engine.weight_regions()]
