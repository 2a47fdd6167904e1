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
    dist.all_gather(outs, t, group=group)
    return torch.cat(outs).cpu().numpy()


def env_rank() -> tuple[int, int, int]:
    """(rank, local_rank, world) from torchrun's environment (1 process if unset)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))
