"""bench.py's algorithmic work figures against SURVEY.md §8d (the roofline numerators)."""
import importlib.util
import os

from mapsum.config import LLAMA32_3B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(bench)


def test_prefill_flops_match_survey():
    # §8d: 1.1546e13 (linear) + 7.22e11 (attention) + lm_head on the last token ~= 1.2268e13
    f = bench.prefill_flops_per_chunk(LLAMA32_3B, 2048)
    assert abs(f - 1.2268e13) / 1.2268e13 < 1e-3


def test_decode_weight_bytes_match_survey():
    # §8d: W = 6,425,149,440 B of fp16 weights per decode step incl. the tied lm_head
    cfg, B = LLAMA32_3B, 8
    act = bench.gemv_bytes_per_step(cfg, B) - bench.gemv_bytes_per_step(cfg, 0)
    w = bench.gemv_bytes_per_step(cfg, 0) + cfg.vocab * cfg.hidden * 2
    assert w == 6_425_149_440
    assert 0 < act < 1e-2 * w  # activations are ~0.4 % of the weight stream at B = 8
    lm = bench.lm_head_bytes_per_step(cfg, B)
    assert lm == cfg.vocab * cfg.hidden * 2 + 2 * B * cfg.hidden + 4 * B * cfg.vocab


def test_q4_k_m_bytes_between_4_5_and_6_6_bits():
    cfg = LLAMA32_3B
    q = bench.qgemv_bytes_per_step(cfg, 0)
    n = bench.gemv_bytes_per_step(cfg, 0) / 2  # weights
    assert 144 / 256 <= q / n <= 224 / 256


def test_decode_weight_bytes_helper():
    assert bench.decode_weight_bytes(LLAMA32_3B) == 6_425_149_440
    q = bench.decode_weight_bytes(LLAMA32_3B, quant=True)
    assert 0.25 < q / 6_425_149_440 < 0.45


def test_docs_mode_shards_every_chunk_once():
    """configs[2]: 512 docs x 8 chunks over N ranks, chunk i -> rank i mod N."""
    for world in (1, 2, 8):
        args = bench.parse_args(["--docs", "512", "--gpus", str(world)])
        parts = [bench.local_units(args, r, world) for r in range(world)]
        flat = sorted((u.doc, u.chunk) for p in parts for u in p)
        assert flat == [(d, c) for d in range(512) for c in range(8)]
        assert {len(p) for p in parts} == {4096 // world}
    args = bench.parse_args([])
    assert [(u.doc, u.chunk) for u in bench.local_units(args, 3, 4)] == [(3, c) for c in range(8)]


def test_synthetic_chunks_are_placement_independent():
    a = bench.synthetic_chunks(3, 64, doc=5, vocab=128256, bos=128000, first_chunk=2)
    b = bench.synthetic_chunks(1, 64, doc=5, vocab=128256, bos=128000, first_chunk=3)
    assert a[1].tolist() == b[0].tolist() and len(a[0]) == 64


def test_gpus_flag_launches_ranks(monkeypatch):
    """`python bench.py --gpus N` without torchrun starts N ranks itself (before any GPU
    call in the parent) instead of silently running one."""
    seen = {}
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: seen.setdefault("cmd", cmd) and 0)
    monkeypatch.setattr(bench.sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench._spawn_ranks(4) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "2"]


def _bench_rank_worker(rank, world, port, q):
    """The bench's per-rank map step on CPU: its sharding, a FakeEngine standing in for
    libmapsum, pack_results and the gather over gloo."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from mapsum.dist import gather_summaries, pack_results, unpack_results
    from test_host import FakeEngine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    args = bench.parse_args(["--docs", "3", "--prompt-len", "32", "--gen-len", "4"])
    units = bench.local_units(args, rank, world)
    max_rows = max(len(bench.local_units(args, r, world)) for r in range(world))
    chunks = [bench.synthetic_chunks(1, 32, u.doc, 128256, 128000, first_chunk=u.chunk)[0] for u in units]
    res = FakeEngine().generate(chunks, 4)
    rows = gather_summaries(pack_results(units, [r.ids for r in res], 4), max_rows)
    if rank == 0:
        q.put(unpack_results(rows))
    dist.destroy_process_group()


def test_bench_rank_logic_world2_gloo():
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bench_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(60)
    assert sorted(got) == [(d, c) for d in range(3) for c in range(8)]
    for (d, c), ids in got.items():
        want = bench.synthetic_chunks(1, 32, d, 128256, 128000, first_chunk=c)[0][::-1][:4]
        assert ids == want.tolist()


def test_pmc_traffic_matches_rows_and_regime():
    """The roofline's PMC traffic is quoted only from a pass over the same launches: the same
    rows in flight (the engine's max_batch), hence the same decode regime (GEMV below 24 rows,
    skinny GEMM at >= 24), and the same prompt length."""
    t8, src8 = bench.pmc_traffic("f16", 8, 2048)
    assert src8 and src8.endswith("pmc_traffic_f16.json") and t8 > 57_000_000
    t128, src128 = bench.pmc_traffic("f16", 128, 2048)
    assert src128 and src128.endswith("pmc_traffic_f16_b128.json") and t128 > t8
    assert bench.pmc_traffic("f16", 64, 2048) == (None, None)  # no pass at 64 rows
    assert bench.pmc_traffic("f16", 8, 1024) == (None, None)
