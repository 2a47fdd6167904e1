"""Host-side chunking throughput: the pipeline's token-length
RecursiveCharacterTextSplitter(12000, 200) over synthetic Vietnamese documents of the
corpus' average size (54,566 tokens, metadata/doc_metadata.json:2-10), with the plain
per-piece ``len(tokenizer.encode(t))`` vs mapsum.splitter.TokenLength (batched, memoised).

    python tools/bench_splitter.py [--docs 8]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "map-reduced-approach-for-vietnamese-long-document-summarization_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from mapsum.hierarchical import SEPARATORS, RecursiveCharacterTextSplitter  # noqa: E402
from mapsum.splitter import TokenLength  # noqa: E402
from test_splitter import viet_doc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=8)
    ap.add_argument("--vocab", type=int, default=4000)
    a = ap.parse_args()
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    from mapsum.tokenizer import Tokenizer as MT
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=a.vocab, special_tokens=["<|begin_of_text|>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator([viet_doc(s, 40) for s in range(40)], tr)
    tok = MT.from_object(tk)
    docs = []
    for s in range(a.docs):  # grow each doc to ~54.6k tokens
        d, n = "", 0
        while n < 54566:
            d = (d + "\n\n" if d else "") + viet_doc(1000 * s + n, 20)
            n = len(tok.encode(d))
        docs.append(d)
    toks = sum(len(tok.encode(d)) for d in docs)
    for size in (12000, 2048):  # the pipeline's chunk_size (:994-998) and the bench unit (§8d)
        res = {}
        for name, mk in [("plain", lambda: (lambda t: len(tok.encode(t)))), ("batched", lambda: TokenLength(tok))]:
            sp = RecursiveCharacterTextSplitter(size, 200, mk(), SEPARATORS)
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                chunks = [sp.split_text(d) for d in docs]
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
                sp.length = mk()  # cold length cache every round
            res[name] = chunks
            n = sum(len(c) for c in chunks)
            print(f"chunk_size {size:5d} {name:8s}: {a.docs} docs ({toks} tokens), {n} chunks in {best:.3f} s = "
                  f"{n / best:.1f} chunks/s, {toks / best / 1e3:.0f} k tokens/s", flush=True)
        assert res["plain"] == res["batched"]
    print("engine consumption for comparison: configs[2] 33.5 chunks/s per MI355X x 2048 tokens = 68.6 k prompt "
          "tokens/s per GPU, 549 k tokens/s on 8 GPUs (profiles/r02/v26_config2_B128.json)")


if __name__ == "__main__":
    main()
