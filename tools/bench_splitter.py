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
    res = {}
    for name, mk in [("plain", lambda: (lambda t: len(tok.encode(t)))), ("batched", lambda: TokenLength(tok))]:
        sp = RecursiveCharacterTextSplitter(12000, 200, mk(), SEPARATORS)
        t0 = time.perf_counter()
        chunks = [sp.split_text(d) for d in docs]
        dt = time.perf_counter() - t0
        res[name] = chunks
        n = sum(len(c) for c in chunks)
        print(f"{name:8s}: {a.docs} docs, {n} chunks in {dt:.3f} s = {n / dt:.1f} chunks/s", flush=True)
    assert res["plain"] == res["batched"]


if __name__ == "__main__":
    main()
