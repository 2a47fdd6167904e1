"""The pipeline's token-length splitter (mapsum/splitter.py; reference
run_full_evaluation_pipeline.py:344-361): the batched, memoised length function gives the
same chunks as the plain ``len(tokenizer.encode(text))`` with far fewer tokenizer calls.
The Llama-3.2 tokenizer is not available offline: a byte-level BPE trained here stands in
(same library, same ``encode`` semantics incl. the BOS that makes ``len(encode(""))`` 1)."""
import random

import pytest

from mapsum.hierarchical import SEPARATORS, RecursiveCharacterTextSplitter
from mapsum.splitter import TokenLength, pipeline_splitter, split_documents

WORDS = ("Việt Nam kinh tế xã hội lịch sử văn hóa chính sách phát triển người dân đất nước "
         "năm thế kỷ chiến tranh hòa bình giáo dục khoa học công nghệ nông nghiệp").split()


def viet_doc(seed, paragraphs=40):
    rnd = random.Random(seed)
    paras = []
    for _ in range(paragraphs):
        sents = []
        for _ in range(rnd.randrange(2, 9)):
            sents.append(" ".join(rnd.choice(WORDS) for _ in range(rnd.randrange(6, 30))).capitalize()
                         + rnd.choice([".", "!", "?", ";"]))
        paras.append(" ".join(sents))
    return "\n\n".join(paras)


@pytest.fixture(scope="module")
def tok():
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    from mapsum.tokenizer import Tokenizer as MT
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=600, special_tokens=["<|begin_of_text|>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator([viet_doc(s, 10) for s in range(5)], tr)
    return MT.from_object(tk)


def test_length_counts_bos_like_hf_encode(tok):
    tl = TokenLength(tok)
    assert tl("") == 1  # len(tokenizer.encode("")) == 1: the BOS alone
    t = "Việt Nam kinh tế."
    assert tl(t) == len(tok.encode(t, add_bos=False)) + 1


@pytest.mark.parametrize("size,overlap", [(12000, 200), (300, 40), (80, 0), (25, 5)])
def test_batched_equals_plain(tok, size, overlap):
    doc = viet_doc(size + overlap)
    plain = RecursiveCharacterTextSplitter(size, overlap, lambda t: len(tok.encode(t)), SEPARATORS)
    tl = TokenLength(tok)
    batched = RecursiveCharacterTextSplitter(size, overlap, tl, SEPARATORS)
    a, b = plain.split_text(doc), batched.split_text(doc)
    assert a == b and len(a) >= 1
    if size < 12000:
        assert tl.batches > 0 and tl.calls < len(a)  # pieces measured in batches, not one by one
        for c in b:  # every chunk fits unless it is one unsplittable piece
            assert tl(c) <= size + 1 or len(c.split()) == 1


def test_pipeline_splitter_defaults(tok):
    sp = pipeline_splitter(tok)
    assert (sp.chunk_size, sp.chunk_overlap, sp.separators) == (12000, 200, SEPARATORS)
    docs = [viet_doc(s, 300) for s in range(2)]
    chunks = split_documents(docs, tok, chunk_size=2000, chunk_overlap=200)
    assert [len(c) > 1 for c in chunks] == [True, True]
    for d, cs in zip(docs, chunks):  # nothing lost: every word of the doc is in some chunk
        assert set(d.split()) <= set(" ".join(cs).split())
