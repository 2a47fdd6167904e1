"""TEST INFRASTRUCTURE ONLY -- CPU restatement (oracle) of the map-phase hot path.

Nothing in the product path may import this package.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` use it,
and only as the checker / the timed CPU reference.

What it restates:
  * A1/A7/A8/A9 -- the arithmetic behind the per-chunk ``OllamaLLM._call``
    (``run_full_evaluation_pipeline.py:80-106``): Llama-3.2 prefill + greedy
    decode.  The arithmetic lives in Ollama/llama.cpp (EXT, not vendored, not
    pinned), so this is a restatement of the *published*
    Llama-3.2 architecture, pinned against ``transformers.LlamaForCausalLM``
    on seeded tiny models (``tests/golden/make_golden.py``).  Parity against
    Ollama itself is **unpinned** (no Ollama, no GGUF, no tokenizer here).
  * the synthetic-weight generator shared with the engine (``synth.py``).
"""
