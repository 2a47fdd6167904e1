"""mapsum -- MI355X-native map-phase engine for the Vietnamese map-reduce summarizer.

Drop-in for the per-chunk ``OllamaLLM._call`` of the reference runners
(run_full_evaluation_pipeline.py:66-117, runners/run_summarization_ollama_mapreduce.py:23-60):
``mapsum.compat.OllamaLLM`` keeps the prompt-in/summary-out contract and runs every
chunk through ``libmapsum.so`` (hand-written gfx950 HIP kernels behind a C-ABI).
"""
from .config import CONFIGS, LLAMA32_3B, TINY, ModelConfig  # noqa: F401

__all__ = ["ModelConfig", "LLAMA32_3B", "TINY", "CONFIGS"]
