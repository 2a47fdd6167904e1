"""Ollama wire shim (mapsum/server.py): the reference's own HTTP calls
(run_full_evaluation_pipeline.py:81-94 generate, :199-233 tags) against a shim backed by
the CPU test engine."""
import concurrent.futures
import time

import pytest
import requests

from mapsum import compat
from mapsum.server import OllamaShim
from test_host import FakeEngine, toy_tokenizer  # noqa: F401  (fixture)


class SlowEngine(FakeEngine):
    def step(self):
        time.sleep(0.05)  # lets concurrent requests pile up into one step
        return super().step()


@pytest.fixture
def shim(toy_tokenizer):  # noqa: F811
    eng = SlowEngine()
    be = compat.MapBackend(eng, toy_tokenizer)
    with OllamaShim({"llama3.2:3b": be}, port=0) as s:
        yield f"http://127.0.0.1:{s.port}", be, eng


def _call(url, prompt, n=1000):
    # exactly the reference's request (pipeline.py:83-94)
    payload = {"model": "llama3.2:3b", "prompt": prompt, "stream": False, "options": {"num_predict": n}}
    resp = requests.post(f"{url}/api/generate", json=payload, timeout=30)
    resp.raise_for_status()
    return resp.json()["response"]


def test_generate_matches_backend(shim):
    url, be, _ = shim
    prompt = "Tóm tắt nội dung văn bản tiếng Việt."
    assert _call(url, prompt) == be.generate([prompt], 1000)[0]


def test_tags_lists_model(shim):
    url, _, _ = shim
    r = requests.get(f"{url}/api/tags", timeout=10)
    r.raise_for_status()
    assert [m["name"] for m in r.json()["models"]] == ["llama3.2:3b"]


def test_concurrent_requests_are_batched(shim):
    url, be, eng = shim
    prompts = [f"Tóm tắt {i} nội dung" for i in range(8)]
    with concurrent.futures.ThreadPoolExecutor(8) as ex:
        got = list(ex.map(lambda p: _call(url, p), prompts))
    assert got == [be.generate([p], 1000)[0] for p in prompts]
    assert max(eng.batches) > 1


def test_errors(shim, toy_tokenizer):  # noqa: F811
    url, _, _ = shim
    r = requests.post(f"{url}/api/generate", json={"model": "nope", "prompt": "x", "stream": False}, timeout=10)
    assert r.status_code == 404
    with pytest.raises(requests.HTTPError):
        r.raise_for_status()

    class Broken(FakeEngine):
        def step(self):
            raise RuntimeError("libmapsum ms_step failed (-5): device lost")
    with OllamaShim({"m": compat.MapBackend(Broken(), toy_tokenizer)}, port=0) as s:
        r = requests.post(f"http://127.0.0.1:{s.port}/api/generate",
                          json={"model": "m", "prompt": "x", "stream": False}, timeout=10)
        assert r.status_code == 500 and "device lost" in r.json()["error"]


def test_done_reason_reports_truncation(shim):
    """Ollama answers done_reason "length" when num_predict cut the output, "stop" at EOS
    (the FakeEngine finishes every chunk with "length")."""
    url, _, _ = shim
    payload = {"model": "llama3.2:3b", "prompt": "Tóm tắt", "stream": False, "options": {"num_predict": 3}}
    r = requests.post(f"{url}/api/generate", json=payload, timeout=30)
    r.raise_for_status()
    assert r.json()["done_reason"] == "length"
