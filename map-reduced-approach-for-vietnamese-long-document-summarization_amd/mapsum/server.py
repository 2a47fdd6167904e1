"""Ollama wire shim: the two routes the reference calls, served from a libmapsum engine
(SURVEY.md §8b "wire-level", §8f rank 4), so the unchanged pipeline can point
``ollama_url`` here.

  POST /api/generate  {"model", "prompt", "stream": false, "options": {"num_predict"}}
                      -> {"model", "response", "done": true, "done_reason", ...}
                      (run_full_evaluation_pipeline.py:81-94; the caller reads only
                      ["response"] and applies clean_thinking_tokens itself, :94-106)
  GET  /api/tags      -> {"models": [{"name": ...}]}   (:199-233, the availability check)

Requests from concurrent clients are batched: every request thread hands its prompt to
one asyncio loop that drives ``MapBackend.agenerate``, so requests that arrive together
share engine steps.  Errors are HTTP 500 with {"error": msg}, which the reference turns
into an exception through ``raise_for_status`` (:91).
"""
from __future__ import annotations

import asyncio
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

DEFAULT_NUM_PREDICT = 128  # EXT Ollama's default when options.num_predict is absent


class OllamaShim:
    def __init__(self, backends: dict, host: str = "127.0.0.1", port: int = 11434):
        """backends: model name -> mapsum.compat.MapBackend."""
        self.backends = backends
        self.loop = asyncio.new_event_loop()
        self._loop_thread = threading.Thread(target=self.loop.run_forever, daemon=True)
        shim = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):  # quiet
                pass

            def _send(self, code, obj, ctype="application/json"):
                body = (obj if isinstance(obj, (bytes, bytearray)) else json.dumps(obj, ensure_ascii=False).encode())
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):
                if self.path.rstrip("/") == "/api/tags":
                    self._send(200, {"models": [{"name": n, "model": n} for n in shim.backends]})
                elif self.path in ("/", ""):
                    self._send(200, b"Ollama is running", "text/plain")
                else:
                    self._send(404, {"error": "not found"})

            def do_POST(self):
                if self.path.rstrip("/") != "/api/generate":
                    return self._send(404, {"error": "not found"})
                try:
                    n = int(self.headers.get("Content-Length", "0"))
                    req = json.loads(self.rfile.read(n) or b"{}")
                    code, resp = shim.generate(req)
                except json.JSONDecodeError as e:
                    code, resp = 400, {"error": f"invalid JSON: {e}"}
                if code == 200 and req.get("stream", True):
                    # Ollama streams NDJSON by default; one final chunk carries everything
                    return self._send(200, (json.dumps(resp, ensure_ascii=False) + "\n").encode(),
                                      "application/x-ndjson")
                self._send(code, resp)

        self.httpd = ThreadingHTTPServer((host, port), Handler)
        self.port = self.httpd.server_address[1]
        self._http_thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    def generate(self, req: dict):
        model = req.get("model")
        be = self.backends.get(model)
        if be is None:
            return 404, {"error": f"model '{model}' not found"}
        prompt = req.get("prompt")
        if not isinstance(prompt, str):
            return 400, {"error": "prompt must be a string"}
        n = int((req.get("options") or {}).get("num_predict", DEFAULT_NUM_PREDICT))
        t0 = time.perf_counter()
        try:
            fut = asyncio.run_coroutine_threadsafe(be.agenerate_full(prompt, n), self.loop)
            text, finish = fut.result()
        except Exception as e:  # noqa: BLE001 -- reported to the client as Ollama does
            return 500, {"error": str(e)}
        dt = time.perf_counter() - t0
        return 200, {"model": model, "created_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
                     "response": text, "done": True,
                     "done_reason": "length" if finish == "length" else "stop",
                     "total_duration": int(dt * 1e9)}

    def start(self):
        self._loop_thread.start()
        self._http_thread.start()
        return self

    def close(self):
        self.httpd.shutdown()
        self.httpd.server_close()
        self.loop.call_soon_threadsafe(self.loop.stop)
        self._loop_thread.join(timeout=5)

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.close()
