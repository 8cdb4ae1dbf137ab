"""Golden byte streams of the REFERENCE server driving the mi355x adapter (P19).

Run in the build container only (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_server_golden.py

Imports ``Morpheus_Client.server`` from /root/reference (stubs only for packages the image
lacks: ``dotenv`` no-op, ``snac`` never called, ``websockets`` never connected), from a
temporary working directory so its ``.env`` bootstrap (config.py:9-33) writes nothing.
It registers ``project_morpheus_amd.adapter.MxTTSAdapter`` -- unchanged, its synthesis source
replaced by the deterministic PCM of tests/_server_fake.py -- into the reference registry
through ``project_morpheus_amd.adapter.register`` and selects it as the server's adapter
(server.py:92 ``current_adapter_name``; the ``POST /config`` route would also persist to
.env, so it is not used).  Recorded with starlette's TestClient:

* ``POST /v1/audio/speech`` bodies (RIFF header + orchestrated PCM, server.py:161-190) for a
  short and a > 1000-char input, and the constructor arguments the server passed;
* every Orchestrator pull of the short request: ``token_window`` and the base64 PCM of the
  structured log entry (orchestrator/core.py:89-117), captured from the reference logger;
* ``/ws/tts`` frames (server.py:209-222);
* ``GET /adapters`` (server.py:236-239) with the mi355x descriptor.

Output: ``tests/golden/server_golden.json`` (inputs + expected outputs only).
"""
from __future__ import annotations

import base64
import hashlib
import json
import logging
import os
import sys
import tempfile
import types

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "server_golden.json")
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))  # the repo (our package)
sys.path.insert(0, os.path.dirname(HERE))                   # tests/ (_server_fake)


def load_reference_server():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("dotenv", types.SimpleNamespace(load_dotenv=lambda *a, **k: None))

    class _NoSNAC:
        @classmethod
        def from_pretrained(cls, *_a, **_k):
            return cls()

        def eval(self):
            return self

        def to(self, *_a, **_k):
            return self

    sys.modules.setdefault("snac", types.SimpleNamespace(SNAC=_NoSNAC))
    sys.modules.setdefault("websockets", types.SimpleNamespace(connect=None))
    sys.path.insert(0, REF)
    import Morpheus_Client.server as server  # noqa: E402
    return server


class _Capture(logging.Handler):
    def __init__(self):
        super().__init__(logging.INFO)
        self.entries = []

    def emit(self, record):
        try:
            self.entries.append(json.loads(record.getMessage()))
        except ValueError:
            pass


def main():
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            server = load_reference_server()
            from starlette.testclient import TestClient

            import _server_fake as F
            from project_morpheus_amd.adapter import register
            reg = server.adapter_registry
            register(reg)  # the drop-in boundary: registry.register("mi355x", ...)
            reg._registry["mi355x"].constructor = F.GoldenAdapter  # deterministic source
            server.current_adapter_name = "mi355x"
            cap = _Capture()
            lg = logging.getLogger("Morpheus_Client.orchestrator.core")
            lg.addHandler(cap)
            lg.setLevel(logging.INFO)
            client = TestClient(server.app)
            golden = {"source": REF, "speech": [], "ws": [], "adapters": None}
            long_text = "A sentence for the long-form switch. " * 30
            for text, voice in (("Hello world", "leo"), (long_text, "nobody")):
                F.CALLS.clear()
                cap.entries.clear()
                r = client.post("/v1/audio/speech", json={"input": text, "voice": voice})
                body = r.content
                golden["speech"].append({
                    "input": text, "voice": voice, "status": r.status_code,
                    "content_type": r.headers["content-type"],
                    "body_b64": base64.b64encode(body).decode(),
                    "body_sha256": hashlib.sha256(body).hexdigest(),
                    "adapter_calls": [list(c) for c in F.CALLS],
                    "pulls": [{"chunk_id": e["chunk_id"], "adapter": e["adapter"],
                               "token_window": e["token_window"], "pcm": e["pcm"]}
                              for e in cap.entries]})
            # the reference route returns without closing the socket (server.py:209-222),
            # which leaves a TestClient reader waiting: record the frames it sends and close
            # after its stream has ended (the frames themselves are the reference's)
            sent = []
            orig = server.websocket_pcm_stream

            async def recording(websocket, pcm_iter, sample_rate=server.SAMPLE_RATE):
                real = websocket.send_bytes

                async def send_bytes(b):
                    sent.append(bytes(b))
                    await real(b)
                websocket.send_bytes = send_bytes
                await orig(websocket, pcm_iter, sample_rate=sample_rate)
                await websocket.close()

            server.websocket_pcm_stream = recording
            with client.websocket_connect("/ws/tts?prompt=Hi%20there&voice=tara") as ws:
                try:
                    while True:
                        ws.receive_bytes()
                except Exception:
                    pass
            frames = sent
            golden["ws"].append({"prompt": "Hi there", "voice": "tara",
                                 "frames_b64": [base64.b64encode(f).decode() for f in frames]})
            golden["adapters"] = client.get("/adapters").json()
        finally:
            os.chdir(cwd)
    with open(OUT, "w") as fh:
        json.dump(golden, fh, indent=1)
    print(f"wrote {OUT}: {[len(s['pulls']) for s in golden['speech']]} pulls, "
          f"{len(golden['ws'][0]['frames_b64'])} ws frames")


if __name__ == "__main__":
    main()
