"""project_morpheus_amd — MI355X-native Orpheus TTS hot path (drop-in for Morpheus tts_engine).

Layout:
  csrc/           HIP kernels for gfx950 + the C ABI (include/morpheus_mx.h)
  build.py        in-tree hipcc build of libmorpheus_mx.so (per-TU objects)
  _lib.py         ctypes binding of libmorpheus_mx.so (no CPU fallback)
  engine.py       LlmEngine / SnacDecoder / Synthesizer (one stream, hipGraph steps)
  batching.py     BatchSynthesizer: continuous batching (online submit + offline run)
  service.py      per-GPU Service over one BatchSynthesizer (shared by every adapter)
  dispatch.py     GpuPool: one worker process per GPU, least-loaded request dispatch
  sharding.py     long-form jobs over ranks (torch.distributed gather + ordered stitch)
  schedule.py     speechpipe token parsing + window schedule (host logic)
  speechpipe.py   drop-in module for Morpheus_Client/tts_engine/speechpipe.py
  adapter.py      MxTTSAdapter + describe/voice_mapper/register for adapter_registry
  completions.py  /v1/completions SSE token stream (remote_backend wire format)
  server.py       ASGI app: /v1/audio/speech (4096-B pulls or a control-plane stream hook) + /v1/completions
  inference.py    generation params, voices, prompt framing, long-form split/stitch
  stitcher.py     stitch_chunks (orchestrator/stitcher.py contract)
  weights.py      HF / snac state-dict loaders, synthetic weights, fp8 quantisation
  gguf.py         GGUF v3 reader / writer (F32, F16, BF16, Q8_0) for llama.cpp checkpoints
  config.py       model constants and environment knobs
"""
__version__ = "0.1.0"
