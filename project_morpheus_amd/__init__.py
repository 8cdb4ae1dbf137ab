"""project_morpheus_amd — MI355X-native Orpheus TTS hot path (drop-in for Morpheus tts_engine).

Layout:
  csrc/         HIP kernels for gfx950 + the C ABI (include/morpheus_mx.h)
  _lib.py       ctypes binding of libmorpheus_mx.so (no CPU fallback)
  engine.py     LlmEngine / SnacDecoder / Synthesizer (the per-GPU decoder loop)
  schedule.py   speechpipe token parsing + window schedule (host logic)
  speechpipe.py drop-in module for Morpheus_Client/tts_engine/speechpipe.py
  adapter.py    MxTTSAdapter + describe/voice_mapper/register for adapter_registry
  inference.py  generation params, voices, prompt framing, long-form split/stitch
  stitcher.py   stitch_chunks (orchestrator/stitcher.py contract)
  parallel.py   batch-sharding of utterances across GPUs (one process per GPU)
"""
__version__ = "0.1.0"
