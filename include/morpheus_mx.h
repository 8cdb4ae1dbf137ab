/*
 * morpheus_mx.h — C ABI of libmorpheus_mx.so, the MI355X-native Orpheus TTS hot path.
 *
 * Drop-in boundary for the reference's L0 arithmetic.  The reference has
 * no native code of its own; these entry points replace the third-party engines it binds:
 *
 *   mx_llm_*   replaces the Orpheus decoder loop's LLM engine:
 *                vLLM AsyncLLMEngine.generate  Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:117
 *                (SamplingParams engine_class.py:106-112), llama.cpp Llama(...)/text_to_speech
 *                Morpheus_Client/tts_engine/llama_local.py:42-52,77, and the remote
 *                /v1/completions stream Morpheus_Client/tts_engine/remote_backend.py:64-117.
 *   mx_snac_*  replaces snac.SNAC.decode(codes) + slice + PCM16 in convert_to_audio
 *                Morpheus_Client/tts_engine/speechpipe.py:76-129 (model load :41-49).
 *
 * Conventions: return 0 on success, a negative code on error (message via *_last_error);
 * no exceptions cross the ABI.  All device I/O pointers are caller-owned device memory (or
 * host-mapped memory from mx_host_alloc); weights passed to *_set_weight are copied and
 * packed into context-owned storage.  Streams are hipStream_t passed as void*.  One context
 * per (GPU, host thread); contexts are not re-entrant.  The host engine calls these from
 * its own thread (never from the asyncio event loop), mirroring llama_local.py:79.
 */
#ifndef MORPHEUS_MX_H
#define MORPHEUS_MX_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MX_OK 0
#define MX_ERR_ARG (-1)
#define MX_ERR_HIP (-2)
#define MX_ERR_STATE (-3)
#define MX_ERR_OOM (-4)

#define MX_DTYPE_F32 0
#define MX_DTYPE_BF16 1
#define MX_DTYPE_FP8 2   /* OCP e4m3 (e4m3fn) bytes */

#define MX_WEIGHTS_BF16 0
#define MX_WEIGHTS_FP8 1 /* e4m3 matrices + one fp32 dequant scale per output row */

typedef struct mx_llm mx_llm;
typedef struct mx_snac mx_snac;

/* Llama-3 decoder shape (Orpheus-3B: 3072/28/24/8/128/8192/156940), limits and eps. */
typedef struct mx_llm_config {
  int32_t hidden, layers, heads, kv_heads, head_dim, ffn, vocab;
  int32_t max_slots;    /* concurrent utterance streams (KV slots) */
  int32_t max_pos;      /* positions per slot (n_ctx, llama_local.py:45) */
  int32_t max_batch;    /* decode rows per step */
  int32_t max_prefill;  /* prompt tokens per prefill call */
  float eps;            /* RMSNorm eps (1e-5) */
  int32_t tied;         /* lm_head shares the embedding table */
  int32_t wdtype;       /* MX_WEIGHTS_BF16 | MX_WEIGHTS_FP8 (BASELINE configs[4]) */
} mx_llm_config;

/* Per-stream generation parameters (engine_class.py:106-112 SamplingParams; inference.py:75-105).
 * temperature <= 0 selects greedy decoding (argmax after the penalty; the parity mode).
 * Otherwise: logits / temperature -> nucleus of mass top_p -> one draw from a Philox4x32-10
 * stream keyed by `seed` and counted by position (definition in csrc/sample_kernels.hip). */
typedef struct mx_sampling {
  float temperature;
  float top_p;
  float repetition_penalty; /* HF/vLLM rule on the prompt + generated set (1.1 in Orpheus) */
  uint64_t seed;
} mx_sampling;

/* ---- library / memory -------------------------------------------------------------- */
const char* mx_version(void);
int mx_host_alloc(size_t bytes, void** host_ptr, void** dev_ptr); /* pinned, device-mapped */
int mx_host_free(void* host_ptr);

/* ---- LLM decoder (replaces vLLM / llama.cpp decode) -------------------------------- */
int mx_llm_create(int device, const mx_llm_config* cfg, mx_llm** out);
/* names: embed, norm, lm_head (untied), l{i}.{attn_norm,wq,wk,wv,wo,mlp_norm,wg,wu,wd}.
 * MX_WEIGHTS_FP8 engines: every matrix but embed comes as MX_DTYPE_FP8 bytes plus
 * "<name>.scale" (fp32, one per output row: W = scale[row] * e4m3); lm_head is always given
 * (the tied embedding stays bf16 for the token lookup). */
int mx_llm_set_weight(mx_llm* ctx, const char* name, const void* dev_data, int64_t numel,
                      int dtype);
/* RoPE tables [n_pos][head_dim/2] fp32 (host memory), llama3-scaled frequencies. */
int mx_llm_set_rope(mx_llm* ctx, const float* cos_host, const float* sin_host, int n_pos);
/* Checks every weight is present and builds the fragment-major copies the multi-row GEMM
 * streams (2x the matrix bytes in HBM).  Weights are frozen afterwards: mx_llm_set_weight
 * then returns MX_ERR_STATE. */
int mx_llm_finalize(mx_llm* ctx);
/* Prefill prompt ids (host) into `slot`, bind the slot to decode row `row`, set the slot's
 * generation parameters, pick the first token.  Enqueued on `stream`. */
int mx_llm_prefill(mx_llm* ctx, int slot, int row, const int32_t* ids_host, int n_ids,
                   const mx_sampling* params, void* stream);
/* One decode step for rows [0, n_rows), each under its slot's parameters (hipGraph-captured
 * per row count and attention grid; replayed). */
int mx_llm_decode(mx_llm* ctx, int n_rows, void* stream);
/* After the host has waited for a step: MX_ERR_HIP if a persistent-engine launch (option
 * b1_engine) gave up on a bounded wait since the last check.  Such a step commits nothing (its
 * history entry reads -1, the row does not advance); this call waits for `stream`, clears the
 * engine's attention tickets and re-reads the row positions, so the next mx_llm_decode
 * recomputes the step.  mx_llm_decode performs the same check before it enqueues. */
int mx_llm_check(mx_llm* ctx, void* stream);
/* Same step launched eagerly (no graph) with HIP events around every launch; adds the
 * elapsed milliseconds per launch class to ms_by_class[k] (k < n_classes; classes:
 * 0 qkv, 1 attention, 2 o-proj, 3 gate/up, 4 down, 5 lm_head+argmax, 6 commit, 7 the
 * persistent engine launch when option b1_engine is on).
 * Synchronises the stream.  Used by bench.py for the roofline of individual kernels. */
int mx_llm_decode_profiled(mx_llm* ctx, int n_rows, void* stream, double* ms_by_class,
                           int n_classes);
/* Tuning knobs (capi.hip mx_llm_set_option; unknown keys and out-of-range values fail with
 * MX_ERR_ARG): "legacy_gemv", "gemv_wpb", "rpw_o", "rpw_gu", "rpw_down", "head_b1",
 * "o_merge", "att_cpw", "att_nw", "att_cpw_batch", "att_nw_batch", "att_b1_short" (one-row
 * attention may split the context into 64- / 96-position pieces: 2 / 1), "att_b1_nw6" (one-row
 * attention may take 192-position splits on 6-wave blocks past L 1,024), "att_nw6" (multi-row
 * attention may pick 6-wave blocks: the shortest split covering the context), "gemv_balance"
 * (one-row qkv / merging o-proj: the waves per block that load the most loaded CU least), "rows_frag",
 * "rows_merge", "rows_head_mt", "rows_head_target", "rows_target", "rows_target_qkv", "rows_target_o",
 * "rows_target_gu", "rows_target_down" (the target for one kind of layer launch), "rows_nt_max", "rows_nt1",
 * "rows_pw", "rows_pw_f8", "rows_lds_pad", "rows_atomic" (o-proj / down at >= 2 rows: K ranges
 * add into the residual with float atomics, no split-K seam), "rows_qkv_parts" (decode at >= 2
 * rows: the qkv K ranges' raw partials summed, scaled, RoPE'd and appended by the attention
 * launch, no split-K seam), "b1_engine" (one-row steps as ONE persistent
 * launch, engine_b1.hip), "engine_slots" (its LDS ring slots), "engine_depth" (ring slots in
 * flight per loader wave, 2 or 3), "engine_loaders" (loader waves, 1 or 2), "engine_trace" (record the engine's phase timeline),
 * "engine_timeout" (bound of every engine wait, 100 MHz ticks; 0 = 50 ms), "engine_dbg" (timing
 * experiments: 1 = no hand-off waits, 2 = no weight stream; outputs invalid), "bench_one_layer"
 * (diagnostic: the GEMV probes below sweep layer 0 only, its weights resident on die).  Drops
 * the captured graphs so the next mx_llm_decode re-captures with the new choice. */
int mx_llm_set_option(mx_llm* ctx, const char* key, int value);
/* Diagnostic (option engine_trace on): after a device sync, copy the last engine launch's
 * timeline, 12 stamps of the 100 MHz clock per (CU, layer) -- consumer: layer start, input
 * ready, qkv done, attention done, o input ready, o done, gate/up input ready, gate/up done,
 * down input ready, down done; loader: layer start, layer streamed -- into host_out
 * ([grid][layers][12], n entries available); *grid_out = the engine's grid. */
int mx_llm_engine_trace(mx_llm* ctx, uint64_t* host_out, int n, int* grid_out);
/* Roofline probe: mean microseconds per launch of the decode GEMV/GEMM `which` (0 qkv,
 * 1 o-proj, 2 gate/up, 3 down, 4 the one-row o-proj merging 8 attention splits, 5 lm_head +
 * penalty + argmax) for `n_rows` rows (1..max_batch), timed over one hipGraph of
 * `reps` sweeps across all layers' weights (as in a decode step); *bytes_out = weight
 * bytes per launch.  Clobbers decode-row state and KV position 0 of the first n_rows
 * slots: only on an idle context. */
int mx_llm_bench_gemv(mx_llm* ctx, int which, int n_rows, int reps, float* us_out,
                      double* bytes_out);
/* Diagnostic: per-block phase stamps (s_memrealtime, 100 MHz) of the multi-row GEMM launch of
 * mx_llm_bench_gemv's last layer, replayed inside its sweep: host_out[block * 8 + k], k = 0
 * entry, 1 first activation staged, 2 first weight sub-chunk consumed, 3 main loop done,
 * 4 split-K partial published + ticket, 5 K ranges merged, 6 epilogue done (0 = not
 * reached).  n_rows >= 2; *blocks_out = grid size (<= cap_blocks).  The stamps exist only in
 * the diagnostic build (MORPHEUS_MX_ROWS_TRACE=1, libmorpheus_mx_trace.so); the product
 * library returns MX_ERR_STATE. */
int mx_llm_bench_gemv_trace(mx_llm* ctx, int which, int n_rows, uint64_t* host_out,
                            int cap_blocks, int* blocks_out);
/* Diagnostic: mx_llm_bench_gemv's all-layer multi-row sweep (n_rows >= 2; which 0-3, 5)
 * replayed on nstreams (1..4) streams at once, each with its own split-K workspace (values
 * meaningless): wall microseconds per launch of one stream's sweep. */
int mx_llm_bench_gemv_streams(mx_llm* ctx, int which, int n_rows, int reps, int nstreams,
                              float* us_out);
/* Diagnostic: mean microseconds of one eager attention launch (layer 0) for n_rows rows of
 * length L, `cpw` 32-position chunks per wave (split = 128*cpw), experiment flags `debug`
 * (0 = product kernel).  Clobbers decode-row state: only on an idle context. */
int mx_llm_bench_attention(mx_llm* ctx, int L, int n_rows, int cpw, int debug, int reps,
                           float* us_out);
/* Park decode row `row` on the scratch slot (stream ended / barge-in reset). */
int mx_llm_release_row(mx_llm* ctx, int row, void* stream);
/* Row compaction (stream-ordered on `stream`, between steps): the stream bound to row `src`
 * continues in the parked row `dst` -- same KV slot, position, token and next input; `src`
 * is parked.  Lets a step run the row class of the live stream count instead of the highest
 * row index in use (replaces nothing in the reference: vLLM's scheduler compacts its batch
 * internally, engine_class.py:114-134).  MX_ERR_STATE if `dst` is live. */
int mx_llm_move_row(mx_llm* ctx, int dst, int src, void* stream);
/* Host view of decode row `row`: *active = 1 while a stream is bound to it (prefill until
 * release), *next_pos = the position its next token takes. */
int mx_llm_row_state(const mx_llm* ctx, int row, int* active, int* next_pos);
/* Host-mapped token history [max_slots][max_pos] int32 written by the device. */
int32_t* mx_llm_history(mx_llm* ctx);
/* Parity/debug: keep a copy of the penalised logits of each decode row (enable before the
 * first mx_llm_decode; costs one extra write per vocab entry) and read one row back. */
int mx_llm_debug_logits(mx_llm* ctx, int enable);
int mx_llm_read_logits(mx_llm* ctx, int row, float* host_out, void* stream);
const char* mx_llm_last_error(const mx_llm* ctx);
void mx_llm_destroy(mx_llm* ctx);

/* ---- SNAC 24 kHz decoder (replaces SNAC.decode + slice + int16) --------------------- */
int mx_snac_create(int device, int max_frames, int max_batch, mx_snac** out);
/* names: q{i}.codebook [4096*8], q{i}.out_proj.w [768*8], q{i}.out_proj.b, in.dw.w [768*7],
 * in.dw.b, in.pw.w [1024*768], in.pw.b, b{k}.alpha, b{k}.up.w [Cin*Cout*2s], b{k}.up.b,
 * b{k}.noise.w, b{k}.r{j}.{alpha1,dw.w,dw.b,alpha2,pw.w,pw.b}, out.alpha, out.conv.w, out.conv.b
 * (weight norm already folded; layouts as torch Conv1d / ConvTranspose1d weights). */
int mx_snac_set_weight(mx_snac* ctx, const char* name, const void* dev_data, int64_t numel,
                       int dtype);
int mx_snac_finalize(mx_snac* ctx);
/* Decode `batch` windows of n_frames frames each.  frames: [batch][7*n_frames] SNAC codes in
 * speechpipe token order (0..4095; the caller applies the range check of speechpipe.py:108-111).
 * noise: [batch][sum of the 4 NoiseBlock lengths] or NULL: fresh N(0,1) drawn from `seeds[b]`
 * per window (device-accessible [batch], e.g. host-mapped; a window's noise then depends on
 * its own seed only) or, with seeds NULL, from `seed` over the whole batch.
 * pcm: [batch][hi-lo] int16 of samples [lo,hi) (NULL to skip); audio: [batch][2048*n_frames]
 * fp32 full window (NULL to skip).  With audio NULL only the positions [lo,hi) depend on are
 * computed past the first DecoderBlock (the same PCM within fp32 summation order). */
int mx_snac_decode(mx_snac* ctx, const int32_t* frames, int n_frames, int batch,
                   const float* noise, uint64_t seed, const uint64_t* seeds, int16_t* pcm,
                   float* audio, int lo, int hi, void* stream);
const char* mx_snac_last_error(const mx_snac* ctx);
void mx_snac_destroy(mx_snac* ctx);

#ifdef __cplusplus
}
#endif
#endif /* MORPHEUS_MX_H */
