"""Pin the LLM oracle (oracle/llama_ref.py) against transformers' LlamaForCausalLM.

Same seeded fp32 weights, llama3 RoPE scaling, GQA; the oracle's bf16 KV rounding is
disabled for this comparison (transformers keeps fp32 K/V).  Also checks the product's
RoPE table (project_morpheus_amd.config) equals the oracle's.
"""
import numpy as np
import pytest
import torch

from oracle import llama_ref as L
from project_morpheus_amd import config as C
from project_morpheus_amd.weights import synthetic_llm_weights


def small_cfg(**kw):
    d = dict(hidden=256, layers=2, heads=4, kv_heads=2, head_dim=64, ffn=512, vocab=300,
             rope_theta=500000.0)
    d.update(kw)
    return d


def _hf_model(cfgd, w):
    transformers = pytest.importorskip("transformers")
    hc = transformers.LlamaConfig(
        hidden_size=cfgd["hidden"], num_hidden_layers=cfgd["layers"],
        num_attention_heads=cfgd["heads"], num_key_value_heads=cfgd["kv_heads"],
        head_dim=cfgd["head_dim"], intermediate_size=cfgd["ffn"], vocab_size=cfgd["vocab"],
        rms_norm_eps=1e-5, rope_theta=cfgd["rope_theta"], tie_word_embeddings=True,
        max_position_embeddings=4096,
        rope_scaling={"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                      "high_freq_factor": 4.0, "original_max_position_embeddings": 8192},
        attn_implementation="eager")
    m = transformers.LlamaForCausalLM(hc).float().eval()
    sd = {"model.embed_tokens.weight": w["embed"], "model.norm.weight": w["norm"],
          "lm_head.weight": w["embed"]}
    for i in range(cfgd["layers"]):
        a, p = f"model.layers.{i}.", f"l{i}."
        sd.update({a + "input_layernorm.weight": w[p + "attn_norm"],
                   a + "post_attention_layernorm.weight": w[p + "mlp_norm"],
                   a + "self_attn.q_proj.weight": w[p + "wq"], a + "self_attn.k_proj.weight": w[p + "wk"],
                   a + "self_attn.v_proj.weight": w[p + "wv"], a + "self_attn.o_proj.weight": w[p + "wo"],
                   a + "mlp.gate_proj.weight": w[p + "wg"], a + "mlp.up_proj.weight": w[p + "wu"],
                   a + "mlp.down_proj.weight": w[p + "wd"]})
    m.load_state_dict({k: v.float() for k, v in sd.items()}, strict=False)
    return m


def test_oracle_matches_transformers_logits():
    d = small_cfg()
    pc = C.OrpheusConfig(hidden=d["hidden"], layers=d["layers"], heads=d["heads"],
                         kv_heads=d["kv_heads"], head_dim=d["head_dim"], ffn=d["ffn"],
                         vocab=d["vocab"])
    w = synthetic_llm_weights(pc, seed=7, std=0.05, norm_jitter=0.5)
    rc = L.RefConfig(hidden=d["hidden"], layers=d["layers"], heads=d["heads"],
                     kv_heads=d["kv_heads"], head_dim=d["head_dim"], ffn=d["ffn"],
                     vocab=d["vocab"])
    ids = [5, 17, 99, 3, 250, 42, 7, 7, 180, 11]
    hf = _hf_model(d, w)
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0]
    ref = L.LlamaRef(rc, w, max_pos=64, round_kv=False)
    got = ref.forward(ids, [0] * len(ids), list(range(len(ids))))
    assert torch.allclose(got, want, atol=2e-4, rtol=1e-4), (got - want).abs().max()
    # incremental decode (KV cache) == full forward
    ref.free(0)
    ref.forward(ids[:6], [0] * 6, list(range(6)))
    inc = torch.stack([ref.forward([t], [0], [6 + i])[0] for i, t in enumerate(ids[6:])])
    assert torch.allclose(inc, want[6:], atol=2e-4, rtol=1e-4)


def test_rope_tables_agree():
    cfg = C.OrpheusConfig()
    cos, sin = C.rope_tables(cfg, 3000)
    rc = L.RefConfig()
    oc, os_ = L.rope_cos_sin(rc, torch.arange(3000))
    assert np.array_equal(cos, oc.numpy()) and np.array_equal(sin, os_.numpy())


def test_penalty_and_greedy_tie_break():
    logits = torch.tensor([1.0, 2.0, -1.0, 2.2, 2.0])
    out = L.apply_penalty(logits, [3, 2], 1.1)
    assert out[3] == pytest.approx(2.0) and out[2] == pytest.approx(-1.1)
    assert int(torch.argmax(out)) == 1  # first of the equal maxima


def test_param_count_orpheus():
    cfg = C.OrpheusConfig()
    assert cfg.params() == 3_300_691_968
    assert cfg.kv_bytes_per_position() == 114_688


def test_teacher_forced_rows_match_per_row_generation():
    """The batched teacher-forced oracle (one forward per step for all rows, optional shared
    prefix computed once) gives each row the logits of its own greedy_generate run."""
    d = small_cfg()
    pc = C.OrpheusConfig(hidden=d["hidden"], layers=d["layers"], heads=d["heads"],
                         kv_heads=d["kv_heads"], head_dim=d["head_dim"], ffn=d["ffn"],
                         vocab=d["vocab"])
    w = synthetic_llm_weights(pc, seed=9, std=0.05, norm_jitter=0.5)
    rc = L.RefConfig(hidden=d["hidden"], layers=d["layers"], heads=d["heads"],
                     kv_heads=d["kv_heads"], head_dim=d["head_dim"], ffn=d["ffn"],
                     vocab=d["vocab"])
    rng = np.random.default_rng(3)
    prefix = [int(x) for x in rng.integers(0, d["vocab"], 20)]
    prompts = [prefix + [int(x) for x in rng.integers(0, d["vocab"], 2 + 3 * r)]
               for r in range(4)]
    forced = [[int(x) for x in rng.integers(0, d["vocab"], 7)] for _ in prompts]
    # fp32 KV here: the products' summation order differs between one-row and batched
    # forwards, and with the bf16 KV cache a last-ulp difference can flip a rounding
    # (1e-4 here, the effect the GPU tests' 5e-3 absorbs)
    for shared in (0, 20):
        ref = L.LlamaRef(rc, w, max_pos=128, round_kv=False)
        got = L.teacher_forced_rows(ref, prompts, forced, 1.1, shared_prefix=shared)
        for r, p in enumerate(prompts):
            one = L.LlamaRef(rc, w, max_pos=128, round_kv=False)
            _, want = L.greedy_generate(one, p, 7, 1.1, return_logits=True, forced=forced[r])
            for k in range(7):
                assert torch.allclose(got[r][k], want[k], atol=1e-5, rtol=1e-5), (shared, r, k, float((got[r][k] - want[k]).abs().max()))
