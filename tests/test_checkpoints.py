"""Checkpoint loaders on CPU: HF Llama safetensors, snac 1.2.x state dicts, llama.cpp GGUF.

No real checkpoint exists here, so each test writes seeded synthetic weights
in the external layout -- HF names + config.json; snac 1.2.x module paths with weight-norm
``weight_g`` / ``weight_v`` (and the newer ``parametrizations`` names); GGUF v3 with Q8_0
blocks and llama.cpp's rotary row permutation -- loads them back and checks the engine-named
weights, and the oracles' outputs on them, against the originals.
"""
import json
import math
import os

import numpy as np
import torch

from oracle import llama_ref as L
from oracle import snac_ref
from project_morpheus_amd import config as C
from project_morpheus_amd import gguf as G
from project_morpheus_amd.weights import (load_hf_llm, load_snac_state_dict,
                                          synthetic_llm_weights, synthetic_snac_weights)

CFG = C.OrpheusConfig(hidden=256, layers=2, heads=4, kv_heads=2, ffn=512, vocab=600)


def _ref(cfg, w):
    return L.LlamaRef(L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                                  kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab,
                                  eps=cfg.eps, rope_theta=cfg.rope_theta,
                                  rope_scaling=cfg.rope_scaling), w, max_pos=64)


def _logits(cfg, w, prompt=(5, 17, 99, 3, 250)):
    return _ref(cfg, w).forward(list(prompt), [0] * len(prompt), list(range(len(prompt))))


def test_hf_safetensors_round_trip(tmp_path):
    from safetensors.torch import save_file
    w = synthetic_llm_weights(CFG, seed=3, std=0.05, norm_jitter=0.5)
    names = {"embed": "model.embed_tokens.weight", "norm": "model.norm.weight"}
    hf = {}
    for k, v in w.items():
        if k in names:
            hf[names[k]] = v
            continue
        i, f = k[1:].split(".", 1)
        a = f"model.layers.{i}."
        hf[a + {"attn_norm": "input_layernorm.weight",
                "mlp_norm": "post_attention_layernorm.weight",
                "wq": "self_attn.q_proj.weight", "wk": "self_attn.k_proj.weight",
                "wv": "self_attn.v_proj.weight", "wo": "self_attn.o_proj.weight",
                "wg": "mlp.gate_proj.weight", "wu": "mlp.up_proj.weight",
                "wd": "mlp.down_proj.weight"}[f]] = v
    save_file({k: v.contiguous() for k, v in hf.items()}, str(tmp_path / "model.safetensors"))
    json.dump({"hidden_size": CFG.hidden, "num_hidden_layers": CFG.layers,
               "num_attention_heads": CFG.heads, "num_key_value_heads": CFG.kv_heads,
               "intermediate_size": CFG.ffn, "vocab_size": CFG.vocab, "rms_norm_eps": 1e-5,
               "rope_theta": 500000.0, "rope_scaling": CFG.rope_scaling,
               "tie_word_embeddings": True, "head_dim": 128},
              open(tmp_path / "config.json", "w"))
    cfg = C.OrpheusConfig.from_hf(str(tmp_path))
    assert (cfg.hidden, cfg.layers, cfg.heads, cfg.kv_heads, cfg.ffn, cfg.vocab, cfg.tied) == \
        (CFG.hidden, CFG.layers, CFG.heads, CFG.kv_heads, CFG.ffn, CFG.vocab, True)
    got = load_hf_llm(str(tmp_path))
    assert set(got) == set(w)
    for k in w:
        assert torch.equal(got[k], w[k]), k
    assert torch.equal(_logits(cfg, got), _logits(CFG, w))


def _snac_1_2_state_dict(sw, parametrized=False):
    """Engine SNAC weights -> a snac 1.2.x ``SNAC.state_dict()`` (24 kHz, noise, depthwise):
    every WN conv as (g, v) with v = w * c_o (c_o > 0 per output channel), g = ||v|| / c_o."""
    g = torch.Generator().manual_seed(9)
    sd = {}

    def wn(prefix, w, shape=None):
        w = w if shape is None else w.reshape(shape)
        c = 0.5 + torch.rand((w.shape[0],) + (1,) * (w.dim() - 1), generator=g)
        v = w * c
        gg = v.norm(dim=tuple(range(1, v.dim())), keepdim=True) / c
        if parametrized:
            sd[prefix + ".parametrizations.weight.original0"] = gg
            sd[prefix + ".parametrizations.weight.original1"] = v
        else:
            sd[prefix + ".weight_g"] = gg
            sd[prefix + ".weight_v"] = v

    for i in range(3):
        q = f"quantizer.quantizers.{i}."
        sd[q + "codebook.weight"] = sw[f"q{i}.codebook"]
        wn(q + "out_proj", sw[f"q{i}.out_proj.w"], (768, 8, 1))
        sd[q + "out_proj.bias"] = sw[f"q{i}.out_proj.b"]
        sd[q + "in_proj.weight_g"] = torch.ones(8, 1, 1)       # encoder side, unused
        sd[q + "in_proj.weight_v"] = torch.ones(8, 768, 1)
    d = "decoder.model."
    wn(d + "0", sw["in.dw.w"])
    sd[d + "0.bias"] = sw["in.dw.b"]
    wn(d + "1", sw["in.pw.w"], (1024, 768, 1))
    sd[d + "1.bias"] = sw["in.pw.b"]
    for b in range(4):
        m, p, co = f"{d}{2 + b}.block.", f"b{b}.", 512 >> b
        sd[m + "0.alpha"] = sw[p + "alpha"].reshape(1, -1, 1)
        wn(m + "1", sw[p + "up.w"])
        sd[m + "1.bias"] = sw[p + "up.b"]
        wn(m + "2.linear", sw[p + "noise.w"], (co, co, 1))
        for j in range(3):
            r, q = f"{m}{3 + j}.block.", f"{p}r{j}."
            sd[r + "0.alpha"] = sw[q + "alpha1"].reshape(1, -1, 1)
            wn(r + "1", sw[q + "dw.w"])
            sd[r + "1.bias"] = sw[q + "dw.b"]
            sd[r + "2.alpha"] = sw[q + "alpha2"].reshape(1, -1, 1)
            wn(r + "3", sw[q + "pw.w"], (co, co, 1))
            sd[r + "3.bias"] = sw[q + "pw.b"]
    sd[d + "6.alpha"] = sw["out.alpha"].reshape(1, -1, 1)
    wn(d + "7", sw["out.conv.w"])
    sd[d + "7.bias"] = sw["out.conv.b"]
    return sd


def test_snac_state_dict_round_trip(tmp_path):
    from safetensors.torch import save_file
    sw = synthetic_snac_weights(seed=4)
    codes = np.random.default_rng(0).integers(0, 4096, size=14)
    c0, c1, c2 = [int(codes[0]), int(codes[7])], [int(x) for x in codes[[1, 4, 8, 11]]], \
        [int(x) for x in codes[[2, 3, 5, 6, 9, 10, 12, 13]]]
    want = snac_ref.decode(sw, c0, c1, c2, noise=snac_ref.window_noise(7, 2))
    for par in (False, True):
        sd = _snac_1_2_state_dict(sw, parametrized=par)
        f = tmp_path / f"snac{int(par)}.safetensors"
        save_file({k: v.contiguous() for k, v in sd.items()}, str(f))
        got = load_snac_state_dict(str(f))
        assert set(got) == set(sw)
        for k in sw:
            torch.testing.assert_close(got[k], sw[k], rtol=1e-5, atol=1e-6, msg=k)
        audio = snac_ref.decode(got, c0, c1, c2, noise=snac_ref.window_noise(7, 2))
        assert float((audio - want).pow(2).mean().sqrt()) < 1e-6


def test_gguf_q8_0_round_trip(tmp_path):
    w = synthetic_llm_weights(CFG, seed=5, std=0.05, norm_jitter=0.5)
    f = str(tmp_path / "orpheus-q8_0.gguf")
    G.export_gguf(f, CFG, w, tokens=[f"t{i}" for i in range(CFG.vocab)])
    cfg, got = G.load_gguf_llm(f, dtype="float32")
    assert (cfg.hidden, cfg.layers, cfg.heads, cfg.kv_heads, cfg.ffn, cfg.vocab, cfg.tied) == \
        (CFG.hidden, CFG.layers, CFG.heads, CFG.kv_heads, CFG.ffn, CFG.vocab, True)
    assert set(got) == set(w)

    def q8(a):  # what the file holds: Q8_0 of the (llama.cpp-permuted) matrix, dequantised
        blk = np.frombuffer(G.quantize_q8_0(a), dtype=np.uint8).reshape(-1, 34)
        d = blk[:, :2].copy().view("<f2").astype(np.float32)
        return (d * blk[:, 2:].view(np.int8).astype(np.float32)).reshape(a.shape)

    for k, v in w.items():
        a = v.float().numpy()
        if a.ndim == 1:
            want = a
        elif k.endswith(".wq") or k.endswith(".wk"):
            nh = CFG.heads if k.endswith(".wq") else CFG.kv_heads
            want = G._unpermute_rope(q8(G._permute_rope(a, nh)), nh)
        else:
            want = q8(a)
        np.testing.assert_array_equal(got[k].numpy(), want, err_msg=k)
        if a.ndim == 2:  # Q8_0 is a faithful 8-bit code of the weights
            assert np.abs(got[k].numpy() - a).max() <= np.abs(a).max() / 127 * 0.51 + 1e-6
    # the permutation is undone: the oracle on the GGUF weights matches the oracle on the
    # dequantised originals in HF layout, logit for logit
    hf_layout = {k: torch.from_numpy(q8(v.float().numpy())) if v.dim() == 2 else v.float()
                 for k, v in w.items()}
    torch.testing.assert_close(_logits(cfg, got), _logits(CFG, hf_layout), rtol=0, atol=2e-5)
