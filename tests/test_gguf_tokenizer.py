"""Tokenizer from a GGUF file alone (§8(f4)): the reference CPU path needs only
``LLAMA_MODEL_PATH`` to a GGUF (llama_local.py:42-52, .env.example:10), whose metadata holds
the byte-level BPE vocabulary.  A small Llama-3-style BPE is trained here with ``tokenizers``
(Llama-3 split regex, byte-level, ``ignore_merges``, special tokens), written into a GGUF with
``write_gguf`` as llama.cpp's converter stores it (tokens, merges, token_type, bos id), and
``Tokenizer(<file>.gguf)`` must encode exactly as the trained tokenizer does."""
import json

import pytest

from project_morpheus_amd.gguf import GGML_F32, write_gguf
from project_morpheus_amd.tokenizer import LLAMA3_SPLIT, Tokenizer

CORPUS = [
    "tara: Hello world, this is a test of the Orpheus voice.",
    "Numbers 12345 and 3.14159, dates 2025-08-24, emails a.b@c.de!",
    "Don't stop; it's fine, we'll see. I'm here, you're there, they've gone.",
    "Unicode: café naïve über 中文 日本語 emoji \U0001F600.",
    "New\nlines\r\nand\ttabs   and    spaces.",
] * 40
SPECIAL = ["<|begin_of_text|>", "<|eot_id|>", "<custom_token_0>", "<custom_token_4097>"]


@pytest.fixture(scope="module")
def trained(tmp_path_factory):
    from tokenizers import Regex, Tokenizer as HFTok, decoders, models, pre_tokenizers, trainers
    tk = HFTok(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_SPLIT), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, trim_offsets=True, use_regex=False)])
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=600, special_tokens=SPECIAL,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator(CORPUS, trainer=tr)
    j = json.loads(tk.to_str())
    j["model"]["ignore_merges"] = True          # as Llama-3's tokenizer.json
    ref = HFTok.from_str(json.dumps(j))
    vocab = j["model"]["vocab"]
    tokens = [None] * len(vocab)
    for t, i in vocab.items():
        tokens[i] = t
    merges = [m if isinstance(m, str) else " ".join(m) for m in j["model"]["merges"]]
    types = [3 if t in SPECIAL else 1 for t in tokens]
    path = str(tmp_path_factory.mktemp("gguf") / "tiny.gguf")
    meta = {"general.architecture": "llama", "tokenizer.ggml.model": "gpt2",
            "tokenizer.ggml.pre": "llama-bpe", "tokenizer.ggml.tokens": tokens,
            "tokenizer.ggml.merges": merges, "tokenizer.ggml.token_type": types,
            "tokenizer.ggml.bos_token_id": vocab["<|begin_of_text|>"]}
    import numpy as np
    write_gguf(path, meta, {"output_norm.weight": (np.ones(32, np.float32), GGML_F32)})
    return ref, path, vocab


def test_gguf_tokenizer_matches_trained_bpe(trained):
    ref, path, vocab = trained
    tok = Tokenizer(path)
    assert not tok.synthetic
    texts = CORPUS[:5] + ["", " ", "tara: Hello world", "x" * 50, "  leading and trailing  ",
                          "<custom_token_0><custom_token_4097> mixed <|eot_id|> text",
                          "The year 1999999 had 3 digits-groups", "Zoë's café's"]
    for t in texts:
        want = ref.encode(t, add_special_tokens=False).ids
        got = tok.encode(t)
        assert got[0] == vocab["<|begin_of_text|>"]
        assert got[1:] == want, t
        assert tok.decode(got[1:]) == ref.decode(want, skip_special_tokens=False)


def test_llama_model_path_gguf_is_picked_up(trained, monkeypatch):
    _, path, vocab = trained
    monkeypatch.setenv("LLAMA_MODEL_PATH", path)
    tok = Tokenizer(None)
    assert not tok.synthetic and tok.encode("hi")[0] == vocab["<|begin_of_text|>"]


def test_non_bpe_gguf_vocab_is_rejected():
    from project_morpheus_amd.tokenizer import hf_tokenizer_from_gguf_meta
    with pytest.raises(ValueError):
        hf_tokenizer_from_gguf_meta({"tokenizer.ggml.model": "llama",
                                     "tokenizer.ggml.tokens": ["a"]})
