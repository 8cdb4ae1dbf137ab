"""CPU check of the speaking weights (tests/_speaking.py) that drive the composed GPU parity
test (tests/test_gpu_composed.py): the oracle's own greedy decode emits the designed script,
with a wide argmax margin at every step, and the script walks the reference schedule's edge
cases (speechpipe.py:146-293) as designed."""
import numpy as np

from _speaking import STARTS, four_scripts, make_script, speaking_config, speaking_weights
from oracle import llama_ref as L
from oracle import speechpipe_ref as SP
from project_morpheus_amd import config as C
from project_morpheus_amd import inference as I


def test_oracle_greedy_speaks_the_script():
    cfg = speaking_config()
    script = make_script(7)
    w = speaking_weights(cfg, {C.START_OF_SPEECH: script})
    ref = L.LlamaRef(L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                                 kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab,
                                 tied=False), w, max_pos=256)
    prompt = I.prompt_ids([1001, 1002, 1003])
    assert prompt[-1] == C.START_OF_SPEECH
    toks, logits = L.greedy_generate(ref, prompt, len(script) + 4, 1.1,
                                     stop_ids=C.STOP_IDS, return_logits=True)
    assert toks == script
    margins = [float(np.diff(np.sort(lg.numpy())[-2:])[0]) for lg in logits]
    assert min(margins) > 5.0  # no near-tie: GPU and oracle must agree token for token

    # the schedule on the model's own tokens: text / special / code-0 ids skipped, the
    # 4097 code makes the windows that hold it invalid (first window retried until valid)
    strings = [f"<custom_token_{t - C.CUSTOM_TOKEN_BASE}>" if t >= C.CUSTOM_TOKEN_BASE
               else "text" for t in toks]
    wins = []
    SP.decode_stream(strings, lambda c0, c1, c2: np.zeros(2048 * len(c0), np.float32),
                     windows_out=wins)
    codes = [SP.parse_custom_token(s, 0) for s in strings]
    assert any(c is None for c in codes)                 # text ids
    bad = [win for win in wins if not SP.codes_valid(*SP.deinterleave(win))]
    good = [win for win in wins if SP.codes_valid(*SP.deinterleave(win))]
    assert bad and good
    assert len(good[0]) == 7 and 4097 not in good[0]     # first window after the retries


def test_four_disjoint_scripts_share_one_model():
    """The B = 4 batch test's weights: each start id leads to its own script."""
    cfg = speaking_config()
    scripts = four_scripts()
    w = speaking_weights(cfg, dict(zip(STARTS, scripts)))
    ref = L.LlamaRef(L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                                 kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab,
                                 tied=False), w, max_pos=256)
    for b, start in enumerate(STARTS):
        prompt = [1001 + b, 1002, start]
        toks = L.greedy_generate(ref, prompt, len(scripts[b]) + 4, 1.1, stop_ids=C.STOP_IDS)
        assert toks == scripts[b], b
