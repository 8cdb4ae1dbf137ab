"""CPU checks of the fp8 weight quantizer (weights.quantize_fp8 / dequantize_fp8)."""
import torch

from project_morpheus_amd import config as C
from project_morpheus_amd.weights import dequantize_fp8, quantize_fp8


def _cfg():
    return C.OrpheusConfig(hidden=1024, layers=2, heads=8, kv_heads=2, ffn=2048, vocab=1000)


def test_fp8_quantizer_roundtrip():
    w = {"embed": torch.randn(8, 1024), "l0.wq": torch.randn(16, 1024) * 0.02}
    q = quantize_fp8(w, _cfg())
    assert q["l0.wq"].dtype == torch.float8_e4m3fn and q["lm_head"].dtype == torch.float8_e4m3fn
    d = dequantize_fp8(q)
    assert torch.allclose(d["l0.wq"], w["l0.wq"], rtol=0.07, atol=1e-6)
    assert d["embed"] is w["embed"]


def test_fp8_scale_is_row_absmax_over_448():
    w = {"embed": torch.randn(4, 1024), "l0.wd": torch.randn(32, 1024)}
    q = quantize_fp8(w, _cfg())
    amax = w["l0.wd"].abs().amax(dim=1)
    assert torch.equal(q["l0.wd.scale"], amax / 448.0)
    assert q["l0.wd"].float().abs().amax() <= 448.0
