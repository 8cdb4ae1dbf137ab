"""CPU emulation: can prefill run on the CDNA4 fp8 MFMA (e4m3 x e4m3) and keep the oracle
tolerance?    Weights are e4m3 with a per-row scale either way; the
question is the ACTIVATION operand.  The fp8->bf16 path in use feeds the bf16 MFMA with x
split into 3 bf16 parts (fp32-exact products).  An fp8 MFMA needs x in e4m3: one part
(W8A8, per-row activation scale), or x = s (p0 + p1 2^-k + ...) split into several e4m3 parts.

For a Llama-3.2-3B-shaped projection (K = 3072 / 8192) on random activations with realistic
outliers, prints the max relative error of y = W x against the fp32 product of the same
dequantised weights, per activation encoding.  The decode / prefill logits tolerance is 5e-3
absolute on logits of magnitude ~1-10 (tests/test_gpu_llm.py), i.e. ~1e-3 relative per GEMM
stacked over 28 layers."""
import torch

torch.manual_seed(0)
E4M3_MAX = 448.0


def e4m3(x):
    return x.to(torch.float8_e4m3fn).to(torch.float32)


def split_fp8(x, parts):
    """x (rows, K) -> sum of `parts` e4m3 terms with one power-of-two scale per term and row."""
    out = torch.zeros_like(x)
    r = x.clone()
    for _ in range(parts):
        amax = r.abs().amax(dim=1, keepdim=True).clamp_min(1e-30)
        s = torch.exp2(torch.floor(torch.log2(E4M3_MAX / amax)))
        q = e4m3(r * s) / s
        out += q
        r = r - q
    return out


def main():
    for K in (3072, 8192):
        N, R = 1024, 64
        w = torch.randn(N, K) * 0.02
        ws = w.abs().amax(dim=1, keepdim=True) / E4M3_MAX
        wq = e4m3(w / ws) * ws                       # the engine's e4m3 weights, dequantised
        x = torch.randn(R, K)
        x[:, torch.randint(0, K, (8,))] *= 30.0      # a few outlier channels, as in LLM activations
        ref = x.double() @ wq.double().T
        den = ref.abs().max().item()
        for name, xa in (("bf16x3 (in use)", None), ("e4m3 x1 (W8A8)", split_fp8(x, 1)),
                         ("e4m3 x2", split_fp8(x, 2)), ("e4m3 x3", split_fp8(x, 3)),
                         ("e4m3 x4", split_fp8(x, 4))):
            if xa is None:
                b0 = x.to(torch.bfloat16).float()
                b1 = (x - b0).to(torch.bfloat16).float()
                b2 = (x - b0 - b1).to(torch.bfloat16).float()
                xa = b0 + b1 + b2
            y = xa.double() @ wq.double().T
            err = (y - ref).abs().max().item() / den
            print(f"K={K:5d}  {name:16s}  max |dy| / max |y| = {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
