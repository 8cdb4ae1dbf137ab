"""CPU emulation of the SNAC conv-GEMM operand splits (bf16 parts per operand, products kept
when part indices sum below `terms`) against the fp32 oracle (diagnostic)."""
import sys, numpy as np, torch
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch.nn.functional as F0
from oracle import snac_ref
from project_morpheus_amd.weights import synthetic_snac_weights

def bf(x): return x.to(torch.bfloat16).to(torch.float32)
def split(x, n):
    parts=[]; r=x
    for _ in range(n):
        h=bf(r); parts.append(h); r=r-h
    return parts

MODE = None
class FP:
    def __getattr__(self, k): return getattr(F0, k)
    @staticmethod
    def conv1d(x, w, b=None, **kw):
        if kw.get('groups',1)!=1 or w.shape[-1]!=1 or MODE is None: return F0.conv1d(x,w,b,**kw)
        return _apply(lambda xx, ww: F0.conv1d(xx.double(), ww.double(), None, **kw), x, w, b)
    @staticmethod
    def conv_transpose1d(x, w, b=None, **kw):
        if MODE is None: return F0.conv_transpose1d(x,w,b,**kw)
        return _apply(lambda xx, ww: F0.conv_transpose1d(xx.double(), ww.double(), None, **kw), x, w, b, ch_dim=1)
def _apply(f, x, w, b, ch_dim=None):
    nx, nw, terms = MODE
    xs, ws = split(x, nx), split(w, nw)
    out = 0
    for i,xp in enumerate(xs):
        for j,wp in enumerate(ws):
            if i+j < terms: out = out + f(xp, wp)
    out = out.float()
    if b is not None: out = out + b.reshape(1,-1,1)
    return out
snac_ref.F = FP()
w = synthetic_snac_weights(seed=3)
p = {k: (v.float() if torch.is_tensor(v) else v) for k,v in w.items()}
rng = np.random.default_rng(1)
n=7
for trial in range(2):
    c = rng.integers(0,4096,size=7*n).tolist()
    c0=[c[7*f] for f in range(n)]; c1=[c[7*f+j] for f in range(n) for j in (1,4)]; c2=[c[7*f+j] for f in range(n) for j in (2,3,5,6)]
    noise = snac_ref.window_noise(11+trial, n)
    MODE=None; ref = snac_ref.decode(p,c0,c1,c2,noise)
    for mode in [(2,2,2),(3,2,3),(3,3,3),(2,2,3)]:
        MODE=mode; out = snac_ref.decode(p,c0,c1,c2,noise)
        d=(out-ref).abs()
        pr=(ref*32767).trunc(); po=(out*32767).trunc()
        print(trial, mode, 'rms %.2e max %.2e pcm_max %d ref_absmax %.3f' % (d.pow(2).mean().sqrt(), d.max(), (pr-po).abs().max(), ref.abs().max()))
