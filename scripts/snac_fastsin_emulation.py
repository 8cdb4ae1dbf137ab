"""CPU emulation of the device Snake (hardware sine on an fp32 revolution-reduced argument) against
the fp32 oracle's torch.sin (diagnostic)."""
import sys, os, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import snac_ref
from project_morpheus_amd.weights import synthetic_snac_weights
orig = snac_ref.snake
def fast_snake(x, alpha):
    a = alpha.reshape(1, -1, 1).float()
    ax = (a * x).float()
    rev = (ax * torch.tensor(1/(2*np.pi), dtype=torch.float32)).float()
    fr = rev - torch.floor(rev)   # fp32
    s = torch.sin(fr.double() * 2 * np.pi).float()
    return x + (a + 1e-9).reciprocal() * s * s
w = synthetic_snac_weights(seed=3)
p = {k: (v.float() if torch.is_tensor(v) else v) for k,v in w.items()}
rng = np.random.default_rng(1); n = 7
for trial in range(3):
    c = rng.integers(0,4096,size=7*n).tolist()
    c0=[c[7*f] for f in range(n)]; c1=[c[7*f+j] for f in range(n) for j in (1,4)]; c2=[c[7*f+j] for f in range(n) for j in (2,3,5,6)]
    noise = snac_ref.window_noise(11+trial, n)
    snac_ref.snake = orig; ref = snac_ref.decode(p,c0,c1,c2,noise)
    snac_ref.snake = fast_snake; out = snac_ref.decode(p,c0,c1,c2,noise)
    d=(out-ref).abs(); pr=(ref*32767).trunc(); po=(out*32767).trunc()
    print('rms %.2e max %.2e pcm_max %d' % (d.pow(2).mean().sqrt(), d.max(), (pr-po).abs().max()))
