"""Which HIP kernel instantiations one decode / prefill launch sequence runs.

A restatement of the library's host-side dispatch, so that the parity tests' coverage of
the kernels the bench runs can be checked on the CPU (tests/test_kernel_coverage.py):

* ``capi.hip``: ``att_b1_shape``, ``att_cpw_auto`` / ``att_cpw_pick``, the o-proj merge
  choice of ``enqueue_layers`` (``b1_merge`` / ``rows_merge``), ``enqueue_head``;
* ``llm_kernels.hip``: ``launch_gemv`` / ``launch_gemv1`` / ``launch_gemv1_t``,
  ``launch_attention``;
* ``mx_rows_v4.inc`` / ``rows_v4_*.hip``: ``rows_tiles``, ``rows_nkc``, ``rows_target_of``,
  ``launch_rows_k`` / ``launch_rows_sub``, ``rows_merge_ok``, ``launch_rows_head``;
* ``head_b1.hip``: ``launch_head_b1``.

Kernel keys are the rocprofv3 names without ``void mx::`` and the argument list, e.g.
``v4::gemm_rows_kernel<1, 1, 1, false, 3, true, 2, 4>``, so they can be compared with the
committed kernel-trace summaries under profiles/.
"""
from __future__ import annotations

from dataclasses import dataclass

EPI_STORE, EPI_RESID, EPI_SILU, EPI_QKV, EPI_ARGMAX = 0, 1, 2, 3, 4


@dataclass(frozen=True)
class Dims:
    hidden: int
    heads: int
    kv_heads: int
    ffn: int
    vocab: int

    @property
    def grp(self):
        return self.heads // self.kv_heads


ORPHEUS = Dims(3072, 24, 8, 8192, 156940)
ORPHEUS_16K = Dims(3072, 24, 8, 8192, 16384)   # the long-context tests' vocabulary
SMALL = Dims(512, 4, 2, 1024, 1000)
SMALL_5K = Dims(512, 4, 2, 1024, 5000)
SMALL_156K = Dims(512, 4, 2, 1024, 156940)
FP8_SMALL = Dims(1024, 8, 2, 2048, 1000)

# library option defaults (capi.hip struct mx_llm)
DEFAULTS = dict(att_cpw=0, att_nw=4, att_nw_batch=8, att_cpw_batch=0, o_merge=1,
                rows_merge=1, gemv_wpb=4, rows_pw=2, rows_pw_f8=2, rows_target=0,
                rows_nt_max=0, rows_nt1=2, rows_head_target=0, rows_head_mt=1, head_b1=1, rpw_o=0,
                rpw_gu=0, rpw_down=0, legacy_gemv=0, b1_engine=0, engine_slots=7, rows_atomic=1,
                rows_qkv_parts=1, att_nw6=1, gemv_balance=1, att_b1_short=1,
                att_b1_nw6=1)
# (rows_atomic and rows_qkv_parts select the residual projections' split-K epilogue at run time inside the same
# instantiation -- float atomics into h / raw partials summed by the attention, or the
# seam -- so they change no kernel key)


def _b(v):
    return "true" if v else "false"


# ---- attention shape (capi.hip) -------------------------------------------------------
def att_b1_shape(max_len, o):
    if o["att_cpw"] > 0:
        return o["att_nw"], o["att_cpw"]
    shapes = ((2, 1), (3, 1), (4, 1), (6, 1), (4, 2), (4, 4), (8, 4), (8, 8))
    first = {2: 0, 1: 1}.get(o.get("att_b1_short", 0), 2)
    for nw, cpw in shapes[first:]:
        if (nw, cpw) == (6, 1) and not o.get("att_b1_nw6", 0):
            continue
        if (max_len + 32 * nw * cpw - 1) // (32 * nw * cpw) <= 8:
            return nw, cpw
    return 8, 8


def att_cpw_pick(want, nw):
    if nw != 8:
        return 1 if want <= 1 else 2 if want <= 2 else 4
    if want <= 4:
        return 1 if want < 1 else want
    return 6 if want <= 6 else 8


def att_shape(d, R, max_len, o):
    """(waves, chunks per wave, splits) of the attention launch over R rows."""
    if R == 1:
        nw, cpw = att_b1_shape(max_len, o)
    else:
        nw = o["att_nw_batch"]
        if o["att_cpw_batch"] > 0:
            cpw = o["att_cpw_batch"]
        else:
            pairs = R * d.kv_heads
            splits = 1 if pairs > 64 else max(1, 256 // pairs)
            chunks = (max_len + 31) // 32
            if o.get("att_nw6", 0) and splits > 1:  # capi.hip att_batch_shape
                for nw, cpw in ((6, 1), (8, 1), (6, 2), (8, 2), (6, 3), (8, 3), (8, 4), (8, 6), (8, 8)):
                    if (chunks + nw * cpw - 1) // (nw * cpw) <= splits:
                        break
            else:
                cpw = att_cpw_pick((chunks + splits * nw - 1) // (splits * nw), nw)
    S = 32 * nw * cpw
    return nw, cpw, (max_len + S - 1) // S


# ---- multi-row GEMM generation 4 (mx_rows_v4.inc) -------------------------------------
_SUBS = (1, 2, 3, 4, 6, 8, 12, 16, 24)


def rows_nkc(N, K, R, MT, NT, target):
    subs = K // 128
    tiles = -(-N // (128 * MT)) * -(-R // (16 * NT))
    nkc = 1
    while tiles * nkc < target and subs % (2 * nkc) == 0 and subs // (2 * nkc) >= 2:
        nkc *= 2
    while tiles * nkc < target and subs % (3 * nkc) == 0 and subs // (3 * nkc) >= 2:
        nkc *= 3
    while (subs // nkc) not in _SUBS and subs % (2 * nkc) == 0:
        nkc *= 2
    return nkc


def rows_tiles(R, nt_max):
    nt = 1 if R <= 16 else 2 if R <= 32 else 4
    if nt_max > 0 and nt > nt_max:
        nt = nt_max
    return 1, nt


def rows_target_of(epi, o):
    if epi == EPI_ARGMAX and o["rows_head_target"] > 0:
        return o["rows_head_target"]
    if o["rows_target"] > 0:
        return o["rows_target"]
    return 128 if epi == EPI_QKV else 192


def _rows_key(MT, NT, epi, norm, sub, f8, o, nsm=0):
    pw = min(o["rows_pw_f8"] if f8 else o["rows_pw"], sub)
    pw = 2 if pw >= 2 else 1
    return f"v4::gemm_rows_kernel<{MT}, {NT}, {epi}, {_b(norm)}, {sub}, {_b(f8)}, {pw}, {nsm}>"


def target_opts(o, kind):
    """capi.hip nt_cap: options rows_target_{qkv,o,gu,down} override rows_target per kind."""
    names = ("rows_target_qkv", "rows_target_o", "rows_target_gu", "rows_target_down")
    if kind is not None and kind < 4 and o.get(names[kind], 0) > 0:
        return dict(o, rows_target=o[names[kind]])
    return o


def nt_max_of(o, kind, R, f8=False):
    """capi.hip nt_cap: option rows_nt1 puts this kind's 17-32-row launches on 16-row tiles
    (kind: 0 qkv, 1 o-proj, 2 gate/up, 3 down, 4 lm_head; None: not a layer launch); above 32
    rows the layer launches take 32-row tiles (rows_nt_max 0 = auto) with e4m3 weights or at
    most 128 rows."""
    if kind is not None and (o["rows_nt1"] >> kind) & 1 and R <= 32:
        return 1
    if o["rows_nt_max"] == 0 and kind is not None and kind < 4 and R > 32 and (f8 or R <= 128):
        return 2
    return o["rows_nt_max"]


def rows_launch(N, K, R, epi, norm, f8, o, merge_nsm=0, kind=None):
    """launch_gemm_rows_v4 -> the instantiation (None where it returns NotSupported)."""
    mt, nt = rows_tiles(R, nt_max_of(o, kind, R, f8))
    o = target_opts(o, kind)
    if epi == EPI_ARGMAX and norm and o["rows_head_mt"] == 2 and nt in (1, 2):
        mt = 2
    if K % 128:
        return None
    nkc = rows_nkc(N, K, R, mt, nt, rows_target_of(epi, o))
    if merge_nsm:
        assert epi == EPI_RESID and mt == 1 and nt == 1 and K // 128 // nkc == 3
        return _rows_key(1, 1, EPI_RESID, False, 3, f8, o, 2 if merge_nsm <= 2 else 4)
    sub = K // 128 // nkc
    if sub not in _SUBS:
        return None
    return _rows_key(mt, nt, epi, norm, sub, f8, o)


def rows_merge_ok(d, R, nsplit, o):
    mt, nt = rows_tiles(R, nt_max_of(o, 1, R))
    o = target_opts(o, 1)
    K = d.heads * 128
    if R < 2 or nt != 1 or K % 128 or nsplit < 1 or nsplit > 4:
        return False
    return K // 128 // rows_nkc(d.hidden, K, R, mt, nt, rows_target_of(EPI_RESID, o)) == 3


# ---- one-row GEMV (llm_kernels.hip) ---------------------------------------------------
def gemv1_launch(N, K, epi, norm, f8, o, rpw=0, nsm=0):
    epc = 1024 if f8 else 512
    if K % epc:
        return None
    kch = K // epc
    if rpw == 0:
        rpw = 2 if epi == EPI_QKV else (4 if f8 else 2) if epi == EPI_SILU else 1
    ok = {(2, EPI_QKV, True), (1, EPI_RESID, False), (2, EPI_RESID, False), (2, EPI_SILU, True),
          (4, EPI_SILU, True), (1, EPI_STORE, False), (1, EPI_STORE, True)}
    if kch not in (1, 2, 3, 4, 6, 8, 16) or (rpw, epi, norm) not in ok or N % rpw:
        return None
    G = N // rpw
    if nsm:
        if not (kch in ((1, 3) if f8 else (1, 2, 6)) and epi == EPI_RESID and not norm):
            raise ValueError("the merging o-proj has no instantiation for this width")
        m = 2 if nsm <= 2 else 4 if nsm <= 4 else 8
        wpb = 6 if o.get("gemv_balance", 0) and gemv_wpb_balanced(G, (8, 6)) == 6 else 8
        return f"gemv1_kernel<{kch}, {rpw}, {epi}, {_b(norm)}, {wpb}, {_b(f8)}, {m}>"
    wpb = o["gemv_wpb"]
    if epi == EPI_QKV and o.get("gemv_balance", 0) and gemv_wpb_balanced(G, (4, 5, 8)) == 5:
        wpb = 5
    return f"gemv1_kernel<{kch}, {rpw}, {epi}, {_b(norm)}, {wpb}, {_b(f8)}, 0>"


CUS = 256  # MI355X compute units (option gemv_balance queries the device)


def gemv_wpb_balanced(G, cand):
    """llm_kernels.hip gemv_wpb_balanced: fewest waves on the most loaded CU, first wins ties."""
    best, best_w = 0, 1 << 30
    for w in cand:
        per_cu = -(-(-(-G // w)) // CUS) * w
        if per_cu < best_w:
            best, best_w = w, per_cu
    return best


def gemv_launch(N, K, R, epi, norm, f8, o, rpw=0, nsm=0, kind=None):
    """launch_gemv: the kernel one projection / lm_head launch runs."""
    if R == 1 and epi != EPI_ARGMAX and not o["legacy_gemv"]:
        k = gemv1_launch(N, K, epi, norm, f8, o, rpw, nsm)
        if k or nsm:
            return k
    if R == 1 and epi == EPI_ARGMAX and norm and o["head_b1"] and not o["legacy_gemv"]:
        if K == 3072:
            return "head1::head_b1_kernel<3, 4, true>" if f8 else "head1::head_b1_kernel<6, 2, false>"
    if R == 1 and epi == EPI_ARGMAX and norm and f8 and K % 1024 == 0:
        return "gemv_kernel<1, 8, 4, true, true>"
    if (R >= 2 and not o["legacy_gemv"]) or f8:
        k = rows_launch(N, K, R, epi, norm, f8, o, kind=kind)
        if k or f8:
            return k
    rt = 1 if R == 1 else 4
    rpw_g = 4 if epi == EPI_ARGMAX else 2
    return f"gemv_kernel<{rt}, {rpw_g}, {epi}, {_b(norm)}, false>"


# ---- one forward (capi.hip enqueue_layers / enqueue_head) -----------------------------
PREFILL_TAG = " [prefill]"


def forward_keys(d, R, max_len, f8, opts=None, head_rows=None, sample=False):
    """Kernel keys of one forward over R rows whose longest attention span is max_len
    (decode: R rows, lm_head over R rows; prefill: R = prompt length, lm_head on 1 row:
    head_rows = 1).  The attention key of a prefill carries PREFILL_TAG: its rows share one
    KV slot at consecutive positions, so it does not stand in for a decode launch of the same
    instantiation (rows on separate slots)."""
    o = dict(DEFAULTS, **(opts or {}))
    H, QD = d.hidden, d.heads * 128
    keys = set()
    if R == 1 and head_rows is None and o["b1_engine"]:  # capi.hip enqueue_decode
        keys.add(f"eng::engine_kernel<{_b(f8)}, {d.grp}>")
        keys.add(gemv_launch(d.vocab, H, 1, EPI_ARGMAX, True, f8, o))
        return keys
    keys.add(gemv_launch(QD + 2 * d.kv_heads * 128, H, R, EPI_QKV, True, f8, o, kind=0))
    nw, cpw, nsplit = att_shape(d, R, max_len, o)
    keys.add(f"attn_kernel<{d.grp}, {cpw}, {nw}>" + (PREFILL_TAG if head_rows == 1 and R > 1 else ""))
    b1_merge = R == 1 and not o["legacy_gemv"] and o["o_merge"] and nsplit <= 8
    rmerge = (R >= 2 and nsplit > 1 and not o["legacy_gemv"] and o["rows_merge"]
              and rows_merge_ok(d, R, nsplit, o))
    if b1_merge:
        keys.add(gemv_launch(H, QD, 1, EPI_RESID, False, f8, o,
                             rpw=o["rpw_o"] or 2, nsm=nsplit))
    elif rmerge:
        keys.add(rows_launch(H, QD, R, EPI_RESID, False, f8, o, merge_nsm=nsplit, kind=1))
    else:
        keys.add(gemv_launch(H, QD, R, EPI_RESID, False, f8, o, rpw=o["rpw_o"], kind=1))
    keys.add(gemv_launch(2 * d.ffn, H, R, EPI_SILU, True, f8, o, rpw=o["rpw_gu"], kind=2))
    keys.add(gemv_launch(H, d.ffn, R, EPI_RESID, False, f8, o, rpw=o["rpw_down"], kind=3))
    hr = R if head_rows is None else head_rows
    keys.add(gemv_launch(d.vocab, H, hr, EPI_ARGMAX, True, f8, o, kind=4))
    if sample:
        keys.add("sample_kernel")
    if None in keys:
        raise ValueError(f"no instantiation for R={R} L={max_len} f8={f8} dims={d}")
    return keys


def decode_keys(d, R, max_len, f8, opts=None, sample=False):
    """One decode step (mx_llm_decode: the graph is captured at max_len rounded up to the
    split length, which selects the same shapes)."""
    return forward_keys(d, R, max_len, f8, opts, sample=sample)


def prefill_keys(d, n, f8, opts=None, sample=False):
    """mx_llm_prefill of an n-id prompt: n rows through the layers, lm_head on the last."""
    return forward_keys(d, n, n, f8, opts, head_rows=1, sample=sample)


def run_keys(d, f8, lens, steps, opts=None):
    """Prompts of `lens` ids prefilled on their own rows, then `steps` tokens per row: the
    first from the prefill, then steps - 1 decode steps over all rows together (the helpers
    of tests/test_gpu_llm.py / test_gpu_fp8.py).  Decode step k's longest span is
    max(lens) + k."""
    keys = set()
    for n in sorted(set(lens)):
        keys |= prefill_keys(d, n, f8, opts)
    for k in range(1, steps):
        keys |= decode_keys(d, len(lens), max(lens) + k, f8, opts)
    return keys
