"""Per-layer parity pin: the GPU residual stream after
every stage against the CPU oracle, on the golden fixtures' inputs.

For each stage s (0 = embeddings + LN, reference bert.cpp:865-898; s = l + 1 =
encoder layer l, bert.cpp:900-993) the test compares, per sentence:

  chained : GPU X_s vs the oracle's X_s (both from the same token ids) —
            max ulp and 1 - cos, the error the stage has accumulated;
  local   : GPU X_s vs oracle.layer(l, GPU X_{s-1}) — the error layer l adds
            by itself, with its input held equal;
  spread  : oracle.layer(l, GPU X_{s-1}) under ggml's plain-C summation
            order vs the AVX2 order on that same input — how far two ggml
            builds land apart on this very layer (the f32-order noise floor
            that Q8 re-quantisation amplifies);
  codes   : the GPU's own Q8 / fp16 activations of X_s against the oracle
            quantiser (ggml quantize_row_q8_x, AVX2) applied to the GPU's X_s:
            must be bit-identical at every stage.  A code that differs where
            the input is identical is a quantiser bug, not order noise.

The per-stage table is printed and written to gpurun_out/layer_parity_<case>.json
(DESIGN.md §4 "Per-layer parity").
"""
import json
import os

import numpy as np
import pytest

import bertlib
from make_golden import ensure_model, load_case, sha256

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG = os.environ.get("BERT_AMD_PARITY_DIAG") == "1"


def cos_rows(a, b):
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    return float((a * b).sum() / np.linalg.norm(a) / np.linalg.norm(b))


def max_ulp(a, b):
    """Largest difference in units of the last place of the row's largest
    magnitude (a value near zero that changes sign is not counted as 2^31 ulp)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    scale = np.spacing(np.abs(b).max(axis=-1, keepdims=True))
    return int(np.ceil((np.abs(a.astype(np.float64) - b) / scale).max()))


# (case, sentences of the fixture to use, load options): C3 on the fused QKV +
# attention kernel (fuse_min 0: a 4-sentence batch would otherwise take the
# unfused pair), C2 F16, and the 24-layer C5 whose 1 - cos ~2e-3 this explains
CASES = [
    ("c5_bge_q4_1", [0], {"i8": "all"}),
    ("c3_minilm_q4_0", [0, 1], {"fuse_min": 0}),
    ("c3_minilm_q4_0", [0], {"fuse_min": 1000}),
    ("c2_minilm_f16", [0], {"fuse_min": 0}),
    ("minilm_q4_1", [0, 1], {"fuse_min": 0}),
    ("c5_bge_q4_1", [0], {}),
    # Q4_1's scale products on the bf16 MFMA (W_Q4_1B) held to the same acceptance
    ("c5_bge_q4_1", [0], {"q41bf": 1}),
    ("minilm_q4_1", [0, 1], {"fuse_min": 0, "q41bf": 1}),
    ("c5_bge_q4_1", [0], {"q41bf": 0}),
]


def _tag(c):
    t = c[0] + ("-i8all" if c[2].get("i8") == "all" else "-fused" if c[2].get("fuse_min") == 0 else "-pair")
    return t + (f"-q41bf{c[2]['q41bf']}" if "q41bf" in c[2] else "")


@pytest.mark.parametrize("case,sents,opts", CASES, ids=[_tag(c) for c in CASES])
def test_layer_by_layer_parity(case, sents, opts, model_dir):
    import oracle
    meta, toks, want = load_case(case)
    p = ensure_model(model_dir, meta["shape"], meta["ftype"], meta["w_std"], meta.get("n_layer"))
    assert sha256(p) == meta["model_sha256"]
    toks = [toks[i] for i in sents]
    m = bertlib.BertModel(p, options=opts)
    try:
        X, q, d = m.debug_layers(toks)
    finally:
        m.close()
    orc = oracle.Oracle(p)
    wt = orc.wtype  # ggml type: 0 f32, 1 f16, 2 q4_0, 3 q4_1
    q4 = wt in (2, 3)
    S = X.shape[0]
    offs = np.concatenate([[0], np.cumsum([len(t) for t in toks])])
    rows = []
    for si, t in enumerate(toks):
        r0, r1 = offs[si], offs[si + 1]
        ref = orc.eval_layers(t)  # [S, n, E]
        for s in range(S):
            g = X[s, r0:r1]
            row = {"sentence": si, "stage": s, "chained_ulp": max_ulp(g, ref[s]),
                   "chained_1mcos": 1 - cos_rows(g, ref[s])}
            # codes: the GPU's activation form of its own X_s, bit for bit
            if q4:
                dq, _, qq = oracle.quantize_q8(g, q8_1=(wt == 3))
                row["code_mismatch"] = int(np.count_nonzero(q[s, r0:r1].ravel() != qq))
                row["scale_mismatch"] = int(np.count_nonzero(d[s, r0:r1].astype(np.float32).ravel() != dq))
            elif wt == 1:
                row["code_mismatch"] = int(np.count_nonzero(q[s, r0:r1].view(np.uint16) !=
                                                            g.astype(np.float16).view(np.uint16)))
                row["scale_mismatch"] = 0
            if s > 0:
                x_in = X[s - 1, r0:r1]
                loc = orc.layer(s - 1, x_in)
                row["local_ulp"] = max_ulp(g, loc)
                row["local_1mcos"] = 1 - cos_rows(g, loc)
                # ggml's plain-C and 16-lane (AVX-512) summation orders on the same input
                spreads = []
                for var in ("generic", "lanes16"):
                    oracle.set_dot_variant(var)
                    try:
                        alt = orc.layer(s - 1, x_in)
                    finally:
                        oracle.set_dot_variant("avx2")
                    spreads.append((1 - cos_rows(alt, loc), max_ulp(alt, loc)))
                    # the GPU's own layer against that build's layer on the same input
                    row[f"local_{var}_1mcos"] = 1 - cos_rows(g, alt)
                if DIAG:
                    # diagnostic (BERT_AMD_PARITY_DIAG=1): the oracle with the GPU's attention
                    # operand form (oracle.set_attn_form, not a ggml build) under each order
                    oracle.set_attn_form("gpu_operands")
                    try:
                        for var in ("avx2", "generic"):
                            oracle.set_dot_variant(var)
                            row[f"local_{var}_gpuattn_1mcos"] = 1 - cos_rows(g, orc.layer(s - 1, x_in))
                    finally:
                        oracle.set_dot_variant("avx2")
                        oracle.set_attn_form("ggml")
                row["spread_1mcos"] = max(sp[0] for sp in spreads)
                row["spread_ulp"] = max(sp[1] for sp in spreads)
            rows.append(row)
    tag = _tag((case, sents, opts))
    print(f"\n{tag}: stage, chained ulp / 1-cos, local ulp / 1-cos, ggml spread ulp / 1-cos, code mismatches")
    for r in rows:
        print(f"  s{r['sentence']} stage {r['stage']:2d}: {r['chained_ulp']:>10d} {r['chained_1mcos']:.2e} | "
              f"{r.get('local_ulp', 0):>10d} {r.get('local_1mcos', 0):.2e} | "
              f"{r.get('spread_ulp', 0):>10d} {r.get('spread_1mcos', 0):.2e} | {r.get('code_mismatch', '-')}")
    out = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, f"layer_parity_{tag}.json"), "w") as f:
            json.dump(rows, f, indent=1)
    # the integer stage conversions are exact everywhere
    assert all(r.get("code_mismatch", 0) == 0 and r.get("scale_mismatch", 0) == 0 for r in rows), \
        [r for r in rows if r.get("code_mismatch", 0) or r.get("scale_mismatch", 0)]
    # the embedding stage is f32-exact up to one ulp (test_embed_stage_bit_exact)
    assert all(r["chained_ulp"] <= 1 for r in rows if r["stage"] == 0)
    # each layer's own error is f32-order noise, not a defect: a wrong block,
    # scale or mask shows up as 1 - cos >= 1e-4 on one layer, whereas Q8
    # re-quantisation turns an f32 rounding difference into single code flips
    # worth ~1e-7 here — the same quantum by which ggml's own builds differ
    # (spread column); and over all layers the GPU is no further from the AVX2
    # build than ggml's other builds are (means of the local columns)
    loc = [r["local_1mcos"] for r in rows if r["stage"]]
    spr = [r["spread_1mcos"] for r in rows if r["stage"]]
    print(f"mean local 1-cos {np.mean(loc):.2e}, mean ggml spread {np.mean(spr):.2e}, max local {max(loc):.2e}")
    for var in ("generic", "lanes16") + (("avx2_gpuattn", "generic_gpuattn") if DIAG else ()):
        lv = [r[f"local_{var}_1mcos"] for r in rows if r["stage"]]
        print(f"  mean local 1-cos vs the {var} build {np.mean(lv):.2e} (max {max(lv):.2e}, "
              f"layers where the GPU equals it bit for bit: {sum(v == 0.0 for v in lv)} of {len(lv)})")
    # (measured, round 5: max local 1.6e-6 on C5; mean local / mean spread
    # 0.83 - 1.13 across the fixtures and forms)
    assert max(loc) <= 4e-6, loc
    assert np.mean(loc) <= max(1.5 * np.mean(spr), 2e-7), (np.mean(loc), np.mean(spr))
