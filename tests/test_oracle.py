"""Pin the CPU oracle (oracle/bert_oracle.c) before trusting it as the checker.

The reference cannot be built or run here (ggml / tokenizers-cpp are
un-vendored submodules) and holds no embedding golden vectors,
so the oracle is pinned by:
  1. bit-level checks of its ggml primitives (fp16 conversion, ggml_init
     tables, Q8 quantiser) against numpy;
  2. an independent numpy restatement of the whole path (tests/numpy_ref.py,
     third GGUF reader, float64 accumulation);
  3. a semantic cross-check against transformers.BertModel built locally with
     the same weights (no download);
  4. reproducibility of the committed golden fixtures (any thread count).
"""
import ctypes
import os

import numpy as np
import pytest

import bertlib
import numpy_ref
import oracle
from make_golden import CASES, ensure_model, load_case


def cos(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return (a * b).sum(-1) / np.linalg.norm(a, axis=-1) / np.linalg.norm(b, axis=-1)


def test_fp16_conversion_bit_exact():
    L = oracle.lib()
    h = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    want = h.view(np.float16).astype(np.float32)
    got = np.array([L.oracle_f16_to_f32(int(x)) for x in h], np.float32)
    finite = np.isfinite(want)
    assert np.array_equal(got[finite].view(np.uint32), want[finite].view(np.uint32))
    assert np.all(np.isnan(got[~finite & np.isnan(want)]))
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.normal(0, 1, 20000), rng.normal(0, 1e-5, 5000), rng.normal(0, 3e4, 2000),
                         [0.0, -0.0, 65504, 65520, 65519.99, 1e-8, 2 ** -24, 2 ** -25, 3 * 2 ** -26, 1e9]])
    xs = xs.astype(np.float32)
    got = np.array([L.oracle_f32_to_f16(float(x)) for x in xs], np.uint16)
    assert np.array_equal(got, xs.astype(np.float16).view(np.uint16))


def test_ggml_tables_match_restatement():
    L = oracle.lib()
    gelu, expt = numpy_ref.tables()
    h = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    x = h.view(np.float16).astype(np.float32)
    og = np.array([L.oracle_tab_gelu(int(v)) for v in h], np.uint16).view(np.float16).astype(np.float32)
    oe = np.array([L.oracle_tab_exp(int(v)) for v in h], np.uint16).view(np.float16).astype(np.float32)
    same = lambda a, b: (a == b) | (np.isnan(a) & np.isnan(b))  # noqa: E731
    assert same(oe, expt).all()
    # glibc tanhf (oracle, like ggml) vs numpy's own f32 tanh: 1 + tanh(x) cancels for
    # x < -1.5, so their last-ulp differences reach the fp16 GELU there (and only there)
    tail = x < -1.5
    assert same(og, gelu)[~tail].all()
    bad = tail & ~same(og, gelu)
    assert bad.sum() < 300
    ulp = np.abs(og[bad].astype(np.float16).view(np.int16).astype(np.int32) -
                 gelu[bad].astype(np.float16).view(np.int16).astype(np.int32))
    assert np.all(ulp <= 8)


def test_q8_quantiser_matches_restatement():
    rng = np.random.default_rng(3)
    x = rng.normal(0, 2, (37, 384)).astype(np.float32)
    x[3, 32:64] = 0.0  # all-zero block: d = 0, q = 0
    x[5, :32] = np.float32(0.5) * np.arange(32, dtype=np.float32)  # exact ties
    for q81 in (False, True):
        d, s, q = oracle.quantize_q8(x, q81)
        rd, rs, rq = numpy_ref.quant_q8(x, q81)
        assert np.array_equal(q.reshape(rq.shape), rq.astype(np.int8))
        assert np.array_equal(d, rd.ravel())
        if q81:
            assert np.array_equal(s, rs.ravel())


SMALL = {"f32": 1e-6, "f16": 1e-6, "q4_0": 3e-5, "q4_1": 3e-5}


@pytest.mark.parametrize("ftype", list(SMALL))
def test_oracle_matches_numpy_restatement(ftype, model_dir):
    p = os.path.join(model_dir, f"pin_minilm_l2_{ftype}.gguf")
    if not os.path.exists(p):
        bertlib.synth_model(p, "minilm", ftype, n_layer=2, seed=99)
    rng = np.random.default_rng(5)
    toks = [[101] + rng.integers(1000, 30522, n - 2).tolist() + [102] for n in (5, 31, 64, 128)]
    got = oracle.Oracle(p).eval_batch(toks, 4)
    m = numpy_ref.Model(p)
    want = np.stack([m.eval(t) for t in toks])
    c = cos(got, want)
    assert np.all(1 - c < SMALL[ftype]), (ftype, 1 - c)
    assert np.allclose(np.linalg.norm(got, axis=1), 1, atol=1e-6)


def test_oracle_semantics_vs_transformers_bert(model_dir):
    """Wiring check: transformers.BertModel (tanh GELU) with the same f32 weights,
    mean-pooled and L2-normalised, agrees up to ggml's fp16 GELU/exp tables."""
    torch = pytest.importorskip("torch")
    tr = pytest.importorskip("transformers")
    p = os.path.join(model_dir, "pin_minilm_l2_f32.gguf")
    if not os.path.exists(p):
        bertlib.synth_model(p, "minilm", "f32", n_layer=2, seed=99)
    g = numpy_ref.GGUF(p)
    cfg = tr.BertConfig(vocab_size=30522, hidden_size=384, num_hidden_layers=2, num_attention_heads=12,
                        intermediate_size=1536, hidden_act="gelu_pytorch_tanh", max_position_embeddings=512,
                        type_vocab_size=2, layer_norm_eps=1e-12, hidden_dropout_prob=0.0,
                        attention_probs_dropout_prob=0.0)
    cfg._attn_implementation = "eager"
    model = tr.BertModel(cfg, add_pooling_layer=False).eval().double()
    sd = {}
    for name, (ne, typ, off) in g.tensors.items():
        w = g.f32(name)
        sd[name] = torch.from_numpy(np.ascontiguousarray(w)).double()
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected and all("position_ids" in k or "token_type_ids" in k for k in missing), (missing, unexpected)
    rng = np.random.default_rng(8)
    toks = [[101] + rng.integers(1000, 30522, n - 2).tolist() + [102] for n in (9, 64, 128)]
    got = oracle.Oracle(p).eval_batch(toks, 4)
    for t, g_ in zip(toks, got):
        with torch.no_grad():
            h = model(input_ids=torch.tensor([t]), token_type_ids=torch.zeros(1, len(t), dtype=torch.long)
                      ).last_hidden_state[0].numpy()
        m = h.mean(0)
        m = m / np.linalg.norm(m)
        assert 1 - cos(g_, m) < 2e-5


@pytest.mark.parametrize("case", [c for c in CASES if CASES[c][0] == "minilm"])
def test_golden_fixtures_reproduce(case, model_dir):
    meta, toks, emb = load_case(case)
    p = ensure_model(model_dir, meta["shape"], meta["ftype"], meta["w_std"])
    o = oracle.Oracle(p)
    assert np.array_equal(o.eval_batch(toks, 3), emb)  # thread-count independent, bit-exact


@pytest.mark.parametrize("case", ["c3_minilm_q4_0", "minilm_q4_1", "c2_minilm_f16"])
def test_ggml_order_spread_reproduces(case, model_dir):
    """The fixtures' ggml_order_spread_1mcos (how far ggml@8ca2c19's plain-C
    and 16-lane builds land from its AVX2 build on the fixture's inputs; the
    GPU parity bound of tests/test_gpu_parity.py parity_bound) is reproduced
    by the oracle's alternate summation orders, and the default order is
    still the AVX2 checker; the variant embeddings stored in the fixture
    (emb_generic, emb_lanes16) are the variants' outputs, bit for bit."""
    from make_golden import load_variants, order_spread, order_variants
    meta, toks, want = load_case(case)
    p = ensure_model(model_dir, meta["shape"], meta["ftype"], meta["w_std"], meta.get("n_layer"))
    var = order_variants(p, toks)
    stored = load_variants(case)
    assert set(stored) == set(var) == {"generic", "lanes16"}
    for k in var:
        assert np.array_equal(var[k], stored[k]), k
    got = order_spread(var, want)
    np.testing.assert_allclose(got, meta["ggml_order_spread_1mcos"], rtol=1e-9, atol=1e-15)
    assert np.array_equal(oracle.Oracle(p).eval_batch(toks, 0), want)
    assert max(got) > 0.0  # the orders really differ


@pytest.mark.skipif(not oracle.simd_available(), reason="host CPU lacks AVX2/FMA/F16C")
@pytest.mark.parametrize("case", ["c1_minilm_f32", "c2_minilm_f16", "c3_minilm_q4_0", "minilm_q4_1",
                                  "c3_minilm_q4_0_ragged"])
def test_simd_oracle_bitwise_scalar(case, model_dir):
    """The AVX2-intrinsics form of the checker (bert_oracle.c oracle_set_simd:
    ggml's AVX2 instructions, the CPU baseline bench.py times) gives the scalar
    AVX2-order checker's embeddings bit for bit — every golden fixture's
    stored vectors — on every weight type, including sentence lengths that are
    not multiples of 32 (the f32 dots' fma tails) and of 4 (the Q4 path's
    4-token groups)."""
    meta, toks, emb = load_case(case)
    p = ensure_model(model_dir, meta["shape"], meta["ftype"], meta["w_std"], meta.get("n_layer"))
    o = oracle.Oracle(p)
    try:
        oracle.set_simd(True)
        got = o.eval_batch(toks, 3)
    finally:
        oracle.set_simd(False)
    assert np.array_equal(got, emb)
    assert np.array_equal(o.eval_batch(toks[:2], 3), emb[:2])  # scalar again after switching back
