"""GPU parity: build/libbert.so (HIP kernels, gfx950) vs the CPU oracle.

Every call goes through the C ABI (bert_eval_batch / bert_eval / bert_encode /
bert_amd_eval_device).  Tolerance (BASELINE.json north_star): cosine
similarity >= 0.9999 per sentence against the ggml-semantics oracle; the
measured deviation is ~1e-5.  Properties checked at full size:
unit norm, determinism, batch invariance (a sentence's embedding does not
depend on what else is in the batch), replica sharding invariance.
"""
import os

import numpy as np
import pytest

import bertlib
from make_golden import CASES, CHAOTIC, SEED, ensure_model, load_case, sentence, sha256

pytestmark = pytest.mark.gpu

COS_TOL = 0.9999


def cos(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return (a * b).sum(-1) / np.linalg.norm(a, axis=-1) / np.linalg.norm(b, axis=-1)


_models = {}


def get_model(model_dir, shape, ftype, w_std=0.05, n_layer=None):
    key = (shape, ftype, w_std, n_layer)
    if key not in _models:
        for k in list(_models):  # keep at most one big model resident at a time
            if k[0] != "minilm":
                _models.pop(k)[1].close()
        p = ensure_model(model_dir, shape, ftype, w_std, n_layer)
        _models[key] = (p, bertlib.BertModel(p))
    return _models[key]


@pytest.fixture(scope="module", autouse=True)
def _cleanup():
    yield
    for _, m in _models.values():
        m.close()
    _models.clear()


@pytest.mark.parametrize("case", list(CASES))
def test_golden_vectors(case, model_dir):
    meta, toks, want = load_case(case)
    p, m = get_model(model_dir, meta["shape"], meta["ftype"], meta["w_std"], meta.get("n_layer"))
    assert sha256(p) == meta["model_sha256"], "generator is not reproducing the fixture's model on this host"
    got = m.eval_batch(toks)
    assert np.all(np.isfinite(got))
    c = cos(got, want)
    print(f"{case}: 1-cos min/mean {1 - c.max():.2e}/{1 - c.mean():.2e} max {1 - c.min():.2e} "
          f"maxabs {np.abs(got - want).max():.2e}")
    if case in CHAOTIC:
        # intrinsic sensitivity: an exact float64 restatement lands this far from the
        # oracle; the GPU must not be further than twice that (and never NaN/garbage)
        bound = np.maximum(2.0 * np.asarray(meta["exact_restatement_1mcos"]), 1 - COS_TOL)
        assert np.all(1 - c <= bound), (case, 1 - c, bound)
    else:
        assert c.min() >= COS_TOL, (case, 1 - c)
    assert np.allclose(np.linalg.norm(got, axis=1), 1.0, atol=1e-5)


def test_live_oracle_random_ragged(model_dir):
    """Random lengths (not multiples of 16/64), fresh ids: GPU vs oracle run now."""
    import oracle
    p, m = get_model(model_dir, "minilm", "q4_0")
    rng = np.random.default_rng(2024)
    lens = [3, 15, 16, 17, 63, 65, 100, 127, 200, 333]
    toks = [[101] + rng.integers(1000, 30522, n - 2).tolist() + [102] for n in lens]
    got = m.eval_batch(toks)
    want = oracle.Oracle(p).eval_batch(toks, 0)
    c = cos(got, want)
    assert c.min() >= COS_TOL, 1 - c


@pytest.mark.parametrize("ftype", ["f32", "f16", "q4_0", "q4_1"])
def test_every_weight_type_vs_oracle(ftype, model_dir):
    import oracle
    p, m = get_model(model_dir, "minilm", ftype)
    toks = [sentence(100 + i, n, 30522) for i, n in enumerate([8, 40, 128])]
    c = cos(m.eval_batch(toks), oracle.Oracle(p).eval_batch(toks, 0))
    assert c.min() >= COS_TOL, (ftype, 1 - c)


@pytest.mark.parametrize("case", ["c3_minilm_q4_0", "c3_minilm_q4_0_ragged", "minilm_q4_1", "minilm_q4_0_std01"])
def test_int8_gemm_path_golden(case, model_dir, monkeypatch):
    """The opt-in int8-MFMA Q4 GEMMs (env BERT_AMD_I8=1: gemm_i8.hip, scales
    applied in-kernel per block like ggml_vec_dot_q4_x_q8_x) against the same
    golden fixtures, and bitwise deterministic."""
    meta, toks, want = load_case(case)
    p = ensure_model(model_dir, meta["shape"], meta["ftype"], meta["w_std"], meta.get("n_layer"))
    monkeypatch.setenv("BERT_AMD_I8", "1")
    m = bertlib.BertModel(p)
    try:
        got = m.eval_batch(toks)
        assert np.array_equal(got, m.eval_batch(toks))
    finally:
        m.close()
    c = cos(got, want)
    print(f"int8 {case}: 1-cos max {1 - c.min():.2e}")
    if case in CHAOTIC:
        assert np.all(1 - c <= np.maximum(2.0 * np.asarray(meta["exact_restatement_1mcos"]), 1 - COS_TOL))
    else:
        assert c.min() >= COS_TOL, (case, 1 - c)


def test_batch_invariance_and_determinism(model_dir):
    p, m = get_model(model_dir, "minilm", "q4_0")
    toks = [sentence(i, n, 30522) for i, n in enumerate([5, 128, 64, 17, 512, 128])]
    full = m.eval_batch(toks)
    again = m.eval_batch(toks)
    assert np.array_equal(full, again)
    for i in (0, 1, 4):
        assert np.array_equal(m.eval(toks[i]), full[i])
    rev = m.eval_batch(toks[::-1])
    assert np.array_equal(rev[::-1], full)


def test_full_size_north_star_batch(model_dir):
    """BASELINE config 3 at full size: 1024 x 128 Q4_0; size-independent properties
    on all rows and oracle parity on a sample of rows."""
    import oracle
    p, m = get_model(model_dir, "minilm", "q4_0")
    toks = [sentence(i, 128, 30522) for i in range(1024)]
    out = m.eval_batch(toks)
    assert np.all(np.isfinite(out))
    assert np.allclose(np.linalg.norm(out, axis=1), 1.0, atol=1e-5)
    sample = [0, 1, 511, 1023]
    want = oracle.Oracle(p).eval_batch([toks[i] for i in sample], 0)
    c = cos(out[sample], want)
    assert c.min() >= COS_TOL, 1 - c
    fx_meta, fx_toks, fx_emb = load_case("c3_minilm_q4_0")  # fixture = sentences 0..3 of this batch
    assert [t for t in fx_toks] == toks[:4]
    assert cos(out[:4], fx_emb).min() >= COS_TOL


def test_device_resident_api_matches_host_api(model_dir):
    torch = pytest.importorskip("torch")
    p, m = get_model(model_dir, "minilm", "q4_0")
    toks = [sentence(i, n, 30522) for i, n in enumerate([128, 77, 1, 300])]
    host = m.eval_batch(toks)
    offs = np.zeros(len(toks) + 1, np.int32)
    offs[1:] = np.cumsum([len(t) for t in toks])
    d_tok = torch.tensor(np.concatenate(toks), dtype=torch.int32, device="cuda")
    d_off = torch.tensor(offs, dtype=torch.int32, device="cuda")
    d_out = torch.empty(len(toks), m.n_embd, dtype=torch.float32, device="cuda")
    m.eval_device(d_tok.data_ptr(), d_off.data_ptr(), offs, len(toks), d_out.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy(), host)


def test_two_replicas_shard_like_one(model_dir):
    """bert_amd_load with devices [0, 0]: two replicas, two host threads, the
    batch split by token count — results identical to one replica."""
    p, m = get_model(model_dir, "minilm", "q4_0")
    m2 = bertlib.BertModel(p, devices=[0, 0])
    try:
        assert m2.n_devices == 2
        toks = [sentence(i, n, 30522) for i, n in enumerate([128, 9, 256, 64, 2, 500, 128])]
        assert np.array_equal(m2.eval_batch(toks), m.eval_batch(toks))
    finally:
        m2.close()


def test_error_paths_leave_output_untouched(model_dir):
    p, m = get_model(model_dir, "minilm", "q4_0")
    too_long = [101] + [2000] * 600 + [102]  # > n_max_tokens (512): reference prints and returns
    out = m.eval_batch([too_long])
    assert np.all(np.isnan(out))
    bad_id = [101, 40000, 102]
    assert np.all(np.isnan(m.eval_batch([bad_id])))


def test_encode_path_and_tokenizer(model_dir):
    """bert_encode_batch (tokenise + eval, as sample_dylib.py / server.cpp call it)
    equals bert_eval_batch on bert_tokenize's ids."""
    p, m = get_model(model_dir, "minilm", "q4_0")
    texts = ["Should I get health insurance?", "Québec", "ba ce di fo gu " * 40, "x"]
    emb = m.encode(texts)
    ids = [m.tokenize(t) for t in texts]
    assert ids[1][0] == 101 and ids[1][-1] == 102
    assert np.array_equal(emb, m.eval_batch(ids))
    assert np.array_equal(m.encode(texts[0]), emb[0])


def test_q8_scale_division_exhaustive():
    """kernels.hip q8_scales: the short forms of ggml's d = amax/127 and
    id = 127/amax equal IEEE division for every positive finite f32 (the
    reciprocal form inside [2^-101, 2^101), where the kernels use it)."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "div_check")
    assert os.path.exists(exe), "build/div_check missing: run make"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120).stdout
    print(out)
    assert "x/127 mismatches 0;" in out and "127/x mismatches (x in [2^-101, 2^101)) 0," in out
