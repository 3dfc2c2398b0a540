"""The drop-in boundary on CPU: library loads and exports every declared
symbol, the GGUF contract of the reference loader, the synthetic generator's
determinism, bert_model_quantize, failure behaviour without a GPU, and the
reference's own C++ consumers compiling unchanged against include/."""
import ctypes
import hashlib
import json
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

import bertlib
from gguf_reader import GGUF

HAS_GPU = False
try:
    import torch

    HAS_GPU = torch.cuda.is_available()
except Exception:
    pass


def declared_functions(path):
    src = open(path).read()
    return sorted(set(re.findall(r"BERT_API\s+[\w\s\*]+?\b(\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol(repo):
    L = bertlib.lib()
    decl = declared_functions(os.path.join(repo, "include", "bert.h")) + \
        declared_functions(os.path.join(repo, "include", "bert_amd.h"))
    assert set(bertlib.ABI_SYMBOLS) <= set(decl)
    assert set(bertlib.EXT_SYMBOLS) <= set(decl)
    for name in decl:
        assert hasattr(L, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", bertlib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if " T " in line}
    for name in decl:
        if name == "bert_params_parse":  # C++ reference parameter: mangled like the reference's
            assert any("bert_params_parse" in e for e in exported)
        else:
            assert name in exported, name


def test_no_internal_symbols_leak():
    nm = subprocess.run(["nm", "-D", "--defined-only", bertlib.LIB_PATH], capture_output=True, text=True).stdout
    exported = [line.split()[-1] for line in nm.splitlines() if " T " in line]
    leaked = [e for e in exported if "bertamd" in e]
    assert not leaked, leaked[:5]


def sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def test_synth_is_deterministic_and_matches_fixture(model_dir, repo):
    a = os.path.join(model_dir, "det_a.gguf")
    b = os.path.join(model_dir, "det_b.gguf")
    bertlib.synth_model(a, "minilm", "q4_0", seed=20250117, w_std=0.05)
    bertlib.synth_model(b, "minilm", "q4_0", seed=20250117, w_std=0.05)
    assert sha(a) == sha(b)
    z = np.load(os.path.join(repo, "tests", "golden", "c3_minilm_q4_0.npz"), allow_pickle=False)
    assert json.loads(str(z["meta"]))["model_sha256"] == sha(a)


def test_gguf_contract_of_reference_loader(model_dir):
    """Keys and tensor shapes the reference loader demands (bert.cpp:496-578, 623-652)."""
    p = os.path.join(model_dir, "contract.gguf")
    bertlib.synth_model(p, "minilm", "f16", n_layer=2)
    g = GGUF(p)
    for k in ["bert.context_length", "bert.embedding_length", "bert.feed_forward_length",
              "bert.attention.head_count", "bert.block_count", "bert.attention.layer_norm_epsilon",
              "tokenizer.ggml.model", "tokenizer.ggml.tokens", "tokenizer.ggml.scores",
              "tokenizer.ggml.token_type", "blob.tokenizer.json"]:
        assert k in g.kv, k
    E, I, V = 384, 1536, 30522
    assert len(g.kv["tokenizer.ggml.tokens"]) == V
    t = g.tensors
    assert t["embeddings.word_embeddings.weight"][0] == [E, V]
    assert t["embeddings.token_type_embeddings.weight"][0] == [E, 2]
    assert t["embeddings.position_embeddings.weight"][0] == [E, 512]
    assert t["encoder.layer.1.intermediate.dense.weight"][0] == [E, I]
    assert t["encoder.layer.1.output.dense.weight"][0] == [I, E]
    # f16 conversion rule of convert-to-gguf.py:314-321: only 2-D *.weight tensors
    assert t["encoder.layer.0.attention.self.query.weight"][1] == 1
    assert t["encoder.layer.0.attention.self.query.bias"][1] == 0
    assert t["embeddings.LayerNorm.weight"][1] == 0
    assert len(t) == 5 + 16 * 2


def q4_0_ref(x):
    """ggml quantize_row_q4_0_reference restated in numpy."""
    b = x.reshape(-1, 32).astype(np.float32)
    idx = np.argmax(np.abs(b), axis=1)
    mx = b[np.arange(len(b)), idx]
    d = (mx / np.float32(-8)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(d != 0, np.float32(1) / np.where(d != 0, d, 1), 0).astype(np.float32)
    q = np.minimum(15, np.trunc(b * idv[:, None] + np.float32(8.5)).astype(np.int32))
    qs = (q[:, :16] | (q[:, 16:] << 4)).astype(np.uint8)
    return d.astype(np.float16), qs


def test_bert_model_quantize_matches_reference_quantiser(model_dir):
    f32 = os.path.join(model_dir, "quant_src_f32.gguf")
    q = os.path.join(model_dir, "quant_dst_q4_0.gguf")
    direct = os.path.join(model_dir, "quant_direct_q4_0.gguf")
    bertlib.synth_model(f32, "minilm", "f32", n_layer=1, seed=7)
    bertlib.synth_model(direct, "minilm", "q4_0", n_layer=1, seed=7)
    assert bertlib.quantize(f32, q, "q4_0")
    gq, gs, gd = GGUF(q), GGUF(f32), GGUF(direct)
    for name, (ne, typ, off) in gs.tensors.items():
        tq = gq.tensors[name]
        want_q = name.endswith("weight") and len(ne) == 2
        assert tq[1] == (2 if want_q else typ), name
        # quantising the f32 file == quantising the same f32 master in the generator
        assert np.array_equal(gq.raw(name)[2], gd.raw(name)[2]), name
    # and the quantiser equals the numpy restatement of ggml's reference quantiser
    w = gs.f32("encoder.layer.0.attention.self.key.weight")
    d, qs = q4_0_ref(w.ravel())
    blk = gq.raw("encoder.layer.0.attention.self.key.weight")[2].reshape(-1, 18)
    assert np.array_equal(blk[:, :2].copy().view(np.float16).ravel(), d)
    assert np.array_equal(blk[:, 2:], qs)
    assert gq.kv["general.file_type"] == 2
    assert not bertlib.lib().bert_model_quantize(f32.encode(), q.encode(), 7)  # invalid ftype -> false


@pytest.mark.skipif(HAS_GPU, reason="checks the no-GPU failure path")
def test_load_without_gpu_fails_loudly(model_dir):
    p = os.path.join(model_dir, "nogpu.gguf")
    bertlib.synth_model(p, "minilm", "q4_0", n_layer=1)
    L = bertlib.lib()
    assert not L.bert_load_from_file(p.encode())
    assert "no HIP device" in bertlib.last_error()
    with pytest.raises(RuntimeError):
        bertlib.BertModel(p)


def test_load_rejects_bad_files(model_dir):
    L = bertlib.lib()
    assert not L.bert_load_from_file(b"/nonexistent/model.gguf")
    bad = os.path.join(model_dir, "bad.gguf")
    open(bad, "wb").write(b"GGUF" + b"\0" * 64)
    assert not L.bert_load_from_file(bad.encode())


REF = "/root/reference"


def _compile_ref(repo, src, out, extra=("-L", None, "-lbert")):
    cmd = ["g++", "-std=c++17", "-O1", "-I", os.path.join(repo, "include"), src, "-o", str(out)]
    if extra:
        cmd += ["-L", os.path.join(repo, "build"), "-lbert", "-Wl,-rpath," + os.path.join(repo, "build")]
    else:
        cmd += ["-ldl"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, (src, r.stderr[-2000:])


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "examples")), reason="reference checkout absent")
def test_reference_consumers_compile_unchanged(repo, tmp_path):
    """The reference's consumer programs build unchanged against include/ and
    link build/libbert.so: examples/main.cpp, server.cpp, test_tokenizer.cpp,
    test_embedding.cpp (bert.h + ggml.h), models/quantize.cpp (includes
    "ggml/ggml.h", reference models/quantize.cpp:1) and examples/dylib.cpp
    (dlopen's the library by path, reference examples/dylib.cpp:8: no link)."""
    for ex in ["main.cpp", "server.cpp", "test_tokenizer.cpp", "test_embedding.cpp"]:
        _compile_ref(repo, os.path.join(REF, "examples", ex), tmp_path / ex.replace(".cpp", ""))
    _compile_ref(repo, os.path.join(REF, "models", "quantize.cpp"), tmp_path / "quantize")
    _compile_ref(repo, os.path.join(REF, "examples", "dylib.cpp"), tmp_path / "dylib", extra=None)


@pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "models", "quantize.cpp")), reason="reference checkout absent")
def test_reference_quantize_program_equals_library_quantiser(repo, model_dir, tmp_path):
    """The reference's own quantize program (models/quantize.cpp, compiled
    unchanged, whose work is bert_model_quantize: models/quantize.cpp:47) run on
    an f32 GGUF writes the same bytes as bert_model_quantize called through
    ctypes, for q4_0 and q4_1 (type 2 / 3, models/quantize.cpp:23-24); a bad
    type fails with exit code 1 as in the reference."""
    exe = tmp_path / "quantize"
    _compile_ref(repo, os.path.join(REF, "models", "quantize.cpp"), exe)
    f32 = os.path.join(model_dir, "refq_src_f32.gguf")
    bertlib.synth_model(f32, "minilm", "f32", n_layer=1, seed=11)
    for ftype, code in (("q4_0", "2"), ("q4_1", "3")):
        via_prog = tmp_path / f"prog_{ftype}.gguf"
        via_lib = tmp_path / f"lib_{ftype}.gguf"
        r = subprocess.run([str(exe), f32, str(via_prog), code], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "quantize time" in r.stdout
        assert bertlib.quantize(f32, str(via_lib), ftype)
        assert via_prog.read_bytes() == via_lib.read_bytes(), ftype
    r = subprocess.run([str(exe), f32, str(tmp_path / "bad.gguf"), "7"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1


@pytest.mark.parametrize("n_rep", [1, 2, 3, 8])
def test_shard_cuts_balance_and_cover(n_rep):
    """bert_eval_batch's split over replicas (runtime.cpp shard_cuts, reference
    bert.cpp:1065-1107: sentences are independent): contiguous slices that
    cover the batch exactly once, in order, each within one sentence of the
    token-balanced share — on the shape bert_encode_batch hands it (lengths
    sorted ascending, bert.cpp:1163-1196), on uniform and on ragged batches,
    and when there are fewer sentences than replicas."""
    rng = np.random.default_rng(n_rep)
    cases = [np.sort(rng.integers(1, 513, 4096)), np.full(1024, 128), rng.integers(1, 129, 777),
             np.sort(rng.integers(2, 41, 300)), np.array([512, 1, 1, 1]), np.array([5]), np.array([], np.int64)]
    for lens in cases:
        cut = bertlib.shard_cuts(lens, n_rep)
        assert len(cut) == n_rep + 1 and cut[0] == 0 and cut[-1] == len(lens)
        assert all(a <= b for a, b in zip(cut, cut[1:]))
        total = int(lens.sum())
        mx = int(lens.max()) if len(lens) else 0
        for r in range(n_rep):
            share = int(lens[cut[r]:cut[r + 1]].sum())
            assert share <= total / n_rep + mx, (r, share, total / n_rep, mx)
            # no replica is left idle while another holds more than a share plus one sentence
        if len(lens) >= n_rep and total >= n_rep * mx:
            assert all(cut[r + 1] > cut[r] for r in range(n_rep)), cut
    with pytest.raises(ValueError):
        bertlib.shard_cuts([1, 2], 0)
