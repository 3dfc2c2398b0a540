"""Generate the committed golden fixtures tests/golden/*.npz (test infrastructure).

For every case: write the deterministic synthetic GGUF (bertlib.synth_model,
splitmix64-seeded), draw the token ids the way SURVEY.md §8(d) prescribes
([CLS] + uniform ids in [1000, V) from splitmix64(20250117 + sentence) + [SEP]),
and evaluate them with the CPU oracle (oracle/bert_oracle.c).  The fixture
stores inputs, oracle outputs and the sha256 of the model file, so the GPU
tests can regenerate the same model on the box and prove it is byte-identical
before comparing.  The reference itself cannot be built or run here
(DESIGN.md §5), so these vectors pin the GPU path to the oracle, and the
oracle is pinned separately (tests/test_oracle.py).

Run:  python tests/golden/make_golden.py [case ...]
      python tests/golden/make_golden.py --spread [case ...]   (only add the ggml-order variants and spread)

Each fixture also holds the oracle's embeddings under ggml's other build orders
(emb_generic: the plain-C fallback, emb_lanes16: the AVX-512 width), so the GPU
tests can report and pin how close the GPU lands to each named build.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "embedding.cpp_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import bertlib  # noqa: E402

SEED = 20250117

# name -> (shape, ftype, w_std, sentence lengths[, n_layer override])
CASES = {
    "c1_minilm_f32": ("minilm", "f32", 0.05, [16, 32, 7]),
    "c2_minilm_f16": ("minilm", "f16", 0.05, [128, 128, 128, 128]),
    "c3_minilm_q4_0": ("minilm", "q4_0", 0.05, [128, 128, 128, 128]),
    "c3_minilm_q4_0_ragged": ("minilm", "q4_0", 0.05, [1, 2, 17, 64, 129, 300, 512]),
    "minilm_q4_1": ("minilm", "q4_1", 0.05, [128, 40]),
    "minilm_q4_0_std01": ("minilm", "q4_0", 0.1, [128, 60]),
    "c4_e5_f16": ("e5-base", "f16", 0.05, [256, 256]),
    "c5_bge_q4_1": ("bge-large", "q4_1", 0.05, [512, 512]),
    "c5_bge_q4_1_l2": ("bge-large", "q4_1", 0.05, [512, 77], 2),
    # short sentences on the head-dim-64 shapes: the fused QKV + attention kernel
    "c4_e5_f16_short": ("e5-base", "f16", 0.05, [1, 7, 33, 64, 100, 128]),
    "c5_bge_q4_1_l2_short": ("bge-large", "q4_1", 0.05, [5, 40, 128], 2),
}

# Cases whose Q8 re-quantisation amplifies ANY f32-level rounding difference
# (weights at 2x the trained scale; 24 layers of Q4_1): for them the fixture
# also records how far an exact float64 restatement (tests/numpy_ref.py) lands
# from the oracle, and the GPU is held to that intrinsic level.
CHAOTIC = {"minilm_q4_0_std01", "c5_bge_q4_1"}


def splitmix64(state: int):
    state = (state + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return state, z ^ (z >> 31)


def sentence(index: int, n: int, n_vocab: int) -> list[int]:
    """[CLS] r_1 .. r_{n-2} [SEP]; r uniform in [1000, n_vocab) from splitmix64(SEED + index)."""
    if n == 1:
        return [101]
    st = SEED + index
    ids = [101]
    for _ in range(n - 2):
        st, z = splitmix64(st)
        ids.append(1000 + z % (n_vocab - 1000))
    return ids + [102]


def sha256(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 22), b""):
            h.update(chunk)
    return h.hexdigest()


def model_path(d: str, shape: str, ftype: str, w_std: float, n_layer=None) -> str:
    lay = f"_l{n_layer}" if n_layer else ""
    return os.path.join(d, f"{shape}_{ftype}_s{SEED}_w{w_std:g}{lay}.gguf")


def ensure_model(d: str, shape: str, ftype: str, w_std: float, n_layer=None) -> str:
    p = model_path(d, shape, ftype, w_std, n_layer)
    if not os.path.exists(p):
        over = {"n_layer": n_layer} if n_layer else {}
        bertlib.synth_model(p, shape, ftype, seed=SEED, w_std=w_std, **over)
    return p


def load_case(name: str):
    z = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    offs = z["offsets"]
    toks = [z["tokens"][offs[i]:offs[i + 1]].tolist() for i in range(len(offs) - 1)]
    return meta, toks, z["emb"]


def order_variants(path: str, toks) -> dict:
    """The oracle's embeddings under ggml's other summation orders
    (oracle.DOT_VARIANTS except the AVX2 checker: plain-C fallback, 16-lane
    width) — what two other valid ggml CPU builds of the reference output."""
    import oracle
    o = oracle.Oracle(path)
    out = {}
    try:
        for v in oracle.DOT_VARIANTS:
            if v == "avx2":
                continue
            oracle.set_dot_variant(v)
            out[v] = o.eval_batch(toks, 0).astype(np.float32)
    finally:
        oracle.set_dot_variant("avx2")
    return out


def order_spread(variants: dict, emb) -> list[float]:
    """Per sentence, the largest 1 - cos between the AVX2 oracle (`emb`) and
    the same semantics under the other summation orders ggml@8ca2c19 builds
    use: how far two valid ggml CPU runs of the reference land apart on this
    input."""
    emb = np.asarray(emb, np.float64)
    worst = np.zeros(len(emb))
    for a in variants.values():
        a = a.astype(np.float64)
        c = (a * emb).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(emb, axis=1)
        worst = np.maximum(worst, 1 - c)
    return [float(x) for x in worst]


def save(name: str, tokens, offsets, emb, meta: dict, variants: dict):
    np.savez_compressed(os.path.join(HERE, name + ".npz"), tokens=tokens, offsets=offsets, emb=emb,
                        meta=np.array(json.dumps(meta)), **{f"emb_{k}": v for k, v in variants.items()})


def load_variants(name: str) -> dict:
    """The fixture's embeddings under ggml's other build orders: {"generic": .., "lanes16": ..}."""
    z = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    return {k[4:]: z[k] for k in z.files if k.startswith("emb_")}


def add_spread(name: str, model_dir: str):
    """Add the variant embeddings and ggml_order_spread_1mcos to an existing
    fixture (inputs/outputs unchanged)."""
    meta, toks, emb = load_case(name)
    path = ensure_model(model_dir, meta["shape"], meta["ftype"], meta["w_std"], meta.get("n_layer"))
    assert sha256(path) == meta["model_sha256"]
    var = order_variants(path, toks)
    meta["ggml_order_spread_1mcos"] = order_spread(var, emb)
    z = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    save(name, z["tokens"], z["offsets"], z["emb"], meta, var)
    print(f"{name}: ggml order spread {meta['ggml_order_spread_1mcos']}", flush=True)


def make(name: str, model_dir: str):
    import oracle  # test infrastructure only

    shape, ftype, w_std, lens = CASES[name][:4]
    n_layer = CASES[name][4] if len(CASES[name]) > 4 else None
    hp = dict(bertlib.SHAPES[shape])
    if n_layer:
        hp["n_layer"] = n_layer
    path = ensure_model(model_dir, shape, ftype, w_std, n_layer)
    toks = [sentence(i, n, hp["n_vocab"]) for i, n in enumerate(lens)]
    t0 = time.time()
    emb = oracle.Oracle(path).eval_batch(toks, 0)
    dt = time.time() - t0
    offs = np.zeros(len(toks) + 1, np.int32)
    offs[1:] = np.cumsum([len(t) for t in toks])
    meta = dict(case=name, shape=shape, hparams=hp, ftype=ftype, seed=SEED, w_std=w_std, lengths=lens,
                n_layer=n_layer, model_sha256=sha256(path), oracle_seconds=round(dt, 2),
                generator="bertlib.synth_model (csrc/synth.cpp)", oracle="oracle/bert_oracle.c")
    var = order_variants(path, toks)
    meta["ggml_order_spread_1mcos"] = order_spread(var, emb)
    if name in CHAOTIC:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import numpy_ref
        m = numpy_ref.Model(path)
        ex = np.stack([m.eval(t) for t in toks]).astype(np.float64)
        c = (ex * emb).sum(1) / np.linalg.norm(ex, axis=1) / np.linalg.norm(emb, axis=1)
        meta["exact_restatement_1mcos"] = [float(1 - v) for v in c]
    save(name, np.concatenate(toks).astype(np.int32), offs, emb.astype(np.float32), meta, var)
    print(f"{name}: {len(toks)} sentences, oracle {dt:.1f}s", flush=True)


def main():
    args = sys.argv[1:]
    spread_only = "--spread" in args
    names = [a for a in args if not a.startswith("--")] or list(CASES)
    model_dir = os.environ.get("BERT_AMD_MODEL_DIR") or os.path.join(tempfile.gettempdir(), "bert_amd_models")
    os.makedirs(model_dir, exist_ok=True)
    for n in names:
        (add_spread if spread_only else make)(n, model_dir)


if __name__ == "__main__":
    main()
