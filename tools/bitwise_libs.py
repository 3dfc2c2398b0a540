"""Bitwise comparison of library builds (development A/B on the GPU box).

    python3 tools/bitwise_libs.py lib_a.so lib_b.so[@BERT_AMD_KEY=VALUE,...] ...

Each library runs in its own process (BERT_AMD_LIB) on the same synthetic
MiniLM Q4_0 / Q4_1 models and the same batches (the headline shape, a ragged
8..128-token batch, one 16-token sentence); every later library's embeddings
must equal the first's byte for byte.  A variant that only re-arranges the
arithmetic (e.g. i8_core.h I8_FOLD) has to pass this before it is timed.
"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out):
    sys.path.insert(0, os.path.join(REPO, "embedding.cpp_amd"))
    import bertlib

    d = os.environ.get("BERT_AMD_MODEL_DIR", "/tmp/bert_amd_models")
    os.makedirs(d, exist_ok=True)
    rng = np.random.default_rng(7)
    batches = {
        "fixed": [[101] + rng.integers(1000, 30522, 126).tolist() + [102] for _ in range(512)],
        "ragged": [[101] + rng.integers(1000, 30522, int(n) - 2).tolist() + [102] for n in rng.integers(8, 129, 400)],
        "one": [[101] + rng.integers(1000, 30522, 14).tolist() + [102]],
        "few": [[101] + rng.integers(1000, 30522, n - 2).tolist() + [102] for n in (5, 40, 77, 128)],
    }
    res = {}
    for ft in os.environ.get("BITWISE_FTYPES", "q4_0,q4_1").split(","):
        path = os.path.join(d, f"bitwise_minilm_{ft}.gguf")
        if not os.path.exists(path):
            bertlib.synth_model(path, "minilm", ft, seed=20250117, w_std=0.05)
        m = bertlib.BertModel(path, devices=[0])
        for k, b in batches.items():
            res[f"{ft}_{k}"] = m.eval_batch(b)
        m.close()
    np.savez(out, **res)


def main():
    libs = sys.argv[1:]
    outs = []
    for i, spec in enumerate(libs):
        # "lib.so" or "lib.so@KEY=VALUE,KEY=VALUE": environment options for that run
        lib, _, envs = spec.partition("@")
        out = f"/tmp/bitwise_{i}.npz"
        env = dict(os.environ, BERT_AMD_LIB=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in envs.split(",") if kv)
        subprocess.run([sys.executable, __file__, "--child", out], env=env, check=True, timeout=300)
        outs.append(np.load(out))
    ok = True
    for lib, o in zip(libs[1:], outs[1:]):
        for k in outs[0].files:
            a, b = outs[0][k], o[k]
            same = a.tobytes() == b.tobytes()
            ok &= same
            print(f"{lib} {k}: {'bitwise equal' if same else 'DIFFERS max %.3g' % np.abs(a - b).max()}", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        main()
