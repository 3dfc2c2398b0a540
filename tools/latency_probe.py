"""Single-sentence latency (bert_eval, the reference server's per-request path)
under the small-batch options: small_rows (32-row int8 GEMM tiles) and
graph_seqs (captured HIP graph per batch shape).  Development A/B; prints one
JSON line per configuration.

    python3 tools/latency_probe.py [--runs 200] [--shape minilm --ftype q4_0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedding.cpp_amd"))
import bertlib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="minilm")
ap.add_argument("--ftype", default="q4_0")
ap.add_argument("--runs", type=int, default=200)
ap.add_argument("--model-dir", default=os.environ.get("BERT_AMD_MODEL_DIR", "/tmp/bert_amd_models"))
ap.add_argument("--configs", default="0:0,2048:0,2048:8,0:8", help="small_rows:graph_seqs pairs")
ap.add_argument("--lengths", default="16,128")
ap.add_argument("--opts", default="", help="extra options, k=v[,k=v]")
args = ap.parse_args()

os.makedirs(args.model_dir, exist_ok=True)
path = os.path.join(args.model_dir, f"{args.shape}_{args.ftype}_s20250117_w0.05.gguf")
if not os.path.exists(path):
    tmp = f"{path}.tmp{os.getpid()}"
    bertlib.synth_model(tmp, args.shape, args.ftype, seed=20250117, w_std=0.05)
    os.replace(tmp, path)
m = bertlib.BertModel(path, devices=[0])
for kv in filter(None, args.opts.split(",")):
    k, v = kv.split("=")
    m.set_option(k, int(v))
rng = np.random.default_rng(7)
ref = {}
for cfg in args.configs.split(","):
    sr, gs = (int(x) for x in cfg.split(":"))
    m.set_option("small_rows", sr)
    m.set_option("graph_seqs", gs)
    res = {"small_rows": sr, "graph_seqs": gs, "opts": args.opts}
    for n in (int(x) for x in args.lengths.split(",")):
        toks = [101] + rng.integers(1000, 30000, n - 2).tolist() + [102]
        for _ in range(20):
            e = m.eval(toks)
        ts = []
        for _ in range(args.runs):
            t0 = time.perf_counter()
            m.eval(toks)
            ts.append(time.perf_counter() - t0)
        res[f"n{n}_us_median"] = round(float(np.median(ts)) * 1e6, 1)
        res[f"n{n}_us_p10"] = round(float(np.percentile(ts, 10)) * 1e6, 1)
        key = n
        if key not in ref:
            ref[key] = (toks, e)
        else:
            res[f"n{n}_bitwise_vs_first"] = bool(np.array_equal(m.eval(ref[key][0]), ref[key][1]))
    print(json.dumps(res), flush=True)
m.close()
