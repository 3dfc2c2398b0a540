#!/usr/bin/env python3
"""Phase stamps of the producer / consumer kernel INSIDE the pipeline
(development): a -DPHASE_STAMPS variant of libbert.so (tools/variant_lib.sh
stamps "-DPHASE_STAMPS=1") runs the C3 batch (1024 x 128, MiniLM Q4_0,
device-resident, one row group) and the stamps of its last qkv_attention
launch are reported like tools/stamps.h (median cycles per phase over
workgroups and periods; wave 0 = producer, wave last = consumer).
   BERT_AMD_LIB=build/var/stamps/libbert.so python3 tools/pipe_stamps.py [names...]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embedding.cpp_amd"))
sys.path.insert(0, REPO)
import bertlib  # noqa: E402
from bench import splitmix_tokens  # noqa: E402

STAMP_TILES, B, N = 32, 1024, 128


def main():
    import torch
    names = sys.argv[1:] or ["main|pass1", "V|pass2", "QK|store", "->period"]
    path = os.path.join(os.environ.get("BERT_AMD_MODEL_DIR", "/tmp/bert_amd_models"), "minilm_q4_0_s20250117_w0.05.gguf")
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        bertlib.synth_model(path, "minilm", "q4_0")
    dev = torch.device("cuda", 0)
    m = bertlib.BertModel(path, devices=[0])
    m.set_option("split", 0)
    toks = splitmix_tokens(0, B, N, 30522)
    offs = (np.arange(B + 1) * N).astype(np.int32)
    d_tok = torch.from_numpy(toks.ravel()).to(dev)
    d_off = torch.from_numpy(offs).to(dev)
    d_out = torch.empty(B, 384, dtype=torch.float32, device=dev)
    buf = torch.zeros(B * STAMP_TILES * 2 * 16, dtype=torch.int64, device=dev)
    f = m.lib.bert_amd_dev_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(3):
        m.eval_device(d_tok.data_ptr(), d_off.data_ptr(), offs, B, d_out.data_ptr(), 0)
    torch.cuda.synchronize()
    assert f(ctypes.c_void_p(buf.data_ptr()), B) == 0
    m.eval_device(d_tok.data_ptr(), d_off.data_ptr(), offs, B, d_out.data_ptr(), 0)
    torch.cuda.synchronize()
    assert f(ctypes.c_void_p(0), 0) == 0
    # blocks >= 512 only: the persistent GEMMs (<= 256 workgroups) stamp the same buffer
    h = buf.cpu().numpy().astype(np.uint64).reshape(B, STAMP_TILES, 2, 16)[512:]
    # STAMP_SLOTS="0,3,4,1,2": the slots in program order (default 0 .. len(names) - 1)
    order = [int(x) for x in os.environ.get("STAMP_SLOTS", "").split(",") if x] or list(range(len(names)))
    h = h[:, :, :, order + [k for k in range(16) if k not in order]]
    ns = len(names)
    for w in (0, 1):
        out, tot = [], 0.0
        for k in range(1, ns + 1):
            a = h[:, :, w, k - 1].astype(np.float64)
            if k < ns:
                b = h[:, :, w, k].astype(np.float64)
            else:
                b = np.concatenate([h[:, 1:, w, 0], np.zeros((h.shape[0], 1), np.uint64)], axis=1).astype(np.float64)
            ok = (a > 0) & (b > a)
            md = float(np.median((b - a)[ok])) if ok.any() else 0.0
            tot += md
            out.append(f"{names[k - 1]} {md:.0f}")
        print(f"  wave {'last' if w else '0   '}: " + "  ".join(out) + f"  | period {tot:.0f} cyc", flush=True)
    m.close()


if __name__ == "__main__":
    main()
