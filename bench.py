#!/usr/bin/env python3
"""bench.py — BASELINE.json's headline metric on MI355X.

Metric: embeddings/sec at seq_len=128, batch=1024 (all-MiniLM-L6-v2 Q4_0 shape,
synthetic deterministic weights: no checkpoints offline), plus cosine
similarity vs the ggml-semantics CPU oracle.  One "step" = one pass of the
embedding path (bert_amd_eval_device: embed+LN, 6 x {QKV, attention, O+LN,
FFN-up+GELU, FFN-down+LN}, mean-pool+L2) over one batch of 1024 sentences x 128
tokens already resident in HBM.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
one process per GPU, each rank evaluates its own 1024 sentences (weak scaling;
sentences are independent, reference bert.cpp:1065, so there is no data-path
collective); RCCL is used only for the barrier and the max-over-ranks time.

Prints exactly one JSON line on rank 0 (everything else goes to stderr).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "embedding.cpp_amd"))

import bertlib  # noqa: E402

SEED = 20250117
METRIC = "embeddings/sec at seq_len=128 batch=1024; cosine-sim vs ggml CPU ref"
PEAK_FP16_TFLOPS = 2516.6  # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP32_MFMA_TFLOPS = 157.3
PEAK_INT8_TOPS = 2 * PEAK_FP16_TFLOPS  # i8 MFMA: 2x the bf16 rate per clock (MI355X_MICROARCH.md MFMA table)
PEAK_HBM_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def splitmix_tokens(first_index: int, n_sent: int, seq: int, n_vocab: int) -> np.ndarray:
    """Sentence s: [101, r_1..r_{seq-2}, 102], r uniform in [1000, V) from
    splitmix64(SEED + s) — identical to tests/golden/make_golden.py:sentence."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        st = (np.uint64(SEED) + np.arange(first_index, first_index + n_sent, dtype=np.uint64))
        out = np.empty((n_sent, seq), np.int64)
        out[:, 0] = 101
        out[:, -1] = 102
        for j in range(1, seq - 1):
            st = (st + np.uint64(0x9E3779B97F4A7C15)) & M
            z = st
            z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M
            z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M
            z = z ^ (z >> np.uint64(31))
            out[:, j] = (np.uint64(1000) + z % np.uint64(n_vocab - 1000)).astype(np.int64)
    return out.astype(np.int32)


def shard(rank: int, batch: int) -> int:
    """First global sentence index of this rank's batch (weak scaling: rank r
    owns sentences [r*batch, (r+1)*batch))."""
    return rank * batch


def max_over_ranks(x: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def library_sharding(rank: int, world: int, cpu_barrier, work):
    """bench's N > 1 library-sharding step (reference bert.cpp:1065: sentences are
    independent): rank 0 runs `work()` — bert_amd_load over every device of the
    node + bert_eval_batch on the global batch — while the other ranks wait in
    `cpu_barrier` (a gloo barrier: it blocks on the CPU, so the waiting ranks do
    not spin on their GPUs the way an RCCL barrier would, and it fails with a
    timeout error instead of hanging if rank 0 dies).  Returns work()'s result
    on rank 0, None elsewhere."""
    res = None
    try:
        if rank == 0:
            res = work()
    finally:
        cpu_barrier()
    return res


def lib_shard_work(model_cls, path, devices, gtoks, B, out_rank0, workload):
    """Rank 0's part of library_sharding: time bert_eval_batch over the global
    batch (host buffers, median of 5 after 2 warm-ups) on a context replicated
    over `devices`, and check its first B rows against rank 0's own shard."""
    gm = model_cls(path, devices=devices)
    try:
        run, gemb = gm.prepared_batch(list(gtoks))
        for _ in range(2):
            run()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            run()
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts))
        n = len(gtoks)
        return dict(value=round(n / med, 1), unit="embeddings/s", devices=gm.n_devices, workload=workload,
                    ms_median=round(med * 1e3, 3), runs=5, bitwise_vs_rank0=bool(np.array_equal(gemb[:B], out_rank0)),
                    note="bert_amd_load(devices=0..N-1) + bert_eval_batch on host buffers "
                         "(H2D ids and D2H embeddings included)")
    finally:
        gm.close()


def build_info() -> dict:
    """The library this run measures: sha256 of build/libbert.so and the git
    HEAD it was built from (build/BUILD_INFO, written by make)."""
    import hashlib
    info = {}
    try:
        with open(bertlib.LIB_PATH, "rb") as f:
            info["lib_sha256"] = hashlib.sha256(f.read()).hexdigest()
    except OSError:
        pass
    bi = os.path.join(os.path.dirname(bertlib.LIB_PATH), "BUILD_INFO")
    if os.path.exists(bi):
        with open(bi) as f:
            info["git_head"] = f.read().strip()
        built = [w[4:] for w in info["git_head"].split() if w.startswith("src=")]
        if built:
            info["src_matches_tree"] = built[0] == src_hash()
    return info


def src_hash() -> str:
    """sha256 (first 16 hex digits) of the library's sources in this tree, the
    same file list and order as the Makefile's SRC_HASH_FILES."""
    import glob
    import hashlib
    pats = ["embedding.cpp_amd/csrc/*.hip", "embedding.cpp_amd/csrc/*.cpp", "embedding.cpp_amd/csrc/*.h",
            "embedding.cpp_amd/csrc/*.inc", "include/*.h", "include/ggml/*.h"]
    files = sorted(set(os.path.relpath(f, REPO) for p in pats for f in glob.glob(os.path.join(REPO, p))))
    h = hashlib.sha256()
    for f in files + ["Makefile"]:
        with open(os.path.join(REPO, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def kernel_flops(name: str, B: int, N: int, hp: dict) -> float:
    return sum(f for f, _ in kernel_parts(name, B, N, hp, {}, "q4_0"))


def kernel_parts(name: str, B: int, N: int, hp: dict, arith: dict, ftype: str) -> list:
    """Algorithmic work of one launch split by the MFMA arithmetic it runs on:
    [(flops, peak TFLOP/s)].  `arith` is the library's resolved choice per
    projection (bert_amd_get_option: i8_qkv / i8_up / i8_o / i8_down): a Q4
    projection on the int8-MFMA GEMMs is priced at the int8 peak, one on the
    split-fp16 GEMMs at the fp16 peak; attention (split-fp16 K.Q and P.V) at
    the fp16 peak; F32 GEMMs at the fp32 MFMA peak."""
    E, I = hp["n_embd"], hp["n_intermediate"]
    M = B * N
    q4 = ftype in ("q4_0", "q4_1")
    gemm_peak = PEAK_FP32_MFMA_TFLOPS if ftype == "f32" else PEAK_FP16_TFLOPS

    def proj(key):
        return PEAK_INT8_TOPS if q4 and arith.get(key) else gemm_peak

    # i8_qkv: the producer / consumer kernel and its unfused twin, or the unfused
    # int8 QKV GEMM of option i8=qkv (older callers pass only qkva_ntw: 0 = int8)
    qkv_int8 = q4 and bool(arith["i8_qkv"] if "i8_qkv" in arith else arith.get("qkva_ntw") == 0)
    qkv = (2.0 * M * E * 3 * E, PEAK_INT8_TOPS if qkv_int8 else gemm_peak)
    att = (4.0 * B * N * N * E, PEAK_FP16_TFLOPS)
    return {
        "gemm_qkv": [qkv],
        "gemm_o_ln": [(2.0 * M * E * E, proj("i8_o"))],
        "gemm_up_gelu": [(2.0 * M * E * I, proj("i8_up"))],
        "gemm_down_ln": [(2.0 * M * I * E, proj("i8_down"))],
        "attention": [att],
        "qkv_attention": [qkv, att],
    }.get(name, [])


def dtype_label(ftype: str, arith: dict) -> str:
    """The MFMA arithmetic of the step: Q4 models run their int8-MFMA
    projections (exact Q4 x Q8 block dots) beside split-fp16 ones and fp16
    attention."""
    if ftype in ("q4_0", "q4_1"):
        i8 = any(arith.get(k) for k in ("i8_qkv", "i8_up", "i8_o", "i8_down")) or (
            "i8_qkv" not in arith and arith.get("qkva_ntw") == 0)
        return "int8+fp16" if i8 else "fp16"
    return "fp32+fp16" if ftype == "f32" else "fp16"


def dtype_note(ftype: str, arith: dict) -> str:
    if ftype in ("q4_0", "q4_1"):
        names = {"qkv": arith["i8_qkv"] if "i8_qkv" in arith else arith.get("qkva_ntw") == 0,
                 "o": arith.get("i8_o"), "up": arith.get("i8_up"),
                 "down": arith.get("i8_down")}
        i8 = [k for k, v in names.items() if v]
        f16 = [k for k, v in names.items() if not v]
        s = "Q4 x Q8 as ggml vec_dot_q4_x_q8_x: "
        if i8:
            s += f"{'/'.join(i8)} on int8 MFMA (exact block isum, per-block d_w*d_a fold in f32)"
            bf = [k for k in ("qkv", "o", "up", "down") if arith.get(f"q41bf_{k}")]
            if bf:
                s += f" ({'/'.join(bf)}: Q4_1 scale products as exact bf16 partial products on the bf16 MFMA)"
        if f16:
            s += ("; " if i8 else "") + (f"{'/'.join(f16)} with Q4 weights as exact fp16 hi/lo pairs x Q8 integers "
                                         "on fp16 MFMA (per-block d_a fold)")
    else:
        s = f"{ftype} GEMM on {'fp16' if ftype == 'f16' else 'f32'} MFMA, f32 accumulate"
    return s + "; attention split-fp16 MFMA (f32-level); LN/softmax sums f64"


def mixed_roofline(parts: list, avg_s: float) -> dict:
    """frac = (sum of F_i / P_i) / t: the launch's ideal time at each part's
    own peak over its measured time.  `peak` is the matching effective peak
    (F / ideal time), so achieved / peak == frac."""
    fl = sum(f for f, _ in parts)
    ideal = sum(f / (p * 1e12) for f, p in parts)
    dts = sorted({"int8" if p == PEAK_INT8_TOPS else "fp32" if p == PEAK_FP32_MFMA_TFLOPS else "fp16"
                  for _, p in parts}, key=["int8", "fp16", "fp32"].index)
    return dict(achieved=round(fl / avg_s / 1e12, 1), peak=round(fl / ideal / 1e12, 1), frac=round(ideal / avg_s, 4),
                flops_per_launch=fl, peak_dtype="+".join(dts),
                parts=[dict(flops=f, peak=p) for f, p in parts])


def kernel_bytes(name: str, B: int, N: int, hp: dict, ftype: str) -> float:
    """Algorithmic HBM bytes per launch (each operand read once, each output written once)."""
    E, I, L = hp["n_embd"], hp["n_intermediate"], hp["n_layer"]
    M = B * N
    act = {"q4_0": 1 + 2 / 32, "q4_1": 1 + 4 / 32, "f16": 2, "f32": 4}[ftype]  # bytes/elem of GEMM inputs
    wb = {"q4_0": 18 / 32, "q4_1": 20 / 32, "f16": 2, "f32": 4}[ftype]
    return {
        "gemm_qkv": M * E * act + 3 * E * E * wb + M * 3 * E * 4,
        "gemm_o_ln": M * E * act + E * E * wb + 2 * M * E * 4 + M * E * act,
        "gemm_up_gelu": M * E * act + E * I * wb + M * I * act,
        "gemm_down_ln": M * I * act + E * I * wb + 2 * M * E * 4 + M * E * act,
        "attention": M * 3 * E * 4 + M * E * act,
        "qkv_attention": M * E * act + 3 * E * E * wb + M * E * act,
        "embed_ln": M * 4 + M * E * (4 + act) + M * E * 4,  # f32 word rows (pos/type tables stay cached)
        "pool_l2": M * E * 4 + B * E * 4,
    }.get(name, 0.0) if L else 0.0


def pmc_traffic(csv_path: str, kernel_substr):
    """Average corrected HBM bytes per dispatch of one kernel from a rocprofv3
    --pmc FETCH_SIZE / WRITE_SIZE counter CSV (gfx950: FETCH_SIZE counts half the
    bytes of a wide coalesced read — MI355X_MICROARCH.md §HBM — so it is doubled;
    both counters are in KB).  kernel_substr: a symbol fragment, or a list of
    them of which the first that occurs in the CSV is used."""
    import csv
    frags = [kernel_substr] if isinstance(kernel_substr, str) else list(kernel_substr)
    rows = []
    for p in csv_path.split(","):
        if os.path.exists(p):
            with open(p) as f:
                rows += [(r.get("Kernel_Name", ""), r.get("Counter_Name", ""), r.get("Counter_Value", 0))
                         for r in csv.DictReader(f)]
    for frag in frags:
        vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
        for name, cn, v in rows:
            if frag in name and cn in vals:
                vals[cn].append(float(v))
        if vals["FETCH_SIZE"] and vals["WRITE_SIZE"]:
            return (2.0 * np.mean(vals["FETCH_SIZE"]) + np.mean(vals["WRITE_SIZE"])) * 1024.0
    return None


# name fragments of the dominant kernels' mangled symbols (for PMC CSV lookup)
KERNEL_SYMBOL = {
    "gemm_qkv": "gemm_kernel<2, 0,", "gemm_o_ln": "gemm_kernel<2, 2,", "gemm_up_gelu": "i8_up_gelu_kernel",
    "gemm_down_ln": "i8_ln384_kernel", "attention": "attention_short_kernel", "qkv_attention": ["qkv_attention_pc_kernel", "qkv_attention_kernel"], "embed_ln": "embed_ln_kernel",
    "pool_l2": "pool_l2_kernel",
}


def consumer_line(model, hp, n_texts, rank, dev, stream, torch):
    import ctypes
    L = model.lib
    words = []
    for i in range(1000, hp["n_vocab"]):
        w = L.bert_vocab_id_to_token(model.ctx, i).decode("utf-8", "replace")
        if w.isalpha() and w.islower() and not w.startswith("##"):
            words.append(w)
    rng = np.random.default_rng(SEED + 7 + rank)
    lens = rng.integers(8, 129, n_texts)  # framed token counts: [CLS] + words + [SEP]
    texts = [" ".join(rng.choice(words, n - 2)) for n in lens]
    n = len(texts)
    c_texts = (ctypes.c_char_p * n)(*[t.encode("utf-8") for t in texts])
    # tokeniser alone (bert_tokenize per text through ctypes, one thread)
    buf = (ctypes.c_int32 * hp["n_max_tokens"])()
    nt = ctypes.c_int32(0)
    t0 = time.perf_counter()
    toks = []
    for i in range(n):
        L.bert_tokenize(model.ctx, c_texts[i], buf, ctypes.byref(nt), hp["n_max_tokens"])
        toks.append(np.frombuffer(buf, np.int32, nt.value).copy())
    t_tok = time.perf_counter() - t0
    ntoks = np.array([len(t) for t in toks])
    framed_ok = bool(np.array_equal(ntoks, lens))
    emb = np.zeros((n, hp["n_embd"]), np.float32)
    ptrs = (bertlib.F_P * n)(*[emb[i].ctypes.data_as(bertlib.F_P) for i in range(n)])
    threads = int(os.environ.get("OMP_NUM_THREADS", 0) or 8)
    res = dict(texts=n, mean_tokens=round(float(ntoks.mean()), 2), lengths="uniform 8..128 tokens (seeded)",
               framing_ok=framed_ok, n_threads=threads,
               tokenizer=dict(texts_per_s=round(n / t_tok, 1), tokens_per_s=round(float(ntoks.sum()) / t_tok, 1),
                              note="bert_tokenize per text via ctypes, one thread"))
    ref = None
    for bs in (16, 256, n):
        L.bert_encode_batch(model.ctx, threads, bs, n, c_texts, ptrs)  # warm-up (workspace growth)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            L.bert_encode_batch(model.ctx, threads, bs, n, c_texts, ptrs)
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts))
        if ref is None:
            ref = emb.copy()
        res[f"encode_batch_{'all' if bs == n else bs}"] = dict(value=round(n / med, 1), unit="embeddings/s",
                                                              ms_median=round(med * 1e3, 2),
                                                              bitwise_vs_batch16=bool(np.array_equal(emb, ref)))
    # the same sentences device-resident, one batch (eval_device)
    offs = np.zeros(n + 1, np.int32)
    offs[1:] = np.cumsum(ntoks)
    d_tok = torch.from_numpy(np.concatenate(toks)).to(dev)
    d_off = torch.from_numpy(offs).to(dev)
    d_out = torch.empty(n, hp["n_embd"], dtype=torch.float32, device=dev)
    for _ in range(2):
        model.eval_device(d_tok.data_ptr(), d_off.data_ptr(), offs, n, d_out.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(5):
        model.eval_device(d_tok.data_ptr(), d_off.data_ptr(), offs, n, d_out.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    dres = n * 5 / (time.perf_counter() - t0)
    res["device_resident_same_sentences"] = dict(value=round(dres, 1), unit="embeddings/s")
    res["batch16_frac_of_device"] = round(res["encode_batch_16"]["value"] / dres, 4)
    res["bitwise_vs_device"] = bool(np.array_equal(d_out.cpu().numpy(), ref))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--shape", default="minilm", choices=list(bertlib.SHAPES))
    ap.add_argument("--ftype", default="q4_0", choices=list(bertlib.FTYPES))
    ap.add_argument("--w-std", type=float, default=0.05)
    ap.add_argument("--model-dir", default=os.environ.get("BERT_AMD_MODEL_DIR", "/tmp/bert_amd_models"))
    ap.add_argument("--cpu-sample", type=int, default=256, help="sentences for the CPU oracle baseline (0: skip)")
    ap.add_argument("--cpu-sample-scalar", type=int, default=64,
                    help="of those, sentences for the scalar form of the oracle (timed beside the SIMD form)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--profile-steps", type=int, default=5)
    ap.add_argument("--pmc-csv", default=os.environ.get("BENCH_PMC_CSV", ""))
    ap.add_argument("--host-runs", type=int, default=10, help="timed bert_eval_batch runs (host buffers), 0: skip")
    ap.add_argument("--load-replicas", type=int, default=8, help="time a load with this many replicas on one device")
    ap.add_argument("--latency-runs", type=int, default=100, help="single-sentence bert_eval runs per length, 0: skip")
    ap.add_argument("--ragged-steps", type=int, default=10, help="variable-length batch steps, 0: skip")
    ap.add_argument("--consumer-texts", type=int, default=4096,
                    help="texts for the bert_encode_batch (consumer path) line, 0: skip")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="development: every rank on device 0, gloo instead of RCCL (N > 1 code paths on a 1-GPU box)")
    ap.add_argument("--lib-shard", type=int, default=1,
                    help="N>1: rank 0 also times the library's own sharding (bert_amd_load over all N devices)")
    args = ap.parse_args()

    import torch

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    gpu = 0 if args.rehearse_one_gpu else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    cpu_group = None
    if world > 1:
        import datetime
        import torch.distributed as dist
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
            # CPU-side waits (library_sharding) go through gloo, not RCCL
            cpu_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(minutes=20))

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    hp = bertlib.SHAPES[args.shape]
    os.makedirs(args.model_dir, exist_ok=True)
    path = os.path.join(args.model_dir, f"{args.shape}_{args.ftype}_s{SEED}_w{args.w_std:g}.gguf")
    if local_rank == 0 and not os.path.exists(path):
        tmp = f"{path}.tmp{os.getpid()}"
        bertlib.synth_model(tmp, args.shape, args.ftype, seed=SEED, w_std=args.w_std)
        os.replace(tmp, path)
    barrier()
    while not os.path.exists(path):  # other nodes' local rank 0 (single node: already there)
        time.sleep(0.1)

    # the library reports the load on stdout (as the reference's bert_load_from_file
    # does); keep stdout for the one JSON line
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        l0 = time.perf_counter()
        model = bertlib.BertModel(path, devices=[gpu])
        load_s = time.perf_counter() - l0
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
    B, N = args.batch, args.seq
    first = shard(rank, B)
    toks = splitmix_tokens(first, B, N, hp["n_vocab"])
    offs = (np.arange(B + 1, dtype=np.int64) * N).astype(np.int32)
    d_tok = torch.from_numpy(toks.ravel()).to(dev)
    d_off = torch.from_numpy(offs).to(dev)
    d_out = torch.empty(B, hp["n_embd"], dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        model.eval_device(d_tok.data_ptr(), d_off.data_ptr(), offs, B, d_out.data_ptr(), stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    t1 = time.perf_counter()
    dt = max_over_ranks(t1 - t0, dev)
    value = world * B * args.steps / dt
    ms_per_step = dt / args.steps * 1e3
    out = d_out.cpu().numpy()

    # per-kernel durations: HIP events recorded by the library around every launch,
    # on the launch stream, in a separate pass of profile-steps steps right after
    # the timed region (the timed region itself carries no events)
    log(f"timed: {value:.1f} emb/s; per-kernel event pass")
    # one row group in this pass (the timed steps run two on two streams,
    # DESIGN.md §3): every profiled launch covers the whole batch alone, so its
    # duration is the kernel's own and the roofline below is per launch
    model.set_option("split", 0)
    model.profile(True)
    for _ in range(args.profile_steps):
        step()
    torch.cuda.synchronize(dev)
    prof = model.profile_read()
    model.profile(False)
    model.set_option("split", int(os.environ.get("BERT_AMD_SPLIT", "1")[:1] != "0"))
    arith = {k: model.get_option(k) for k in ("qkva_ntw", "i8_qkv", "i8_up", "i8_o", "i8_down", "q41bf_qkv",
                                              "q41bf_o", "q41bf_up", "q41bf_down")}
    kern = {}
    for name, (ms, cnt) in prof.items():
        parts = kernel_parts(name, B, N, hp, arith, args.ftype)
        by = kernel_bytes(name, B, N, hp, args.ftype)
        avg_s = ms / max(cnt, 1) / 1e3
        kern[name] = dict(avg_us=round(avg_s * 1e6, 2), launches_per_step=cnt // max(args.profile_steps, 1),
                          share=round(ms / max(sum(v[0] for v in prof.values()), 1e-9), 4),
                          gbs=round(by / avg_s / 1e9, 1) if by else None)
        if parts:
            mr = mixed_roofline(parts, avg_s)
            kern[name].update(tflops=mr["achieved"], mfma_frac=mr["frac"], peak_dtype=mr["peak_dtype"])
    dominant = max(prof, key=lambda k: prof[k][0]) if prof else None

    roofline = None
    hbm_step = None
    if dominant:
        avg_s = prof[dominant][0] / prof[dominant][1] / 1e3
        parts = kernel_parts(dominant, B, N, hp, arith, args.ftype)
        if parts:
            # priced on the arithmetic each part runs (mixed_roofline); e.g. the
            # producer / consumer kernel: QKV at the int8 peak, attention at fp16
            roofline = dict(kernel=dominant, bound="mfma", unit="TFLOP/s", **mixed_roofline(parts, avg_s),
                            formula="frac = sum(F_i / peak_i) / t_launch; peak = F / sum(F_i / peak_i)")
        else:
            by = kernel_bytes(dominant, B, N, hp, args.ftype)
            ach = by / avg_s / 1e9
            roofline = dict(kernel=dominant, bound="hbm", achieved=round(ach, 1), peak=PEAK_HBM_GBS, unit="GB/s",
                            frac=round(ach / PEAK_HBM_GBS, 4), bytes_per_launch=by)
        traffic, tsrc = None, None
        # profiles/pmc_traffic.json: corrected FETCH_SIZE x2 + WRITE_SIZE per launch
        # measured by tools/profile_round.sh (separate rocprofv3 --pmc passes) on the
        # library it records (lib_sha256, git_head); it is used only for the same
        # workload, and marked stale when this run's library is a different build
        pt, stale = None, None
        pf = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(pf):
            with open(pf) as f:
                pt = json.load(f)
            if pt.get("workload") != f"{args.shape} {args.ftype} batch={B} seq_len={N}":
                pt = None
            else:
                stale = pt.get("lib_sha256") != build_info().get("lib_sha256")
        if args.pmc_csv:
            traffic = pmc_traffic(args.pmc_csv, KERNEL_SYMBOL.get(dominant, dominant))
            tsrc = args.pmc_csv
        elif pt and dominant in pt.get("bytes_per_launch", {}):
            traffic = pt["bytes_per_launch"][dominant]
            tsrc = (f"profiles/pmc_traffic.json ({pt.get('source', '')}; git {pt.get('git_head', '?')})"
                    + (" STALE: measured on a different build of libbert.so" if stale else ""))
        roofline["traffic"] = traffic
        roofline["traffic_source"] = tsrc
        roofline["traffic_stale"] = bool(stale) if (traffic is not None and not args.pmc_csv) else False
        # whole-step achieved HBM (north_star): PMC bytes of one step's launches
        # (profiles/pmc_traffic.json bytes_per_step) over this run's ms_per_step
        if pt and pt.get("bytes_per_step"):
            bps = float(pt["bytes_per_step"])
            gbs = bps / (ms_per_step * 1e-3) / 1e9
            hbm_step = dict(bytes_per_step=round(bps), achieved_GBs=round(gbs, 1), peak_GBs=PEAK_HBM_GBS,
                            frac=round(gbs / PEAK_HBM_GBS, 4), stale=bool(stale),
                            source=f"profiles/pmc_traffic.json ({pt.get('source', '')}; git {pt.get('git_head', '?')}) "
                                   f"over this run's ms_per_step")
        roofline["algorithmic_bytes_per_launch"] = kernel_bytes(dominant, B, N, hp, args.ftype)

    # whole-path MFMA fraction: F(N) = L(8NE^2 + 4NEI + 4N^2E) per sentence
    E, I, L = hp["n_embd"], hp["n_intermediate"], hp["n_layer"]
    f_sent = L * (8 * N * E * E + 4 * N * E * I + 4 * N * N * E)
    path_frac = f_sent * value / (world * PEAK_FP16_TFLOPS * 1e12)
    # the same step priced on the arithmetic each projection runs (int8 / fp16):
    # the ideal step time at those peaks over the measured ms_per_step
    ideal_step = L * sum(f / (p * 1e12) for k in ("gemm_qkv", "attention", "gemm_o_ln", "gemm_up_gelu", "gemm_down_ln")
                         for f, p in kernel_parts(k, B, N, hp, arith, args.ftype))
    path_frac_mixed = ideal_step / (ms_per_step * 1e-3)

    # the reference ABI path (bert_eval_batch: host token lists in, host rows out,
    # pinned H2D of the ids and D2H of the embeddings included), SURVEY §8(d):
    # 3 warm-ups, median of 10 — reported beside `value`, never as it
    host_api = None
    if args.host_runs > 0:
        log("host-API timing (bert_eval_batch)")
        tl = toks  # [B, N] int32: bertlib builds the row pointer arrays by address arithmetic
        for _ in range(3):
            model.eval_batch(tl)
        ts = []
        for _ in range(args.host_runs):
            h0 = time.perf_counter()
            model.eval_batch(tl)
            ts.append(time.perf_counter() - h0)
        med = float(np.median(ts))
        host_api = dict(value=round(B / med, 1), unit="embeddings/s", ms_median=round(med * 1e3, 3),
                        ms_min=round(min(ts) * 1e3, 3), runs=args.host_runs,
                        note="bert_eval_batch on host buffers, per GPU: ids H2D + embeddings D2H included")

    # single-sentence latency: the reference server's path (examples/server.cpp:114
    # -> bert_encode -> bert_eval, one text per request; bert.cpp:1020-1028):
    # bert_eval on host buffers, median of `latency_runs` after 10 warm-ups, at
    # N = 16 / 32 / 128 tokens, with the kernel launches one call makes
    latency = None
    if args.latency_runs > 0:
        log("single-sentence latency (bert_eval)")
        latency = {}
        for n_tok in (16, 32, 128):
            sent = toks[0][:n_tok].copy()
            sent[-1] = 102
            for _ in range(10):
                model.eval(sent)
            ts = []
            for _ in range(args.latency_runs):
                h0 = time.perf_counter()
                model.eval(sent)
                ts.append(time.perf_counter() - h0)
            model.profile(True)
            model.eval(sent)
            lp = model.profile_read()
            model.profile(False)
            latency[f"n{n_tok}"] = dict(us_median=round(float(np.median(ts)) * 1e6, 1),
                                        us_p10=round(float(np.percentile(ts, 10)) * 1e6, 1),
                                        us_p90=round(float(np.percentile(ts, 90)) * 1e6, 1),
                                        launches_per_call=int(sum(c for _, c in lp.values())),
                                        device_us=round(sum(ms for ms, _ in lp.values()) * 1e3, 1),
                                        kernel_us={k: round(ms * 1e3 / max(c, 1), 1) for k, (ms, c) in lp.items()})
        latency["note"] = ("bert_eval, one sentence, host buffers (ids H2D + embedding D2H + stream sync), "
                           f"median of {args.latency_runs}; device_us = sum of the call's kernel durations "
                           "(HIP events, separate profiled call)")

    # variable-length batches (server / MTEB-like sentences), same sentence
    # count, device-resident like the headline: lengths uniform in [8, 128],
    # and short ones in [8, 40] (several share a fused QKV+attention tile)
    def ragged_line(lo, hi, salt):
        rng = np.random.default_rng(SEED + rank + salt)
        lens = rng.integers(lo, hi + 1, B)
        rtoks = [toks[i][:n].copy() for i, n in enumerate(lens)]
        for t in rtoks:
            t[-1] = 102
        roffs = np.zeros(B + 1, np.int32)
        roffs[1:] = np.cumsum(lens)
        rd_tok = torch.from_numpy(np.concatenate(rtoks)).to(dev)
        rd_off = torch.from_numpy(roffs).to(dev)
        for _ in range(3):
            model.eval_device(rd_tok.data_ptr(), rd_off.data_ptr(), roffs, B, d_out.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        r0 = time.perf_counter()
        for _ in range(args.ragged_steps):
            model.eval_device(rd_tok.data_ptr(), rd_off.data_ptr(), roffs, B, d_out.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        rdt = (time.perf_counter() - r0) / args.ragged_steps
        return dict(value=round(B / rdt, 1), unit="embeddings/s", ms_per_step=round(rdt * 1e3, 4),
                    tokens_per_s=round(float(lens.sum()) / rdt, 1), lengths=f"uniform {lo}..{hi} (seeded)",
                    mean_len=round(float(lens.mean()), 2), steps=args.ragged_steps)

    ragged = ragged_short = None
    if args.ragged_steps > 0:
        log("variable-length batch timing")
        ragged = ragged_line(8, 128, 0)
        ragged_short = ragged_line(8, 40, 1)
        # the same 8..128 batch through bert_eval_batch on host buffers: the
        # library may reorder it (fused-kernel tile packing), outputs per sentence
        rng = np.random.default_rng(SEED + rank)
        lens = rng.integers(8, 129, B)
        rtoks = [toks[i][:n].copy() for i, n in enumerate(lens)]
        for t in rtoks:
            t[-1] = 102
        run, remb = model.prepared_batch(rtoks)
        for _ in range(2):
            run()
        ts = []
        for _ in range(max(3, args.host_runs)):
            t0 = time.perf_counter()
            run()
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts))
        ragged["host_api"] = dict(value=round(B / med, 1), unit="embeddings/s", ms_median=round(med * 1e3, 3),
                                  unit_norm=bool(np.allclose(np.linalg.norm(remb, axis=1), 1.0, atol=1e-5)),
                                  note="bert_eval_batch, host buffers, same lengths")

    # the reference consumers' path (examples/sample_dylib.py:42 batch 16,
    # benchmarks/run_mteb.py:19,89 batch os.cpu_count()): bert_encode_batch on
    # synthetic texts of whole vocabulary words (one token each, 8..128 tokens
    # framed), host tokenisation and host buffers included, against the same
    # sentences device-resident in one batch
    consumer = None
    if args.consumer_texts > 0 and rank == 0:
        log("consumer path timing (bert_encode_batch)")
        consumer = consumer_line(model, hp, args.consumer_texts, rank, dev, stream, torch)

    cpu = None
    parity = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # CPU checker + baseline only (never the measured path)
        # the CPUs this job may use: OMP_NUM_THREADS where the launcher sets the share (16 on the
        # GPU box, whose os.cpu_count() is the whole host), else the affinity mask
        avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
        threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", 0) or avail)
        log(f"cpu baseline: {min(args.cpu_sample, B)} sentences on {threads} threads")
        S = min(args.cpu_sample, B)
        orc = oracle.Oracle(path)
        sample = [toks[i].tolist() for i in range(S)]
        orc.eval_batch(sample[:1], threads)  # warm-up (page-in of the model file)
        cpu_model = ""
        try:
            with open("/proc/cpuinfo") as f:
                cpu_model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
        except OSError:
            pass
        # the scalar AVX2-order checker on a smaller sample (it is 5-7x slower), then the same
        # checker in AVX2 intrinsics (ggml's AVX2 instructions, bitwise equal:
        # tests/test_oracle.py::test_simd_oracle_bitwise_scalar) on the whole sample
        Ss = max(1, min(S, args.cpu_sample_scalar))
        c0 = time.perf_counter()
        ref_s = orc.eval_batch(sample[:Ss], threads)
        c1 = time.perf_counter()
        scalar = dict(value=round(Ss / (c1 - c0), 3), unit="embeddings/s", cores=threads, kind="port",
                      sample=f"first {Ss} of the {B} sentences, scalar C form of the checker",
                      seconds=round(c1 - c0, 2))
        simd = oracle.simd_available()
        if simd:
            oracle.set_simd(True)
            try:
                c0 = time.perf_counter()
                ref = orc.eval_batch(sample, threads)
                c1 = time.perf_counter()
            finally:
                oracle.set_simd(False)
            cpu = dict(value=round(S / (c1 - c0), 3), unit="embeddings/s", cores=threads, kind="port",
                       form="simd restatement",
                       sample=f"first {S} of the {B} sentences (seq_len {N}), oracle/bert_oracle.c in AVX2 "
                              f"intrinsics (ggml's AVX2 vec_dot instructions: maddubs/madd/cvt/fma per Q4 block, "
                              f"8-lane f32 fma dots, F16C; bitwise the scalar checker), one sentence at a time, "
                              f"{threads} OpenMP threads = the CPU share of this job, -O3 -march=x86-64-v3",
                       seconds=round(c1 - c0, 2), cpu_model=cpu_model, host_cpus=os.cpu_count(), scalar=scalar,
                       simd_bitwise_scalar=bool(np.array_equal(ref[:Ss], ref_s)))
        else:
            ref = ref_s
            S = Ss
            cpu = dict(scalar, cpu_model=cpu_model, host_cpus=os.cpu_count(), form="scalar restatement")
        a = out[:S].astype(np.float64)
        c = (a * ref).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(ref, axis=1)
        parity = dict(cos_min=float(c.min()), cos_mean=float(c.mean()), n=S,
                      max_abs=float(np.abs(out[:S] - ref).max()))

    # model load: one replica (above) vs 8 replicas on this one device
    # (rehearsal of an 8-GPU bert_load_from_file: the weights are repacked
    # once and uploaded by one thread per replica, runtime.cpp Stager)
    load = None
    if rank == 0 and args.load_replicas > 1:
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            l0 = time.perf_counter()
            m1 = bertlib.BertModel(path, devices=[gpu])
            l1 = time.perf_counter() - l0
            m1.close()
            l0 = time.perf_counter()
            mr = bertlib.BertModel(path, devices=[gpu] * args.load_replicas)
            lr = time.perf_counter() - l0
            mr.close()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        load = dict(first_load_s=round(load_s, 3), one_replica_s=round(l1, 3), replicas=args.load_replicas,
                    replicas_s=round(lr, 3),
                    note=f"bert_amd_load wall time; first_load_s: the process's first load (runtime init, "
                         f"cold file); then one replica and {args.load_replicas} replicas all on device {gpu}, "
                         "warm (one repack, one upload thread per replica)")

    # N > 1: the library's own sharding, the path drop-in consumers get
    # (bert_amd_load over every device of the node + bert_eval_batch on host
    # buffers: one thread per device, slices balanced by token count), on the
    # global batch world x B; rank 0 only, the other ranks idle on the CPU
    lib_shard = None
    if world > 1 and args.lib_shard:
        import torch.distributed as dist
        if rank == 0:
            log(f"library sharding over {world} devices")
        devices = [0] * world if args.rehearse_one_gpu else list(range(world))
        lib_shard = library_sharding(
            rank, world, lambda: dist.barrier(group=cpu_group),
            lambda: lib_shard_work(bertlib.BertModel, path, devices, splitmix_tokens(0, world * B, N, hp["n_vocab"]),
                                   B, out, f"{args.shape} {args.ftype} global batch={world * B} seq_len={N}"))

    if rank == 0:
        res = {
            "metric": METRIC, "value": round(value, 1), "unit": "embeddings/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": dtype_label(args.ftype, arith),
            "dtype_note": dtype_note(args.ftype, arith),
            "data": "synthetic (deterministic splitmix64 token ids and weights; no checkpoints offline)",
            "config": {"workload": f"{args.shape} {args.ftype} batch={B} seq_len={N} per GPU",
                       "model": f"all-MiniLM-L6-v2 shape ({args.shape}), synthetic weights" if args.shape == "minilm"
                       else f"{args.shape} shape, synthetic weights",
                       "global_batch": B * world, "seq_len": N, "parallelism": f"dp{world}"},
            "roofline": roofline,
            "build": build_info(),
            "pipeline_mfma_frac": round(path_frac, 4),
            "pipeline_mfma_frac_mixed": round(path_frac_mixed, 4),
            "step_hbm": hbm_step,
            "kernels": kern,
            "kernels_note": "per-kernel HIP-event pass with one row group (bert_amd_set_option split 0); the timed steps "
                            "run two row groups on two streams (runtime.cpp run_pipeline)",
            "cosine_vs_oracle": parity,
            "host_api": host_api,
            "latency": latency,
            "ragged": ragged,
            "ragged_short": ragged_short,
            "consumer": consumer,
            "library_sharding": lib_shard,
            "load": load,
            "cpu_baseline": cpu,
        }
        print(json.dumps(res), flush=True)
    model.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
