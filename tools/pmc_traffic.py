"""Per-launch HBM traffic of the bench's kernels from separate rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE passes (tools/profile_round.sh), corrected as
MI355X_MICROARCH.md prescribes for gfx950 (FETCH_SIZE counts half of the
bytes of wide coalesced reads: doubled; both counters in KB), written as
profiles/pmc_traffic.json for bench.py's roofline.traffic.
python tools/pmc_traffic.py <fetch dir> <write dir> <workload> <out.json> [source note]"""
import hashlib
import json
import os
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from hbm_summary import load  # noqa: E402

# bench.py kernel names -> fragments of the mangled kernel symbols
NAMES = {
    "qkv_attention": ["qkv_attention_pc_kernel", "qkv_attention_kernel"],
    "gemm_up_gelu": ["i8_up_gelu_kernel", "q4r_up_gelu_kernel", "gemm_kernelILi2ELi1", "gemm_kernel<2, 1,"],
    # default C3 build: o-proj on the split-fp16 LN GEMM, down on the int8 one
    "gemm_o_ln": ["gemm_kernelILi2ELi2", "gemm_kernel<2, 2,", "i8_ln384_kernel"],
    "gemm_down_ln": ["i8_ln384_kernel", "gemm_kernelILi2ELi2", "gemm_kernel<2, 2,"],
    "embed_ln": ["embed_ln_kernel"],
    "pool_l2": ["pool_l2_kernel"],
}


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    out = {"workload": sys.argv[3], "source": sys.argv[5] if len(sys.argv) > 5 else "", "bytes_per_launch": {},
           "fetch_bytes": {}, "write_bytes": {},
           "note": "FETCH_SIZE x2 + WRITE_SIZE, KB -> bytes, per dispatch; each name takes the kernels of "
                   "its first symbol fragment that occurs (o-proj: split-fp16 LN GEMM, down: int8 LN GEMM)"}
    # the build these counters describe (bench.py marks the traffic stale for any other build)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(repo, "build", "libbert.so")
    if os.path.exists(lib):
        with open(lib, "rb") as f:
            out["lib_sha256"] = hashlib.sha256(f.read()).hexdigest()
    bi = os.path.join(repo, "build", "BUILD_INFO")
    if os.path.exists(bi):
        with open(bi) as f:
            out["git_head"] = f.read().strip()
    out["kernel_symbols"] = sorted(set(fetch) | set(write))
    for name, frags in NAMES.items():
        fv, wv = [], []
        keys = set(fetch) | set(write)
        for f in frags:
            hit = [k for k in keys if f in k]
            if hit:
                for k in hit:
                    fv += list(fetch.get(k, {}).values())
                    wv += list(write.get(k, {}).values())
                break
        if fv and wv:
            fb = 2.0 * sum(fv) / len(fv) * 1024.0
            wb = sum(wv) / len(wv) * 1024.0
            out["fetch_bytes"][name] = round(fb)
            out["write_bytes"][name] = round(wb)
            out["bytes_per_launch"][name] = round(fb + wb)
    # whole step: every layer kernel launches n_layer (6) times per step, embed and pool once
    per_step = {"embed_ln": 1, "pool_l2": 1}
    bl = out["bytes_per_launch"]
    step = list(NAMES)
    if all(k in bl for k in step):
        out["bytes_per_step"] = round(sum(bl[k] * per_step.get(k, 6) for k in step))
    with open(sys.argv[4], "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["bytes_per_launch"]))


if __name__ == "__main__":
    main()
