"""SQ issue / wait counters of the four big kernels (development; DESIGN.md §3
"Issue floors").  Reads two rocprofv3 --pmc pass directories over bench.py
(one row group) and the same round's kernel-trace stats for the wall time:

  python3 tools/sq_counters.py <cycles pass dir> <instructions pass dir> <kernel_stats.csv | bench.json> <out.json> <source>

Round 6: o-proj and FFN-down both run i8_ln384_kernel (int8 O by default), so
its dispatches are dealt out in dispatch order (o, down in every layer; one row
group) and the wall times come from the bench line's per-name event times when
a bench JSON is given (rocprof's stats merge the two).

SQ_WAVE_CYCLES and the disjoint SQ_WAIT_ANY / SQ_WAIT_INST_ANY /
SQ_ACTIVE_INST_ANY buckets give the share of wave cycles parked, stalled at
issue and issuing; GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / wall is the
clock; a wave64 VALU instruction holds its SIMD 2 cycles, so
valu_issue_frac = 2 x VALU instructions / (1024 SIMDs x wall cycles);
SQ_VALU_MFMA_BUSY_CYCLES (summed over SIMDs) / (1024 x wall cycles) is the
matrix pipe's busy share."""
import collections
import csv
import glob
import json
import os
import sys

# (symbol fragment, label, bench.py kernel name)
KERNELS = [("qkv_attention_pc_kernel", "qkv_attention (qkv_attention_pc_kernel)", "qkv_attention"),
           ("gemm_kernel", "gemm_o_ln (gemm_kernel split-fp16)", "gemm_o_ln"),
           ("i8_up_gelu_kernel", "gemm_up_gelu (i8_up_gelu_kernel)", "gemm_up_gelu"),
           ("i8_ln384_kernel", "gemm_down_ln (i8_ln384_kernel)", "gemm_down_ln")]
O_I8 = "gemm_o_ln (i8_ln384_kernel, int8)"
SHARED = "i8_ln384_kernel"  # o-proj (even dispatches) and FFN-down (odd) when O is int8


def label(name):
    for k, v, _ in KERNELS:
        if k in name:
            return v
    return None


def per_dispatch(root):
    """{kernel label: {counter: average per dispatch}} (rows of one dispatch summed)."""
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = label(row["Kernel_Name"])
                if k:
                    vals[k][(row["Counter_Name"], row.get("Dispatch_Id", ""))] += float(row["Counter_Value"])
    split_o = "gemm_o_ln (gemm_kernel split-fp16)" not in vals
    out = {}
    for k, d in vals.items():
        groups = {k: d}
        if split_o and SHARED in k:  # dispatches in order: o, down, o, down, ...
            ids = sorted({i for _, i in d}, key=lambda x: int(x) if str(x).isdigit() else 0)
            rank = {i: n for n, i in enumerate(ids)}
            groups = {O_I8: {key: v for key, v in d.items() if rank[key[1]] % 2 == 0},
                      k: {key: v for key, v in d.items() if rank[key[1]] % 2 == 1}}
        for gk, gd in groups.items():
            per = collections.defaultdict(list)
            for (c, _), v in gd.items():
                per[c].append(v)
            out[gk] = {c: sum(v) / len(v) for c, v in per.items()}
    return out


def walls(src):
    """wall us per label: a bench.py JSON line (per-name event times) or a rocprof kernel-stats CSV"""
    w = {}
    if src.endswith(".json"):
        with open(src) as fh:
            kern = json.loads(fh.read().strip().splitlines()[-1])["kernels"]
        for _, v, name in KERNELS:
            if name in kern:
                w[v] = kern[name]["avg_us"]
        if "gemm_o_ln" in kern:
            w[O_I8] = kern["gemm_o_ln"]["avg_us"]
        return w
    with open(src) as fh:
        for row in csv.DictReader(fh):
            k = label(row["Name"])
            if k and k not in w:
                w[k] = float(row["AverageNs"]) / 1e3
    return w


def main(cyc_dir, ins_dir, stats_csv, out, source):
    a, b, w = per_dispatch(cyc_dir), per_dispatch(ins_dir), walls(stats_csv)
    res = {}
    for k in [v for _, v, _ in KERNELS] + [O_I8]:
        if k not in a or k not in b or k not in w:
            continue
        c = {**a[k], **b[k]}
        wall = w[k]
        clock = c["GRBM_GUI_ACTIVE"] / 8 / (wall * 1e3)  # GHz
        cyc = wall * 1e3 * clock  # wall cycles
        wc = c["SQ_WAVE_CYCLES"]
        res[k] = {
            "wall_us": round(wall, 1),
            "clock_GHz": round(clock, 3),
            "wave_cycles_parked": round(c["SQ_WAIT_ANY"] / wc, 3),
            "wave_cycles_issue_stalled": round(c["SQ_WAIT_INST_ANY"] / wc, 3),
            "wave_cycles_issuing": round(c["SQ_ACTIVE_INST_ANY"] / wc, 3),
            "valu_insts": c["SQ_INSTS_VALU"],
            "mfma_insts": c["SQ_INSTS_MFMA"],
            "lds_insts": c["SQ_INSTS_LDS"],
            "salu_insts": c["SQ_INSTS_SALU"],
            "vmem_insts": c["SQ_INSTS_VMEM"],
            "valu_per_mfma": round(c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"], 1),
            "valu_issue_frac_of_wall": round(2 * c["SQ_INSTS_VALU"] / (1024 * cyc), 3),
            "mfma_busy_frac_of_wall": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), 3),
        }
    doc = {"source": source + "; " + __doc__.split("\n\n")[2].replace("\n", " ").strip(), "kernels": res}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
