"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh) per kernel: average counter
value per dispatch, plus derived ratios.  FETCH_SIZE is doubled (gfx950
reports half the bytes of wide streaming reads: MI355X_MICROARCH.md, HBM)."""
import collections
import csv
import glob
import os
import sys

SHORT = [("gemm_kernelILi2ELi0", "gemm_qkv"), ("gemm_kernelILi2ELi1", "gemm_up_gelu"),
         ("gemm_kernelILi2ELi2", "gemm_ln"), ("attention_short", "attention"), ("embed_ln", "embed_ln"),
         ("pool_l2", "pool_l2")]


def short(name):
    for k, v in SHORT:
        if k in name:
            return v
    return name[:40]


def main(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                c = row["Counter_Name"]
                vals[k][(c, row.get("Dispatch_Id", ""))].append(float(row["Counter_Value"]))
    for k in sorted(vals):
        per = collections.defaultdict(list)
        for (c, _), v in vals[k].items():
            per[c].append(sum(v))
        avg = {c: sum(v) / len(v) for c, v in per.items()}
        if "FETCH_SIZE" in avg:
            avg["FETCH_SIZE"] *= 2 * 1024  # KB -> B, x2 gfx950 correction
        if "WRITE_SIZE" in avg:
            avg["WRITE_SIZE"] *= 1024
        print(f"== {k}")
        for c in sorted(avg):
            print(f"   {c:28s} {avg[c]:.4g}")
        g = avg.get
        if g("SQ_WAVE_CYCLES"):
            w = g("SQ_WAVE_CYCLES")
            print(f"   wait_any/wave {g('SQ_WAIT_ANY', 0) / w:.3f}  wait_inst/wave {g('SQ_WAIT_INST_ANY', 0) / w:.3f}"
                  f"  active/wave {g('SQ_ACTIVE_INST_ANY', 0) / w:.3f}")
        if g("SQ_INSTS_MFMA"):
            print(f"   valu/mfma {g('SQ_INSTS_VALU', 0) / g('SQ_INSTS_MFMA'):.2f}  lds/mfma {g('SQ_INSTS_LDS', 0) / g('SQ_INSTS_MFMA'):.2f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
