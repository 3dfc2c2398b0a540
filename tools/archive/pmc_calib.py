"""counted / moved for build/pmc_calib's kernels (tools/pmc_calib.sh): raw
FETCH_SIZE and WRITE_SIZE (KB, no correction applied) against the bytes each
kernel moves.  python tools/pmc_calib.py <gpurun_out/pmc_calib>"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(__file__))
from hbm_summary import load  # noqa: E402

NAMES = [("st16_kernel", "st16", "w"), ("st8_kernel", "st8", "w"), ("st_kernel<unsigned int>", "st4", "w"),
         ("st_kernel<unsigned short>", "st2", "w"), ("ld16_kernel", "ld16", "r"), ("ld8_kernel", "ld8", "r"),
         ("ld4_kernel", "ld4", "r"), ("st4_rows_kernel", "st4_rows", "w"), ("st8_ln_kernel", "st8_ln", "w"),
         ("scratch_kernel", "scratch", "w")]


def main():
    out = sys.argv[1]
    moved = {}
    for line in open(os.path.join(out, "plain.log")):
        m = re.match(r"bytes (.*) (\d+)$", line.strip())
        if m:
            for k in m.group(1).split():
                moved[k] = int(m.group(2))
    fetch, write = load(os.path.join(out, "FETCH_SIZE"), "FETCH_SIZE"), load(os.path.join(out, "WRITE_SIZE"), "WRITE_SIZE")
    print(f"{'kernel':10s} {'moved_MB':>9s} {'FETCH_MB':>9s} {'WRITE_MB':>9s} {'counted/moved':>14s}")
    for frag, short, kind in NAMES:
        def pick(per):
            for k, d in per.items():
                if frag in k:
                    return sum(d.values()) / max(len(d), 1) * 1024.0
            return float("nan")
        f, w = pick(fetch), pick(write)
        mv = moved.get(short, float("nan"))
        ratio = (w if kind == "w" else f) / mv
        print(f"{short:10s} {mv / 1e6:9.1f} {f / 1e6:9.1f} {w / 1e6:9.1f} {ratio:14.3f}")


if __name__ == "__main__":
    main()
