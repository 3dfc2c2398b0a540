"""Text table of tests/test_layer_parity.py's per-stage records
(gpurun_out/layer_parity_<case>.json) -> stdout (profiles/rNN_layer_parity.txt).
python tools/layer_parity_table.py gpurun_out/layer_parity_*.json"""
import json
import os
import sys

print("# tests/test_layer_parity.py on one MI355X (ulp: in units of the row's largest magnitude)")
for path in sorted(sys.argv[1:]):
    rows = json.load(open(path))
    print("== " + os.path.basename(path)[len("layer_parity_"):-len(".json")])
    print("sent stage | chained ulp  1-cos | local ulp  1-cos | ggml spread ulp  1-cos | code/scale mismatches")
    for r in rows:
        print(f"s{r['sentence']} {r['stage']:2d} | {r['chained_ulp']:>9d} {r['chained_1mcos']:.2e} | "
              f"{r.get('local_ulp', 0):>9d} {r.get('local_1mcos', 0):.2e} | "
              f"{r.get('spread_ulp', 0):>9d} {r.get('spread_1mcos', 0):.2e} | "
              f"{r.get('code_mismatch', '-')}/{r.get('scale_mismatch', '-')}")
