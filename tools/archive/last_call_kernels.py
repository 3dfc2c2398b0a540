"""Per-kernel durations of the last bert_eval call in a rocprofv3
--kernel-trace CSV (the call = the last embed_ln_kernel onwards).

    python3 tools/last_call_kernels.py <kernel_trace.csv> [json_out]
"""
import csv
import json
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = max(i for i, r in enumerate(rows) if "embed_ln" in r["Kernel_Name"])
call = rows[first:]
t0 = int(call[0]["Start_Timestamp"])
out = []
for r in call:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    name = r["Kernel_Name"].split("(")[0]
    out.append({"kernel": name, "start_us": round((int(r["Start_Timestamp"]) - t0) / 1000, 2), "us": round(d, 2)})
    print(f"{out[-1]['start_us']:8.1f} {d:6.2f} {name}")
span = (int(call[-1]["End_Timestamp"]) - t0) / 1000
print(f"kernels {len(call)}  sum {sum(o['us'] for o in out):.1f} us  span {span:.1f} us")
if len(sys.argv) > 2:
    json.dump({"kernels": out, "span_us": round(span, 1)}, open(sys.argv[2], "w"), indent=1)
