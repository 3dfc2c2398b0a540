"""Development sweep (not shipped): bert_encode_batch consumer-path rate at
n_batch_size 16 / 256 for several encode_lanes x encode_merge settings, on the
bench's synthetic texts (bench.consumer_line).  One model load, options set
per context with bert_amd_set_option.  Usage: python tools/consumer_sweep.py
[lanes,merge[,merge_rows] ...]  e.g. 2,4 4,4 4,8 2,32,512"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from bench import bertlib  # noqa: E402


def main():
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    hp = bertlib.SHAPES["minilm"]
    d = os.environ.get("BERT_AMD_MODEL_DIR", "/tmp/bert_amd_models")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"minilm_q4_0_s{bench.SEED}_w0.05.gguf")
    if not os.path.exists(path):
        bertlib.synth_model(path, "minilm", "q4_0", seed=bench.SEED, w_std=0.05)
    model = bertlib.BertModel(path, devices=[0])
    stream = torch.cuda.current_stream(dev).cuda_stream
    combos = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(2, 4)]
    for c in combos:
        lanes, merge, rows = (c + (256,))[:3]
        model.set_option("encode_lanes", lanes)
        model.set_option("encode_merge", merge)
        model.set_option("encode_merge_rows", rows)
        r = bench.consumer_line(model, hp, 4096, 0, dev, stream, torch)
        print(json.dumps(dict(lanes=lanes, merge=merge, rows=rows, b16=r["encode_batch_16"]["value"],
                              b256=r["encode_batch_256"]["value"], all=r["encode_batch_all"]["value"],
                              dev=r["device_resident_same_sentences"]["value"],
                              frac16=r["batch16_frac_of_device"], bitwise=r["bitwise_vs_device"])), flush=True)


if __name__ == "__main__":
    main()
