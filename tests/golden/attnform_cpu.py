# CPU experiment (round 5): the oracle with the GPU kernels' attention operand form
# (oracle.set_attn_form("gpu_operands")) against the three ggml build orders stored in the fixtures.
import os, sys, json, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for _p in ("oracle", "tests/golden", "embedding.cpp_amd"):
    sys.path.insert(0, os.path.join(REPO, _p))
import numpy as np, oracle
from make_golden import load_case, ensure_model, load_variants
def cos(a,b):
    a=np.asarray(a,np.float64); b=np.asarray(b,np.float64)
    return (a*b).sum(1)/np.linalg.norm(a,axis=1)/np.linalg.norm(b,axis=1)
out={}
for case in ['c3_minilm_q4_0','minilm_q4_1','c5_bge_q4_1_l2','c5_bge_q4_1']:
    meta,toks,want=load_case(case); var=load_variants(case)
    p=ensure_model(os.environ.get('BERT_AMD_MODEL_DIR', '/tmp/bert_amd_models'),meta['shape'],meta['ftype'],meta['w_std'],meta.get('n_layer'))
    o=oracle.Oracle(p)
    res={}
    for v in ['avx2','generic']:
        oracle.set_dot_variant(v); oracle.set_attn_form('gpu_operands')
        t0=time.time(); g=o.eval_batch(toks,0)
        oracle.set_attn_form('ggml'); oracle.set_dot_variant('avx2')
        res[f'{v}+gpu_operands vs avx2']=float((1-cos(g,want)).max())
        res[f'{v}+gpu_operands vs generic']=float((1-cos(g,var['generic'])).max())
        res[f'{v}+gpu_operands vs lanes16']=float((1-cos(g,var['lanes16'])).max())
        res[f'{v}+gpu_operands seconds']=round(time.time()-t0,1)
    out[case]=res
    print(case, json.dumps(res), flush=True)
json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "profiles", "r05_attnform_cpu.json"), "w"), indent=1)
