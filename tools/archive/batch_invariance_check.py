import sys, os, numpy as np
sys.path[:0]=['embedding.cpp_amd','tests/golden','tests']
import bertlib
from make_golden import ensure_model, sentence
p=ensure_model('/tmp/bert_amd_models','minilm','q4_0',0.05)
m=bertlib.BertModel(p)
toks=[sentence(i,n,30522) for i,n in enumerate([128,9,256,64,2,500,128])]
full=m.eval_batch(toks)
for i,t in enumerate(toks):
    a=m.eval(t)
    print(i,len(t),np.array_equal(a,full[i]), float(np.abs(a-full[i]).max()))
sh=[t for t in toks if len(t)<=128]
b=m.eval_batch(sh)
print('short-only vs full', [np.array_equal(b[k], full[i]) for k,i in enumerate([0,1,3,4,6])])
m2=bertlib.BertModel(p, devices=[0,0])
f2=m2.eval_batch(toks)
print('2rep', [np.array_equal(f2[i], full[i]) for i in range(len(toks))])
