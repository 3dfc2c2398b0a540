cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
echo "== 4 consumers (pairs0)"; BERT_AMD_LIB=build/var/st0/libbert.so timeout -k 10 200 python3 tools/pipe_stamps.py work sync+split Y || exit 1
echo "== pairs"; BERT_AMD_LIB=build/var/st1/libbert.so timeout -k 10 200 python3 tools/pipe_stamps.py work sync+split Y || exit 1
echo "== pairs, consumer B detail (slots 0,3,4,5,1,2)"; STAMP_SLOTS=0,3,4,5,1,2 BERT_AMD_LIB=build/var/st1/libbert.so timeout -k 10 200 python3 tools/pipe_stamps.py scores+mxx exp waitA PV Xsync+store Y || exit 1
