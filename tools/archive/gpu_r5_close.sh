#!/bin/bash
# Round-5 closing measurements (GPU box), in two calls (gpurun's 20-minute limit):
#   a: the bench line, rocprofv3 kernel summary, PMC FETCH / WRITE passes and the
#      bench line with that traffic folded in (tools/profile_round.sh r05);
#   b: the C2 / C4 / C5 config lines, the FFN-down PMC pass without the two-tile
#      pipeline (build/var/lnp0), and the N > 1 rehearsal (two ranks on one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
case "$1" in
a)
  bash tools/gpu_steps.sh profile 1000 "bash tools/profile_round.sh r05" ;;
b)
  bash tools/gpu_steps.sh \
    configs 600 "CFG_OUT=gpurun_out/cfg bash tools/configs_bench.sh" \
    pmc_lnp0 300 "cd /tmp && B=\$GRAFT_REPO_ROOT/bench.py; A='--steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 --ragged-steps 0 --host-runs 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0'; export BERT_AMD_SPLIT=0 BERT_AMD_LIB=\$GRAFT_REPO_ROOT/build/var/lnp0/libbert.so; timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/lnp0/fetch -o lnp0 -- python3 \$B \$A && timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/lnp0/write -o lnp0 -- python3 \$B \$A && python3 \$GRAFT_REPO_ROOT/tools/hbm_summary.py \$GRAFT_REPO_ROOT/gpurun_out/lnp0/fetch \$GRAFT_REPO_ROOT/gpurun_out/lnp0/write 'lnp0: FFN-down LN kernel without the two-tile pipeline (no scratch)' > \$GRAFT_REPO_ROOT/gpurun_out/lnp0_pmc_hbm.txt" \
    rehearse 300 "python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 --cpu-sample 0 --ragged-steps 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0 > gpurun_out/rehearse2.json" ;;
*) echo "usage: $0 a|b"; exit 2 ;;
esac
