"""The N>1 path of bench.py on CPU: world_size-2 torch.distributed over gloo.

bench.py shards sentences across ranks with no data-path collective (weak
scaling: rank r owns sentences [r*B, (r+1)*B), reference bert.cpp:1065 keeps no
state across sentences); the only collectives are the barrier and the
max-over-ranks step time.  Here each rank runs the CPU oracle (test
infrastructure) on its shard and the union is compared with a single-process
run of the same global batch: per-sentence results must not depend on the
sharding.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

B_PER_RANK, SEQ = 2, 12


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, model_path, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import oracle

        first = bench.shard(rank, B_PER_RANK)
        toks = bench.splitmix_tokens(first, B_PER_RANK, SEQ, 30522)
        emb = oracle.Oracle(model_path).eval_batch([t.tolist() for t in toks], 1)
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), emb)
        np.save(os.path.join(out_dir, f"tok{rank}.npy"), toks)
        t = bench.max_over_ranks(float(rank + 1) * 1.5)
        with open(os.path.join(out_dir, f"max{rank}.txt"), "w") as f:
            f.write(repr(t))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process(tmp_path, model_dir):
    import bench
    import bertlib
    import oracle
    from make_golden import sentence

    path = os.path.join(model_dir, "multirank_minilm_q4_0.gguf")
    if not os.path.exists(path):
        bertlib.synth_model(path, "minilm", "q4_0", seed=bench.SEED, w_std=0.05, n_layer=2)
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), path, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    # the collective the bench uses for timing: max over ranks
    for r in range(world):
        assert float((tmp_path / f"max{r}.txt").read_text()) == 3.0
    # shards are disjoint, contiguous and equal to the bench's global token stream
    toks = np.concatenate([np.load(tmp_path / f"tok{r}.npy") for r in range(world)])
    assert toks.shape == (world * B_PER_RANK, SEQ)
    for i in range(world * B_PER_RANK):
        assert toks[i].tolist() == sentence(i, SEQ, 30522)
    # union of per-rank results == one process over the whole batch (bitwise: the oracle is deterministic)
    got = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    want = oracle.Oracle(path).eval_batch([t.tolist() for t in toks], 1)
    assert np.array_equal(got, want)
