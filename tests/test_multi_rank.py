"""The N>1 path of bench.py on CPU: world_size-2 torch.distributed over gloo.

bench.py shards sentences across ranks with no data-path collective (weak
scaling: rank r owns sentences [r*B, (r+1)*B), reference bert.cpp:1065 keeps no
state across sentences); the only collectives are the barrier and the
max-over-ranks step time.  Here each rank runs the CPU oracle (test
infrastructure) on its shard and the union is compared with a single-process
run of the same global batch: per-sentence results must not depend on the
sharding.  The library-sharding step SCALE runs at N > 1 (bench.library_sharding
+ lib_shard_work: rank 0 times a context replicated over every device while
the other ranks wait in a gloo barrier) is driven through bench's own code with
a CPU stand-in for the library's BertModel.
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
        # bench's library-sharding step: rank 0 evaluates the global batch on a
        # (stand-in) context over `world` devices, the other rank waits in gloo
        gtoks = bench.splitmix_tokens(0, world * B_PER_RANK, SEQ, 30522)
        res = bench.library_sharding(
            rank, world, lambda: dist.barrier(),
            lambda: bench.lib_shard_work(OracleModel, model_path, list(range(world)), gtoks, B_PER_RANK, emb, "test"))
        with open(os.path.join(out_dir, f"libshard{rank}.txt"), "w") as f:
            f.write(repr(res))
        # a failing rank 0 still releases the waiting ranks (no hang), and the error surfaces on rank 0
        def boom():
            raise RuntimeError("rank 0 failure")
        try:
            bench.library_sharding(rank, world, lambda: dist.barrier(), boom)
            outcome = "returned"
        except RuntimeError as e:
            outcome = str(e)
        with open(os.path.join(out_dir, f"fail{rank}.txt"), "w") as f:
            f.write(outcome)
        dist.barrier()
    finally:
        dist.destroy_process_group()


class OracleModel:
    """CPU stand-in with bertlib.BertModel's surface for bench.lib_shard_work:
    a context "replicated" over `devices` whose bert_eval_batch is the oracle
    (the library's sharding itself needs GPUs: tests/test_gpu_parity.py)."""

    def __init__(self, path, devices):
        import oracle
        self.o = oracle.Oracle(path)
        self.n_devices = len(devices)

    def prepared_batch(self, token_lists):
        emb = np.full((len(token_lists), self.o.n_embd), np.nan, np.float32)

        def run():
            emb[:] = self.o.eval_batch([np.asarray(t).tolist() for t in token_lists], 1)
            return emb

        return run, emb

    def close(self):
        pass


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
    # library sharding: rank 0 measured the global batch over both devices, bitwise
    # equal to its own shard; the waiting rank got nothing and did not hang
    lib0 = eval((tmp_path / "libshard0.txt").read_text())
    assert lib0["devices"] == world and lib0["bitwise_vs_rank0"] and lib0["value"] > 0
    assert (tmp_path / "libshard1.txt").read_text() == "None"
    assert (tmp_path / "fail0.txt").read_text() == "rank 0 failure"
    assert (tmp_path / "fail1.txt").read_text() == "returned"
    # union of per-rank results == one process over the whole batch (bitwise: the oracle is deterministic)
    got = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    want = oracle.Oracle(path).eval_batch([t.tolist() for t in toks], 1)
    assert np.array_equal(got, want)
