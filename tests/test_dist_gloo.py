"""World-size-2 gloo test of the multi-GPU protocol on CPU.

Batches are split round-robin with no data-path collective; the only
communication is the barrier and the max-over-ranks of the timed region that
bench.py uses.  Each rank classifies its shard with the oracle (the CPU checker;
the GPU path is exercised by the -m gpu tests) and the union must equal the
single-process result."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import mosrx
import oracle_py as O


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    d = bench.Dist(world, rank)
    t = mosrx.Trace(mosrx.TRACE_IMIX, 12_000, nflows=3000)
    batches = mosrx.split_batches(t.frames, t.off, t.len, 1000)
    mine = bench.job_batches(len(batches), world, rank)     # the split bench.py runs
    d.barrier()
    res = {b: O.classify(batches[b][0], batches[b][1], batches[b][2]) for b in mine}
    d.barrier()
    m = d.max(float(rank + 1))
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), m=m,
             **{f"b{b}": r.view(np.uint8) for b, r in res.items()})
    d.close()


@pytest.mark.parametrize("world", [2])
def test_round_robin_shards_cover_job(tmp_path, world):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    t = mosrx.Trace(mosrx.TRACE_IMIX, 12_000, nflows=3000)
    whole = O.classify(t.frames, t.off, t.len)
    got = {}
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        assert float(z["m"]) == world          # max over ranks
        for k in z.files:
            if k.startswith("b"):
                b = int(k[1:])
                assert b not in got              # disjoint
                got[b] = z[k]
    assert sorted(got) == list(range(12))        # complete
    joined = np.concatenate([got[b] for b in range(12)]).view(mosrx.RESULT_DTYPE)
    assert np.array_equal(joined.view(np.uint8), whole.view(np.uint8))


def test_bench_job_split_is_round_robin():
    """bench.py's own split of the job (config #5): rank r of W takes job batches
    r, r + W, ...; the shards are disjoint, cover the job, and each rank's resident
    contents are seeded by the job batch index (batch 0 = the default trace)."""
    import bench
    for world in (1, 2, 4, 8):
        shards = [bench.job_batches(world * 8, world, r) for r in range(world)]
        assert sorted(b for sh in shards for b in sh) == list(range(world * 8))
        assert all(sh == list(range(r, world * 8, world)) for r, sh in enumerate(shards))
    assert bench.job_seed(mosrx.TRACE_IMIX, 0) == 0
    seeds = {bench.job_seed(mosrx.TRACE_IMIX, b) for b in range(64)}
    assert len(seeds) == 64
    a = mosrx.Trace(mosrx.TRACE_IMIX, 300, nflows=50, seed=bench.job_seed(mosrx.TRACE_IMIX, 3))
    b = mosrx.Trace(mosrx.TRACE_IMIX, 300, nflows=50, seed=bench.job_seed(mosrx.TRACE_IMIX, 3))
    c = mosrx.Trace(mosrx.TRACE_IMIX, 300, nflows=50, seed=bench.job_seed(mosrx.TRACE_IMIX, 4))
    assert np.array_equal(a.frames, b.frames) and not np.array_equal(a.frames, c.frames)


def test_shard_plan():
    assert mosrx.shard_plan(10, 4, 1) == [1, 5, 9]
    allb = sorted(b for r in range(8) for b in mosrx.shard_plan(37, 8, r))
    assert allb == list(range(37))
    with pytest.raises(ValueError):
        mosrx.shard_plan(4, 2, 2)


def _leg_worker(rank, world, port, out_dir):
    """Each rank runs one end-to-end leg (bench.Dist.leg), its timed region between
    barriers: rank r moves (r + 1) * 1000 frames of 100 bytes in about 0.2 * (r + 1) s."""
    import json
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    d = bench.Dist(world, rank)

    def fn(sync):
        time.sleep(0.3 * (1 - rank))          # set-up of different lengths: the timed regions still start together
        sync()
        t0 = time.perf_counter()
        time.sleep(0.2 * (rank + 1))
        dt = time.perf_counter() - t0
        sync()
        return {"frames": (rank + 1) * 1000, "bytes": (rank + 1) * 100_000, "seconds": dt}
    mine, agg = d.leg(fn)
    spread = d.gather([float(rank + 1), 10.0 * rank])
    with open(os.path.join(out_dir, f"leg{rank}.json"), "w") as fh:
        json.dump({"mine": mine, "agg": agg, "spread": spread}, fh)
    d.close()


def test_bench_leg_aggregate_over_ranks(tmp_path):
    """The N>1 end-to-end figure: every rank's frames and bytes summed over the
    longest rank's wall time (the job ends with its last rank), and each rank's
    own rate as min / max; every rank computes the same aggregate."""
    import json
    world = 2
    mp.start_processes(_leg_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    outs = [json.load(open(tmp_path / f"leg{r}.json")) for r in range(world)]
    agg = outs[0]["agg"]
    assert outs[1]["agg"] == agg
    assert agg["ranks"] == 2 and agg["frames"] == 3000
    wall = agg["seconds"]
    assert 0.4 <= wall < 0.7                                   # the slower rank's ~0.4 s timed region
    assert abs(agg["mpkts"] - 3000 / wall / 1e6) < 1e-2
    assert abs(agg["gbps"] - 300_000 / wall / 1e9) < 1e-2
    assert agg["per_rank_mpkts"]["min"] <= agg["per_rank_mpkts"]["max"]
    assert outs[0]["spread"] == [[1.0, 0.0], [2.0, 10.0]]       # gather: rank order, every rank


def test_aggregate_rows():
    import bench
    a = bench.aggregate([[1e6, 1e9, 0.5], [3e6, 2e9, 1.0]])
    assert a["frames"] == 4_000_000 and a["seconds"] == 1.0
    assert a["mpkts"] == 4.0 and a["gbps"] == 3.0
    assert a["per_rank_mpkts"] == {"min": 2.0, "max": 3.0}
