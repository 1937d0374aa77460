"""Multi-GPU drivers: one process per GPU over torch.distributed (RCCL = backend "nccl" on ROCm).

SURVEY.md §8(e). ImageProjection and the feature stage are independent per scan, so batches of
scans are sharded across ranks as replicas with no collective on the data path (`shard_range`).
The one real exchange step is the scan-to-map LM with every scan's correspondences split over
the ranks: `sharded_scan2map` runs MapOptimization::scan2MapOptimization's iteration loop
(MO:1578-1608) with ONE all-reduce (sum) per LM iteration of the [P, LLSR_NE_WORDS] int64
fixed-point normal equations (include/llsr.h, llsr_scan2map_shard_*). Every rank then solves the
same 6x6 systems, so there is no broadcast, and the ranks stop after the same iteration because
they hold the same state. Integer sums make the result bit-identical for any world size.
"""
from __future__ import annotations

import time

from ._abi import NE_WORDS


def world_and_rank(group=None) -> tuple[int, int]:
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def shard_range(n: int, rank: int, world: int) -> range:
    """Replica sharding: the contiguous block of the n items rank `rank` of `world` owns."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return range(lo, hi)


class HipShardEngine:
    """This rank's share of a scan-to-map batch on its HIP device (llsr_scan2map_shard_*).

    `stream` must be the stream torch runs the collective and the buffer updates on, i.e.
    torch's current stream, and a non-default one: the ABI reads a NULL stream as the handle's
    own stream, which is not ordered with torch's legacy default stream."""

    def __init__(self, pipeline, ptrs: dict, P: int, stream: int):
        if not stream:
            raise ValueError("HipShardEngine needs a non-default stream (run under torch.cuda.stream(...))")
        self.pipe, self.ptrs, self.P, self.stream = pipeline, ptrs, P, stream

    def new_ne(self, device):
        import torch
        return torch.zeros((self.P, NE_WORDS), dtype=torch.int64, device=device)

    def begin(self):
        self.pipe.scan2map_shard_begin(self.ptrs, self.P, self.stream)

    def partial(self, rank: int, world: int, ne):
        self.pipe.scan2map_shard_partial(rank, world, ne.data_ptr(), self.stream)

    def step(self, ne, poll: bool) -> int:
        return self.pipe.scan2map_shard_step(ne.data_ptr(), poll, self.stream)

    def end(self):
        self.pipe.scan2map_shard_end(self.stream)


def sharded_scan2map(engine, ne, iter_max: int, group=None, poll: int = 4, force_collective: bool = False) -> int:
    """Run one split-correspondence scan-to-map batch; `ne` is the [P, NE_WORDS] int64 exchange
    buffer (on the engine's device for RCCL, a CPU tensor for gloo). The engine must be bound to
    the same stream torch uses for the collective (the current stream). Returns the LM
    iterations run (the loop stops early once every problem converged). At world 1 the
    all-reduce is an identity and is skipped unless force_collective (which runs it through the
    initialised process group, e.g. a one-rank RCCL group)."""
    import torch.distributed as dist
    world, rank = world_and_rank(group)
    collective = world > 1 or (force_collective and dist.is_available() and dist.is_initialized())
    engine.begin()
    it = 0
    while it < iter_max:
        engine.partial(rank, world, ne)
        if collective:
            dist.all_reduce(ne, op=dist.ReduceOp.SUM, group=group)
        it += 1
        active = engine.step(ne, poll=(it % poll == 0 or it == iter_max))
        if active == 0:
            break
    engine.end()
    return it


def max_over_ranks(seconds: float, device=None, group=None) -> float:
    """The bench contract's max-over-ranks of a timed region."""
    world, _ = world_and_rank(group)
    if world == 1:
        return seconds
    import torch
    import torch.distributed as dist
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def allreduce_latency_us(ne, reps: int = 50, group=None) -> float:
    """Mean wall time of one all-reduce of the exchange buffer (synchronised per call); 0.0 when no
    process group is initialised (a one-rank group is measured: RCCL still runs the collective)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return 0.0
    cuda = ne.is_cuda
    ne.zero_()
    for _ in range(5):
        dist.all_reduce(ne, group=group)
    if cuda:
        torch.cuda.synchronize(ne.device)
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_reduce(ne, group=group)
        if cuda:
            torch.cuda.synchronize(ne.device)
    return (time.perf_counter() - t0) / reps * 1e6
