"""Multi-GPU sharding of a sieve sweep: one process per GPU, rows split by rank.

Assignments are regenerated per rank from the counter-based generator (row i of rank r is global
candidate index r * rows_per_rank + i), so no input moves between GPUs.  The one exchange per
step is the per-tape result: the smallest satisfying global index (MIN; MH_NO_HIT = all ones is
mapped to INT64_MAX for the reduction) and the number of satisfying rows (SUM), 16 B per tape,
over RCCL ("nccl" backend) on the GPUs or gloo on the CPU.  The minimum over shards is the global
minimum, so results are identical for any number of ranks.
"""
from __future__ import annotations

from typing import Tuple

INT64_MAX = (1 << 63) - 1


def shard_range(rank: int, world: int, rows_per_rank: int) -> Tuple[int, int]:
    """(global index of this rank's first row, rows) — weak scaling: every rank sweeps
    rows_per_rank candidates."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world of %d" % (rank, world))
    return rank * rows_per_rank, rows_per_rank


def strong_shard_range(rank: int, world: int, total_rows: int) -> Tuple[int, int]:
    """(global index of this rank's first row, rows) — strong scaling: `total_rows` candidates
    (config 5: 2^26 in total over the node's GPUs) split into `world` contiguous shards that
    differ by at most one row; rank r's rows keep their global indices, so the reduced results
    equal one GPU's sweep of all `total_rows`."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world of %d" % (rank, world))
    q, r = divmod(total_rows, world)
    first = rank * q + min(rank, r)
    return first, q + (1 if rank < r else 0)


def allreduce_results(first_hit, hit_count, group=None) -> None:
    """In place over all ranks: first_hit = MIN (NO_HIT stays NO_HIT), hit_count = SUM.
    first_hit / hit_count are int64 tensors holding the u64 results (NO_HIT reads -1)."""
    import torch
    import torch.distributed as dist

    f = torch.where(first_hit == -1, torch.full_like(first_hit, INT64_MAX), first_hit)
    dist.all_reduce(f, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hit_count, op=dist.ReduceOp.SUM, group=group)
    first_hit.copy_(torch.where(f == INT64_MAX, torch.full_like(f, -1), f))


def setup_exchange(ctx, rank: int, world: int, device=None):
    """The per-step result exchange of a multi-rank sweep (bench.py): the library's own RCCL
    communicator (``mh_comm_init``: rank 0's unique id reaches the others through
    torch.distributed) when every rank can open it, else torch.distributed's all-reduce of the
    same MIN / SUM (allreduce_results).  Returns (exchange, reasons): "library" or "torch", and
    on the torch fallback the failure message of every rank that could not open the
    communicator ("rank r: ..."), gathered to every rank -- bench.py puts them in its JSON line
    (``exchange_fallback``), so a scaling number taken on the fallback says so.  `ctx` needs
    ``comm_init(uid, rank, world)``; the unique id comes from ``native.comm_unique_id``."""
    import torch
    import torch.distributed as dist

    from . import native

    box, why = [None], None
    if rank == 0:
        try:
            box = [native.comm_unique_id()]
        except Exception as e:  # noqa: BLE001 - depends on the node's RCCL
            why = "rank 0: mh_comm_unique_id: %s" % e
    dist.broadcast_object_list(box, src=0)
    if box[0] is not None:
        try:
            ctx.comm_init(box[0], rank, world)
        except Exception as e:  # noqa: BLE001
            why = "rank %d: mh_comm_init: %s" % (rank, e)
    elif why is None:
        why = "rank %d: no communicator id from rank 0" % rank
    reasons = [None] * world
    dist.all_gather_object(reasons, why)
    failed = [r for r in reasons if r]
    flag = torch.tensor([0 if failed else 1], dtype=torch.int32,
                        device=device if device is not None else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 1:
        return "library", []
    return "torch", failed
