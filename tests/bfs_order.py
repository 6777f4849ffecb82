"""Query sequences in the order LASER's default strategy asks them (test / measurement helper).

LASER runs breadth-first by default (mythril/interfaces/cli.py:417-419: ``--strategy bfs``), and
after each JUMPI it asks ``is_possible`` for both successor states (laser/ethereum/svm.py:243-262):
the state's path plus the condition, then plus its negation; a state found infeasible is dropped.
``bfs_queries`` yields the roots of every query of such a run over a binary JUMPI tree: the first
``prefix`` constraints asked in LASER order (one path: each query its parent plus one), then one
level per remaining constraint in which every open state, in FIFO order, asks both of its
branches back to back.  The caller drops a state by adding ``tuple(roots)`` to ``dropped``
before asking for the next query; at most ``k`` of the surviving new states stay open (drawn
with ``seed`` among all of them, kept in BFS order), so open paths part at many depths.
"""
from __future__ import annotations

import random
from typing import Iterator, List, Optional, Sequence, Set


def bfs_queries(nodes: Sequence[int], negs: Sequence[int], prefix: int, k: int,
                seed: int = 0, dropped: Optional[Set[tuple]] = None) -> Iterator[List[int]]:
    """nodes[j] / negs[j]: the j-th JUMPI condition and its negation (term nodes)."""
    rng = random.Random(seed)
    dropped = set() if dropped is None else dropped
    for i in range(1, prefix + 1):
        yield list(nodes[:i])
    open_ = [list(nodes[:prefix])]
    for j in range(prefix, len(nodes)):
        nxt = []
        for s in open_:
            for c in (nodes[j], negs[j]):
                q = s + [c]
                yield q
                if tuple(q) not in dropped:
                    nxt.append(q)
        if len(nxt) > k:
            keep = sorted(rng.sample(range(len(nxt)), k))
            nxt = [nxt[i] for i in keep]
        if not nxt:
            return
        open_ = nxt
