"""Batched healer repair: the reference healer's EC repair (cmd/healer/poller.go:
227-309, auditAndRepairEC) for a whole scan's worth of damaged objects at once
(SURVEY.md §8f rank 2).

The reference audits one object per goroutine, at most 10 at a time
(poller.go:49-65), and calls ``h.ec.Reconstruct(shards)`` per object (:282).
Here the audit results of many objects are evaluated with the same rules and
every object that needs repair goes to the GPU in as few batched launches as
their shard lengths allow (rs_co_reconstruct_many).  Fetching shards from and
writing them back to storage nodes stays with the caller (out of scope: HTTP).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from .coalescer import CoalescingService
from .ec import ECError

HEALTHY = "healthy"
REPAIRED = "repaired"
DATA_LOSS = "data_loss"
FAILED = "failed"


@dataclass
class RepairResult:
    key: str
    status: str
    missing: List[int] = field(default_factory=list)
    repaired: Dict[int, bytes] = field(default_factory=dict)  # shard index -> bytes to write back
    error: Optional[str] = None


class BatchHealer:
    def __init__(self, svc: CoalescingService):
        self.svc = svc

    def repair(self, audits: Sequence[Tuple[str, List[Optional[bytes]]]]) -> List[RepairResult]:
        """audits: (main key, K+M shards as fetched; None/empty = fetch failed).
        Per object, poller.go's steps: 2. evaluate (nothing missing -> healthy;
        fewer than K available -> "critical data loss"); 3. Reconstruct; 4. the
        missing shards to write back."""
        k, m = self.svc.k, self.svc.m
        out: List[RepairResult] = []
        todo, todo_idx = [], []
        for key, shards in audits:
            shards = [None if s is None or len(s) == 0 else bytearray(s) for s in shards]
            missing = [i for i, s in enumerate(shards) if s is None]  # poller.go:240-246
            if not missing:
                out.append(RepairResult(key, HEALTHY))
                continue
            if len(shards) - len(missing) < k:  # poller.go:256-262
                out.append(RepairResult(key, DATA_LOSS, missing, error="critical data loss: not enough shards"))
                continue
            out.append(RepairResult(key, REPAIRED, missing))
            todo.append(shards)
            todo_idx.append(len(out) - 1)
        errs = self.svc.ReconstructMany(todo) if todo else []
        for shards, i, err in zip(todo, todo_idx, errs):
            r = out[i]
            if err is not None:  # poller.go:282-285
                r.status, r.error = FAILED, str(err)
                continue
            r.repaired = {j: bytes(shards[j]) for j in r.missing}
        return out
