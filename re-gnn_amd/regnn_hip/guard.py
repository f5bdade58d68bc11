"""Collective-consistent failure handling for the data-parallel NS path.

The reference is single-process (mag/regnn_ns.py:392-420: zero_grad -> forward -> nll -> backward
-> Adam); the build inserts one gradient all-reduce per step between the backward and Adam
(:406-407). With several ranks, a rank that raises while its peers sit in a collective leaves them
blocked until the process group's timeout. The rules here:

* every stage that can fail on one rank is run by ``Guard.stage``: the exception is caught, the
  collectives the peers are issuing in that stage (``always``: e.g. the step's gradient
  exchange) are still issued, and all ranks then agree on the outcome with one eager SUM
  all-reduce of the failure flags (the number of ranks that failed);
* if any rank failed, every rank raises ``RankFailure`` (a SystemExit with a non-zero code), so
  the whole job ends with a non-zero exit on every rank instead of hanging; the failing rank's
  own traceback is printed first;
* the agreement itself is guarded: if its all-reduce (or reading its result) raises -- a peer
  that died, a device left in a faulted state -- this rank raises ``RankFailure`` too, so it
  exits with ``EXIT_CODE`` rather than a plain RuntimeError;
* a rank whose device faults hard (the process is killed, or it hangs inside a HIP call) never
  reaches the agreement: its peers' agreement all-reduce then fails at the process group's
  timeout (``pg_timeout``), which ends them through the rule above;
* nothing here re-executes a process (no exec of any kind after the GPU was touched).

One rank: ``stage`` runs fn and lets its exception propagate unchanged.
"""
import sys
import traceback
from datetime import timedelta

import torch

EXIT_CODE = 3                                # the exit status of every rank after a failure


class RankFailure(SystemExit):
    """raised on every rank after a stage failed on at least one of them."""

    def __init__(self, what, ranks_failed, local_exc=None):
        super().__init__(EXIT_CODE)
        self.what, self.ranks_failed, self.local_exc = what, ranks_failed, local_exc

    def __str__(self):
        if self.ranks_failed < 0:
            return f"stage '{self.what}': the ranks could not agree (collective failed)"
        return f"stage '{self.what}' failed on {self.ranks_failed} rank(s)"


def pg_timeout(default_s=600):
    """the process group's timeout (env REGNN_DIST_TIMEOUT seconds): a collective whose peer
    died or never arrives errors out after it instead of blocking forever."""
    import os
    return timedelta(seconds=float(os.environ.get("REGNN_DIST_TIMEOUT", default_s)))


class Guard:
    """stage(what, fn, always=None) -> fn's result; see the module docstring.

    world: ranks in the default process group; device: where the agreement flag lives
    (the GPU for RCCL / "nccl", the CPU for gloo)."""

    def __init__(self, world=None, device=None):
        import torch.distributed as dist
        self.dist = dist
        on = dist.is_available() and dist.is_initialized()
        self.world = int(world if world is not None else (dist.get_world_size() if on else 1))
        if device is None:
            device = "cpu"
            if on and dist.get_backend() == "nccl":
                device = torch.device("cuda", torch.cuda.current_device())
        self.device = device

    def agree(self, ok, what="stage"):
        """True on every rank when ok holds on every rank; else RankFailure on every rank."""
        if self.world <= 1:
            return True
        try:
            flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=self.device)
            self.dist.all_reduce(flag, op=self.dist.ReduceOp.SUM)
            n_bad = int(flag.item())
        except Exception as e:               # noqa: BLE001 (a dead peer, a faulted device)
            rank = self.dist.get_rank() if self.dist.is_initialized() else -1
            print(f"[rank {rank}] the agreement after '{what}' failed: {e}", file=sys.stderr,
                  flush=True)
            raise RankFailure(what, -1, e) from e
        if n_bad:
            raise RankFailure(what, n_bad)
        return True

    def stage(self, what, fn, always=None):
        if self.world <= 1:
            out = fn()
            if always is not None:
                always()
            return out
        out, exc = None, None
        try:
            out = fn()
        except Exception as e:               # noqa: BLE001 (any failure ends the whole job)
            exc = e
            rank = self.dist.get_rank()
            print(f"[rank {rank}] stage '{what}' failed:", file=sys.stderr, flush=True)
            traceback.print_exc()
        if always is not None:
            # the peers issue these collectives in this stage: issue them too (the failed rank's
            # operands may be garbage; the agreement below discards the step on every rank)
            try:
                always()
            except Exception:                # noqa: BLE001
                exc = exc or RuntimeError(f"{what}: collective failed")
                traceback.print_exc()
        try:
            self.agree(exc is None, what)
        except RankFailure as rf:
            rf.local_exc = exc
            raise
        return out
