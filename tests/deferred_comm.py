"""A transport for the sharded multiply whose transfers complete only at wait() (tests only).

sharded.TorchComm over gloo on CPU tensors finishes a batch of sends and receives almost at
once, so on the CPU a stage that runs before its exchange has landed -- or that overwrites a
buffer still being sent -- reads the right bytes anyway, and the overlapped orderings of
sharded.ShardedMul.run (exchange #1 beside operand 2's column passes, exchange #2 beside the
next row chunk) degenerate to synchronous ones.  RCCL on GPUs does not: its transfers run on
the communicator's stream while the rank's own stream goes on computing.

DeferredComm makes the hazard visible on the CPU:
  * exchange(wait=False) snapshots every send view and fills every receive view with a
    poison pattern (a stage reading it before wait() computes garbage -> wrong product);
  * wait() first checks that no send view changed since the exchange was issued (raises
    SendOverwritten: the compute wrote into bytes still in flight), then moves the
    snapshots through the real gloo exchange into the receive views (a stage that wrote a
    receive view early has its bytes overwritten -> wrong product).
Ranks issue and wait their exchanges in the same program order, so the deferred gloo
batches pair up across ranks exactly as the immediate ones would.
"""
import torch


class SendOverwritten(RuntimeError):
    pass


def _aliases(a, b):
    return a.numel() and b.numel() and a.data_ptr() == b.data_ptr() and a.numel() == b.numel()


class _Pending:
    def __init__(self, items):
        self.items = items      # [(snapshots, live send views, receive views)]


class DeferredComm:
    def __init__(self, inner):
        self.inner = inner      # sharded.TorchComm (gloo)
        self.issued = 0         # exchanges issued with wait=False (the tests check the async paths ran)

    def exchange(self, plan, wait=True):
        items = []
        for send, recv in plan:
            snaps = [s.clone() for s in send]
            for d, r in enumerate(recv):
                if r.numel() and not any(_aliases(r, s) for s in send):
                    r.view(torch.uint8).fill_(0x5A)   # (any dtype: every byte 0x5A)
            items.append((snaps, list(send), list(recv)))
        tok = _Pending(items)
        if wait:
            self.wait([tok])
            return []
        self.issued += 1
        return [tok]

    def wait(self, toks):
        for tok in toks:
            for snaps, live, _ in tok.items:
                for a, b in zip(snaps, live):
                    if not torch.equal(a, b):
                        raise SendOverwritten("a send buffer changed while its transfer was in flight")
            self.inner.exchange([(snaps, recv) for snaps, _, recv in tok.items], wait=True)

    def all_gather(self, t):
        return self.inner.all_gather(t)
