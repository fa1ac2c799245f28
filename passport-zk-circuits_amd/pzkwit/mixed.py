"""Mixed verification-flow batches.

Real passport batches mix signature flows: RSA-2048 (SIGNATURE_TYPE 1), RSA-4096 (2) and ECDSA
secp256r1 (20) documents arrive interleaved. Each flow is a different RegisterIdentityBuilder
instance (different witness layout and size), so a mixed batch is

  * grouped by instance parameters (one `native.Instance` per distinct parameter set), every
    group run as one device batch, results returned in the caller's order;
  * sharded across ranks by COST, not by count: the path is HBM-write-bound, so a witness
    costs its .wtns bytes (ECDSA 176 MB, RSA-4096 ~97 MB, RSA-2048 72 MB at the canonical
    shifts). `shard_by_cost` gives each rank a contiguous run of the batch whose total bytes
    are within one witness of the even split, so 8 GPUs finish together.

The reference runs each passport through its own compiled circuit in a serial loop
(test/automatisationTest.js:24-51); there is no mixing logic to mirror beyond picking the circuit
from the passport's signature type (test/process_passport.js:157-240).
"""
import numpy as np

from . import native


def params_key(params):
    return tuple(sorted(params.items()))


def witness_cost(params, _cache={}):
    """Bytes one witness of `params` writes (.wtns body), from the host layout (no device)."""
    k = params_key(params)
    if k not in _cache:
        _cache[k] = 32 * native.layout_witness_size(params)
    return _cache[k]


def shard_by_cost(costs, world, rank):
    """Contiguous shard [lo, hi) of items with per-item `costs` for `rank`: boundaries at the item
    whose cumulative cost first reaches r/world of the total (so every shard is within one item's
    cost of the even split, and shards tile the batch in order)."""
    c = np.cumsum(np.asarray(costs, dtype=np.float64))
    total = c[-1] if len(c) else 0.0

    def bound(r):
        if r <= 0:
            return 0
        if r >= world:
            return len(costs)
        return int(np.searchsorted(c, total * r / world, side="left")) + 1 if total else 0

    lo, hi = bound(rank), bound(rank + 1)
    return min(lo, hi), hi


class MixedBatch:
    """Runs a list of (params, input_row) items, grouped per instance. `instances` are created on
    first use and reused across calls; a call creates every instance its items need before it runs
    any of them, so the library sees the whole set of register instances sharing the device when it
    picks their stream sets (runtime.cpp ensure_chain_streams)."""

    def __init__(self):
        self.instances = {}

    def instance(self, params):
        k = params_key(params)
        if k not in self.instances:
            self.instances[k] = native.Instance(native.PZK_CIRCUIT_REGISTER, 0, params)
        return self.instances[k]

    def run_host(self, items):
        """items: [(params, row (nIn, 32) uint8)]. Returns ([witness (nW, 32) uint8], status int32[n]),
        in item order."""
        groups = {}
        for i, (prm, row) in enumerate(items):
            groups.setdefault(params_key(prm), (prm, []))[1].append(i)
        wits = [None] * len(items)
        status = np.zeros(len(items), dtype=np.int32)
        for prm, _ in groups.values():
            self.instance(prm)
        for prm, idx in groups.values():
            inst = self.instance(prm)
            rows = np.stack([items[i][1] for i in idx])
            w, st = inst.witness_batch_host(rows)
            for k, i in enumerate(idx):
                wits[i] = w[k]
                status[i] = st[k]
        return wits, status
