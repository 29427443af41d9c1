"""Launch plans: record the C-ABI launch sequence of a fixed-shape GPU region once, replay it
without the Python layer logic.

The relay sampler (2 x UNet + control: ~900 launches, many of them short at the 8x8..32x32 UNet
levels) and the VAE decoder are a fixed sequence of librdeic_hip launches for a given batch
shape. Eagerly, each launch pays ~20-30 us of Python (descriptor building, shape checks, tensor
allocation); the short UNet kernels then leave the GPU waiting on the host. A LaunchPlan runs
the region once eagerly (autotuning, weight packing, workspaces), then once more recording every
`_lib.call` (the function pointer and its already-converted ctypes arguments) while all tensors
of the region are allocated from a private torch MemPool, so the recorded device pointers stay
valid and unshared. replay() re-issues the recorded calls on the same stream: ~2 us of host time
per launch, no allocation. Unlike a captured hipGraph, each launch stays an ordinary stream
launch, so bench.py's HIP events still bracket every conv / attention / GroupNorm kernel (ROCm's
torch refuses timing events inside graph capture: tools/probe/graph_events.py).

Requirements on a recorded region: every GPU operation goes through `_lib.call` (no torch
kernels: constants are prepared outside), fixed shapes, and host work (coder round trips,
pinned copies, event waits) only inside `host_step`, which runs it and records it at its place
in the sequence: the entropy coder's compress / decompress regions interleave launches with
host steps. tests/test_plan_gpu.py checks replay == eager bit for bit.
"""
from __future__ import annotations

import weakref

import torch

from . import _lib, ops

# MemPool lifetime. A plan's pool must outlive every tensor allocated from it: returning a block to
# a destroyed pool aborts inside the caching allocator (a noexcept path, so SIGABRT). Models, plans
# and their tensors form reference cycles, so the cyclic GC frees them in arbitrary order and at
# arbitrary points (it once ran inside another plan's recording). Pools are therefore owned by this
# registry, not by the plan, and are destroyed only by _sweep_pools() (called when a new plan is
# made, never inside a pool context) once their plan is gone and no block of theirs is allocated.
_POOLS: list = []  # [(weakref to LaunchPlan, MemPool)]


def _pool_in_use(pool) -> bool:
    return any(seg["allocated_size"] for seg in torch.cuda.memory_snapshot(pool.id))


def _sweep_pools() -> None:
    keep = [(ref, pool) for ref, pool in _POOLS if ref() is not None or _pool_in_use(pool)]
    _POOLS[:] = keep  # the dropped pools are destroyed here, with no pool routing allocations


class _HostStep:
    __slots__ = ("fn",)

    def __init__(self, fn):
        self.fn = fn

    def __call__(self):
        self.fn()
        return 0


def host_step(fn) -> None:
    """Run a host-side step now; inside a recording, also append it to the plan so replay() runs
    it at the same point of the launch sequence. Library calls made by the step itself (the
    rANS coders) belong to the step and are not recorded as launches."""
    rec = _lib.RECORDER
    if rec is not None:
        rec.append(("<host>", _HostStep(fn), (), None))
    _lib.RECORDER = None
    try:
        fn()
    finally:
        _lib.RECORDER = rec


class LaunchPlan:
    def __init__(self):
        self.calls = []
        _sweep_pools()
        self.pool = torch.cuda.MemPool()
        _POOLS.append((weakref.ref(self), self.pool))
        self.out = None

    def record(self, fn, *args):
        with torch.cuda.use_mem_pool(self.pool):
            prev, _lib.RECORDER = _lib.RECORDER, self.calls
            try:
                self.out = fn(*args)
            finally:
                _lib.RECORDER = prev
        return self.out

    def replay(self):
        prof = ops.PROFILE
        for name, fn, args, tag in self.calls:
            if prof is not None and tag is not None:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                ev0.record()
                rc = fn(*args)
                ev1.record()
                ops.record_profile(tag, ev0, ev1)
            else:
                rc = fn(*args)
            if rc:
                _lib.check(name, rc)
        return self.out

    def __len__(self):
        return len(self.calls)


class PlanCache:
    """key -> (plan, static inputs). run() copies the inputs into the plan's static tensors and
    replays; the first call for a key warms up eagerly and records."""

    def __init__(self):
        self.plans = {}

    def run(self, key, fn, inputs, before=None):
        """before(): resets per-call host state (e.g. reopens the rANS decoders) ahead of each
        execution of the region: the warm-up, the recording and every replay."""
        ent = self.plans.get(key)
        if ent is None:
            statics = [t.clone() for t in inputs]
            if before is not None:
                before()
            fn(*statics)  # eager warm-up: autotune caches, packed weights, split-K workspace
            plan = LaunchPlan()
            if before is not None:
                before()
            out = plan.record(fn, *statics)
            self.plans[key] = (plan, statics, ops.stream_ptr())
            return out
        plan, statics, stream = ent
        if stream != ops.stream_ptr():
            # the recorded launches (and the events of its host steps) are bound to that stream
            raise RuntimeError("launch plan replayed on a different stream than it was recorded on: "
                               "use one RDEIC.session() per stream")
        if before is not None:
            before()
        for s, t in zip(statics, inputs):
            if s.data_ptr() != t.data_ptr():
                s.copy_(t)
        return plan.replay()

    def clear(self):
        self.plans.clear()
