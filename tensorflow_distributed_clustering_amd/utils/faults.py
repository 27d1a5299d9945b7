"""Fault injection for the failure-handling paths.

``TDC_FAULT`` is a comma list of ``kind@when[:rank]``:

* ``crash@N``      raise :class:`InjectedFault` after iteration N completes
* ``oom@setup``    raise an out-of-memory error while the engine is being built
* ``oom@N``        raise an out-of-memory error inside iteration N's local step (the
                   engines flag it in the all-reduce buffer, every rank rolls back to the
                   centroids before the step and continues streamed)

``:rank`` restricts the fault to one rank (default: every rank).  Each entry fires at
most once per process, so a retry after an injected setup OOM goes through.
"""
from __future__ import annotations

import os
from typing import Set

import torch


class InjectedFault(RuntimeError):
    pass


_FIRED: Set[str] = set()


def _entries():
    spec = os.environ.get("TDC_FAULT", "").strip()
    for e in filter(None, (x.strip() for x in spec.split(","))):
        kind, _, rest = e.partition("@")
        when, _, rank = rest.partition(":")
        yield e, kind, when, (int(rank) if rank else None)


def oom_error(msg: str):
    cls = getattr(torch.cuda, "OutOfMemoryError", None) or getattr(torch, "OutOfMemoryError", RuntimeError)
    return cls(msg)


def maybe_fail(when: str, rank: int = 0, kinds=("crash", "oom")) -> None:
    for e, kind, w, r in _entries():
        if w != str(when) or (r is not None and r != rank) or e in _FIRED or kind not in kinds:
            continue
        _FIRED.add(e)
        if kind == "crash":
            raise InjectedFault(f"injected crash ({e})")
        if kind == "oom":
            raise oom_error(f"injected out of memory ({e})")


def is_oom(exc: BaseException) -> bool:
    cls = getattr(torch.cuda, "OutOfMemoryError", None)
    if cls is not None and isinstance(exc, cls):
        return True
    return isinstance(exc, RuntimeError) and "out of memory" in str(exc).lower()
