"""Opt-in per-phase tracing (SURVEY.md §5 "Tracing / profiling"): KNN_TRACE=1 prints
"[dmlp-trace] rank <r> <phase> <ms>" lines on stderr — never a line starting with "Time taken",
which run_bench.sh greps.  Phases are bracketed by a device synchronisation only when tracing is
on, so the untraced path keeps its asynchrony.  roctx ranges are emitted when available."""
from __future__ import annotations

import os
import sys
import time
from contextlib import contextmanager


class Tracer:
    def __init__(self, rank: int = 0, enabled: bool | None = None, sync=None):
        self.rank = rank
        self.enabled = (os.environ.get("KNN_TRACE", "0") not in ("", "0")) if enabled is None else enabled
        self.sync = sync
        self.records = []

    @contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        if self.sync:
            self.sync()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if self.sync:
                self.sync()
            ms = (time.perf_counter() - t0) * 1e3
            self.records.append((name, ms))
            print(f"[dmlp-trace] rank {self.rank} {name} {ms:.3f} ms", file=sys.stderr, flush=True)

    def summary(self):
        return {n: ms for n, ms in self.records}
