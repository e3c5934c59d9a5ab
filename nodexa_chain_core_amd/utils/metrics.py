"""Engine metrics: counters / gauges with labels, a JSON-lines log and Prometheus text.

Parity: the reference exposes mining telemetry only as `getmininginfo.hashespersec`
(nHashesDone / elapsed, src/miner.cpp:685-687, src/rpc/mining.cpp:209-250) and
`getnetworkhashps`; SURVEY §5 asks the new engine for per-GPU MH/s, shares/s,
stale rate, DAG build time and collective latency as a JSON-lines metrics log.

    m = metrics.REGISTRY
    m.inc("miner_hashes_total", n, device="gpu0")
    m.set("dag_build_seconds", 0.61, device="gpu0", epoch=384)
    metrics.JsonlWriter(path, interval_s=10).start()   # -metricslog=<path>

Rates are derived in `snapshot()` from the counter deltas between snapshots, so the
log carries both totals and per-interval rates (hashes/s, shares/s).
"""
from __future__ import annotations

import json
import threading
import time

Labels = tuple[tuple[str, str], ...]


def _labels(kw: dict) -> Labels:
    return tuple(sorted((k, str(v)) for k, v in kw.items()))


class Registry:
    def __init__(self) -> None:
        self._lock = threading.Lock()
        self._counters: dict[tuple[str, Labels], float] = {}
        self._gauges: dict[tuple[str, Labels], float] = {}
        self._last: tuple[float, dict[tuple[str, Labels], float]] = (time.time(), {})
        self.started = time.time()

    def inc(self, name: str, value: float = 1.0, **labels) -> None:
        k = (name, _labels(labels))
        with self._lock:
            self._counters[k] = self._counters.get(k, 0.0) + value

    def set(self, name: str, value: float, **labels) -> None:
        with self._lock:
            self._gauges[(name, _labels(labels))] = float(value)

    def counter(self, name: str, **labels) -> float:
        with self._lock:
            return self._counters.get((name, _labels(labels)), 0.0)

    def gauge(self, name: str, default: float | None = None, **labels) -> float | None:
        with self._lock:
            return self._gauges.get((name, _labels(labels)), default)

    def total(self, name: str) -> float:
        with self._lock:
            return sum(v for (n, _), v in self._counters.items() if n == name)

    def reset(self) -> None:
        with self._lock:
            self._counters.clear()
            self._gauges.clear()
            self._last = (time.time(), {})

    def snapshot(self) -> dict:
        """Totals, gauges and per-second rates since the previous snapshot."""
        now = time.time()
        with self._lock:
            t0, prev = self._last
            dt = max(now - t0, 1e-9)
            counters = dict(self._counters)
            gauges = dict(self._gauges)
            self._last = (now, counters)

        def fmt(d):
            return [{"name": n, "labels": dict(lb), "value": v} for (n, lb), v in sorted(d.items())]

        rates = [{"name": n + "_per_s", "labels": dict(lb), "value": (v - prev.get((n, lb), 0.0)) / dt}
                 for (n, lb), v in sorted(counters.items())]
        return {"time": now, "uptime_s": now - self.started, "interval_s": dt, "counters": fmt(counters),
                "gauges": fmt(gauges), "rates": rates}

    def prometheus(self) -> str:
        """Text exposition format (one sample per line)."""
        lines = []
        with self._lock:
            items = [(n, lb, v, "counter") for (n, lb), v in self._counters.items()] + \
                    [(n, lb, v, "gauge") for (n, lb), v in self._gauges.items()]
        seen = set()
        for n, lb, v, kind in sorted(items):
            name = "nodexa_" + n
            if name not in seen:
                lines.append(f"# TYPE {name} {kind}")
                seen.add(name)
            lab = ",".join(f'{k}="{val}"' for k, val in lb)
            lines.append(f"{name}{{{lab}}} {v}" if lab else f"{name} {v}")
        return "\n".join(lines) + "\n"


REGISTRY = Registry()


class JsonlWriter:
    """Appends one `REGISTRY.snapshot()` per interval to a JSON-lines file (-metricslog)."""

    def __init__(self, path: str, interval_s: float = 10.0, registry: Registry | None = None):
        self.path, self.interval = path, float(interval_s)
        self.registry = registry or REGISTRY
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def write_once(self) -> dict:
        snap = self.registry.snapshot()
        with open(self.path, "a") as f:
            f.write(json.dumps(snap) + "\n")
        return snap

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            try:
                self.write_once()
            except OSError:
                pass

    def start(self) -> "JsonlWriter":
        self._thread = threading.Thread(target=self._run, name="metrics-log", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
        try:
            self.write_once()  # final snapshot on shutdown
        except OSError:
            pass
