"""Tiny thread-safe Prometheus-style metrics registry (counters + latency summaries)."""
from __future__ import annotations

import threading


def _lbl(labels: dict | None) -> str:
    if not labels:
        return ""
    return "{" + ",".join(f'{k}="{v}"' for k, v in sorted(labels.items())) + "}"


class Metrics:
    def __init__(self):
        self._lock = threading.Lock()
        self.counters: dict = {}
        self.sums: dict = {}
        self.samples: dict = {}

    def inc(self, name: str, labels: dict | None = None, v: float = 1.0):
        k = (name, _lbl(labels))
        with self._lock:
            self.counters[k] = self.counters.get(k, 0.0) + v

    def observe(self, name: str, value: float, labels: dict | None = None):
        k = (name, _lbl(labels))
        with self._lock:
            s = self.sums.setdefault(k, [0, 0.0])
            s[0] += 1
            s[1] += value
            buf = self.samples.setdefault(k, [])
            buf.append(value)
            if len(buf) > 2048:
                del buf[:1024]

    def quantile(self, name: str, q: float, labels: dict | None = None) -> float | None:
        buf = sorted(self.samples.get((name, _lbl(labels)), []))
        if not buf:
            return None
        return buf[min(len(buf) - 1, int(q * len(buf)))]

    def render(self) -> str:
        lines = []
        with self._lock:
            for (n, l), v in sorted(self.counters.items()):
                lines.append(f"{n}{l} {v}")
            for (n, l), (c, s) in sorted(self.sums.items()):
                lines.append(f"{n}_count{l} {c}")
                lines.append(f"{n}_sum{l} {s}")
                buf = sorted(self.samples[(n, l)])
                for q in (0.5, 0.99):
                    qv = buf[min(len(buf) - 1, int(q * len(buf)))]
                    ql = l[:-1] + f',quantile="{q}"' + "}" if l else f'{{quantile="{q}"}}'
                    lines.append(f"{n}{ql} {qv}")
        return "\n".join(lines) + "\n"


METRICS = Metrics()
