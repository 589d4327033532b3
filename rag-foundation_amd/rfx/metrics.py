"""Call counters/latency in the reference's shape (gemini_api_calls_total{operation,status},
gemini_api_latency_seconds{operation}, backend/app/metrics.py:6-7).  The host app can hand its
own prometheus objects to set_metrics(); by default a private registry is used so importing this
package never collides with the app's metric names."""
import time
from contextlib import contextmanager

_calls = None
_latency = None


def _default():
    global _calls, _latency
    if _calls is None:
        try:
            from prometheus_client import CollectorRegistry, Counter, Histogram
            reg = CollectorRegistry()
            _calls = Counter("gemini_api_calls_total", "rfx adapter calls", ["operation", "status"], registry=reg)
            _latency = Histogram("gemini_api_latency_seconds", "rfx adapter latency", ["operation"], registry=reg)
        except Exception:  # prometheus_client missing: metrics become no-ops
            _calls, _latency = False, False
    return _calls, _latency


def set_metrics(calls_total, latency) -> None:
    global _calls, _latency
    _calls, _latency = calls_total, latency


@contextmanager
def observe(operation: str):
    calls, lat = _default()
    start = time.perf_counter()
    status = "ok"
    try:
        yield
    except Exception:
        status = "error"
        raise
    finally:
        if calls:
            calls.labels(operation, status).inc()
        if lat:
            lat.labels(operation).observe(time.perf_counter() - start)
