"""Prometheus exposition of a verifier context's counters (cmtv_stats).

CometBFT publishes its node metrics through Prometheus with a namespace and a
per-package subsystem (consensus/metrics.go:16-18, 100-110: namespace
"cometbft", subsystem "consensus"). The verifier follows the same scheme with
subsystem "cmtverify", so a node that binds libcmtverify can register one
collector next to its own and scrape both from the same endpoint:

    from prometheus_client import REGISTRY
    from cometbft_amd.metrics import StatsCollector
    REGISTRY.register(StatsCollector(ctx, labels={"chain_id": "..."}))

The collector reads cmtv_stats at scrape time (one C call, no polling
thread). Counters follow Prometheus naming (`_total`; seconds, not ms).
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

from prometheus_client import CollectorRegistry, generate_latest
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily

NAMESPACE = "cometbft"
SUBSYSTEM = "cmtverify"

# cmtv_stats field -> (metric suffix, kind, help)
_FIELDS = [
    ("calls", "calls_total", "counter", "Verification calls served by the context."),
    ("signatures", "signatures_total", "counter", "Signatures verified."),
    ("invalid", "invalid_signatures_total", "counter", "Signatures rejected."),
    ("kernel_launches", "kernel_launches_total", "counter", "Verification kernel launches."),
    ("keyed_launches", "keyed_launches_total", "counter", "Launches of the registered-key kernels."),
    ("cache_hits", "verdict_cache_hits_total", "counter", "Verdicts served by the verdict cache."),
    ("sharded_calls", "sharded_calls_total", "counter", "Batches split over more than one device."),
    ("gathers", "bitmap_gathers_total", "counter", "Verdict-bitmap all-gathers (RCCL or peer copy)."),
    ("faults_injected", "faults_injected_total", "counter", "Launches failed by the CMTV_FAULT_AT knob."),
    ("device_failures", "device_failures_total", "counter", "Devices retired after a HIP error."),
    ("reshards", "reshards_total", "counter", "Host batches re-planned over the remaining devices."),
    ("late_k_waves", "late_k_waves_total", "counter",
     "Keyed split-kernel waves that hashed their own signatures instead of waiting for the helper."),
    ("fused_sign_bytes", "fused_sign_bytes_total", "counter",
     "Templated batches whose sign-bytes the verify kernel's helper wave wrote."),
    ("cache_entries", "verdict_cache_entries", "gauge", "Verdicts currently cached."),
    ("n_devices", "devices", "gauge", "Devices driven by the context."),
    ("rccl", "rccl", "gauge", "1 when bitmap gathers run over an RCCL communicator."),
    ("live_devices", "live_devices", "gauge", "Devices still taking work."),
    ("timed_calls", "timed_calls_total", "counter",
     "Calls whose kernel time device_seconds holds (CMTV_TIMING samples one call in N per device)."),
    ("rccl_failures", "rccl_failures_total", "counter",
     "RCCL bitmap all-gathers that failed and fell back to peer copies."),
    ("polled_calls", "polled_calls_total", "counter",
     "Small host batches read off the row kernel's completion flag (no stream synchronisation)."),
]


def _name(suffix: str) -> str:
    return f"{NAMESPACE}_{SUBSYSTEM}_{suffix}"


class StatsCollector:
    """A prometheus_client collector over one Context (cometbft_amd.Context)."""

    def __init__(self, ctx, labels: Optional[Dict[str, str]] = None):
        self._ctx = ctx
        self._labels = dict(labels or {})

    def describe(self) -> Iterable:
        return []  # unchecked collector: families are produced at collect time

    def collect(self) -> Iterable:
        st = self._ctx.stats()
        keys = sorted(self._labels)
        vals = [self._labels[k] for k in keys]
        for field, suffix, kind, doc in _FIELDS:
            fam = (CounterMetricFamily if kind == "counter" else GaugeMetricFamily)(
                _name(suffix[:-6] if kind == "counter" else suffix), doc, labels=keys)
            fam.add_metric(vals, float(st[field]))
            yield fam
        dev = CounterMetricFamily(_name("device_seconds"),
                                  "Summed kernel time of the timed calls (HIP events); mean kernel time = "
                                  "device_seconds / timed_calls.", labels=keys)
        dev.add_metric(vals, st["device_ms"] / 1e3)
        yield dev
        last = GaugeMetricFamily(_name("last_kernel_seconds"), "Kernel time of the most recent timed call.",
                                 labels=keys)
        last.add_metric(vals, st["last_kernel_ms"] / 1e3)
        yield last


def exposition(ctx, labels: Optional[Dict[str, str]] = None) -> bytes:
    """The context's metrics in the Prometheus text format (one scrape)."""
    reg = CollectorRegistry()
    reg.register(StatsCollector(ctx, labels))
    return generate_latest(reg)
