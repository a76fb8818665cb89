"""cometbft_amd.metrics: the Prometheus exposition of cmtv_stats (SURVEY 5
metrics; consensus/metrics.go naming). CPU: a stand-in context object; GPU:
a real context after a verification."""
import numpy as np
import pytest

from cometbft_amd import metrics as M


class _FakeCtx:
    def __init__(self, **kw):
        base = {k: 0 for k in ("calls", "signatures", "invalid", "kernel_launches", "cache_hits", "cache_entries",
                               "keyed_launches", "sharded_calls", "gathers", "faults_injected", "n_devices",
                               "rccl", "fused_sign_bytes", "device_failures", "reshards", "late_k_waves",
                               "live_devices", "timed_calls", "rccl_failures", "polled_calls")}
        base.update(device_ms=0.0, last_kernel_ms=0.0)
        base.update(kw)
        self._st = base

    def stats(self):
        return dict(self._st)


def _parse(text):
    out = {}
    for line in text.decode().splitlines():
        if line and not line.startswith("#"):
            name, val = line.rsplit(" ", 1)
            out[name] = float(val)
    return out


def test_exposition_names_and_units():
    ctx = _FakeCtx(calls=3, signatures=450, invalid=2, device_ms=1.5, last_kernel_ms=0.25, n_devices=2, rccl=1)
    got = _parse(M.exposition(ctx, labels={"chain_id": "test-chain"}))
    lab = '{chain_id="test-chain"}'
    assert got["cometbft_cmtverify_calls_total" + lab] == 3
    assert got["cometbft_cmtverify_signatures_total" + lab] == 450
    assert got["cometbft_cmtverify_invalid_signatures_total" + lab] == 2
    assert got["cometbft_cmtverify_device_seconds_total" + lab] == pytest.approx(1.5e-3)
    assert got["cometbft_cmtverify_last_kernel_seconds" + lab] == pytest.approx(2.5e-4)
    assert got["cometbft_cmtverify_devices" + lab] == 2
    assert got["cometbft_cmtverify_rccl" + lab] == 1


def test_collector_reads_at_scrape_time():
    from prometheus_client import CollectorRegistry, generate_latest

    ctx = _FakeCtx(signatures=1)
    reg = CollectorRegistry()
    reg.register(M.StatsCollector(ctx))
    assert _parse(generate_latest(reg))["cometbft_cmtverify_signatures_total"] == 1
    ctx._st["signatures"] = 7
    assert _parse(generate_latest(reg))["cometbft_cmtverify_signatures_total"] == 7


@pytest.mark.gpu
def test_exposition_of_a_device_context(gpu_ctx, corpus):
    from cometbft_amd import MODE_GO_STDLIB, pack_messages

    before = _parse(M.exposition(gpu_ctx))
    msg, off = pack_messages(corpus["msgs"])
    got = gpu_ctx.verify(corpus["pk"], corpus["sig"], msg, off, MODE_GO_STDLIB)
    after = _parse(M.exposition(gpu_ctx))
    n = len(corpus["msgs"])
    assert after["cometbft_cmtverify_signatures_total"] - before["cometbft_cmtverify_signatures_total"] == n
    assert (after["cometbft_cmtverify_invalid_signatures_total"]
            - before["cometbft_cmtverify_invalid_signatures_total"]) == int(n - np.asarray(got).sum())
    # kernel time is sampled (CMTV_TIMING: one call in 16 per device by default)
    for _ in range(16):
        gpu_ctx.verify(corpus["pk"], corpus["sig"], msg, off, MODE_GO_STDLIB)
    after = _parse(M.exposition(gpu_ctx))
    assert after["cometbft_cmtverify_timed_calls_total"] > before["cometbft_cmtverify_timed_calls_total"]
    assert after["cometbft_cmtverify_device_seconds_total"] > before["cometbft_cmtverify_device_seconds_total"]
