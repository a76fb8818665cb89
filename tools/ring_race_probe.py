"""Timing probe for tests/test_row_ring_gpu.py's race pattern: how long the
spin on stream L lasts, how long the host takes to enqueue the 255 ring-
advancing launches, and whether launches X (stream A) and Y (stream B) ran at
the same time (HIP timing events around each). Prints one JSON line.

    python tools/ring_race_probe.py [--fence 0|1] [--sleep CYCLES]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fence", type=int, default=1)
    ap.add_argument("--sleep", type=int, default=60_000_000)
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--prio", type=int, default=0, help="1: stream A at high priority (its own HW queue)")
    ap.add_argument("--cumask", type=int, default=1,
                    help="1: every stream from hipExtStreamCreateWithCUMask (a dedicated HW queue each)")
    a = ap.parse_args()
    import numpy as np
    import torch

    torch.cuda.init()
    os.environ["CMTV_ROW_FENCE"] = str(a.fence)
    from cometbft_amd import MODE_GO_STDLIB, Context
    from oracle import coracle
    from test_row_gpu import _batch

    ctx = Context(device=0)
    dev = torch.device("cuda:0")
    n = a.n
    jobs = []
    for j in range(2):
        pk, sig, m, off = _batch(n, 7000 + j, flip=0.3)
        exp = coracle.verify_batch(pk, sig, m, off, MODE_GO_STDLIB, nthreads=8)
        jobs.append([torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (pk, sig, m, off.view(np.int32))]
                    + [exp])
    pk1, sig1, m1, off1 = _batch(1, 7100, flip=0.0)
    tc = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (pk1, sig1, m1, off1.view(np.int32))]
    words = (n + 63) // 64
    bx = torch.full((words,), -1, dtype=torch.int64, device=dev)
    by = torch.full((words,), -1, dtype=torch.int64, device=dev)
    bc = torch.full((255,), -1, dtype=torch.int64, device=dev)
    if a.cumask:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from test_row_ring_gpu import hw_queue_streams

        sL, sA, sB, sC = hw_queue_streams(4)
    else:
        sL, sA, sB, sC = (torch.cuda.Stream(device=dev) for _ in range(4))
    if a.prio:
        sA = torch.cuda.Stream(device=dev, priority=-1)
    ev = {k: torch.cuda.Event(enable_timing=True) for k in ("l0", "l1", "xs", "xe", "ys", "ye")}
    torch.cuda.synchronize(dev)

    def launch(t, nn, bm_ptr, stream):
        ctx.verify_device(nn, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), MODE_GO_STDLIB,
                          0, bm_ptr, stream.cuda_stream)

    ev["l0"].record(sL)
    with torch.cuda.stream(sL):
        torch.cuda._sleep(a.sleep)
    ev["l1"].record(sL)
    sA.wait_event(ev["l1"])
    sB.wait_event(ev["l1"])
    ev["xs"].record(sA)
    t0 = time.perf_counter()
    launch(jobs[0], n, bx.data_ptr(), sA)
    ev["xe"].record(sA)
    for i in range(255):
        launch(tc, 1, bc.data_ptr() + 8 * i, sC)
    ev["ys"].record(sB)
    launch(jobs[1], n, by.data_ptr(), sB)
    ev["ye"].record(sB)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    el = lambda p, q: ev[p].elapsed_time(ev[q])  # noqa: E731
    want = lambda exp: np.pad(np.packbits(exp, bitorder="little"),  # noqa: E731
                              (0, 8 * words - (n + 7) // 8)).view(np.int64)
    out = {
        "fence": a.fence,
        "prio": a.prio,
        "cumask": a.cumask,
        "spin_ms": round(el("l0", "l1"), 3),
        "host_enqueue_ms": round(1e3 * t_enq, 3),
        "x_ms": round(el("xs", "xe"), 3),
        "y_ms": round(el("ys", "ye"), 3),
        "x_start_to_y_start_ms": round(el("xs", "ys"), 3),
        "spin_end_to_x_start_ms": round(el("l1", "xs"), 3),
        "x_ok": bool(np.array_equal(bx.cpu().numpy(), want(jobs[0][4]))),
        "y_ok": bool(np.array_equal(by.cpu().numpy(), want(jobs[1][4]))),
        "c_ok": bool((bc.cpu().numpy() == 1).all()),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
