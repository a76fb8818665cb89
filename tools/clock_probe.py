"""Does the configs[1] kernel time depend on how long the GPU has been busy?
Runs the bench step (bench.Devices) in GO / ZIP-215 blocks of 50, then a long
GO block, printing the mean kernel ms of each (libcmtverify HIP events)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from cometbft_amd import Context  # noqa: E402

torch.cuda.set_device(0)  # torch initialises HIP before the library does (as bench.main)
ctx = Context(devices=[0])
D = bench.Devices(ctx, 1, 10_000)
for label, mode, steps in [("go", 0, 50), ("zip", 1, 50), ("go", 0, 50), ("zip", 1, 50), ("go", 0, 50),
                           ("go-long", 0, 2000), ("go", 0, 50), ("zip", 1, 50)]:
    el, kms = bench.timed_steps(ctx, lambda: D.step(ctx, mode), steps, 2, lambda: None)
    print(f"{label:8s} steps={steps:5d} kernel_ms={kms:.4f} ms_per_step={el / steps * 1e3:.4f}", flush=True)
time.sleep(1.0)
el, kms = bench.timed_steps(ctx, lambda: D.step(ctx, 0), 50, 2, lambda: None)
print(f"go-after-1s-idle kernel_ms={kms:.4f} ms_per_step={el / 50 * 1e3:.4f}", flush=True)
