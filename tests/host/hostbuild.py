"""Compile a tests/host checker once, race-free under pytest-xdist.

The binary is rebuilt when it is older than its source or any device header
(cometbft_amd/csrc/*.h, which the checkers include). It is written beside the
target and renamed over it, so a concurrent worker never executes a
half-written file (ETXTBSY)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(src, binary, flags):
    os.makedirs(os.path.dirname(binary), exist_ok=True)
    hdr = os.path.join(ROOT, "cometbft_amd", "csrc")
    deps = [src] + [os.path.join(hdr, f) for f in os.listdir(hdr) if f.endswith(".h")]
    if not os.path.exists(binary) or os.path.getmtime(binary) < max(os.path.getmtime(d) for d in deps):
        tmp = f"{binary}.{os.getpid()}"
        subprocess.run(["g++", "-O2"] + list(flags) + ["-o", tmp, src], check=True)
        os.replace(tmp, binary)
    return binary
