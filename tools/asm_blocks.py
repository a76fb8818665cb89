"""Static instruction census of one kernel in a gfx950 assembly listing.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o k.s kernels.hip
  python tools/asm_blocks.py k.s k_verify_quad [--top 25]

Splits the kernel body into basic blocks (labels), counts VALU / SALU / LDS /
VMEM / DPP / s_waitcnt / s_nop instructions per block and marks the blocks
that end in a backward branch (loop latches) with their loop extent, so a
loop body's per-iteration instruction count can be read off directly.
"""
import re
import sys
from collections import Counter


def kernel_lines(path, name):
    lines, inside = [], False
    with open(path) as f:
        for ln in f:
            if not inside and re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", ln):
                inside = True
                lines.append(ln.rstrip())
                continue
            if inside:
                if ln.startswith(".Lfunc_end"):
                    break
                lines.append(ln.rstrip())
    return lines


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op == "s_waitcnt":
        return "wait"
    if op == "s_nop":
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    lines = kernel_lines(path, name)
    if not lines:
        sys.exit(f"kernel {name} not found")
    blocks, order, cur = {}, [], "entry"
    blocks[cur] = Counter()
    order.append(cur)
    branches = {}
    for ln in lines[1:]:
        s = ln.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            cur = m.group(1)
            blocks[cur] = Counter()
            order.append(cur)
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        c = blocks[cur]
        c[classify(op)] += 1
        if "dpp" in s or "quad_perm" in s or "row_" in s:
            c["dpp"] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            branches.setdefault(cur, []).append(tgt)
    pos = {b: i for i, b in enumerate(order)}
    total = Counter()
    for c in blocks.values():
        total.update(c)
    print(f"{name}: {len(order)} blocks; static totals: " + ", ".join(f"{k}={v}" for k, v in sorted(total.items())))
    loops = []
    for b, tg in branches.items():
        for t in tg:
            if t in pos and pos[t] <= pos[b]:
                body = Counter()
                for x in order[pos[t]: pos[b] + 1]:
                    body.update(blocks[x])
                loops.append((body["valu"], t, b, body))
    print("\nloops (backward branches): valu per iteration, extent")
    for v, t, b, body in sorted(loops, reverse=True)[:top]:
        print(f"  {v:6d} valu  {t} .. {b}  ({pos[b] - pos[t] + 1} blocks)  "
              + " ".join(f"{k}={body[k]}" for k in ("salu", "lds", "vmem", "dpp", "wait", "nop")))
    print("\nlargest blocks:")
    for b in sorted(order, key=lambda x: -blocks[x]["valu"])[:top]:
        c = blocks[b]
        print(f"  {c['valu']:6d} valu  {b}  " + " ".join(f"{k}={c[k]}" for k in ("salu", "lds", "vmem", "dpp", "wait", "nop")))


if __name__ == "__main__":
    main()
