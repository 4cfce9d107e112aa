"""Instruction mix of one loop of a kernel's device assembly: every basic block whose comment names
the loop header ("in Loop: Header=BBx_y", or the header itself), counted once per block.
    python tools/loop_mix.py <asm.s> <kernel symbol prefix> [header label, e.g. BB20_180]
Without a label: the innermost loop around the kernel's first 16-byte load at offset 48 (the
walk-tree node's last quarter, i.e. the per-lane walk's inner-node visit)."""
import re
import collections
import sys


def main():
    path, name = sys.argv[1:3]
    header = sys.argv[3] if len(sys.argv) > 3 else None
    lines = open(path).read().split("\n")
    body, on = [], False
    for l in lines:
        if l.startswith(name) and l.split(";")[0].rstrip().endswith(":"):
            on = True
        elif on and l.startswith(".Lfunc_end"):
            break
        if on:
            body.append(l)
    if header is None:
        at = next(i for i, l in enumerate(body) if "buffer_load_dwordx4" in l and "offset:48" in l)
        for j in range(at, -1, -1):
            m = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", body[j])
            if m:
                header = m.group(1)
                break
            if body[j].startswith(".LBB") and "Loop Header" in (body[j] + body[j + 1]):
                header = body[j].split(":")[0][1:]
                break
        print("loop", header)
    inloop, c = False, collections.Counter()
    for i, l in enumerate(body):
        s = l.strip()
        if s.startswith(".LBB") or s.startswith("; %bb."):
            nxt = l + (body[i + 1] if i + 1 < len(body) else "")
            inloop = ("Header=" + header) in nxt or (s.startswith("." + header + ":"))
            continue
        if not inloop or not s or s.startswith(";"):
            continue
        c[s.split()[0]] += 1
    print("instructions", sum(c.values()))
    for k, v in c.most_common(80):
        print(f"{k:30s}{v}")


if __name__ == "__main__":
    main()
