"""Per-visit instruction budget of the per-lane walk's quantized inner-node visit (innerStepQ) in
k_trace<false, 1, 3> (the exact closest-hit walk), from the device assembly.

    python tools/isa_budget.py [kernel.s]      (default: compiles mrt_kernels.hip to /tmp)

The visit is located by its four 16-byte node loads (buffer_load_dwordx4 ... offset:48 follows
offset:0/16/32) and its 12 v_alignbit near/far rotations; the block from the rotations to the
stack pop of an empty visit is classified by opcode: box tests (alignbit, cvt, fma, min/max, cmp),
child ordering and pushes (cndmask, compares, LDS / spill stores), and control (exec-mask SALU)."""
import collections
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_asm(path, name="_ZN3mrt7k_traceILb0ELi1ELi3E"):
    lines, on = [], False
    for line in open(path):
        if line.startswith(name) and line.split(";")[0].rstrip().endswith(":"):
            on = True
        elif on and line.startswith(".Lfunc_end"):
            break
        if on:
            lines.append(line.rstrip("\n"))
    return lines


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/mrt_kernels.s"
    if len(sys.argv) == 1:
        csrc = os.path.join(HERE, "mobileraytracer_amd", "csrc")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                        "-I../../include", "-fno-slp-vectorize", "--cuda-device-only", "-S", "mrt_kernels.hip", "-o", path],
                       cwd=csrc, check=True, capture_output=True)
    asm = kernel_asm(path)
    # the visit: from the first v_alignbit after the node loads to the block that pops the stack
    first = next(i for i, l in enumerate(asm) if "v_alignbit_b32" in l)
    # up to the label of the empty-visit pop (v_bfrev_b32 ... -2: kRefDone) and its stack refill
    end = next(i for i in range(first, len(asm)) if "v_bfrev_b32" in asm[i])
    body = [l.strip() for l in asm[first:end] if l.strip() and not l.strip().startswith((";", "."))]
    ops = collections.Counter(l.split()[0] for l in body)
    cls = collections.Counter()
    for op, n in ops.items():
        if op.startswith("v_alignbit") or op.startswith("v_cvt") or op.startswith("v_fma") or re.match(r"v_(max|min)3?_f32", op):
            cls["box tests: " + op.split("_e")[0]] += n
        elif op.startswith("v_cmp"):
            cls["compares (hit tests, child order)"] += n
        elif op.startswith("v_cndmask") or op.startswith("v_addc"):
            cls["selects (child order, hit count)"] += n
        elif op.startswith("v_"):
            cls["other VALU (stack addressing, counters)"] += n
        elif op.startswith("ds_") or op.startswith("global_") or op.startswith("buffer_"):
            cls["memory (LDS stack, spill)"] += n
        else:
            cls["SALU / control"] += n
    valu = sum(n for op, n in ops.items() if op.startswith("v_"))
    print(f"k_trace<false, 1, 3> quantized 4-wide visit, {len(body)} instructions in the block, {valu} VALU "
          "(every path through the pushes counted: 1-3 pushes execute per visit)")
    for k, n in sorted(cls.items(), key=lambda kv: -kv[1]):
        print(f"  {n:4d}  {k}")


main()
