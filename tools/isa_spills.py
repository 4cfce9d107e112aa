"""Where a kernel's scratch spills sit: compiles mrt_kernels.hip (extra -D flags from argv) to
device assembly and prints, for each named kernel, its scratch instructions with the nearest
preceding label and whether they fall in the wave-spread triangle tests (the ds_permute /
ds_bpermute region).   usage: python tools/isa_spills.py [-DNAME=V ...]"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("_ZN3mrt7k_traceILb0ELi1ELi3E", "_ZN3mrt8k_shadowILb0ELi1ELi3E")


def main():
    csrc = os.path.join(HERE, "mobileraytracer_amd", "csrc")
    out = "/tmp/mrt_kernels_spills.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                    "-I../../include", "-fno-slp-vectorize", "--cuda-device-only", "-S", "mrt_kernels.hip", "-o", out]
                   + sys.argv[1:], cwd=csrc, check=True, capture_output=True)
    lines = open(out).read().split("\n")
    for name in KERNELS:
        body, on = [], False
        for l in lines:
            if l.startswith(name) and l.split(";")[0].rstrip().endswith(":"):
                on = True
            elif on and l.startswith(".Lfunc_end"):
                break
            if on:
                body.append(l)
        perm = [i for i, l in enumerate(body) if re.search(r"\bds_b?permute", l)]
        lo, hi = (min(perm), max(perm)) if perm else (-1, -1)
        sc = [i for i, l in enumerate(body) if "scratch_" in l]
        inside = sum(1 for i in sc if lo <= i <= hi)
        print(f"{name}: {len(body)} lines, {len(perm)} permutes, {len(sc)} scratch ops ({inside} inside the permute region)")
        for i in sc:
            lab = next((body[j].split(":")[0] for j in range(i, -1, -1) if re.match(r"^\.LBB", body[j])), "?")
            print(f"  {i:6d} {lab:14s} {body[i].strip()[:70]}")


if __name__ == "__main__":
    main()
